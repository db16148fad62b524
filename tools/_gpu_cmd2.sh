set -o pipefail
T=r1r
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for ns in "" 1; do
  touch generic-ebpf_amd/csrc/asm/gen_interp.py
  EBPF_ASM_NOSTORE=$ns make -s -C generic-ebpf_amd > gpurun_out/$T/make.log 2>&1 || exit 1
  for cfg in c0 c4; do
    timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline > gpurun_out/$T/bench_${cfg}_$ns.json 2> gpurun_out/$T/bench.err || { tail -5 gpurun_out/$T/bench.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" gpurun_out/$T/bench_${cfg}_$ns.json "nostore=$ns $cfg"
  done
done
touch generic-ebpf_amd/csrc/asm/gen_interp.py
make -s -C generic-ebpf_amd > gpurun_out/$T/make.log 2>&1
