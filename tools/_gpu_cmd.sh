set -o pipefail
T=r1k
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
python3 -c "import __graft_entry__ as g; g.build()" > gpurun_out/$T/build.log 2>&1 || { tail -20 gpurun_out/$T/build.log; exit 1; }
for nt in 0 1 2 3 0; do
  touch generic-ebpf_amd/csrc/asm/gen_interp.py
  EBPF_ASM_NT=$nt make -s -C generic-ebpf_amd > gpurun_out/$T/make_$nt.log 2>&1 || exit 1
  for cfg in c0 c4 c3; do
    timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline > gpurun_out/$T/bench_${cfg}_$nt.json 2> gpurun_out/$T/bench_$cfg.err || { tail -5 gpurun_out/$T/bench_$cfg.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" gpurun_out/$T/bench_${cfg}_$nt.json "nt=$nt $cfg"
  done
done
