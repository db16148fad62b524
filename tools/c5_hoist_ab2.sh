set -o pipefail
mkdir -p gpurun_out/hoist
run() { n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --config c5 --also= --no-pmc --no-cpu-baseline --steps 20 > gpurun_out/hoist/$n.json 2> gpurun_out/hoist/$n.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r['kernel_ms'], r['frac'], d['check']['verified'])" gpurun_out/hoist/$n.json $n; }
run h16 X=1
run h24 EBPF_LIB=abx/h24.so
run h32 EBPF_LIB=abx/h32.so
run h16b X=1
run h24b EBPF_LIB=abx/h24.so
run h32b EBPF_LIB=abx/h32.so
