#!/bin/bash
# C3L: workgroups per CU (occupancy) A/B, then the SQ counter passes
set -o pipefail
O=gpurun_out/c3locc; mkdir -p $O
run() { n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --config c3l --also= --no-pmc --no-cpu-baseline --steps 30 > $O/$n.json 2> $O/$n.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r['kernel_ms'], r['frac'], d['check']['verified'])" $O/$n.json $n; }
run def X=1
run w4 EBPF_WG_PER_CU=4
run w5 EBPF_WG_PER_CU=5
run w6 EBPF_WG_PER_CU=6
run w8 EBPF_WG_PER_CU=8
run def2 X=1
