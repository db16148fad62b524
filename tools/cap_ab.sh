#!/bin/bash
# The 4-workgroup streaming cap of staged compiled programs, re-checked per config: default vs 6
set -o pipefail
O=gpurun_out/capab; mkdir -p $O
run() { n=$1; c=$2; shift 2
  env "$@" timeout -k 10 120 python -u bench.py --config $c --also= --no-pmc --no-cpu-baseline --steps 30 > $O/$n.json 2> $O/$n.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r['kernel_ms'], r['frac'], d['check']['verified'])" $O/$n.json $n; }
for c in c4 c3 c4c c2; do
  run ${c}_def $c X=1
  run ${c}_w6 $c EBPF_WG_PER_CU=6
  run ${c}_def2 $c X=1
  run ${c}_w6b $c EBPF_WG_PER_CU=6
done
