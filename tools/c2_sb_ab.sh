#!/bin/bash
# C2 (1M packets, a 72-MB launch): superblock length and workgroups per CU A/B
set -o pipefail
O=gpurun_out/c2sb; mkdir -p $O
run() { n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --config c2 --also= --no-pmc --no-cpu-baseline --steps 50 > $O/$n.json 2> $O/$n.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r['kernel_ms'], r['frac'], d['check']['verified'])" $O/$n.json $n; }
for rep in a b; do
  run sb8_$rep X=1
  run sb4_$rep EBPF_SUPERBLOCK=4
  run sb2_$rep EBPF_SUPERBLOCK=2
  run sb8w6_$rep EBPF_WG_PER_CU=6
  run sb4w6_$rep EBPF_SUPERBLOCK=4 EBPF_WG_PER_CU=6
done
