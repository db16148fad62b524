#!/bin/bash
# C3L at its default 5 workgroups per CU: superblock sizes and write phasing (A/B, 3 runs each)
set -u
O=gpurun_out/${TAG:-c3lab2}
mkdir -p "$O"
run() {
  local n=$1; shift
  for r in 1 2 3; do
    env "$@" timeout -k 10 120 python3 bench.py --config c3l --also= --no-pmc --no-cpu-baseline --steps 200 --warmup 20 > "$O/$n.$r.json" 2>/dev/null || return 1
    python3 -c "import json; d=json.load(open('$O/$n.$r.json')); print('$n', d['roofline']['kernel_ms'], d['roofline']['frac'], d['verified'])"
  done
}
run default EBPF_NONE=1 && run sb4 EBPF_SUPERBLOCK=4 && run sb2 EBPF_SUPERBLOCK=2 && run wphase8 EBPF_WPHASE=11,640 && run wphase16 EBPF_WPHASE=12,1024,16
