#!/bin/bash
# C3L A/B: occupancy (workgroups per CU) and write phasing forced on (12-bit period, 1,024-tick
# window, 16 slots: the wide kernel), default line's C3L shape, 3 runs each.
set -u
O=gpurun_out/${TAG:-c3lab}
mkdir -p "$O"
run() { # name, env...
  local n=$1; shift
  for r in 1 2 3; do
    env "$@" timeout -k 10 120 python3 bench.py --config c3l --also= --no-pmc --no-cpu-baseline --steps 200 --warmup 20 > "$O/$n.$r.json" 2>/dev/null || return 1
    python3 -c "import json; d=json.load(open('$O/$n.$r.json')); print('$n', d['roofline']['kernel_ms'], d['roofline']['frac'], d['verified'])"
  done
}
run default EBPF_NONE=1 && run wg4 EBPF_WG_PER_CU=4 && run wg5 EBPF_WG_PER_CU=5 && run wphase16 EBPF_WPHASE=12,1024,16 && run wphase8 EBPF_WPHASE=11,640
