#!/bin/bash
# C3L: keep mode (the staged kernel's next DMA waits for the group's end, so that run-time-offset
# loads whose lanes differ can read the LDS packet buffer) against no keep mode (the DMA right
# after staging; such loads go to global memory) — C3L's cursor is wave-uniform, so its loads
# come from the packet registers either way.  With and without write phasing.  3 runs each.
set -u
O=gpurun_out/${TAG:-c3lkeep}
mkdir -p "$O"
run() {
  local n=$1; shift
  for r in 1 2 3; do
    env "$@" timeout -k 10 120 python3 bench.py --config c3l --also= --no-pmc --no-cpu-baseline --steps 200 --warmup 20 > "$O/$n.$r.json" 2>/dev/null || return 1
    python3 -c "import json; d=json.load(open('$O/$n.$r.json')); print('$n', d['roofline']['kernel_ms'], d['roofline']['frac'], d['verified'])"
  done
}
run default EBPF_NONE=1 && run nokeep EBPF_NOKEEP=1 && run nokeep_wp EBPF_NOKEEP=1 EBPF_WPHASE=12,1024,16 && run nokeep_wg6 EBPF_NOKEEP=1 EBPF_WG_PER_CU=6 && run nokeep_wg4 EBPF_NOKEEP=1 EBPF_WG_PER_CU=4
