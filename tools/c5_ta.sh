#!/bin/bash
# C5: texture-addresser occupancy (is the plain launch TA-issue-bound?), one pass per block
set -o pipefail
O=gpurun_out/c5ta; mkdir -p $O
export TMPDIR=/tmp
i=0
for p in "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  timeout -s KILL 90 rocprofv3 --pmc $p --kernel-trace --kernel-include-regex 'ebpf_jit' --output-format csv -d $O/p$i -o pmc -- python3 bench.py --config c5 --also= --no-pmc --no-cpu-baseline --no-verify --steps 2 --warmup 1 > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
  i=$((i+1))
done
echo done
