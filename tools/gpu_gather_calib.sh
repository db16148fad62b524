#!/bin/bash
# The gather roofline's calibration: tools/ubench/gather (mode 'i': C5's
# IMIX address shape with every lane active; mode 'c':
# per-lane random loads inside 576-B / 1536-B / 64-B packets, and 576-B with one lane in four)
# and C5 under one rocprofv3 --pmc pass each: TCP tag accesses, L1->L2 read requests, TD / TA
# busy, GRBM active; kernel trace only besides (MI355X_MICROARCH.md).
set -eu
export TMPDIR=/tmp
O=gpurun_out/${TAG:-gcal}
mkdir -p "$O"
C="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
timeout -k 10 120 tools/ubench/gather i > "$O/imix_plain.txt"
cat "$O/imix_plain.txt"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$O/pmc_imix" -o pmc -- tools/ubench/gather i > "$O/imix_pmc.txt"
timeout -k 10 120 tools/ubench/gather c > "$O/gather_plain.txt"
cat "$O/gather_plain.txt"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$O/pmc_gather" -o pmc -- tools/ubench/gather c > "$O/gather_pmc.txt"
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --kernel-include-regex 'ebpf_(interp|jit)' --output-format csv \
  -d "$O/pmc_c5" -o pmc -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-pmc --no-verify --also= > "$O/c5.json"
cat "$O/c5.json"
echo done
