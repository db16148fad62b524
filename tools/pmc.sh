#!/bin/bash
# PMC passes (each its own rocprofv3 run, kernel-trace only besides --pmc) over bench.py for
# the configs given; results under gpurun_out/$T/pmc_<cfg>_<pass>/.  Summarise with
# tools/pmc_summary.py.
set -o pipefail
T=${T:-pmc}
export TMPDIR=/tmp
PASSES=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
)
# (EXTRA: one more pass, e.g. "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS")
[ -n "${EXTRA:-}" ] && PASSES+=("$EXTRA")
for cfg in "$@"; do
  i=0
  for p in "${PASSES[@]}"; do
    d=gpurun_out/$T/pmc_${cfg}_$i
    mkdir -p $d
    timeout -k 10 300 rocprofv3 --pmc $p --kernel-trace --kernel-include-regex 'ebpf_(interp|jit)' \
      --output-format csv -d $d -o pmc -- python3 bench.py --config $cfg --no-cpu-baseline --no-pmc --also= \
      --steps 3 --warmup 1 > $d/bench.json 2> $d/err.log || { tail -5 $d/err.log; exit 1; }
    i=$((i+1))
  done
done
