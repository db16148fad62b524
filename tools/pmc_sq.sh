#!/bin/bash
# Issue-side PMC passes (SQ counters, 8 per pass) over bench.py for the configs given; results
# under gpurun_out/$T/pmcsq_<cfg>_<pass>/.  Summarise with tools/pmc_summary.py (same layout).
set -o pipefail
T=${T:-pmcsq}
export TMPDIR=/tmp
PASSES=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_IFETCH"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_IFETCH_LEVEL SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU"
)
for cfg in "$@"; do
  i=0
  for p in "${PASSES[@]}"; do
    d=gpurun_out/$T/pmc_${cfg}_$i
    mkdir -p $d
    timeout -s KILL 120 rocprofv3 --pmc $p --kernel-trace --kernel-include-regex 'ebpf_(interp|jit)' \
      --output-format csv -d $d -o pmc -- python3 bench.py --config $cfg --no-cpu-baseline \
      --steps 3 --warmup 1 ${BENCH_ARGS:-} > $d/bench.json 2> $d/err.log || { tail -5 $d/err.log; exit 1; }
    i=$((i+1))
  done
done
