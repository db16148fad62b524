#!/bin/bash
# Round-1 profiles of the hashtable (C4H) and IMIX (C5) configs: kernel-trace stats + PMC passes.
set -u
export TMPDIR=/tmp
for cfg in c4h c5; do
  d=gpurun_out/prof_$cfg
  mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o prof -- \
      python3 bench.py --config $cfg --no-cpu-baseline --steps 10 --warmup 3 > $d/bench.json 2> $d/err.log \
    || { tail -5 $d/err.log; exit 1; }
done
T=pmc_r1h bash tools/pmc.sh c4h c5 || exit 1
echo done
