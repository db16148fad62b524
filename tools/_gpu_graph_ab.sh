#!/bin/bash
# Graph vs eager step launches, per config (bench lines into gpurun_out/$TAG).
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-graph_ab}
mkdir -p $O
for cfg in ${CFGS:-c2 c4 c3 c5 c4h}; do
  for m in graph eager graph; do
    timeout -k 10 200 python3 bench.py --config $cfg --launch $m --no-cpu-baseline > $O/bench_${cfg}_$m.json 2> $O/bench_${cfg}_$m.err \
      || { tail -5 $O/bench_${cfg}_$m.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['config']['launch'], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" $O/bench_${cfg}_$m.json $cfg $m
  done
done
