#!/bin/bash
# Step cost of the per-step kernel timing events: --time-every 1 / 5 / 1000, C4 and C2.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-te}
mkdir -p $O
for cfg in c4 c2; do
  for k in 1 5 1000 1 5 1000; do
    timeout -k 10 200 python3 bench.py --config $cfg --no-cpu-baseline --time-every $k > $O/bench_${cfg}_$k.json 2> $O/bench_${cfg}_$k.err || { tail -5 $O/bench_${cfg}_$k.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" $O/bench_${cfg}_$k.json $cfg $k
  done
done
