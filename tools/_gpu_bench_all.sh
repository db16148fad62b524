#!/bin/bash
# Bench lines of every config on one box (this round's DESIGN.md table).
set -u
O=gpurun_out/${TAG:-benchall}
mkdir -p $O
for cfg in c4 c0 c3 c2 c5 c4h; do
  timeout -k 10 300 python3 bench.py --config $cfg --steps 30 --warmup 5 ${EXTRA:-} > $O/bench_$cfg.json 2> $O/bench_$cfg.err \
    || { tail -5 $O/bench_$cfg.err; exit 1; }
  grep '^{' $O/bench_$cfg.json | head -1 | cut -c1-200
done
echo done
