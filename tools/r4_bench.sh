#!/bin/bash
# Round-4 bench lines: the default run (C4 + also c2,c3,c5,c4h, PMC traffic and CPU baseline),
# then C4C and C3L with their own roofline lines.
set -u
OUT=gpurun_out/${TAG:-r4b}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== default $(date +%T)"
timeout -k 10 600 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
rc=$?; tail -c 600 "$OUT/bench_default.json"; tail -3 "$OUT/bench_default.err"; [ $rc -eq 0 ] || exit $rc
for c in ${EXTRA:-c4c c3l}; do
  echo "== $c $(date +%T)"
  timeout -k 10 400 python -u bench.py --config $c --also= > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
  rc=$?; tail -c 400 "$OUT/bench_$c.json"; tail -3 "$OUT/bench_$c.err"; [ $rc -eq 0 ] || exit $rc
done
echo "== done $(date +%T)"
