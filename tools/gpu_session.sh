#!/bin/bash
# GPU session: the given pytest selection (TESTS), then optional bench lines (BENCH:
# space-separated configs, each run with --also= and no PMC).  Each GPU step has its own limit;
# the first failure ends the script.
set -u
OUT=gpurun_out/${TAG:-r5}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  echo "== pytest $(date +%T)"
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest -x -v --timeout ${PER_TEST:-120} --timeout-method thread -m gpu $TESTS > "$OUT/pytest.log" 2>&1
  rc=$?; tail -15 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
for c in ${BENCH:-}; do
  echo "== bench $c $(date +%T)"
  timeout -k 10 300 python -u bench.py --config $c --also= --no-pmc --no-cpu-baseline --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
  rc=$?; cat "$OUT/bench_$c.json"; tail -3 "$OUT/bench_$c.err"; [ $rc -eq 0 ] || exit $rc
done
echo "== done $(date +%T)"
