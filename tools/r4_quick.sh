#!/bin/bash
# Quick GPU check: the selected tests, then bench lines (no PMC, no CPU baseline).
set -u
OUT=gpurun_out/${TAG:-r4q}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -q --timeout ${PER_TEST:-120} --timeout-method thread -m gpu $TESTS > "$OUT/pytest.log" 2>&1
  rc=$?; tail -4 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
for c in ${BENCH:-}; do
  timeout -k 10 300 python -u bench.py --config $c --also= --no-pmc --no-cpu-baseline --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$c.err"; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/bench_$c.json'));r=d['roofline'];print('$c', d['value'], 'kernel', r['kernel_ms'], 'frac', r['frac'], 'verified', d.get('verified'))"
done
