#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel-trace summary.
# Every GPU step runs under its own time limit; the first failure ends the script.
set -u
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step build
python3 -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || { tail -20 "$OUT/build.log"; exit 1; }
step pytest-gpu
timeout -k 10 ${TEST_TIMEOUT:-900} python3 -m pytest tests -x -q -m gpu ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -25 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
step smoke
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -3 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
step bench
timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"; [ $rc -eq 0 ] || exit $rc
if [ -n "${PROF:-1}" ]; then
  step rocprof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- \
      python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 ${BENCH_ARGS:-} > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
  rc=$?; tail -3 "$OUT/prof.err"; [ $rc -eq 0 ] || exit $rc
  find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \; | head -20
fi
echo "== done"
