#!/bin/bash
# Window-mode bring-up on the GPU: one small window test first (short limit), then the window
# suite, then C5 bench lines with the window launch on and off, and a kernel trace.
set -u
OUT=gpurun_out/${TAG:-r4w}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== first $(date +%T)"
timeout -k 10 200 python -u -m pytest -x -v --timeout 90 --timeout-method thread -m gpu \
  "tests/test_gpu_window.py::test_window_c5_imix[7]" > "$OUT/first.log" 2>&1
rc=$?; tail -5 "$OUT/first.log"; [ $rc -eq 0 ] || { echo "first rc=$rc"; exit $rc; }
if [ -n "${TESTS:-}" ]; then
  echo "== pytest $(date +%T)"
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -v --timeout ${PER_TEST:-120} --timeout-method thread -m gpu $TESTS > "$OUT/pytest.log" 2>&1
  rc=$?; tail -15 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
for w in 1 0; do
  echo "== bench c5 window=$w $(date +%T)"
  EBPF_WINDOW=$w timeout -k 10 300 python -u bench.py --config c5 --also= --no-pmc --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/bench_c5_w$w.json" 2> "$OUT/bench_c5_w$w.err"
  rc=$?; cat "$OUT/bench_c5_w$w.json"; tail -3 "$OUT/bench_c5_w$w.err"; [ $rc -eq 0 ] || exit $rc
done
echo "== trace $(date +%T)"
EBPF_WINDOW=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt -- python -u bench.py --config c5 --also= --no-pmc --no-cpu-baseline --no-verify --steps 10 --warmup 2 > "$OUT/trace.log" 2>&1
rc=$?; tail -3 "$OUT/trace.log"
echo "== done $(date +%T) rc=$rc"
