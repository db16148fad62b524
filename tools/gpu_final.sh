#!/bin/bash
# The round's final-tree check, one session: the whole GPU suite, smoke(), the default bench line
# (every config, PMC passes, CPU baseline) and the C4 line under rocprofv3 --kernel-trace --stats.
# Each GPU step has its own limit; the first failure ends the script.
set -u
O=gpurun_out/${TAG:-final}
mkdir -p "$O"
export TMPDIR=/tmp
echo "== pytest $(date +%T)"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu_full.log" 2>&1
rc=$?; tail -2 "$O/pytest_gpu_full.log"; [ $rc -eq 0 ] || exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
rc=$?; tail -2 "$O/smoke.log"; [ $rc -eq 0 ] || exit $rc
echo "== bench $(date +%T)"
timeout -k 10 600 python3 -u bench.py > "$O/bench_default.json" 2> "$O/bench_default.err"
rc=$?; cat "$O/bench_default.json"; [ $rc -eq 0 ] || exit $rc
echo "== rocprof $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c4" -o c4 -- python3 bench.py --also= --no-pmc --no-cpu-baseline --steps 30 --warmup 5 > "$O/prof_c4.json" 2> "$O/prof_c4.err"
rc=$?; cat "$O/prof_c4.json"; [ $rc -eq 0 ] || exit $rc
echo "== done $(date +%T)"
