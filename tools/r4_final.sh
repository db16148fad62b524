#!/bin/bash
# Round-4 closing measurement: the default bench line (C4 + the --also lines, PMC traffic, CPU
# baseline), then the same command under rocprofv3 --kernel-trace --stats.
set -u
OUT=gpurun_out/${TAG:-r4f}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== default $(date +%T)"
timeout -k 10 600 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
rc=$?; tail -c 800 "$OUT/bench_default.json"; tail -3 "$OUT/bench_default.err"; [ $rc -eq 0 ] || exit $rc
echo "== rocprof $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o kt -- python3 -u bench.py --no-pmc > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err"
rc=$?; tail -3 "$OUT/bench_prof.err"; [ $rc -eq 0 ] || exit $rc
echo "== done $(date +%T)"
