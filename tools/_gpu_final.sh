#!/bin/bash
# End-of-round evidence on one box: GPU parity tests, smoke, a bench line per config, the
# rocprofv3 kernel-trace summary of the default bench and PMC passes (HBM traffic, SQ mix).
# Every GPU step has its own time limit; the first failure ends the script.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-final}
mkdir -p $O
step() { echo "== $1 ($(date +%T))"; }
step pytest
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
  || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
step smoke
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
step bench
TAG=${TAG:-final}/benchall bash tools/_gpu_bench_all.sh || exit 1
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- \
    python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/prof_bench.json 2> $O/prof.err \
  || { tail -5 $O/prof.err; exit 1; }
[ -n "${SKIP_PMC:-}" ] && { echo "== done, no pmc ($(date +%T))"; exit 0; }
step pmc
T=${TAG:-final}/pmc bash tools/pmc.sh ${PMC_CFGS:-c4 c4h c3 c0} || exit 1
echo "== done ($(date +%T))"
