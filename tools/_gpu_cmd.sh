set -o pipefail
T=r1h
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
python3 -c "import __graft_entry__ as g; g.build()" > gpurun_out/$T/build.log 2>&1 || { tail -20 gpurun_out/$T/build.log; exit 1; }
timeout -k 10 120 python3 tools/asm_smoke.py kat > gpurun_out/$T/smoke_kat.log 2>&1; rc=$?; tail -20 gpurun_out/$T/smoke_kat.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for cfg in c0 c3 c4 c2 c5; do
  timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline > gpurun_out/$T/bench_$cfg.json 2> gpurun_out/$T/bench_$cfg.err || { tail -5 gpurun_out/$T/bench_$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" gpurun_out/$T/bench_$cfg.json $cfg
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o prof -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/$T/prof_bench.json 2> gpurun_out/$T/prof.err || { tail -5 gpurun_out/$T/prof.err; exit 1; }
find gpurun_out/$T/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150 > gpurun_out/$T/kstats.txt
head -6 gpurun_out/$T/kstats.txt
