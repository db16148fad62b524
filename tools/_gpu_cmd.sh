set -o pipefail
T=r1q
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
python3 -c "import __graft_entry__ as g; g.build()" > gpurun_out/$T/build.log 2>&1 || { tail -20 gpurun_out/$T/build.log; exit 1; }
VARIANTS=0,2 timeout -k 10 120 python3 tools/asm_smoke.py kat > gpurun_out/$T/smoke_kat.log 2>&1; rc=$?; grep -c "^ok" gpurun_out/$T/smoke_kat.log; grep FAIL gpurun_out/$T/smoke_kat.log | head -3; [ $rc -eq 0 ] || exit $rc
grep -q FAIL gpurun_out/$T/smoke_kat.log && exit 3
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for v in 0 2; do
for cfg in c0 c3 c4 c2 c5; do
  timeout -k 10 300 python3 bench.py --config $cfg --variant $v --no-cpu-baseline > gpurun_out/$T/bench_${cfg}_$v.json 2> gpurun_out/$T/bench_$cfg.err || { tail -5 gpurun_out/$T/bench_$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" gpurun_out/$T/bench_${cfg}_$v.json "v$v $cfg"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof_c2 -o prof -- python3 bench.py --config c2 --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/$T/prof_c2.json 2> gpurun_out/$T/prof_c2.err || { tail -5 gpurun_out/$T/prof_c2.err; exit 1; }
find gpurun_out/$T/prof_c2 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150
bash tools/_gpu_cmd2.sh
timeout -k 10 200 tools/ubench/pipeline
