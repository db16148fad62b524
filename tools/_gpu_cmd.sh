set -o pipefail
T=r1x
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
python3 -c "import __graft_entry__ as g; g.build()" > gpurun_out/$T/build.log 2>&1 || { tail -20 gpurun_out/$T/build.log; exit 1; }
VARIANTS=0,2 timeout -k 10 120 python3 tools/asm_smoke.py kat > gpurun_out/$T/smoke.log 2>&1; rc=$?; echo "smoke ok=$(grep -c '^ok' gpurun_out/$T/smoke.log)"; grep FAIL gpurun_out/$T/smoke.log | head -3; [ $rc -eq 0 ] || exit $rc
grep -q FAIL gpurun_out/$T/smoke.log && exit 3
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for cfg in c0 c4 c3 c2 c5 c0 c4; do
  timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline > gpurun_out/$T/bench_${cfg}.json 2> gpurun_out/$T/bench.err || { tail -5 gpurun_out/$T/bench.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" gpurun_out/$T/bench_${cfg}.json "$cfg"
done
