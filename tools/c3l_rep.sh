#!/bin/bash
# C3L repeat: the loop/standard GPU tests, then the C3L bench line REPS times (kernel ms per run).
set -u
O=gpurun_out/${TAG:-c3lrep}
mkdir -p "$O"
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
  -k "${TESTS:-standard or loop or c3l or window or cursor}" tests > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
for i in $(seq 1 ${REPS:-3}); do
  echo "== run $i $(date +%T)"
  timeout -k 10 300 python3 bench.py --config c3l --also= --no-cpu-baseline --no-pmc \
    > "$O/bench_$i.json" 2> "$O/bench_$i.err" || { tail -5 "$O/bench_$i.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], r['kernel_ms'], r['frac'], d.get('check',{}).get('verified'))" "$O/bench_$i.json"
done
echo "== general kernel $(date +%T)"
timeout -k 10 300 python3 tools/c3l_general.py > "$O/general.json" 2> "$O/general.err" || { tail -5 "$O/general.err"; exit 1; }
cat "$O/general.json"
echo "== done $(date +%T)"
