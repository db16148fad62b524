#!/bin/bash
# GPU tests, smoke, bench lines (kernel_ms = interpreter kernel alone) and rocprofv3 summaries
# of the same commands for C4 and C2 to compare kernel averages.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-kt}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
echo smoke ok
for cfg in c4 c2 c3 c5 c4h; do
  timeout -k 10 200 python3 bench.py --config $cfg --no-cpu-baseline > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -5 $O/bench_$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" $O/bench_$cfg.json $cfg
done
for cfg in c4 c2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$cfg -o prof -- python3 bench.py --config $cfg --no-cpu-baseline --steps 20 --warmup 3 > $O/prof_$cfg.json 2>$O/prof_$cfg.err || exit 1
  cut -d, -f1-4 $O/prof_$cfg/prof_kernel_stats.csv | grep ebpf_
  python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['roofline']['kernel_ms'])" $O/prof_$cfg.json
done
