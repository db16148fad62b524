#!/bin/bash
# Deep-queue fix check, then histogram second stage rows per block 16 / 32 / 64 (EBPF_HIST_ROWS).
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-hist_ab}
mkdir -p $O
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "deep_async or device_resident" > $O/pytest_deep.log 2>&1 || { tail -20 $O/pytest_deep.log; exit 1; }
tail -1 $O/pytest_deep.log
for cfg in c2 c4; do
  for r in 16 64 32 16 64 32; do
    EBPF_HIST_ROWS=$r timeout -k 10 200 python3 bench.py --config $cfg --no-cpu-baseline --steps 200 > $O/bench_${cfg}_$r.json 2> $O/bench_${cfg}_$r.err \
      || { tail -5 $O/bench_${cfg}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" $O/bench_${cfg}_$r.json $cfg $r
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof16 -o prof -- python3 bench.py --config c2 --no-cpu-baseline --steps 20 > $O/prof16.json 2>$O/prof16.err || exit 1
EBPF_HIST_ROWS=64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof64 -o prof -- python3 bench.py --config c2 --no-cpu-baseline --steps 20 > $O/prof64.json 2>$O/prof64.err || exit 1
