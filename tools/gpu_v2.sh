#!/bin/bash
# GPU box: the GPU suite, then assembly-interpreter (variant 2) benches of C4 / C3 / C4H / C5.
set -o pipefail
T=${TAG:-v2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for cfg in ${CONFIGS:-c4 c3 c4h c5}; do
  for w in ${WGS:-0}; do
    env EBPF_WG_PER_CU=$w timeout -k 10 300 python3 bench.py --config $cfg --variant 2 --also= --no-pmc --steps 30 --no-cpu-baseline \
      > gpurun_out/$T/bench_${cfg}_w$w.json 2> gpurun_out/$T/bench.err || { tail -5 gpurun_out/$T/bench.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('verified'))" \
      gpurun_out/$T/bench_${cfg}_w$w.json "$cfg w$w"
  done
done
