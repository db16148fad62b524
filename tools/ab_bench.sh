#!/bin/bash
# A/B bench of ab/<name>.so variants on one GPU box: CONFIGS (default "c0 c4") x VARIANTS,
# each bench run under its own time limit; PARITY=<name> also runs pytest -m gpu on that variant.
set -o pipefail
T=${TAG:-ab}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
if [ -n "${PARITY:-}" ]; then
  EBPF_LIB=$PWD/ab/$PARITY.so timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/$T/pytest_$PARITY.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest_$PARITY.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
for cfg in ${CONFIGS:-c0 c4}; do
  for v in ${VARIANTS}; do
    EBPF_LIB=$PWD/ab/$v.so timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline ${BENCH_ARGS:-} \
      > gpurun_out/$T/bench_${cfg}_${v}_$rep.json 2> gpurun_out/$T/bench.err || { tail -5 gpurun_out/$T/bench.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" \
      gpurun_out/$T/bench_${cfg}_${v}_$rep.json "$cfg $v"
  done
done
done
