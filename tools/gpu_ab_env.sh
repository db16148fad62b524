#!/bin/bash
# GPU box: parity tests, then A/B benches of the current build under env settings.
#   ENVS="base: nocc:EBPF_JIT_NOCC=1" CONFIGS="c4 c3" TAG=x bash tools/gpu_ab_env.sh
set -o pipefail
T=${TAG:-abenv}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in ${REPS:-1 2}; do
for cfg in ${CONFIGS:-c0 c4}; do
  for ev in ${ENVS:-base:}; do
    name=${ev%%:*}; assign=${ev#*:}
    env $assign timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline ${BENCH_ARGS:-} \
      > gpurun_out/$T/bench_${cfg}_${name}_$rep.json 2> gpurun_out/$T/bench.err || { tail -5 gpurun_out/$T/bench.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" \
      gpurun_out/$T/bench_${cfg}_${name}_$rep.json "$cfg $name"
  done
done
done
