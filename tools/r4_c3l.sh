#!/bin/bash
# C3L (compiled loops) A/B: loop and standard GPU tests, then the C3L bench line with the
# reversed back-edge split and LDS packet loads (keep mode), and with each switched off.
set -u
O=gpurun_out/${TAG:-c3l}
mkdir -p "$O"
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
  -k "${TESTS:-standard or loop or c3l or window}" tests > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
for v in "both:" "nokeep:EBPF_JIT_NOKEEP=1" "norev:EBPF_JIT_NOREVLOOP=1" "neither:EBPF_JIT_NOKEEP=1 EBPF_JIT_NOREVLOOP=1"; do
  name=${v%%:*}; envs=${v#*:}
  echo "== $name $(date +%T)"
  env $envs timeout -k 10 300 python3 bench.py --config c3l --also= --no-cpu-baseline --no-pmc \
    > "$O/bench_$name.json" 2> "$O/bench_$name.err" || { tail -5 "$O/bench_$name.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], r['kernel_ms'], r['frac'], d.get('check',{}).get('verified'))" "$O/bench_$name.json"
done
echo "== done $(date +%T)"
