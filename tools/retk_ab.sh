#!/bin/bash
# Staged result-burst A/B (ab builds with EBPF_ASM_RETK=8 / 1, copied to abx/): kernel ms and
# verification per config; CASES = "cfg:lib[:ENV=val]" items.
set -o pipefail
T=${TAG:-retk}; mkdir -p gpurun_out/$T
for c in ${CASES:-c3l:retk8 c3l:retk1}; do
  IFS=: read cfg lib envs <<< "$c"
  env EBPF_LIB=$PWD/abx/$lib.so $envs timeout -k 10 300 python3 bench.py --config $cfg --also= --no-pmc --steps 30 --no-cpu-baseline > gpurun_out/$T/b.json 2> gpurun_out/$T/err; rc=$?
  [ $rc -le 1 ] || { tail -5 gpurun_out/$T/err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('verified'))" gpurun_out/$T/b.json "$c"
done
