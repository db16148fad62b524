#!/bin/bash
# GPU box: assembly-interpreter (variant 2) benches of ab/<lib>.so builds: LIBS x CONFIGS, REPS.
set -o pipefail
T=${TAG:-v2lib}
mkdir -p gpurun_out/$T
for rep in ${REPS:-1 2}; do
for cfg in ${CONFIGS:-c4}; do
  for lib in ${LIBS}; do
    env EBPF_LIB=$PWD/ab/$lib.so ${ENV:-} timeout -k 10 300 python3 bench.py --config $cfg --variant ${VARIANT:-2} --also= --no-pmc --steps 30 --no-cpu-baseline \
      > gpurun_out/$T/b.json 2> gpurun_out/$T/err || { tail -5 gpurun_out/$T/err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('verified'))" \
      gpurun_out/$T/b.json "$cfg $lib"
  done
done
done
