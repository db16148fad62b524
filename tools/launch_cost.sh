#!/bin/bash
# Build and run the launch-cost probes (tools/launch_cost.c, tools/launch_cost.py) on the GPU box.
set -eu
OUT=gpurun_out/${TAG:-launch_cost}
mkdir -p "$OUT" tools/bin
gcc -O2 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/launch_cost.c -o tools/bin/launch_cost \
  -Lgeneric-ebpf_amd/lib -lebpf -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/generic-ebpf_amd/lib -Wl,-rpath,/opt/rocm/lib
timeout -k 10 120 tools/bin/launch_cost ${K:-2000} | tee "$OUT/launch_cost_c.jsonl"
timeout -k 10 180 python -u tools/launch_cost.py ${K:-2000} c2 | tee "$OUT/launch_cost_py.jsonl"
