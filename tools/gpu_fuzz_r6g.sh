#!/bin/bash
# Round 6: more reference-semantics programs on the compiled path and the assembly interpreter
# (variants 0 and 2: the code generator's value-range facts, the interpreter's superinstructions).
set -eu
O=gpurun_out/${TAG:-fuzz6g}
mkdir -p "$O"
run() {
  local name=$1; shift
  timeout -k 10 900 python3 -u tools/fuzz_gpu.py "$@" > "$O/$name.txt" 2>&1
  grep -E "^[a-z].*programs" "$O/$name.txt" | tail -4
}
run ref0_a --variants 0 --programs 15000 --seed 121
run ref0_b --variants 0 --programs 15000 --seed 122
run ref2_a --variants 2 --programs 15000 --seed 123
run mut2_a --variants 2 --mutate --programs 10000 --seed 124
