#!/bin/bash
# Round 6: the compiled path (variant 0, whose code generator keeps value-range facts) on many
# more random and edited reference programs — where the long campaign found the fused-swap bug.
set -eu
O=gpurun_out/${TAG:-fuzz6e}
mkdir -p "$O"
run() {
  local name=$1; shift
  timeout -k 10 900 python3 -u tools/fuzz_gpu.py --variants 0 "$@" > "$O/$name.txt" 2>&1
  grep -E "^[a-z].*programs" "$O/$name.txt" | tail -4
}
run reference_a --programs 12000 --seed 101
run reference_b --programs 12000 --seed 102
run mutate_a --mutate --programs 10000 --seed 103
run hash_a --hash --programs 6000 --seed 104
