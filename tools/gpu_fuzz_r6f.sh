#!/bin/bash
# Round 6: the compiled path (variant 0) on many more standard-semantics programs (loop-free,
# counted loops, cursor walks; 64- and 72-B strides), edited ones, and loop-write programs.
set -eu
O=gpurun_out/${TAG:-fuzz6f}
mkdir -p "$O"
run() {
  local name=$1; shift
  timeout -k 10 900 python3 -u tools/fuzz_gpu.py --variants 0 "$@" > "$O/$name.txt" 2>&1
  grep -E "^[a-z].*programs" "$O/$name.txt" | tail -4
}
run standard_a --standard --programs 20000 --seed 111
run stdmutate_a --standard --mutate --programs 20000 --seed 112
run loopwrites_a --loopwrites --programs 10000 --seed 113
run loopfetched_a --loopwrites --fetched --programs 10000 --seed 114
run manywrites_a --manywrites --programs 8000 --seed 115
