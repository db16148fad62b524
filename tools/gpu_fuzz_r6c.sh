#!/bin/bash
# Round 6, last tree: every fuzzer mode on fresh seeds, larger campaigns, each under its own limit.
set -eu
O=gpurun_out/${TAG:-fuzz6c}
mkdir -p "$O"
run() {
  local name=$1; shift
  timeout -k 10 600 python3 -u tools/fuzz_gpu.py "$@" > "$O/$name.txt" 2>&1
  grep -E "programs," "$O/$name.txt" | tail -6
}
run reference --programs 2000 --seed 81
run hash --hash --programs 1000 --seed 82
run standard --standard --programs 600 --seed 83
run mutate --mutate --programs 1500 --seed 84
run manywrites --manywrites --programs 600 --seed 85
run loophash --loopwrites --hash --programs 1000 --seed 86
run loopfetched --loopwrites --fetched --programs 1000 --seed 87
