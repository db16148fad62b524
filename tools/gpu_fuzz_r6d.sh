#!/bin/bash
# Round 6, last tree: long fuzz campaigns on fresh seeds (every mode, thousands of programs per
# configuration), each under its own limit.  PART=1 or 2 runs half of them (one gpurun call each).
set -eu
O=gpurun_out/${TAG:-fuzz6d}
mkdir -p "$O"
run() {
  local name=$1; shift
  timeout -k 10 900 python3 -u tools/fuzz_gpu.py "$@" > "$O/$name.txt" 2>&1
  grep -E "^[a-z].*programs" "$O/$name.txt" | tail -6
}
if [ "${PART:-1}" = 1 ]; then
  run reference --programs 8000 --seed 91
  run hash --hash --programs 4000 --seed 92
  run standard --standard --programs 3000 --seed 93
  run mutate --mutate --programs 6000 --seed 94
else
  run stdmutate --standard --mutate --programs 3000 --seed 95
  run manywrites --manywrites --programs 3000 --seed 96
  run loophash --loopwrites --hash --programs 3000 --seed 97
  run loopfetched --loopwrites --fetched --programs 4000 --seed 98
  run loopwrites --loopwrites --programs 4000 --seed 99
fi
