#!/bin/bash
# Round 6: hashtable programs (lookups, forwarded probe values, writes) and hashtable loop writes
# on the compiled path, many more seeds.
set -eu
O=gpurun_out/${TAG:-fuzz6h}
mkdir -p "$O"
run() {
  local name=$1; shift
  timeout -k 10 900 python3 -u tools/fuzz_gpu.py --variants 0 "$@" > "$O/$name.txt" 2>&1
  grep -E "^[a-z].*programs" "$O/$name.txt" | tail -4
}
run hash0_a --hash --programs 15000 --seed 131
run loophash0_a --loopwrites --hash --programs 8000 --seed 132
run manywrites0_b --manywrites --programs 10000 --seed 133
