#!/bin/bash
# Round 6, last session: every fuzzer mode on fresh seeds against the library rebuilt from source
# in a fresh container (the build the round-end GPU tiers load), all three device variants.
set -eu
O=gpurun_out/${TAG:-fuzzfinal}
mkdir -p "$O"
run() {
  local name=$1; shift
  timeout -k 10 300 python3 -u "$@" > "$O/$name.txt" 2>&1
  grep -E "^[a-z].*programs" "$O/$name.txt" | tail -n 6
}
run plain      tools/fuzz_gpu.py --programs 6000 --seed 701
run hash       tools/fuzz_gpu.py --hash --programs 4000 --seed 702
run standard   tools/fuzz_gpu.py --standard --programs 3000 --seed 703
run mutate     tools/fuzz_gpu.py --mutate --programs 4000 --seed 704
run manywrites tools/fuzz_gpu.py --manywrites --programs 3000 --seed 705
run loopwrites tools/fuzz_gpu.py --loopwrites --programs 3000 --seed 706
run fetched    tools/fuzz_gpu.py --loopwrites --fetched --programs 3000 --seed 707
run loophash   tools/fuzz_gpu.py --loopwrites --hash --programs 1500 --seed 708
run facts      tools/fuzz_facts.py --variants 0,1,2 --programs 10000 --seed 709
run facts_maps tools/fuzz_facts.py --maps --variants 0,1,2 --programs 6000 --seed 710
run facts_gen  tools/fuzz_facts.py --general --maps --variants 0,1,2 --programs 6000 --seed 711
run facts_std  tools/fuzz_facts.py --standard --variants 0,1,2 --programs 6000 --seed 712
echo "== done $(date +%T)"
