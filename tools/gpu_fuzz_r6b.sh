#!/bin/bash
# Round 6, after hashtable counters inside loops became counted records: the loop-write fuzzer
# with a hashtable map 0 (every program mixes counters, fetched or not, stores, loads back and
# update calls), and the plain / fetched loop-write campaigns on fresh seeds, each under its own
# limit.
set -eu
O=gpurun_out/${TAG:-fuzz6b}
mkdir -p "$O"
timeout -k 10 900 python3 -u tools/fuzz_gpu.py --loopwrites --hash --programs 400 --seed 71 > "$O/loophash.txt" 2>&1
tail -3 "$O/loophash.txt"
timeout -k 10 600 python3 -u tools/fuzz_gpu.py --loopwrites --programs 300 --seed 72 > "$O/loopwrites.txt" 2>&1
tail -3 "$O/loopwrites.txt"
timeout -k 10 600 python3 -u tools/fuzz_gpu.py --loopwrites --fetched --programs 300 --seed 73 > "$O/loopfetched.txt" 2>&1
tail -3 "$O/loopfetched.txt"
