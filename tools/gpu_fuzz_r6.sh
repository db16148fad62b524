#!/bin/bash
# Round 6's longer fuzz campaigns (tools/fuzz_gpu.py), each under its own limit: reference
# programs with more than 16 map writes on one path, loop programs that read their counters
# back, and the plain loop-write and reference campaigns on fresh seeds.
set -eu
O=gpurun_out/${TAG:-fuzz6}
mkdir -p "$O"
timeout -k 10 900 python3 -u tools/fuzz_gpu.py --manywrites --programs 300 --seed 61 > "$O/manywrites.txt" 2>&1
tail -7 "$O/manywrites.txt"
timeout -k 10 900 python3 -u tools/fuzz_gpu.py --loopwrites --fetched --programs 300 --seed 62 > "$O/loopfetched.txt" 2>&1
tail -3 "$O/loopfetched.txt"
timeout -k 10 900 python3 -u tools/fuzz_gpu.py --programs 300 --seed 63 > "$O/reference.txt" 2>&1
tail -6 "$O/reference.txt"
