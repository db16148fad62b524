#!/bin/bash
# C5 at every occupancy the general kernel allows (EBPF_WG_PER_CU: workgroups of 4 waves per CU),
# plus the default line's PMC passes (roofline.issue / roofline.gather) once.
set -eu
O=gpurun_out/${TAG:-c5occ}
mkdir -p "$O"
for w in 1 2 3 4 5 6; do
  EBPF_WG_PER_CU=$w timeout -k 10 200 python3 bench.py --config c5 --also= --no-pmc --no-cpu-baseline --steps 40 --warmup 5 > "$O/c5_wg$w.json"
  python3 -c "import json,sys; d=json.load(open('$O/c5_wg$w.json')); print('wg/CU $w', d['roofline']['kernel_ms'], d['verified'])"
done
timeout -k 10 400 python3 bench.py --config c5 --also= --no-cpu-baseline --steps 40 --warmup 5 --pmc-dir "$O/pmc" > "$O/c5_default.json"
python3 -c "import json; d=json.load(open('$O/c5_default.json')); r=d['roofline']; print(r['kernel_ms'], r['frac'], json.dumps(r['issue']), json.dumps(r['gather']))"
