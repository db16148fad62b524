# C4H: workgroups per CU (3-6) x write phasing, two rounds.  gpurun_out/c4h/
O=gpurun_out/c4h
mkdir -p $O
B="python bench.py --also= --no-pmc --no-cpu-baseline --steps 30 --warmup 5 --config c4h"
for k in 0 1; do
  for n in 3 4 5 6; do
    EBPF_WG_PER_CU=$n timeout -k 10 200 $B > $O/wg${n}_off_$k.json 2>/dev/null || exit 1
    EBPF_WG_PER_CU=$n EBPF_WPHASE=11,640 timeout -k 10 200 $B > $O/wg${n}_on_$k.json 2>/dev/null || exit 1
  done
done
