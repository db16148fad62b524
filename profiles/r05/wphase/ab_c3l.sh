# C3L: write phasing x occupancy (4 / 5 / 6 workgroups per CU), two rounds.  gpurun_out/c3l_wp/
O=gpurun_out/c3l_wp
mkdir -p $O
B="python bench.py --also= --no-pmc --no-cpu-baseline --steps 60 --warmup 10 --config c3l"
for k in 0 1; do
  for wg in 4 5 6; do
    EBPF_WG_PER_CU=$wg timeout -k 10 200 $B > $O/wg${wg}_off_$k.json 2>/dev/null || exit 1
    EBPF_WG_PER_CU=$wg EBPF_WPHASE=11,640 timeout -k 10 200 $B > $O/wg${wg}_on_$k.json 2>/dev/null || exit 1
  done
done
