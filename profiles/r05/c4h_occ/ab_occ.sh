# occupancy of the uncapped staged launches (C4H, C3L): 5 against 6 workgroups per CU, two rounds
O=gpurun_out/occ
mkdir -p $O
B="python bench.py --also= --no-pmc --no-cpu-baseline --steps 30 --warmup 5"
for k in 0 1; do
  for c in c4h c3l; do
    for n in 5 6; do
      EBPF_WG_PER_CU=$n timeout -k 10 200 $B --config $c > $O/${c}_wg${n}_$k.json 2>/dev/null || exit 1
    done
  done
done
