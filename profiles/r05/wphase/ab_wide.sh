# wide write phasing (16 result slots, ebpf_jit_s64w) against the 8-slot form and off, then a
# period x window sweep of the wide form on C4.  gpurun_out/wide/
O=gpurun_out/wide
mkdir -p $O
B="python bench.py --also= --no-pmc --no-cpu-baseline --steps 30 --warmup 5"
for k in 0 1; do
  for c in c4 c3 c4c; do
    timeout -k 10 200 $B --config $c > $O/${c}_wide_$k.json 2>/dev/null || exit 1
    EBPF_WPHASE=11,640 timeout -k 10 200 $B --config $c > $O/${c}_narrow_$k.json 2>/dev/null || exit 1
    EBPF_WPHASE=0 timeout -k 10 200 $B --config $c > $O/${c}_off_$k.json 2>/dev/null || exit 1
  done
done
for w in 12,768,16 12,1280,16 11,512,16 11,640,16 13,2048,16; do
  EBPF_WPHASE=$w timeout -k 10 200 $B --config c4 > $O/c4_w${w//,/_}.json 2>/dev/null || exit 1
done
