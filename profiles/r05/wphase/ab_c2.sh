# C2 (1M packets, a 16-us launch): superblock size x write phasing with short periods.
# gpurun_out/c2_wp/
O=gpurun_out/c2_wp
mkdir -p $O
B="python bench.py --also= --no-pmc --no-cpu-baseline --steps 2000 --warmup 50 --config c2"
for k in 0 1; do
  for sb in 2 4 8; do
    EBPF_SUPERBLOCK=$sb timeout -k 10 200 $B > $O/sb${sb}_off_$k.json 2>/dev/null || exit 1
    for w in 8,64 9,160 10,320; do
      EBPF_SUPERBLOCK=$sb EBPF_WPHASE=$w timeout -k 10 200 $B > $O/sb${sb}_w${w/,/_}_$k.json 2>/dev/null || exit 1
    done
  done
done
