# C4 at the per-GPU shard sizes of the driver's strong-scaling runs (64M / N packets for N = 2,
# 4, 8): write phasing (default: wide) against off, two rounds.  gpurun_out/shard/
O=gpurun_out/shard
mkdir -p $O
B="python bench.py --also= --no-pmc --no-cpu-baseline --steps 100 --warmup 10 --config c4"
for k in 0 1; do
  for n in 33554432 16777216 8388608; do
    timeout -k 10 200 $B --packets $n > $O/c4_${n}_on_$k.json 2>/dev/null || exit 1
    EBPF_WPHASE=0 timeout -k 10 200 $B --packets $n > $O/c4_${n}_off_$k.json 2>/dev/null || exit 1
  done
done
