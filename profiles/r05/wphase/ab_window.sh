# wide phasing windows on C4 / C3: 1,024 / 1,280 / 1,536 ticks of a 4,096-tick period, three
# alternating rounds.  gpurun_out/window/
O=gpurun_out/window
mkdir -p $O
B="python bench.py --also= --no-pmc --no-cpu-baseline --steps 40 --warmup 5"
for k in 0 1 2; do
  for c in c4 c3; do
    for w in 1024 1280 1536; do
      EBPF_WPHASE=12,$w,16 timeout -k 10 200 $B --config $c > $O/${c}_w${w}_$k.json 2>/dev/null || exit 1
    done
  done
done
