# write phasing A/B (dp_launch.wphase): default (long staged launches) against off, then
# sweeps of period / window and occupancy.  Results: gpurun_out/wphase$T/
O=gpurun_out/wphase${T:-}
mkdir -p $O
B="python bench.py --also= --no-pmc --no-cpu-baseline --steps 30 --warmup 5"
if [ -z "${SWEEP:-}" ]; then
for k in 0 1; do
  for c in c4 c4c c3 c3l c4h c2; do
    timeout -k 10 200 $B --config $c > $O/${c}_on_$k.json 2>/dev/null || exit 1
    EBPF_WPHASE=0 timeout -k 10 200 $B --config $c > $O/${c}_off_$k.json 2>/dev/null || exit 1
  done
done
fi
for c in ${SWEEP_CFGS:-c4}; do
  for w in ${SWEEP:-}; do
    EBPF_WPHASE=$w timeout -k 10 200 $B --config $c > $O/${c}_w${w/,/_}.json 2>/dev/null || exit 1
  done
done
for c in ${OCC_CFGS:-}; do
  for n in 3 5 6; do
    EBPF_WG_PER_CU=$n timeout -k 10 200 $B --config $c > $O/${c}_wg$n.json 2>/dev/null || exit 1
  done
done
