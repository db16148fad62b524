# the same bench line R times per config (box noise / before-after checks).  gpurun_out/rep$T/
O=gpurun_out/rep${T:-}
mkdir -p $O
B="python bench.py --also= --no-pmc --no-cpu-baseline --steps ${STEPS:-60} --warmup 10"
for k in $(seq 1 ${R:-3}); do
  for c in ${CFGS:-c3l c4}; do
    timeout -k 10 200 $B --config $c > $O/${c}_$k.json 2>/dev/null || exit 1
  done
done
