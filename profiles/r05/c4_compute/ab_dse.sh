mkdir -p gpurun_out/r5_dse
for k in 0 1 2; do
  for c in c4 c4c c3 c4h; do
    timeout -k 10 200 python bench.py --config $c --also= --no-pmc --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/r5_dse/${c}_new_$k.json 2>/dev/null || exit 1
    EBPF_LIB=$PWD/abx/libebpf_perm.so timeout -k 10 200 python bench.py --config $c --also= --no-pmc --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/r5_dse/${c}_prev_$k.json 2>/dev/null || exit 1
  done
done
