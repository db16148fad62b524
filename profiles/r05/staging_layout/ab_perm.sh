mkdir -p gpurun_out/r5_perm
for k in 0 1 2; do
  for c in c4 c3 c4h c4c c3l c2; do
    timeout -k 10 200 python bench.py --config $c --also= --no-pmc --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/r5_perm/${c}_perm_$k.json 2>/dev/null || exit 1
    EBPF_LIB=$PWD/abx/libebpf_base.so timeout -k 10 200 python bench.py --config $c --also= --no-pmc --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/r5_perm/${c}_base_$k.json 2>/dev/null || exit 1
  done
done
