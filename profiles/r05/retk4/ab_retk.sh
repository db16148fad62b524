mkdir -p gpurun_out/r5_retk4
for k in 0 1; do
  for c in c3l c4 c4h c4c; do
    timeout -k 10 200 python bench.py --config $c --also= --no-pmc --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r5_retk4/${c}_base_$k.json 2>/dev/null || exit 1
    EBPF_LIB=$PWD/abx/libebpf_retk4.so timeout -k 10 200 python bench.py --config $c --also= --no-pmc --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r5_retk4/${c}_retk4_$k.json 2>/dev/null || exit 1
  done
done
