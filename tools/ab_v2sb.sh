mkdir -p gpurun_out/v2sb
for spec in "rk8 EBPF_SUPERBLOCK=8" "rk8 EBPF_SUPERBLOCK=4" "rk8 EBPF_SUPERBLOCK=2" "rk8 EBPF_SUPERBLOCK=1" "rk1 EBPF_WG_PER_CU=6" "rk1 EBPF_WG_PER_CU=7" "rk1 EBPF_WG_PER_CU=8" "rk2 EBPF_WG_PER_CU=6"; do
  set -- $spec
  env EBPF_LIB=$PWD/ab/$1.so $2 timeout -k 10 300 python3 bench.py --config c4 --variant 2 --also= --no-pmc --steps 30 --no-cpu-baseline > gpurun_out/v2sb/b.json 2> gpurun_out/v2sb/err || { tail -3 gpurun_out/v2sb/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/v2sb/b.json')); print(sys.argv[1], d['value'], d['roofline']['kernel_ms'])" "$spec"
done
