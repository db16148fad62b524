# PMC passes over the C5 bench, path-sorted (on) and plain (off): per-dispatch counters of the
# compiled kernels (the path-sorted step has two: the classifying run, then the main run).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PASSES=(
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
)
for mode in on off; do
  i=0
  for p in "${PASSES[@]}"; do
    d=gpurun_out/ps_pmc/${mode}_$i
    mkdir -p $d
    if [ $mode = off ]; then export EBPF_PATHSORT=0; else export EBPF_PATHSORT=1; fi
    timeout -s KILL 120 rocprofv3 --pmc $p --kernel-include-regex 'ebpf_jit' \
      --output-format csv -d $d -o pmc -- python3 bench.py --config c5 --also= --no-cpu-baseline --no-pmc --no-verify \
      --steps 3 --warmup 1 > $d/bench.json 2> $d/err.log || { tail -5 $d/err.log; exit 1; }
    i=$((i+1))
  done
done
