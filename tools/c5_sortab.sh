# C5 A/B of batch orders on the general kernel: plain, length-sorted without LDS staging
# (EBPF_BUCKET=1 EBPF_BUCKET_NOSPAN=1), length-sorted span-staged (EBPF_BUCKET=1), path-sorted
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --config c5 --also= --no-pmc --no-cpu-baseline --steps 20 > gpurun_out/sab_$n.json 2> gpurun_out/sab_$n.err || exit 1; }
run plain EBPF_PATHSORT=0
run lensort EBPF_BUCKET=1 EBPF_BUCKET_NOSPAN=1
run lenspan EBPF_BUCKET=1
run lensort_xbr EBPF_BUCKET=1 EBPF_BUCKET_NOSPAN=1 EBPF_CC_RUN_XBR=1
run plain2 EBPF_PATHSORT=0
