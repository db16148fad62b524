# C5 A/B: plain, path-sorted, path-sorted with runs continuing past short exits (EBPF_CC_RUN_XBR),
# and hoist rings of 32 / 48 VGPRs (abx/h32.so, abx/h48.so: EBPF_ASM_GENHOIST builds)
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { # name env...
  n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --config c5 --also= --no-pmc --no-cpu-baseline --steps 20 > gpurun_out/ps_ab_$n.json 2> gpurun_out/ps_ab_$n.err || exit 1
}
run plain EBPF_PATHSORT=0
run ps EBPF_PATHSORT=1
run psx EBPF_PATHSORT=1 EBPF_CC_RUN_XBR=1
run ps_h32 EBPF_PATHSORT=1 EBPF_LIB=abx/h32.so
run psx_h32 EBPF_PATHSORT=1 EBPF_CC_RUN_XBR=1 EBPF_LIB=abx/h32.so
run psx_h48 EBPF_PATHSORT=1 EBPF_CC_RUN_XBR=1 EBPF_LIB=abx/h48.so
run plain_h32 EBPF_PATHSORT=0 EBPF_LIB=abx/h32.so
