# C5 plain launch: hoist ring of 16 VGPRs (default, 80 VGPRs: 6 waves per SIMD) vs 8 / 12 (abx/h8.so,
# abx/h12.so: 72 / 76 VGPRs, 7 / 6 waves per SIMD)
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --config c5 --also= --no-pmc --no-cpu-baseline --steps 20 > gpurun_out/hoist_$n.json 2> gpurun_out/hoist_$n.err || exit 1; }
run h16 X=1
run h8 EBPF_LIB=abx/h8.so
run h12 EBPF_LIB=abx/h12.so
run h16b X=1
run h8b EBPF_LIB=abx/h8.so
