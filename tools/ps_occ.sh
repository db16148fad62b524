# C5 path-sorted step time at 1..8 workgroups per CU (EBPF_WG_PER_CU: every launch of the step)
set -o pipefail
cd $GRAFT_REPO_ROOT
for w in 1 2 3 4 6 8; do
  EBPF_PATHSORT=1 EBPF_WG_PER_CU=$w timeout -k 10 120 python -u bench.py --config c5 --also= --no-pmc --no-cpu-baseline --no-verify --steps 20 > gpurun_out/ps_occ_w$w.json 2> gpurun_out/ps_occ_w$w.err || exit 1
done
