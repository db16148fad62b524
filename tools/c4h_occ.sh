# C4H kernel time vs workgroups per CU (the staged compiled kernel admits 6 at 80 VGPRs / 98 SGPRs)
set -o pipefail
cd $GRAFT_REPO_ROOT
for w in 3 4 5 6; do
  EBPF_WG_PER_CU=$w timeout -k 10 200 python -u bench.py --config c4h --also= --no-pmc --no-cpu-baseline --no-verify --steps 20 > gpurun_out/c4h_occ_w$w.json 2> gpurun_out/c4h_occ_w$w.err || exit 1
done
