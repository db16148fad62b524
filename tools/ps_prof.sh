set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ps_prof -o run -- python -u bench.py --config c5 --also= --no-pmc --no-cpu-baseline --no-verify --steps 10 --warmup 3 > gpurun_out/ps_prof.log 2>&1
