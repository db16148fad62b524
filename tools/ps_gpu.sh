set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_pathsort.py -x -v --timeout 200 --timeout-method thread > gpurun_out/ps_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/ps_tests.log
EBPF_PATHSORT=1 timeout -k 10 200 python -u bench.py --config c5 --also= --no-pmc --no-cpu-baseline --steps 30 > gpurun_out/ps_bench_on.json 2> gpurun_out/ps_bench_on.err &&
EBPF_PATHSORT=0 timeout -k 10 200 python -u bench.py --config c5 --also= --no-pmc --no-cpu-baseline --steps 30 > gpurun_out/ps_bench_off.json 2> gpurun_out/ps_bench_off.err
