# Round-end style evidence on the current tree: the GPU suite, smoke, the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/full/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/full/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/full/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1 || { tail -20 gpurun_out/full/smoke.log; exit 1; }
cat gpurun_out/full/smoke.log | tail -1
