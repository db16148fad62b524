set -o pipefail
T=r1l
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
python3 -c "import __graft_entry__ as g; g.build()" > gpurun_out/$T/build.log 2>&1 || { tail -20 gpurun_out/$T/build.log; exit 1; }
timeout -k 10 600 python3 tools/e2e.py > gpurun_out/$T/e2e.json 2> gpurun_out/$T/e2e.err || { tail -5 gpurun_out/$T/e2e.err; exit 1; }
cat gpurun_out/$T/e2e.json
timeout -k 10 600 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -5 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
lscpu > gpurun_out/$T/lscpu.txt; nproc >> gpurun_out/$T/lscpu.txt
