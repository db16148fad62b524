# Interpreter superinstructions: parity (GPU parity tests, fuzz) and C4 on variant 2 with / without fusion
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fuse_parity.log 2>&1 || { tail -20 gpurun_out/fuse_parity.log; exit 1; }
timeout -k 10 300 python -u tools/fuzz_gpu.py --programs 600 > gpurun_out/fuse_fuzz.log 2>&1 || { tail -5 gpurun_out/fuse_fuzz.log; exit 1; }
EBPF_INTERP_FUSE_DEBUG=1 timeout -k 10 120 python -u bench.py --config c4 --variant 2 --also= --no-pmc --no-cpu-baseline --steps 30 > gpurun_out/fuse_c4_v2.json 2> gpurun_out/fuse_c4_v2.err || exit 1
EBPF_INTERP_NOFUSE=1 timeout -k 10 120 python -u bench.py --config c4 --variant 2 --also= --no-pmc --no-cpu-baseline --steps 30 > gpurun_out/fuse_c4_v2_nofuse.json 2> gpurun_out/fuse_c4_v2_nofuse.err || exit 1
timeout -k 10 120 python -u bench.py --config c4 --variant 2 --also= --no-pmc --no-cpu-baseline --steps 30 > gpurun_out/fuse_c4_v2b.json 2> gpurun_out/fuse_c4_v2b.err
