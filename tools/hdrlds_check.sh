set -o pipefail
mkdir -p gpurun_out/hl
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu -k "standard or cursor or parity or fuzz or pcap or window or general" tests > gpurun_out/hl/pytest.log 2>&1 || { tail -30 gpurun_out/hl/pytest.log; exit 1; }
tail -1 gpurun_out/hl/pytest.log
timeout -k 10 200 python3 -u tools/c3l_general.py > gpurun_out/hl/c3l_general_on.json 2>gpurun_out/hl/err1.txt || { tail -5 gpurun_out/hl/err1.txt; exit 1; }
cat gpurun_out/hl/c3l_general_on.json
EBPF_NOHDRLDS=1 timeout -k 10 200 python3 -u tools/c3l_general.py > gpurun_out/hl/c3l_general_off.json 2>gpurun_out/hl/err2.txt || { tail -5 gpurun_out/hl/err2.txt; exit 1; }
cat gpurun_out/hl/c3l_general_off.json
