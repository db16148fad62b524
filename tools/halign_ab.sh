# Interpreter (variant 2) C4: handlers aligned to 4 B (default) / 64 B / 128 B (abx/ha6.so, ha7.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --config c4 --variant 2 --also= --no-pmc --no-cpu-baseline --steps 30 > gpurun_out/ha_$n.json 2> gpurun_out/ha_$n.err || exit 1; }
run a2 X=1
run a6 EBPF_LIB=abx/ha6.so
run a7 EBPF_LIB=abx/ha7.so
run a2b X=1
run a6b EBPF_LIB=abx/ha6.so
