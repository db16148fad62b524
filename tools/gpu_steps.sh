#!/bin/bash
# One GPU call, several steps, each under its own time limit; the first failure ends the call.
#   TAG=<dir under gpurun_out/> bash tools/gpu_steps.sh STEP...
# STEP forms:
#   tests[=<pytest -k expr>]      python -m pytest -m gpu tests (optionally -k)
#   smoke                          __graft_entry__.smoke()
#   bench:<name>:<bench.py args>   one bench line -> $O/bench_<name>.json
#   prof:<name>:<bench.py args>    rocprofv3 --kernel-trace --stats of a short bench run
#   pmc:<name>:<counters>:<bench.py args>   one rocprofv3 --pmc pass (kernel trace only besides)
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-steps}
mkdir -p "$O"
for st in "$@"; do
  echo "== $st ($(date +%T))"
  case "$st" in
    tests*)
      k="${st#tests}"; k="${k#=}"
      timeout -k 10 500 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
        ${k:+-k "$k"} tests > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
      tail -2 "$O/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { tail -5 "$O/smoke.log"; exit 1; }
      tail -1 "$O/smoke.log" ;;
    bench:*)
      rest="${st#bench:}"; name="${rest%%:*}"; args="${rest#*:}"
      timeout -k 10 400 python3 bench.py --pmc-dir "$O/pmc_$name" $args > "$O/bench_$name.json" \
        2> "$O/bench_$name.err" || { tail -5 "$O/bench_$name.err"; cat "$O/bench_$name.json"; exit 1; }
      cat "$O/bench_$name.json" ;;
    prof:*)
      rest="${st#prof:}"; name="${rest%%:*}"; args="${rest#*:}"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$name" -o prof -- \
        python3 bench.py --no-cpu-baseline --no-pmc --no-verify --also= $args > "$O/prof_$name.json" 2> "$O/prof_$name.err" \
        || { tail -5 "$O/prof_$name.err"; exit 1; }
      f=$(ls "$O"/prof_$name/*/prof_kernel_stats.csv "$O"/prof_$name/prof_kernel_stats.csv 2>/dev/null | head -1)
      [ -n "$f" ] && head -4 "$f" ;;
    pmc:*)
      rest="${st#pmc:}"; name="${rest%%:*}"; rest="${rest#*:}"; ctr="${rest%%:*}"; args="${rest#*:}"
      timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --kernel-include-regex 'ebpf_(interp|jit)' \
        --output-format csv -d "$O/pmc_$name" -o pmc -- python3 bench.py --no-cpu-baseline --no-pmc --no-verify --also= \
        $args > "$O/pmc_$name.json" 2> "$O/pmc_$name.err" || { tail -5 "$O/pmc_$name.err"; exit 1; } ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
