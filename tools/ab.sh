#!/bin/bash
# A/B runs of bench.py lines, alternating cases round by round (box drift spreads evenly):
#   tools/ab.sh OUT STEPS ROUNDS CASE...
# CASE = name=config[+VAR=value...][+--bench-arg=value...], e.g.
#   c4_off=c4+EBPF_WPHASE=0   c4h_wg5=c4h+EBPF_WG_PER_CU=5   c4_8m=c4+--packets=8388608
# Each run writes OUT/<name>_<round>.json (one bench line); tools/ab_summary.py OUT tabulates.
# Every run has its own time limit; the first failure ends the script.
set -u
O=$1 STEPS=$2 ROUNDS=$3
shift 3
mkdir -p "$O"
for k in $(seq 0 $((ROUNDS - 1))); do
  for c in "$@"; do
    name=${c%%=*}
    IFS=+ read -r -a parts <<< "${c#*=}"
    cfg=${parts[0]}
    envs=() args=()
    for p in "${parts[@]:1}"; do
      case "$p" in
        --*) args+=("$p") ;;
        *) envs+=("$p") ;;
      esac
    done
    cmd=(timeout -k 10 200 python bench.py --also= --no-pmc --no-cpu-baseline --steps "$STEPS"
         --warmup 5 --config "$cfg" "${args[@]}")
    if [ -n "${DRY:-}" ]; then echo "${envs[*]} ${cmd[*]} > $O/${name}_$k.json"; continue; fi
    ( for e in "${envs[@]}"; do export "$e"; done
      "${cmd[@]}" > "$O/${name}_$k.json" 2>/dev/null ) || exit 1
  done
done
