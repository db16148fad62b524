#!/bin/bash
# C5 window launches: workgroups per CU sweep, then one PMC pass of the window kernel.
set -u
OUT=gpurun_out/${TAG:-r4ws}
mkdir -p "$OUT"
export TMPDIR=/tmp
for wg in ${WGS:-1 2 3 4}; do
  echo "== wg=$wg $(date +%T)"
  EBPF_WINDOW=1 EBPF_WIN_WG=$wg timeout -k 10 200 python -u bench.py --config c5 --also= --no-pmc --no-cpu-baseline --no-verify --steps 20 --warmup 5 > "$OUT/c5_wg$wg.json" 2> "$OUT/c5_wg$wg.err"
  rc=$?; python -c "import json;d=json.load(open('$OUT/c5_wg$wg.json'));print('wg=$wg', d['ms_per_step'], d['roofline']['kernel_ms'])"; [ $rc -eq 0 ] || exit $rc
done
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH"; do
  tag=$(echo $grp | cut -d' ' -f1)
  echo "== pmc $tag $(date +%T)"
  EBPF_WINDOW=${PMC_WINDOW:-1} timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex ebpf_jit --output-format csv -d "$OUT/pmc_$tag" -o pmc -- python -u bench.py --config c5 --also= --no-pmc --no-cpu-baseline --no-verify --steps 2 --warmup 1 > "$OUT/pmc_$tag.log" 2>&1
  rc=$?; tail -2 "$OUT/pmc_$tag.log"; [ $rc -eq 0 ] || exit $rc
done
echo "== done $(date +%T)"
