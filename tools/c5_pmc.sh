#!/bin/bash
# SQ counters of the C5 class probe, regrouped (EBPF_CC_REGROUP=1, p_*_0) and not (p_*_1): CASE=<probe case>
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c5pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="${CTRS:-SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_ANY}"
for rg in 0 1; do
  for c in ${CASES:-imix all64}; do
    if [ $rg = 0 ]; then export EBPF_CC_REGROUP=1; else unset EBPF_CC_REGROUP; fi
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'ebpf_jit' --output-format csv -d $O/p_${c}_$rg -o p -- python $R/tools/c5_class_probe.py $c > $O/p_${c}_$rg.log 2>&1
  done
done
