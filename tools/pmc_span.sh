#!/bin/bash
# PMC passes over the bucketed C5 launch (one rocprofv3 --pmc run per counter group, kernel trace
# only besides): per-dispatch counters of the ebpf kernels, for tools/pmc_classes.py.
export TMPDIR=/tmp EBPF_BUCKET=1
O=gpurun_out/${TAG:-pmcspan}
mkdir -p $O
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_IFETCH"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex 'ebpf_jit' --output-format csv \
    -d $O/p$i -o pmc -- python3 bench.py --config c5 --also= --no-cpu-baseline --no-pmc --no-verify --steps 3 --warmup 1 "$@" \
    > $O/p$i.json 2> $O/p$i.err || { tail -5 $O/p$i.err; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_classes.py $O 3
