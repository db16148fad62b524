#!/bin/bash
# C5 study on one box: occupancy sweep of the class probe, then PMC passes on the IMIX case.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c5s
mkdir -p $O
for w in ${WGS:-1 2 3 4 6}; do
	echo "== wg_per_cu $w" >> $O/occ.txt
	EBPF_WG_PER_CU=$w timeout -k 10 200 python -u $R/tools/c5_class_probe.py ${CASES:-imix all576 all1500} 2>&1 | grep -v amdgpu.ids >> $O/occ.txt
done
cd /tmp && export TMPDIR=/tmp
i=0
for p in "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
	 "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum" \
	 "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
	i=$((i+1))
	timeout -s KILL 120 rocprofv3 --pmc $p --kernel-include-regex 'ebpf_jit' --output-format csv -d $O/pmc$i -o p -- python $R/tools/c5_class_probe.py ${PMC_CASE:-imix} > $O/pmc$i.log 2>&1
done
