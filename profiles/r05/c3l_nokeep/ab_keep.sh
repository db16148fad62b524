# (EBPF_NOKEEP was a temporary host switch for this probe, removed after it lost:
# profiles/r05/c3l_nokeep/README.md)
# C3L: keep mode (run-time-offset loads from the LDS packet buffer, the next DMA at the group's
# end) against none (uniform offsets from the packet registers, others from global memory, the
# next DMA prefetched), x write phasing x 4 / 6 workgroups per CU.  gpurun_out/keep/
O=gpurun_out/keep
mkdir -p $O
B="python bench.py --also= --no-pmc --no-cpu-baseline --steps 60 --warmup 10 --config c3l"
for k in 0 1; do
  timeout -k 10 200 $B > $O/keep_$k.json 2>/dev/null || exit 1
  EBPF_NOKEEP=1 timeout -k 10 200 $B > $O/nokeep_$k.json 2>/dev/null || exit 1
  EBPF_NOKEEP=1 EBPF_WPHASE=12,1024,16 timeout -k 10 200 $B > $O/nokeep_wide_$k.json 2>/dev/null || exit 1
  EBPF_NOKEEP=1 EBPF_WG_PER_CU=4 timeout -k 10 200 $B > $O/nokeep_wg4_$k.json 2>/dev/null || exit 1
  EBPF_NOKEEP=1 EBPF_WG_PER_CU=4 EBPF_WPHASE=12,1024,16 timeout -k 10 200 $B > $O/nokeep_wg4_wide_$k.json 2>/dev/null || exit 1
done
