#!/bin/bash
# Write phasing under other HBM writers, one GPU call: the stream shapes
# of tools/wphase_streams.py, then tools/e2e.py (host buffers: H2D copy engines write HBM during
# the kernels) with phasing on (default) and off (EBPF_WPHASE=0), one shard and two.
set -eu
O=gpurun_out/${TAG:-phasing}
mkdir -p "$O"
timeout -k 10 300 python3 -u tools/wphase_streams.py > "$O/streams.jsonl"
cat "$O/streams.jsonl"
for dv in 0 0,0; do
  for ph in default off; do
    if [ $ph = off ]; then export EBPF_WPHASE=0; else unset EBPF_WPHASE; fi
    timeout -k 10 300 python3 -u tools/e2e.py --pcap-packets 0 --reps 3 --devices $dv > "$O/e2e_${dv/,/_}_$ph.jsonl"
    sed "s/^/$ph /" "$O/e2e_${dv/,/_}_$ph.jsonl"
  done
done
