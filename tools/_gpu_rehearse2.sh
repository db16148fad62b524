#!/bin/bash
# N = 2 rehearsal of bench.py's distributed path on one GPU (both ranks on cuda:0, gloo): the
# overlapped histogram all-reduce, max-over-ranks timing and the histogram check.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-rehearse2}
mkdir -p $O
EBPF_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config c4 --packets 16777216 \
  --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_n2.json 2> $O/bench_n2.err || { tail -20 $O/bench_n2.err; exit 1; }
grep '^{' $O/bench_n2.json | cut -c1-420
