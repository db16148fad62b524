"""N>1 path on CPU: world_size-2 gloo processes shard a C4 batch with shard_bounds, compute
their verdict histograms with the oracle, and all-reduce them; the sum must equal the
single-process histogram (the bench does the same with RCCL and the GPU kernel)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import goldens


def _hist(ret):
    h = np.zeros(257, dtype=np.int64)
    np.add.at(h, np.minimum(ret, 255).astype(np.int64), 1)
    return h


def _worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "tests"), os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    import pkgload
    pkgload.load()
    from generic_ebpf_amd import shard
    from helpers import oracle_run
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    case = [c for c in goldens.load(os.path.join(goldens.GOLDEN_DIR, "workloads.npz"))
            if c.name == "c4"][0]
    lo, hi = shard.shard_bounds(case.count, rank, world)
    sub = goldens.Case("s", case.code, case.relocs, case.maps,
                       case.data[lo * 64: hi * 64], hi - lo, 64, None)
    ret, _, _, _ = oracle_run(sub, nthreads=1)
    h = torch.from_numpy(_hist(ret))
    shard.reduce_hist(h)
    if rank == 0:
        np.save(out, h.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_histogram_equals_single(tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "h.npy")
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    case = [c for c in goldens.load(os.path.join(goldens.GOLDEN_DIR, "workloads.npz"))
            if c.name == "c4"][0]
    np.testing.assert_array_equal(np.load(out), _hist(case.expect_r0))


def test_shard_bounds_cover():
    from generic_ebpf_amd import shard
    for n in (0, 1, 7, 64, 1001):
        for w in (1, 2, 3, 8):
            spans = [shard.shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def _overlap_worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import pkgload
    pkgload.load()
    from generic_ebpf_amd import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bufs = [torch.zeros(257, dtype=torch.int64) for _ in range(2)]
    red = shard.OverlappedHistReduce(bufs)
    steps = 7
    for i in range(steps):   # bench.py's step: acquire, zero + fill, issue
        b = red.acquire(i)
        bufs[b].zero_()
        bufs[b][(i * 3 + rank) % 256] += 10 + i
        bufs[b][256] += rank
        red.issue(b)
    h = red.finish()
    if rank == 0:
        np.save(out, h.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_overlapped_reduce_last_step(tmp_path):
    """The double-buffered asynchronous reduce returns the last step's summed histogram."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "h.npy")
    mp.spawn(_overlap_worker, args=(2, port, out), nprocs=2, join=True)
    want = np.zeros(257, dtype=np.int64)
    last = 6
    for r in range(2):
        want[(last * 3 + r) % 256] += 10 + last
        want[256] += r
    np.testing.assert_array_equal(np.load(out), want)


def test_overlapped_reduce_single_process():
    from generic_ebpf_amd import shard
    bufs = [torch.zeros(257, dtype=torch.int64) for _ in range(2)]
    red = shard.OverlappedHistReduce(bufs)
    assert red.finish() is None
    for i in range(3):
        b = red.acquire(i)
        bufs[b].fill_(i)
        red.issue(b)
    assert int(red.finish()[0]) == 2
