"""bench.py's rank-count-dependent logic at world sizes 4 and 8, on CPU (gloo), with the oracle
standing in for the GPU: the driver runs the bench at N = 1, 2, 4, 8, and only N <= 2 ever ran
before it.

Each rank builds its shard exactly as bench.measure does (shard.shard_bounds, bench.Workload:
the contiguous part [lo, hi) of the global batch, a fixed-size config's distinct packets rotated
by lo % D and tiled, C5's IMIX stream cut at lo / hi), computes what the device would return
for the packets of that shard (the oracle run over Workload.device_packets, the very bytes
bench.py uploads), sums the verdict histograms with an all-reduce and calls bench.verify — the
check that compares a shard's results against the oracle's results for the DISTINCT packets,
re-tiled by its own arithmetic.  The two tilings must agree on every rank: verified, and a single
flipped result on the last rank must make every rank report the mismatch.  C4C also runs
bench.verify_counters against the counter map the shard's packets produce.  bench.DISTINCT is
lowered so that every shard wraps around the distinct set (k > 0 tiles and a remainder r > 0)
and the totals are not multiples of N."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [("c4", 10007, 1153), ("c4c", 9001, 997), ("c3l", 7919, 877), ("c5", 6007, None),
         ("c2", 5003, 613)]


class _CounterMap:
    """Stands in for native.Map in bench.verify_counters: lookup(key) -> (0, value bytes)."""

    def __init__(self, data):
        self.data = data

    def lookup(self, key):
        return 0, self.data[8 * key: 8 * key + 8]


def _worker(rank, world, port, outdir):
    for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import bench
    import pyoracle
    from generic_ebpf_amd import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cpu")
    report = {}
    for cfg, total, distinct in CASES:
        if distinct:
            bench.DISTINCT = distinct
        lo, hi = shard.shard_bounds(total, rank, world)
        w = bench.Workload(cfg, lo, hi, total)
        d_pk, d_offs = w.device_packets(torch, dev)
        maps = w.oracle_maps()
        if cfg == "c4c":
            maps = [maps[0], (8, 256, bytes(8 * 256))]
        op = pyoracle.OracleProgram(w.lay.code, w.lay.relocs, maps, semantics=w.semantics)
        data = d_pk.numpy()
        if d_offs is None:
            ret, flt, _, _ = op.run(data, w.n, 64, None)
        else:
            ret, flt, _, _ = op.run(data, w.n, 0, d_offs.numpy().view(np.uint64))
        d_ret = torch.from_numpy(ret.view(np.int64).copy())
        bins = np.where(flt != 0, 256, np.minimum(ret, 255)).astype(np.int64)
        hist = torch.from_numpy(np.bincount(bins, minlength=257).astype(np.int64))
        dist.all_reduce(hist)
        assert int(hist.sum()) == total
        ok, info = bench.verify(w, torch, d_ret, hist, world, dev)
        r = {"ok": ok, "info": info, "n": w.n, "lo": lo,
             "tiles": (w.n // w.D) if w.offs is None else None,
             "rem": (w.n % w.D) if w.offs is None else None}
        if cfg == "c4c":
            launches = 3   # every launch adds the shard's counts once more
            once = np.frombuffer(op.map_bytes(1), dtype=np.uint64).astype(object)
            data3 = b"".join(int(x * launches % (1 << 64)).to_bytes(8, "little") for x in once)
            r["counters"] = bench.verify_counters(w, [None, _CounterMap(data3)], launches)
        # one flipped result on the last rank: every rank must see the mismatch
        if rank == world - 1 and w.n:
            d_ret[w.n // 2] ^= 1
        ok2, info2 = bench.verify(w, torch, d_ret, hist, world, dev)
        r["flipped_ok"] = ok2
        r["flipped_mismatches"] = info2["ret_mismatches"]
        report[cfg] = r
    with open(os.path.join(outdir, "rank%d.json" % rank), "w") as f:
        json.dump(report, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [4, 8])
def test_bench_shard_verify_tiling_at_world(world, tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    reps = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(world)]
    for cfg, total, distinct in CASES:
        got = [rep[cfg] for rep in reps]
        assert sum(g["n"] for g in got) == total, cfg
        assert len({g["n"] for g in got}) > 1 or total % world == 0, cfg   # uneven shards
        for g in got:
            assert g["ok"], (cfg, g["info"])
            assert not g["flipped_ok"] and g["flipped_mismatches"] == 1, (cfg, g)
        if distinct:   # the shards wrap the distinct set: full tiles and a remainder, rotated starts
            assert any(g["tiles"] > 0 and g["rem"] > 0 for g in got), cfg
            assert any(g["lo"] % distinct for g in got), cfg
        if cfg == "c4c":
            for g in got:
                assert g["counters"]["counters_verified"], g["counters"]
                assert g["counters"]["counted_per_launch"] > 0
