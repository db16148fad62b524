"""Worker for tests/test_multi_gpu.py::test_two_ranks_gloo_equal_one_launch (run under torch.distributed.run, gloo, every rank on
cuda:0): each rank runs its contiguous shard of one C4 / C5 batch on the device
(ebpf_prog_run_batch_dev, the bench's path), the shards' results are gathered to rank 0 and the
histograms summed (the only collective); rank 0 compares them with ONE launch over the whole
batch.  Exit code 0 = equal."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bench  # noqa: E402  (Workload: the bench's shard construction)
from generic_ebpf_amd import native, shard  # noqa: E402


def run(w, env, torch, dev):
    maps = bench.make_maps(env, w.maps)
    prog = native.Prog(env, native.patch_relocs(w.lay.code, w.lay.relocs, [m.handle for m in maps]))
    d_pk, d_offs = w.device_packets(torch, dev)
    d_ret = torch.full((max(w.n, 1),), -1, dtype=torch.int64, device=dev)
    d_hist = torch.full((257,), 777, dtype=torch.int64, device=dev)
    prog.run_batch_dev(0, d_pk.data_ptr(), w.n, 64, d_ret.data_ptr(),
                       None if d_offs is None else d_offs.data_ptr(), None, d_hist.data_ptr(),
                       torch.cuda.current_stream().cuda_stream, hist_overwrite=True)
    torch.cuda.synchronize()
    out = d_ret[: w.n].cpu(), d_hist.cpu()
    prog.destroy()
    for m in maps:
        m.destroy()
    return out


def main():
    import torch
    import torch.distributed as dist
    cfg, total = sys.argv[1], int(sys.argv[2])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    env = native.Env()
    lo, hi = shard.shard_bounds(total, rank, world)
    ret, hist = run(bench.Workload(cfg, lo, hi, total), env, torch, dev)
    sizes = [shard.shard_bounds(total, r, world) for r in range(world)]
    buf = torch.zeros(max(b - a for a, b in sizes), dtype=torch.int64)
    buf[: ret.numel()] = ret
    gathered = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(gathered, buf)
    dist.all_reduce(hist)
    ok = True
    info = {}
    if rank == 0:
        cat = torch.cat([g[: b - a] for g, (a, b) in zip(gathered, sizes)])
        ret1, hist1 = run(bench.Workload(cfg, 0, total, total), env, torch, dev)
        info = {"cfg": cfg, "total": total, "world": world,
                "ret_mismatch": int((cat != ret1).sum()),
                "hist_equal": bool(torch.equal(hist, hist1)),
                "hist_sum": int(hist.sum())}
        ok = info["ret_mismatch"] == 0 and info["hist_equal"] and info["hist_sum"] == total
        print(json.dumps(info), flush=True)
    assert env.destroy() == 0
    flag = torch.tensor([1 if ok else 0])
    dist.broadcast(flag, 0)
    dist.destroy_process_group()
    sys.exit(0 if int(flag[0]) else 1)


if __name__ == "__main__":
    main()
