#!/usr/bin/env python3
"""Device-resident batch eBPF throughput on MI355X (BASELINE.json metric).

One step = one launch of the interpreter over the rank's whole device-resident batch (the
workload named by --config; default C4: the 64-insn VALE-BPF-style classify + one array-map
lookup per packet over 64M x 64 B synthetic packets per GPU) plus the per-step verdict
histogram all-reduce (RCCL) when N > 1.  Packets are synthetic (seeded generator) and resident
in HBM before timing starts.  Multi-GPU: one process per GPU (torch.distributed.run), each
rank runs its own 64M-packet shard (weak scaling), the only collective is the 257-bin
histogram all-reduce, issued asynchronously so that it runs under the next step's kernel.

roofline.kernel_ms is the interpreter kernel alone: HIP events that the library records on the
launch stream just before and after that kernel (ebpf_gpu_time_next_launch), so it compares
with the kernel's average in a rocprofv3 --kernel-trace --stats summary.  Every 5th timed step
carries the events (--time-every): each event pair costs a launch gap.

Prints ONE JSON line on rank 0 (see README / DESIGN.md for the fields).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pkgload  # noqa: E402

pkg = pkgload.load()
from generic_ebpf_amd import native, shard, workloads  # noqa: E402

PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c4", choices=sorted(workloads.CONFIGS))
    ap.add_argument("--packets", type=int, default=0, help="packets per GPU (default per config)")
    ap.add_argument("--variant", type=int, default=0, help="0 = default interpreter, 1 = HIP baseline")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--time-every", type=int, default=5,
                    help="event-time the kernel of every k-th timed step (default 5: a pair of events per step costs C2 7 us of its 21-us step; profiles/r01/te)")
    ap.add_argument("--launch", default="eager", choices=["graph", "eager"],
                    help="eager: direct launches (default); graph: each step replays a captured HIP graph (measured 1.6%% slower on C2-C4, profiles/r01/graph_ab)")
    return ap.parse_args()


DEFAULT_PACKETS = {"nop200": 1 << 24, "alu200": 1 << 24, "c0": 1 << 26, "c2": 1 << 20, "c3": 1 << 24,
                   "c4": 1 << 26, "c5": 1 << 22, "c4h": 1 << 26}
C4H_SLOT_BYTES = 32  # device table slot: u32 used | u32 hash | 4-B key (8-B padded) | 8-B value
DISTINCT = 1 << 22  # distinct synthetic packets generated on the host, tiled in HBM


def build_inputs(cfg, n, rank):
    """Host-side synthetic inputs for one rank: (layout, maps spec, packets u8, offsets|None)."""
    lay = workloads.CONFIGS[cfg]["prog"]()
    maps = []
    if cfg == "c4":
        maps = [(8, 256, workloads.c4_map_values().tobytes())]
    if cfg == "c4h":   # ("hash", key_size, value_size, max_entries, keys, values)
        universe, keys, values = workloads.c4h_table()
        maps = [("hash", 4, 8, len(keys), keys, values)]
        return lay, maps, workloads.packets_c4h(min(n, DISTINCT), universe, seed=4 + 1000 * rank), None
    if cfg == "c5":
        data, offs, _ = workloads.packets_imix(n, seed=5 + rank)
        return lay, maps, data, offs
    d = min(n, DISTINCT)
    rnd = cfg in ("c0", "c2", "nop200", "alu200")
    gen = workloads.packets_random if rnd else workloads.packets_l2l3
    return lay, maps, gen(d, 64, seed=(2 if rnd else 3) + 1000 * rank), None


def cpu_baseline(cfg, lay, maps, pk, offs, budget_s):
    """Oracle (the CPU restatement of the reference interpreter, raw-pointer mode like the
    reference) on a bounded sample of the same workload, all host threads up to 16."""
    import pyoracle
    threads = max(1, min(16, os.cpu_count() or 1))
    if offs is not None:
        n = min(len(offs) - 1, 1 << 18)
        data, offsets = pk[: int(offs[n])], offs[: n + 1]
    else:
        n = min(pk.shape[0], 1 << 20)
        data, offsets = pk[:n].reshape(-1), None
    maps = [pyoracle.HashSpec(m[1], m[2], keys=m[4], values=m[5]) if m[0] == "hash" else m
            for m in maps]
    op = pyoracle.OracleProgram(lay.code, lay.relocs, maps, checked=False)
    op.run(data, n, 64, offsets, nthreads=threads)  # warm
    t0 = time.perf_counter()
    passes = 0
    while True:
        op.run(data, n, 64, offsets, nthreads=threads)
        passes += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": round(n * passes / el / 1e6, 2), "unit": "Mpkt/s", "cores": threads,
            "kind": "port",
            "sample": "%d passes over %d %s packets (%s), %d host threads, %.1f s" % (
                passes, n, cfg.upper(), "IMIX" if offsets is not None else "64 B", threads, el)}


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # nccl (= RCCL) on the node; EBPF_BENCH_BACKEND=gloo rehearses N > 1 on one GPU
        dist.init_process_group(os.environ.get("EBPF_BENCH_BACKEND", "nccl"))
    if world > 1 and os.environ.get("EBPF_BENCH_BACKEND") == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cfg = a.config
    n = a.packets or DEFAULT_PACKETS[cfg]

    lay, maps_spec, pk, offs = build_inputs(cfg, n, rank)
    env = native.Env()
    maps = []
    for spec in maps_spec:
        if spec[0] == "hash":
            _, ks, vs, me, keys, values = spec
            m = native.HashMap(env, ks, vs, me)
            m.fill(keys, values)
        else:
            vs, me, d = spec
            m = native.Map(env, me, vs)
            m.fill(d)
        maps.append(m)
    prog = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    native.set_variant(a.variant)
    prog.prepare(local)

    # device-resident inputs
    if offs is None:
        base = torch.from_numpy(pk.reshape(-1)).to(dev)
        reps = (n + pk.shape[0] - 1) // pk.shape[0]
        d_pk = base.repeat(reps)[: n * 64].contiguous()
        del base
        d_offs = None
        bytes_per_launch = n * 64
        if cfg == "c4h":  # + one table slot per packet that reaches the lookup (IPv4, not ICMP)
            et = (pk[:, 12].astype(np.uint32) << 8) | pk[:, 13]
            reach = float(np.mean((et == 0x0800) & (pk[:, 23] != 1)))
            bytes_per_launch = int(n * 64 + round(n * reach) * C4H_SLOT_BYTES)
    else:
        d_pk = torch.from_numpy(pk).to(dev)
        d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
        sizes = np.diff(offs)
        bytes_per_launch = int(sizes.sum()) + 8 * (n + 1)
    d_ret = torch.empty(n, dtype=torch.int64, device=dev)
    # two histogram buffers: the all-reduce of step i (N > 1) overlaps the launch of step i + 1
    hists = [torch.zeros(257, dtype=torch.int64, device=dev) for _ in range(2)]
    red = shard.OverlappedHistReduce(hists)

    def launch(h, stream):  # the launch sets h to this batch's counts (no memset first)
        prog.run_batch_dev(local, d_pk.data_ptr(), n, 64, d_ret.data_ptr(),
                           None if d_offs is None else d_offs.data_ptr(), None,
                           h.data_ptr(), stream.cuda_stream, hist_overwrite=True)

    # HIP graphs (one per histogram buffer): the zeroing memset, the interpreter and the
    # histogram reduce replay as one submission, with no per-step host launch gaps
    graphs = None
    if a.launch == "graph":
        launch(hists[0], torch.cuda.current_stream())  # map mirrors and program uploaded
        torch.cuda.synchronize()
        try:
            graphs = []
            for h in hists:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    launch(h, torch.cuda.current_stream())
                graphs.append(g)
        except Exception as e:  # capture unsupported: eager launches, said in the bench line
            print("graph capture failed (%s); eager launches" % e, file=sys.stderr)
            graphs = None
            torch.cuda.synchronize()
    stream = torch.cuda.current_stream()

    def step(i, ev=None):
        b = red.acquire(i)
        if graphs is not None:  # events around the replay (histogram reduce in it)
            if ev is not None:
                ev[0].record(stream)
            graphs[b].replay()
            if ev is not None:
                ev[1].record(stream)
        else:
            if ev is not None:  # the library records them around the interpreter kernel alone
                native.time_next_launch(ev[0].cuda_event, ev[1].cuda_event)
            launch(hists[b], stream)
        red.issue(b)

    for i in range(a.warmup):
        step(i)
    red.finish()
    torch.cuda.synchronize()
    timed = list(range(0, a.steps, max(1, a.time_every)))  # steps whose kernel is event-timed
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in timed]
    for e0, e1 in evs:  # torch creates its events at their first record
        e0.record(stream)
        e1.record(stream)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    k = 0
    for i in range(a.steps):
        if k < len(timed) and timed[k] == i:
            step(i, evs[k])
            k += 1
        else:
            step(i)
    d_hist = red.finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in evs]))
    if world > 1:
        t = torch.tensor([el, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, kern_ms = float(t[0]), float(t[1])
    ms_per_step = el * 1e3 / a.steps
    total_pkts = n * world * a.steps
    value = total_pkts / el / 1e6

    hist = d_hist.cpu().numpy()
    faulted = int(hist[256])
    if int(hist.sum()) != n * world:  # every packet lands in exactly one bin of the last step
        raise SystemExit("verdict histogram counts %d packets, expected %d" % (int(hist.sum()), n * world))
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    info = prog.info()
    if rank == 0:
        cpu = None
        if not a.no_cpu_baseline and world == 1:
            maps_for_oracle = maps_spec
            cpu = cpu_baseline(cfg, lay, maps_for_oracle, pk, offs, a.cpu_seconds)
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % cfg)
        if os.path.exists(pmc):
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        out = {
            "metric": "Mpkt/s device-resident (64-insn filter, 64B pkts); achieved HBM GB/s vs peak",
            "value": round(value, 1), "unit": "Mpkt/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": cfg, "desc": workloads.CONFIGS[cfg]["desc"],
                       "packets_per_gpu": n, "packet_bytes": 64 if offs is None else "IMIX",
                       "main_path_insns": lay.main_path_steps, "prog_slots": lay.nslots,
                       "dprog_entries": info.nentries, "variant": a.variant,
                       "parallelism": "dp%d" % world,
                       "launch": "graph" if graphs is not None else "eager", "faulted_packets": faulted},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
                         "traffic": traffic, "kernel_ms": round(kern_ms, 4),
                         "kernel_ms_samples": len(evs),
                         "algorithmic_bytes_per_launch": bytes_per_launch},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    prog.destroy()
    for m in maps:
        m.destroy()
    env.destroy()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
