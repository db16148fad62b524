#!/usr/bin/env python3
"""Host cost of bench.py's launch path for C2, split into what the
library costs and what ctypes / the Python step add.  Prints one JSON line per repetition:

  ctypes_us   : a trivial library call through ctypes (ebpf_gpu_device_count)
  enqueue_us  : the prepared launcher (native.Prog.launcher) alone, K calls, no wait
  step_us     : wall per step, K launches then synchronize (the launcher alone)
  bench_us    : wall per step of bench.py's own step loop shape (acquire, launch, issue; events
                every 2nd step), K steps then synchronize
  kernel_us   : event-timed kernel (median of the timed steps)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import pkgload  # noqa: E402

pkgload.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from generic_ebpf_amd import native, shard, workloads  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    cfg = sys.argv[2] if len(sys.argv) > 2 else "c2"
    n = 1 << 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    lay = workloads.CONFIGS[cfg]["prog"]()
    env = native.Env()
    prog = native.Prog(env, lay.code)
    pk = workloads.packets_random(1 << 16, 64, seed=2)
    d_pk = torch.from_numpy(pk).to(dev).repeat(n >> 16, 1).reshape(-1).contiguous()
    d_ret = torch.empty(n, dtype=torch.int64, device=dev)
    hists = [torch.zeros(257, dtype=torch.int64, device=dev) for _ in range(2)]
    red = shard.OverlappedHistReduce(hists)
    stream = torch.cuda.current_stream()
    launch = prog.launcher(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), None, None,
                           stream.cuda_stream, hist_overwrite=True)
    hptr = [h.data_ptr() for h in hists]
    for _ in range(50):
        launch(hptr[0])
    torch.cuda.synchronize()
    L = native.lib()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(K // 2)]
    for a, b in evs:
        a.record(stream)
        b.record(stream)
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(K):
            L.ebpf_gpu_device_count()
        t1 = time.perf_counter()
        for _ in range(K):
            launch(hptr[0])
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        k = 0
        for i in range(K):
            b = red.acquire(i)
            if i % 2 == 0:
                native.time_next_launch(evs[k][0].cuda_event, evs[k][1].cuda_event)
                k += 1
            launch(hptr[b])
            red.issue(b)
        red.finish()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        ks = float(np.median([a.elapsed_time(b) for a, b in evs])) * 1e3
        print(json.dumps({"cfg": cfg, "calls": K, "ctypes_us": round((t1 - t0) / K * 1e6, 2),
                          "enqueue_us": round((t2 - t1) / K * 1e6, 2),
                          "step_us": round((t3 - t1) / K * 1e6, 2),
                          "bench_us": round((t4 - t3) / K * 1e6, 2), "kernel_us": round(ks, 2)}),
              flush=True)
    prog.destroy()
    env.destroy()


if __name__ == "__main__":
    main()
