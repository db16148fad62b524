#!/usr/bin/env python3
"""Write phasing with other HBM writers on the device.

Phasing makes every wave of a staged streaming launch write its results only inside windows of
the GPU-wide constant clock (asm_runtime.cpp L.wphase).  Its gain needs the whole GPU to write in
the same windows; this measures C4 (64M x 64 B, device-resident) when something else writes HBM
during the kernel, phasing on (default) against off (EBPF_WPHASE=0, read at each launch):

  one      one stream, one 64M launch per step (the bench line's shape)
  halves   two streams, a 32M launch on each per step, concurrent (two launches of the library
           in flight on the device)
  copy     one 64M launch, with a 512 MB device-to-device copy on a second stream in flight

Each step is timed by wall clock between device synchronisations, the best-of and median over
--steps steps reported; every configuration's results are checked equal to the first's.  One JSON
line per (shape, phasing)."""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from generic_ebpf_amd import native, workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 26)
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    n = a.packets
    lay = workloads.CONFIGS["c4"]["prog"]()
    env = native.Env()
    m = native.Map(env, 256, 8)
    m.fill(workloads.c4_map_values().tobytes())
    prog = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [m.handle]))
    prog.prepare(0)
    distinct = torch.from_numpy(workloads.packets_l2l3(1 << 22, 64, seed=3).reshape(-1))
    pk = distinct.to(dev).repeat(n // (1 << 22))
    ret = torch.zeros(n, dtype=torch.int64, device=dev)
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()
    junk_a = torch.empty(1 << 29, dtype=torch.uint8, device=dev)
    junk_b = torch.empty_like(junk_a)
    half = n // 2

    def step(shape):
        if shape == "halves":
            prog.run_batch_dev(0, pk.data_ptr(), half, 64, ret.data_ptr(), stream=s1.cuda_stream)
            prog.run_batch_dev(0, pk.data_ptr() + half * 64, n - half, 64, ret.data_ptr() + half * 8,
                               stream=s2.cuda_stream)
        elif shape == "copy":
            with torch.cuda.stream(s2):
                junk_b.copy_(junk_a)
            prog.run_batch_dev(0, pk.data_ptr(), n, 64, ret.data_ptr(), stream=s1.cuda_stream)
        else:
            prog.run_batch_dev(0, pk.data_ptr(), n, 64, ret.data_ptr(), stream=s1.cuda_stream)

    ref = None
    for shape in ("one", "halves", "copy"):
        for phasing in ("on", "off"):
            if phasing == "off":
                os.environ["EBPF_WPHASE"] = "0"
            else:
                os.environ.pop("EBPF_WPHASE", None)
            for _ in range(3):
                step(shape)
            torch.cuda.synchronize()
            times = []
            for _ in range(a.steps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                step(shape)
                torch.cuda.synchronize()
                times.append((time.perf_counter() - t0) * 1e3)
            out = ret.cpu().numpy()
            if ref is None:
                ref = out.copy()
            same = bool(np.array_equal(out, ref))
            med = statistics.median(times)
            print(json.dumps({"shape": shape, "phasing": phasing, "packets": n,
                              "ms_median": round(med, 4), "ms_best": round(min(times), 4),
                              "gpkt_s_median": round(n / med / 1e6, 1), "results_equal": same}),
                  flush=True)
    os.environ.pop("EBPF_WPHASE", None)
    prog.destroy()
    m.destroy()
    env.destroy()


if __name__ == "__main__":
    main()
