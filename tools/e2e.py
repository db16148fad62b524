#!/usr/bin/env python3
"""End-to-end (host memory in, host memory out) rate of ebpf_prog_run_batch: packets start in a
host buffer (pinned, as a NIC ring or pcap buffer would be, or pageable), results land in a host
array.  Includes H2D, kernel and D2H (chunked, double-buffered on two streams inside the library).
Prints one JSON line per buffer kind."""
import argparse
import json
import os
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
    ap.add_argument("--config", default="c4")
    ap.add_argument("--packets", type=int, default=1 << 26)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pcap-packets", type=int, default=1 << 24,
                    help="also: a pcap capture of this many 64-B frames in host memory turned into a "
                         "batch by ebpf_pcap_batch (pinned), then run (0: skip)")
    ap.add_argument("--devices", default="",
                    help="comma list: ebpf_prog_run_batch_multi over these devices (repeats allowed)")
    a = ap.parse_args()
    import torch
    n = a.packets
    lay = workloads.CONFIGS[a.config]["prog"]()
    env = native.Env()
    maps = []
    if a.config == "c4":
        m = native.Map(env, 256, 8)
        m.fill(workloads.c4_map_values().tobytes())
        maps.append(m)
    prog = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    prog.prepare(0)
    distinct = workloads.packets_l2l3(1 << 22, 64, seed=3)
    for kind in ("pinned", "pageable"):
        t = torch.empty(n * 64, dtype=torch.uint8, pin_memory=(kind == "pinned"))
        host = t.numpy()
        reps = (n + distinct.shape[0] - 1) // distinct.shape[0]
        for r in range(reps):
            lo = r * distinct.shape[0]
            hi = min(n, lo + distinct.shape[0])
            host[lo * 64:hi * 64] = distinct[: hi - lo].reshape(-1)
        rt = torch.empty(n, dtype=torch.int64, pin_memory=(kind == "pinned"))
        ret = rt.numpy().view(np.uint64)
        st = native.BatchStats()
        b = native.PktBatch(host.ctypes.data, None, n, 64, 0)
        devs = [int(x) for x in a.devices.split(",")] if a.devices else None

        def run():
            if devs is None:
                return native.lib().ebpf_prog_run_batch(prog.ptr, native.ctypes.byref(b),
                                                         ret.ctypes.data, None,
                                                         native.ctypes.byref(st))
            d = (native.ctypes.c_int * len(devs))(*devs)
            return native.lib().ebpf_prog_run_batch_multi(prog.ptr, len(devs), d,
                                                           native.ctypes.byref(b), ret.ctypes.data,
                                                           None, native.ctypes.byref(st))
        native._check(run(), "warm")
        first = ret.copy()
        best = None
        for _ in range(a.reps):
            t0 = time.perf_counter()
            native._check(run(), "run")
            el = time.perf_counter() - t0
            if best is None or el < best[0]:
                best = (el, st.kernel_ms, st.total_ms)
        el, kms, tms = best
        assert (ret == first).all() and int(sum(st.hist)) == n
        print(json.dumps({"e2e": kind, "config": a.config, "packets": n,
                          "devices": devs or [0],
                          "mpkt_s": round(n / el / 1e6, 1), "wall_ms": round(el * 1e3, 2),
                          "kernel_ms_sum": round(kms, 2), "h2d_gb_s": round(n * 64 / el / 1e9, 2),
                          "faulted": int(st.faulted)}), flush=True)
        del t, rt
    if a.pcap_packets:
        # a capture in memory: 24-B global header, then per frame a 16-B record header + 64 B
        npk = a.pcap_packets
        rec = np.zeros((npk, 80), dtype=np.uint8)
        hdr = rec[:, :16].view(np.uint32)
        hdr[:, 0] = 1700000000
        hdr[:, 1] = np.arange(npk, dtype=np.uint32) % 1000000
        hdr[:, 2] = 64
        hdr[:, 3] = 64
        reps = (npk + distinct.shape[0] - 1) // distinct.shape[0]
        for r in range(reps):
            lo = r * distinct.shape[0]
            hi = min(npk, lo + distinct.shape[0])
            rec[lo:hi, 16:] = distinct[: hi - lo]
        gh = np.array([0xA1B2C3D4, 0x00040002, 0, 0, 65535, 1], dtype=np.uint32).view(np.uint8)
        cap = np.concatenate([gh, rec.reshape(-1)])
        del rec
        parse_ms = {}
        for pinned in (0, 1):   # the batch in pageable, then pinned memory (kept for the run)
            t0 = time.perf_counter()
            pb = native.PktBatch()
            pi = native.PcapInfo()
            native._check(native.lib().ebpf_pcap_batch(cap.ctypes.data, len(cap), pinned,
                                                       native.ctypes.byref(pb), native.ctypes.byref(pi)),
                          "ebpf_pcap_batch")
            parse = time.perf_counter() - t0
            parse_ms["pinned" if pinned else "pageable"] = round(parse * 1e3, 2)
            if not pinned:
                native.lib().ebpf_pcap_batch_free(native.ctypes.byref(pb))
        ret = np.zeros(npk, dtype=np.uint64)
        st = native.BatchStats()
        native._check(native.lib().ebpf_prog_run_batch(prog.ptr, native.ctypes.byref(pb), ret.ctypes.data,
                                                       None, native.ctypes.byref(st)), "warm")
        best = None
        for _ in range(a.reps):
            t0 = time.perf_counter()
            native._check(native.lib().ebpf_prog_run_batch(prog.ptr, native.ctypes.byref(pb),
                                                           ret.ctypes.data, None,
                                                           native.ctypes.byref(st)), "run")
            el = time.perf_counter() - t0
            best = el if best is None else min(best, el)
        assert int(sum(st.hist)) == npk
        tile = np.tile(first[: distinct.shape[0]], reps)[:npk] if n >= distinct.shape[0] else None
        same = bool(tile is not None and (ret == tile).all())
        native.lib().ebpf_pcap_batch_free(native.ctypes.byref(pb))
        print(json.dumps({"e2e": "pcap", "config": a.config, "packets": npk,
                          "capture_bytes": int(len(cap)), "pcap_to_batch_ms": parse_ms,
                          "mpkt_s_run": round(npk / best / 1e6, 1), "run_ms": round(best * 1e3, 2),
                          "mpkt_s_with_parse": round(npk / (best + parse) / 1e6, 1),
                          "results_equal_64B_batch": same}), flush=True)
        # the same capture run in place (ebpf_pcap_extents: no gather; the upload is the whole
        # capture, record headers included, plus 16 B of extents per record)
        eparse_ms = {}
        for pinned in (0, 1):   # the extents in pageable, then pinned memory (kept for the run)
            t0 = time.perf_counter()
            pe = native.PktBatch()
            pi = native.PcapInfo()
            native._check(native.lib().ebpf_pcap_extents(cap.ctypes.data, len(cap), pinned,
                                                         native.ctypes.byref(pe), native.ctypes.byref(pi)),
                          "ebpf_pcap_extents")
            eparse = time.perf_counter() - t0
            eparse_ms["pinned" if pinned else "pageable"] = round(eparse * 1e3, 2)
            if not pinned:
                native.lib().ebpf_pcap_batch_free(native.ctypes.byref(pe))
        eparse = min(eparse_ms.values()) / 1e3
        ret2 = np.zeros(npk, dtype=np.uint64)
        native._check(native.lib().ebpf_prog_run_batch(prog.ptr, native.ctypes.byref(pe), ret2.ctypes.data,
                                                       None, native.ctypes.byref(st)), "warm")
        best = None
        for _ in range(a.reps):
            t0 = time.perf_counter()
            native._check(native.lib().ebpf_prog_run_batch(prog.ptr, native.ctypes.byref(pe),
                                                           ret2.ctypes.data, None,
                                                           native.ctypes.byref(st)), "run")
            el = time.perf_counter() - t0
            best = el if best is None else min(best, el)
        native.lib().ebpf_pcap_batch_free(native.ctypes.byref(pe))
        print(json.dumps({"e2e": "pcap_extents", "config": a.config, "packets": npk,
                          "capture_bytes": int(len(cap)), "extents_ms": eparse_ms,
                          "mpkt_s_run": round(npk / best / 1e6, 1), "run_ms": round(best * 1e3, 2),
                          "mpkt_s_with_parse": round(npk / (best + eparse) / 1e6, 1),
                          "results_equal_gathered": bool((ret2 == ret).all())}), flush=True)
    prog.destroy()
    for m in maps:
        m.destroy()
    env.destroy()


if __name__ == "__main__":
    main()
