"""Probe: what one C5 packet costs per size class.  Runs the C5 program device-resident on 4M
packets that are all 64 B, all 576 B, all 1500 B, IMIX in generation order and IMIX sorted by
size, and prints the kernel time of each (events around the kernel alone, 10 launches)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
import torch  # noqa: E402
from generic_ebpf_amd import native, workloads  # noqa: E402

n = 1 << 22
only = sys.argv[1:]
lay = workloads.prog_c5()
data, offs, sizes = workloads.packets_imix_range(0, n)
env = native.Env()
p = native.Prog(env, lay.code)
dev = torch.device("cuda:0")


def homogeneous(size):
    """n packets of one IMIX size class, each a copy of a packet of that class."""
    pick = np.flatnonzero(sizes == size)[:4096]
    padded = (size + 63) // 64 * 64
    src = np.stack([data[int(offs[i]):int(offs[i]) + padded] for i in pick])
    d = src[np.arange(n) % len(pick)].reshape(-1)
    o = np.arange(n + 1, dtype=np.uint64) * padded
    return d, o


def reorder(order):
    padded = ((sizes[order].astype(np.uint64) + 63) // 64) * 64
    o = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(padded, out=o[1:])
    d = np.concatenate([data[int(offs[i]):int(offs[i + 1])] for i in order])
    return d, o


cases = [("imix", lambda: (data, offs)),
         ("all64", lambda: homogeneous(64)),
         ("all576", lambda: homogeneous(576)),
         ("all1500", lambda: homogeneous(1500)),
         ("sorted", lambda: reorder(np.argsort(sizes, kind="stable")))]
for name, make in cases:
    if only and name not in only:
        continue
    d, o = make()
    d_pk = torch.from_numpy(d).to(dev)
    d_off = torch.from_numpy(o.view(np.int64)).to(dev)
    d_ret = torch.empty(n, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream()
    for _ in range(3):
        p.run_batch_dev(0, d_pk.data_ptr(), n, 0, d_ret.data_ptr(), d_off.data_ptr(), None, None,
                        st.cuda_stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(10)]
    for a, b in ev:  # torch creates its events at their first record
        a.record(st)
        b.record(st)
    for a, b in ev:
        native.time_next_launch(a.cuda_event, b.cuda_event)
        p.run_batch_dev(0, d_pk.data_ptr(), n, 0, d_ret.data_ptr(), d_off.data_ptr(), None, None,
                        st.cuda_stream)
    torch.cuda.synchronize()
    ms = np.mean([a.elapsed_time(b) for a, b in ev])
    print("%-8s kernel ms %.4f  bytes %.3f GB  %.1f GB/s" % (name, ms, len(d) / 1e9,
                                                          len(d) / ms / 1e6), flush=True)
    del d_pk, d_off, d_ret
p.destroy()
env.destroy()
