"""Probe: is C5 bound by wavefront divergence or by per-lane loads?  Runs the C5 program on the
same IMIX packets in generation order and sorted by size (host-side reorder: waves then see one
size class each), device-resident, and prints the kernel time of both."""
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
lay = workloads.prog_c5()
data, offs, sizes = workloads.packets_imix_range(0, n)
env = native.Env()
p = native.Prog(env, lay.code)
dev = torch.device("cuda:0")
order_sorted = np.argsort(sizes, kind="stable")
for name, order in (("imix", np.arange(n)), ("sorted", order_sorted)):
    padded = ((sizes[order].astype(np.uint64) + 63) // 64) * 64
    o = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(padded, out=o[1:])
    d = np.concatenate([data[int(offs[i]):int(offs[i + 1])] for i in order]) if name != "imix" else data
    d_pk = torch.from_numpy(d).to(dev)
    d_off = torch.from_numpy(o.view(np.int64)).to(dev)
    d_ret = torch.empty(n, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream()
    for _ in range(3):
        p.run_batch_dev(0, d_pk.data_ptr(), n, 0, d_ret.data_ptr(), d_off.data_ptr(), None, None, st.cuda_stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for a, b in ev:  # torch creates its events at their first record
        a.record(st)
        b.record(st)
    for a, b in ev:
        native.time_next_launch(a.cuda_event, b.cuda_event)
        p.run_batch_dev(0, d_pk.data_ptr(), n, 0, d_ret.data_ptr(), d_off.data_ptr(), None, None, st.cuda_stream)
    torch.cuda.synchronize()
    print(name, "kernel ms %.4f" % np.mean([a.elapsed_time(b) for a, b in ev]), flush=True)
p.destroy()
env.destroy()
