"""C3L's loop cost: the C3L program over 16M packets whose IPv4 header lengths are all 5, all 12,
or the bench's mix (half 5, half 6-12), plus C3's program over the same frames; kernel times by
the library's launch events (median of 30)."""
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from generic_ebpf_amd import native, workloads  # noqa: E402


def main():
    import torch
    dev = torch.device("cuda:0")
    n = 1 << 24
    env = native.Env()
    base = workloads.packets_ipv4opt(1 << 22, seed=6)
    sets = {"mix": base.copy()}
    for h in (5, 12):
        p = base.copy()
        v4 = (p[:, 12] == 0x08) & (p[:, 13] == 0x00)
        p[v4, 14] = 0x40 | h
        sets["ihl%d" % h] = p
    progs = {"c3l": workloads.prog_c3l(), "c3": workloads.prog_c3()}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()   # (torch creates its events at their first record; the library re-records them)
    ev1.record()
    for pname, lay in progs.items():
        prog = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, []))
        if pname == "c3l":
            prog.set_semantics(native.SEM_STANDARD)
        for sname, pk in sets.items():
            if pname == "c3" and sname != "mix":
                continue
            d = torch.from_numpy(pk.reshape(-1)).to(dev).repeat(n // pk.shape[0])
            ret = torch.zeros(n, dtype=torch.int64, device=dev)
            s = torch.cuda.current_stream()
            for _ in range(5):
                prog.run_batch_dev(0, d.data_ptr(), n, 64, ret.data_ptr(), stream=s.cuda_stream)
            ts = []
            for _ in range(30):
                native.time_next_launch(ev0.cuda_event, ev1.cuda_event)
                prog.run_batch_dev(0, d.data_ptr(), n, 64, ret.data_ptr(), stream=s.cuda_stream)
                ev1.synchronize()
                ts.append(ev0.elapsed_time(ev1))
            med = statistics.median(ts)
            print("%-4s %-6s kernel %.4f ms  frac %.3f  exec %s" % (
                pname, sname, med, n * 64 / (med * 1e-3) / 8e12, prog.exec_info(0)[0]), flush=True)
        prog.destroy()
    env.destroy()


if __name__ == "__main__":
    main()
