#!/usr/bin/env python3
"""Debug aid (EBPF_LIB=abx/retk1.so): C3L on N packets, staged compiled kernel, keep mode,
launched several times; prints the mismatch pattern against the numpy restatement."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import pkgload  # noqa: E402
pkgload.load()
import torch  # noqa: E402
from generic_ebpf_amd import native, workloads  # noqa: E402

for n in (1 << 22,):
    pk = np.tile(workloads.packets_ipv4opt(1 << 22), (n >> 22, 1))
    want = workloads.c3l_expected(pk)
    data = torch.from_numpy(pk.reshape(-1).copy()).cuda()
    ret = torch.zeros(n, dtype=torch.int64, device="cuda")
    env = native.Env()
    p = native.Prog(env, workloads.prog_c3l().code)
    p.set_semantics(native.SEM_STANDARD)
    hist = torch.zeros(257, dtype=torch.int64, device="cuda")
    native.set_variant(0)
    p.prepare(0)
    launch = p.launcher(0, data.data_ptr(), n, 64, ret.data_ptr(), None, None,
                        torch.cuda.current_stream().cuda_stream, hist_overwrite=True)
    for rep in range(2):
        ret.zero_()
        if rep >= 3:
            a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            native.time_next_launch(a_.cuda_event, b_.cuda_event)
        launch(hist.data_ptr())
        torch.cuda.synchronize()
        got = ret.cpu().numpy().view(np.uint64)
        bad = np.nonzero(got != want)[0]
        print("n", n, "launch", rep, "mismatches", len(bad), "groups", sorted(set((bad // 64).tolist()))[:12])
        for sh in (64, 8192 * 64, 4096 * 64, 16384 * 64):
            j = bad[bad >= sh]
            print("  stale by %d packets: %d of %d" % (sh, int((got[j] == want[j - sh]).sum()), len(j)))
        for i in bad[:4]:
            print("  pkt", i, "want", want[i], "got", got[i], "ihl", pk[i, 14] & 15,
                  "want[i-64]", want[i - 64] if i >= 64 else None)
    p.destroy()
    env.destroy()
