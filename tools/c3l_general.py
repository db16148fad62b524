#!/usr/bin/env python3
"""C3L (the IPv4 header checksum loop) on the general kernels: 16M packets at a 72-B stride (the
C3L frames padded), device-resident, the kernel timed with HIP events around each launch.  Checks
every result against the numpy restatement (workloads.c3l_expected).  Run it twice, with and
without EBPF_NOHDRLDS=1, to compare packet loads at run-time offsets from the LDS header buffer
against global memory.  Prints one JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import pkgload  # noqa: E402

pkgload.load()
import torch  # noqa: E402
from generic_ebpf_amd import native, workloads  # noqa: E402


def main():
    n, stride, distinct = 1 << 24, 72, 1 << 18
    pk = workloads.packets_ipv4opt(distinct)
    want = workloads.c3l_expected(pk)
    rows = np.zeros((distinct, stride), dtype=np.uint8)
    rows[:, :64] = pk
    data = torch.from_numpy(np.tile(rows.reshape(-1), n // distinct)).cuda()
    ret = torch.zeros(n, dtype=torch.int64, device="cuda")
    env = native.Env()
    p = native.Prog(env, workloads.prog_c3l().code)
    p.set_semantics(native.SEM_STANDARD)
    times = []
    for it in range(25):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        p.run_batch_dev(0, data.data_ptr(), n, stride, ret.data_ptr(),
                        stream=torch.cuda.current_stream().cuda_stream)
        b.record()
        torch.cuda.synchronize()
        if it >= 5:
            times.append(a.elapsed_time(b))
    got = ret.cpu().numpy().view(np.uint64).reshape(-1, distinct)
    ok = bool((got == want[None, :]).all())
    ms = float(np.median(times))
    print(json.dumps({"config": "c3l on the general kernel (72-B stride)", "packets": n,
                      "hdrlds": os.environ.get("EBPF_NOHDRLDS") is None, "exec": p.exec_info(0)[0],
                      "ms": round(ms, 4), "gpkt_s": round(n / ms / 1e6, 2), "verified": ok}))
    p.destroy()
    env.destroy()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
