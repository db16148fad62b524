"""Debug: variant-0 mismatches of the hashtable fuzz mode (tools/fuzz_gpu.py --hash)."""
import os
import sys
sys.argv = sys.argv[:1]
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import fuzz_gpu as F
from generic_ebpf_amd import native

env = native.Env()
fails = [126, 1380]
for knob in ("", "EBPF_CC_NOHFWD", "EBPF_JIT_NOCC", "EBPF_JIT_NOSTRUCT", "EBPF_CC_OFF=1", "EBPF_CC_OFF=2",
             "EBPF_CC_OFF=4", "EBPF_CC_OFF=8", "EBPF_CC_OFF=16", "EBPF_CC_OFF=32", "EBPF_CC_NOHOIST"):
    name, _, val = knob.partition("=")
    if name:
        os.environ[name] = val or "1"
    res = []
    for k in fails:
        for lay in ("staged", "general"):
            c = F.case(k, 1, lay, True)
            want, wf, wdata, wmaps = F.oracle(c)
            got, gf, gdata, gmaps = F.device(env, c, 0)
            what = []
            if not np.array_equal(want, got):
                i = int(np.nonzero(want != got)[0][0])
                what.append("ret@%d %x/%x n=%d" % (i, int(want[i]), int(got[i]), int(np.count_nonzero(want != got))))
            if not np.array_equal(wf, gf):
                what.append("faults")
            if not np.array_equal(wdata, gdata):
                what.append("data")
            if wmaps != gmaps:
                what.append("maps")
            res.append((k, lay, what))
    print(knob or "default", res, flush=True)
    if name:
        os.environ.pop(name)
