"""Debug: mutation-mode mismatches (tools/fuzz_gpu.py --mutate): the first differing packet's
results, faults and executed instruction count on the HIP interpreter vs the oracle."""
import sys
sys.argv = sys.argv[:1]
import os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np
import fuzz_gpu as F
from generic_ebpf_amd import native

env = native.Env()
for k in (581, 2491, 2829):
    for lay in ("staged", "general"):
        c = F.case(k, 1, lay, writes=False)
        c.code = F.mutate(c.code, np.random.default_rng(1 * 7777 + k))
        want, wf, wdata, wmaps = F.oracle(c)
        got, gf, gdata, gmaps = F.device(env, c, 1)
        d = np.nonzero((want != got) | (wf != gf))[0]
        info = [(int(i), hex(int(want[i])), hex(int(got[i])), int(wf[i]), int(gf[i])) for i in d[:4]]
        print(k, lay, c.count, "ret/fault mismatches", len(d), info,
              "data", not np.array_equal(wdata, gdata), "maps", wmaps != gmaps, flush=True)
        with open("gpurun_out/mut_%d.bin" % k, "wb") as fh:
            fh.write(c.code)
