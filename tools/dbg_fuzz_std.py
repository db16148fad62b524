"""Debug: variant-0 mismatches of the standard-semantics fuzz mode (tools/fuzz_gpu.py --standard):
which code generator switch makes them go away, and what differs."""
import os
import sys
sys.argv = sys.argv[:1]
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import fuzz_gpu as F  # noqa: F401  (sets up the paths)
import pyoracle
import stdprogs
from generic_ebpf_amd import native

env = native.Env()
fails = [130, 146, 754, 830]


def case(k, seed=1, stride=64):
    s = seed * 100000 + k
    g = np.random.default_rng(s)
    code, rel = stdprogs.gen_program(s, length=int(g.integers(10, 80)), with_map=k % 4 == 0)
    n = int(g.choice([1, 64, 65, 777, 2048]))
    pk = g.integers(0, 256, (n, stride), dtype=np.uint8)
    return code, rel, pk, n


for knob in ("", "EBPF_JIT_NOCC", "EBPF_JIT_NOSTRUCT", "EBPF_CC_OFF=1", "EBPF_CC_OFF=2", "EBPF_CC_OFF=4",
             "EBPF_CC_OFF=8", "EBPF_CC_OFF=16", "EBPF_CC_OFF=32", "EBPF_CC_EXITCALL"):
    name, _, val = knob.partition("=")
    if name:
        os.environ[name] = val or "1"
    res = []
    for k in fails:
        code, rel, pk, n = case(k)
        want, wf, _, _ = pyoracle.OracleProgram(code, rel, [], semantics=1).run(pk.reshape(-1), n, 64)
        p = native.Prog(env, code)
        try:
            p.set_semantics(native.SEM_STANDARD)
            got, gf, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1).copy()), n, 64)
        finally:
            p.destroy()
        d = np.nonzero((want != got) | (wf != gf))[0]
        res.append((k, n, len(d), ("%x/%x f%d/%d" % (int(want[d[0]]), int(got[d[0]]), wf[d[0]], gf[d[0]])) if len(d) else ""))
    print(knob or "default", res, flush=True)
    if name:
        os.environ.pop(name)
