"""Bisect the variant-0 mismatch of the c5ms probe (round 5): variants of the program, each run
on every device variant against the oracle."""
import sys; sys.path[:0] = ['/root/repo', '/root/repo/oracle']
import pkgload; pkgload.load()
import numpy as np, pyoracle
from generic_ebpf_amd import native, workloads as w
n = 1 << 14
data, offs, sizes = w.packets_imix(n)
env = native.Env()
base = dict(ops=("add64_reg",), exits=False)
cases = {
    "add_noexit": dict(base), "nosplit": dict(base, split=False), "notests": dict(base, tests=0),
    "onetest": dict(base, tests=1), "nosplit_notests": dict(base, split=False, tests=0),
    "body8": dict(base, body=8), "body8_nosplit": dict(base, body=8, split=False),
}
for name, kw in cases.items():
    kw = dict(kw)
    body = kw.pop("body", 96)
    nodes, cols = w._meldsim_nodes(7, body, **kw)
    lay = w._asm_std(nodes)
    t = np.zeros((16, max(1, len(cols))), dtype=np.uint32)
    for ci, vals in enumerate(cols):
        for c in range(3):
            for v in range(4):
                t[4 * c + v, ci] = vals[c][v]
    spec = [(4 * t.shape[1], 16, t.tobytes())]
    op = pyoracle.OracleProgram(lay.code, lay.relocs, spec, semantics=1)
    want, wf, _, _ = op.run(data, n, 0, offs, nthreads=8)
    out = []
    for variant in (0, 2):
        m = native.Map(env, 16, 4 * t.shape[1])
        m.fill(t.tobytes())
        p = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [m.handle]))
        p.set_semantics(native.SEM_STANDARD)
        native.set_variant(variant)
        r, f, _ = p.run_batch(np.ascontiguousarray(data.copy()), n, 0, offs)
        out.append("v%d %s mism %d" % (variant, p.exec_info(0)[0], int((r != want).sum())))
        if variant == 0 and (r != want).any():
            i = np.flatnonzero(r != want)[:3]
            out.append("e.g. %s got %s want %s sizes %s" % (i.tolist(), r[i].tolist(), want[i].tolist(), sizes[i].tolist()))
        native.set_variant(0)
        p.destroy()
        m.destroy()
    print(name, out, flush=True)
