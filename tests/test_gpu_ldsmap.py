"""Compiled array-map lookups whose key is proven below max_entries (asm_cc.cpp lookup_stk):
r0 = the value's address with no NULL check, and loads through it read the workgroup's LDS copy
of the map (ldxmap) — in the staged kernel (64-B stride) and in the general kernels (any
stride, offsets), under both semantics.  Round 5: the c5ms probe (workloads.prog_c5meldsim)
found variant 0 wrong where the interpreter was right; these pin the shapes it uses against the
oracle (ebpf_map_array.c:115-124 lookup, ebpf_interpreter.c:327-338 loads)."""
import numpy as np
import pytest

import pyoracle
import stdprogs

pytestmark = pytest.mark.gpu
I = stdprogs.I


def _prog(nloads, std, exit_load):
    """key = pkt[3] & 15 (or, alternating, a constant class * 4 | 2 test bits); r0 = lookup;
    r8 += the words [r0 + 4k] for k < nloads; exit_load: a packet byte decides an early exit
    returning [r0 + 4 * nloads] (a load into r0 through r0)."""
    items = [I("mov64_reg", 7, 1), I("ldxb", 5, 7, 3), I("and64_imm", 5, imm=15),
             I("stxw", 10, 5, -4), ("lddw_map", 1, 0), I("mov64_reg", 2, 10),
             I("add64_imm", 2, imm=-4), I("call", imm=0), I("mov64_imm", 8, imm=0)]
    for k in range(nloads):
        items += [I("ldxw", 4, 0, 4 * k), I("add64_reg", 8, 4)]
        if exit_load and k == nloads // 2:
            items += [I("ldxb", 6, 7, 5), I("jne_imm", 6, imm=7, off="c")]
            items += [I("ldxw", 0, 0, 4 * nloads), I("exit"), ("label", "c")]
    items += [I("mov64_reg", 0, 8), I("exit")]
    return stdprogs.asm(items)


@pytest.mark.parametrize("layout", ["stride64", "stride72", "offsets"])
@pytest.mark.parametrize("exit_load", [False, True])
@pytest.mark.parametrize("words", [13, 72])
def test_lds_map_loads_vs_oracle(gpu, env, layout, exit_load, words):
    """words = 72: a 288-B value size, which is no inline constant: the compiled lookup and loads
    must not read it from a second SGPR (a VOP3 reads one; round 5's c5ms mismatch)."""
    code, rel = _prog(12, True, exit_load)
    g = np.random.default_rng(5)
    vs = 4 * words
    table = g.integers(0, 2**32, (16, words), dtype=np.uint32)
    n = 50000
    if layout == "offsets":
        lens = g.integers(16, 200, n)
        offs = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens, out=offs[1:])
        data, stride = g.integers(0, 256, int(offs[-1]), dtype=np.uint8), 0
    else:
        stride = 64 if layout == "stride64" else 72
        data, offs = g.integers(0, 256, n * stride, dtype=np.uint8), None
    spec = [(vs, 16, table.tobytes())]
    want, wf, _, _ = pyoracle.OracleProgram(code, rel, spec, semantics=1).run(data, n, stride, offs, nthreads=8)
    for variant in (0, 2):
        m = gpu.Map(env, 16, vs)
        m.fill(table.tobytes())
        p = gpu.Prog(env, gpu.patch_relocs(code, rel, [m.handle]))
        try:
            p.set_semantics(gpu.SEM_STANDARD)
            gpu.set_variant(variant)
            got, gf, _ = p.run_batch(np.ascontiguousarray(data.copy()), n, stride, offs)
        finally:
            gpu.set_variant(0)
            p.destroy()
            m.destroy()
        np.testing.assert_array_equal(gf, wf)
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, (variant, bad.size, bad[:5], got[bad[:5]], want[bad[:5]])


@pytest.mark.parametrize("vs", [8, 200])
@pytest.mark.parametrize("stride", [64, 72])
def test_lookup_result_as_update_value(gpu, env, vs, stride):
    """The compiled lookup's r0 itself (not only loads through it): passed as the value pointer
    of map_update_elem(map 1, &key, r0, ANY), which reads value_size bytes there; map 1 after the
    batch must equal the oracle's (a wrong r0 reads elsewhere or faults MEM)."""
    code, rel = stdprogs.asm([
        I("ldxb", 5, 1, 3), I("and64_imm", 5, imm=15), I("stxw", 10, 5, -4),
        ("lddw_map", 1, 0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4), I("call", imm=0),
        I("mov64_reg", 3, 0), ("lddw_map", 1, 1), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4),
        I("mov64_imm", 4, imm=0), I("call", imm=1), I("exit")])
    g = np.random.default_rng(9)
    t0 = g.integers(0, 256, 16 * vs, dtype=np.uint8).tobytes()
    t1 = g.integers(0, 256, 16 * vs, dtype=np.uint8).tobytes()
    n = 4096
    data = g.integers(0, 256, n * stride, dtype=np.uint8)
    op = pyoracle.OracleProgram(code, rel, [(vs, 16, t0), (vs, 16, t1)], semantics=1)
    want, wf, _, _ = op.run(data, n, stride, nthreads=8)
    assert not wf.any()
    for variant in (0, 2):
        ms = [gpu.Map(env, 16, vs), gpu.Map(env, 16, vs)]
        ms[0].fill(t0)
        ms[1].fill(t1)
        p = gpu.Prog(env, gpu.patch_relocs(code, rel, [m.handle for m in ms]))
        try:
            p.set_semantics(gpu.SEM_STANDARD)
            gpu.set_variant(variant)
            got, gf, _ = p.run_batch(np.ascontiguousarray(data.copy()), n, stride)
            after = b"".join(ms[1].lookup(k)[1] for k in range(16))
        finally:
            gpu.set_variant(0)
            p.destroy()
            for m in ms:
                m.destroy()
        np.testing.assert_array_equal(gf, wf)
        np.testing.assert_array_equal(got, want)
        assert after == op.map_bytes(1), variant
