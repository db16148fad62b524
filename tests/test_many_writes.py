"""Many map writes on one loop-free path (tests/manywrites.py).  The
reference runs every ST / STX and map_update_elem it reaches (ebpf_interpreter.c:343-366,
:282-284 -> ebpf_map.c:101-108 -> ebpf_map_array.c:198-211): a loop-free program has no write
limit, on the device either (the 16-write cap belongs to programs with loops only).

CPU: the oracle's batch mode runs them with no fault and equals its sequential mode (the
reference's one-after-the-other run: none of these programs reads a map value, so the batch's
held-back writes cannot change a result), the round-5 probe's known answer, a standard-semantics
loop-free program past 16 writes, and the translation (no EOPNOTSUPP, no cap).
GPU: every variant, staged (64-B stride) and general (CSR offsets) kernels, host-buffer and
device-resident: results, faults and the map against the oracle's batch mode, and against the
sequential mode for batches whose packets write distinct keys.
Stores read back (manywrites.READBACK, round 6): past 16 stores on a path the overlay of the
packet's own stores no longer fits on chip; the portable interpreter runs them with the overlay
spilled to memory (dp_launch.ovl_spill), on every variant, in chunks of its buffer."""
import ctypes
import os

import numpy as np
import pytest

import manywrites as mw
import pyoracle

VARIANTS = [int(v) for v in os.environ.get("EBPF_TEST_VARIANTS", "0,1,2").split(",")]


def _init(vs, me, seed):
    return np.random.default_rng(seed).integers(0, 256, vs * me, dtype=np.uint8).tobytes()


def _oracle(lay, vs, me, init, data, n, stride, offsets=None, sequential=False, semantics=0):
    code, rel = lay if isinstance(lay, tuple) else (lay.code, lay.relocs)
    op = pyoracle.OracleProgram(code, rel, [(vs, me, init)], sequential=sequential, semantics=semantics)
    ret, flt, _, _ = op.run(data, n, stride, offsets, nthreads=1 if sequential else 8)
    return ret, flt, op.map_bytes(0)


def test_oracle_probe_runs_in_batch_mode():
    """One lookup, 20 STDW into the value, r0 = 7: no fault in the batch mode, and every value a
    packet's key reached holds the last store (imm 119, sign-extended)."""
    lay = mw.prog_probe()
    pk = mw.packets(300, 1)
    init = _init(8, 16, 2)
    ret, flt, after = _oracle(lay, 8, 16, init, pk.reshape(-1), len(pk), 64)
    assert not flt.any()
    assert (ret == 7).all()
    want = bytearray(init)
    for k in set(int(p[0]) & 15 for p in pk):
        want[8 * k:8 * k + 8] = (119).to_bytes(8, "little")
    assert after == bytes(want)


@pytest.mark.parametrize("case", sorted(mw.CASES))
def test_oracle_batch_equals_sequential_reference(case):
    mk, vs, me = mw.CASES[case]
    lay = mk()
    pk = mw.packets(3001, 3)
    init = _init(vs, me, 4)
    ret, flt, after = _oracle(lay, vs, me, init, pk.reshape(-1), len(pk), 64)
    sret, sflt, safter = _oracle(lay, vs, me, init, pk.reshape(-1), len(pk), 64, sequential=True)
    assert not flt.any()
    np.testing.assert_array_equal(ret, sret)
    np.testing.assert_array_equal(flt, sflt)
    assert after == safter
    assert after != init


def test_oracle_update_return_codes():
    """the seventh call of each run of seven passes EBPF_NOEXIST: EEXIST (17) on an array, the
    others return 0 (ebpf_map_array.c:185-196)"""
    lay = mw.prog_updates(17)
    pk = mw.packets(50, 5)
    ret, flt, _ = _oracle(lay, 8, 256, _init(8, 256, 6), pk.reshape(-1), len(pk), 64)
    want = 0
    for j in range(17):
        if j % 7 == 6:
            want ^= 17 << (j % 56)
    assert not flt.any() and (ret == want).all()


def test_oracle_standard_loop_free_program_past_16_writes():
    """standard semantics, no backward jump: 24 stores into a value all land, no cap; the same
    stores inside a loop (a backward jump) fault the 17th (EBPF_FAULT_WRITES = 11)"""
    import stdprogs
    I = stdprogs.I
    head = [I("ldxb", 6, 1, 0), I("and64_imm", 6, imm=15), I("stxw", 10, 6, -4), ("lddw_map", 1, 0),
            I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4), I("call", imm=0),
            I("jne_imm", 0, off="hit", imm=0), I("mov64_imm", 0, imm=1), I("exit"), ("label", "hit")]
    flat = stdprogs.asm(head + [I("stb", 0, 0, j % 8, j) for j in range(24)] +
                        [I("mov64_imm", 0, imm=7), I("exit")])
    loop = stdprogs.asm(head + [I("mov64_imm", 7, imm=24), ("label", "L"), I("stb", 0, 0, 3, 9),
                                I("sub64_imm", 7, imm=1), I("jne_imm", 7, imm=0, off="L"),
                                I("mov64_imm", 0, imm=7), I("exit")])
    pk = mw.packets(100, 7)
    init = _init(8, 16, 8)
    ret, flt, after = _oracle(flat, 8, 16, init, pk.reshape(-1), 100, 64, semantics=1)
    assert not flt.any() and (ret == 7).all()
    _, _, safter = _oracle(flat, 8, 16, init, pk.reshape(-1), 100, 64, semantics=1, sequential=True)
    assert after == safter
    ret, flt, after = _oracle(loop, 8, 16, init, pk.reshape(-1), 100, 64, semantics=1)
    assert (flt == 11).all() and after == init


class _Info(ctypes.Structure):
    _fields_ = [("nslots", ctypes.c_uint32), ("nentries", ctypes.c_uint32),
                ("nmaps", ctypes.c_uint32), ("max_stack", ctypes.c_uint32)]


@pytest.mark.parametrize("case", sorted(mw.CASES) + sorted(mw.READBACK))
def test_translation_accepts_many_writes(native, env, case):
    mk, vs, me = (mw.CASES.get(case) or mw.READBACK[case])
    lay = mk()
    m = native.Map(env, me, vs)
    p = native.Prog(env, lay.patched([m.handle]))
    try:
        assert native.lib().ebpf_prog_device_info(p.ptr, ctypes.byref(_Info())) == 0
    finally:
        p.destroy()
        m.destroy()


# ---------------------------------------------------------------- GPU


def _ragged(pk, seed):
    """the same packets' first bytes at CSR offsets, lengths 24..80 (the programs read 0..24)"""
    g = np.random.default_rng(seed)
    n = len(pk)
    sizes = g.integers(24, 81, n).astype(np.uint64)
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(sizes, out=offs[1:])
    data = g.integers(0, 256, int(offs[-1]) + 64, dtype=np.uint8)
    for i in range(n):
        data[int(offs[i]):int(offs[i]) + 24] = pk[i, :24]
    return data, offs


def _device(gpu, lay, vs, me, init, env, data, n, stride, offsets, variant, resident):
    import torch
    m = gpu.Map(env, me, vs)
    m.fill(init)
    p = gpu.Prog(env, lay.patched([m.handle]))
    try:
        gpu.set_variant(variant)
        if resident:
            dev = torch.device("cuda:0")
            d_pk = torch.from_numpy(np.ascontiguousarray(data)).to(dev)
            d_off = None if offsets is None else torch.from_numpy(offsets.view(np.int64)).to(dev)
            d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
            d_flt = torch.zeros(n, dtype=torch.uint8, device=dev)
            p.run_batch_dev(0, d_pk.data_ptr(), n, stride, d_ret.data_ptr(),
                            None if d_off is None else d_off.data_ptr(), d_flt.data_ptr(), None,
                            torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            ret, flt = d_ret.cpu().numpy().view(np.uint64), d_flt.cpu().numpy()
        else:
            ret, flt, _ = p.run_batch(np.ascontiguousarray(data.copy()), n, stride, offsets)
        after = b"".join(m.lookup(k)[1] for k in range(me))
        return ret, flt, after
    finally:
        gpu.set_variant(0)
        p.destroy()
        m.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("layout", ["staged", "general"])
@pytest.mark.parametrize("case", sorted(mw.CASES))
def test_device_many_writes_vs_oracle(gpu, env, variant, layout, case):
    mk, vs, me = mw.CASES[case]
    lay = mk()
    n = (1 << 14) + 13
    pk = mw.packets(n, 11)
    init = _init(vs, me, 12)
    if layout == "staged":
        data, stride, offs = pk.reshape(-1), 64, None
    else:
        (data, offs), stride = _ragged(pk, 13), 0
    want, wf, wafter = _oracle(lay, vs, me, init, data, n, stride, offs)
    assert not wf.any()
    for resident in (False, True):
        ret, flt, after = _device(gpu, lay, vs, me, init, env, data, n, stride, offs, variant, resident)
        np.testing.assert_array_equal(flt, wf)
        np.testing.assert_array_equal(ret, want)
        assert after == wafter, resident


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("case", sorted(mw.CASES))
def test_device_distinct_keys_equal_sequential_reference(gpu, env, variant, case):
    """packets that write distinct keys: the device batch leaves what the reference's one packet
    after the other leaves (the oracle's sequential mode)"""
    lay, vs, me = mw.distinct_case(case, 256)
    pk = mw.distinct_key_packets(256 if not case.startswith("probe") else 16, 14)
    n = len(pk)
    init = _init(vs, me, 15)
    sret, sflt, safter = _oracle(lay, vs, me, init, pk.reshape(-1), n, 64, sequential=True)
    ret, flt, after = _device(gpu, lay, vs, me, init, env, pk.reshape(-1), n, 64, None, variant, False)
    assert not sflt.any()
    np.testing.assert_array_equal(flt, sflt)
    np.testing.assert_array_equal(ret, sret)
    assert after == safter


def test_oracle_readback_sees_own_stores():
    """the read-back programs: r0 from the packet's own stores over the batch-start value, the
    same in the batch and the reference's sequential run when no two packets share a key"""
    for name, (mk, vs, me) in sorted(mw.READBACK.items()):
        lay = mk()
        pk = mw.distinct_key_packets(16, 21)
        init = _init(vs, me, 22)
        ret, flt, after = _oracle(lay, vs, me, init, pk.reshape(-1), 16, 64)
        sret, sflt, safter = _oracle(lay, vs, me, init, pk.reshape(-1), 16, 64, sequential=True)
        assert not flt.any(), name
        np.testing.assert_array_equal(ret, sret)
        assert after == safter, name


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("layout", ["staged", "general"])
@pytest.mark.parametrize("case", sorted(mw.READBACK))
def test_device_readback_vs_oracle(gpu, env, variant, layout, case):
    """past 16 stores read back the overlay is spilled and the portable interpreter runs it (every
    variant); readback120 over 300,007 packets runs in two chunks of the 1-GiB spill buffer"""
    mk, vs, me = mw.READBACK[case]
    lay = mk()
    n = 300007 if case == "readback120" and layout == "staged" else (1 << 14) + 13
    pk = mw.packets(n, 23)
    init = _init(vs, me, 24)
    if layout == "staged":
        data, stride, offs = pk.reshape(-1), 64, None
    else:
        (data, offs), stride = _ragged(pk, 25), 0
    want, wf, wafter = _oracle(lay, vs, me, init, data, n, stride, offs)
    assert not wf.any()
    ret, flt, after = _device(gpu, lay, vs, me, init, env, data, n, stride, offs, variant, False)
    np.testing.assert_array_equal(flt, wf)
    np.testing.assert_array_equal(ret, want)
    assert after == wafter
    m = gpu.Map(env, me, vs)
    p = gpu.Prog(env, lay.patched([m.handle]))
    try:
        gpu.set_variant(variant)
        p.run_batch(np.ascontiguousarray(pk[:64].reshape(-1)), 64, 64)
        ex = p.exec_info(0)[0]
    finally:
        gpu.set_variant(0)
        p.destroy()
        m.destroy()
    if case != "readback16" or variant == 1:   # (16 stores still fit the lanes' own overlay)
        assert ex == "hip"


# ---- the same read-back programs over a hashtable (the spilled overlay on a table's values) ----

def _hash_items(vs, seed, present=12):
    """u32 keys 0..present-1 of the 16 the programs look up (the others miss), random values"""
    g = np.random.default_rng(seed)
    return [(k.to_bytes(4, "little"), g.integers(0, 256, vs, dtype=np.uint8).tobytes())
            for k in range(present)]


def test_oracle_hash_readback_sees_own_stores():
    """over a hashtable: r0 from the packet's own stores, equal to the sequential run when no two
    packets share a key; packets whose key is absent exit with MISS"""
    for name in ("readback17", "readback40"):
        mk, vs, _ = mw.READBACK[name]
        lay = mk()
        pk = mw.distinct_key_packets(16, 31)
        items = _hash_items(vs, 32)
        outs = []
        for seq in (False, True):
            op = pyoracle.OracleProgram(lay.code, lay.relocs, [pyoracle.HashSpec(4, vs, items=items, capacity=16)],
                                        sequential=seq)
            ret, flt, _, _ = op.run(pk.reshape(-1), 16, 64, nthreads=1)
            outs.append((ret, flt))
        np.testing.assert_array_equal(outs[0][0], outs[1][0])
        assert not outs[0][1].any()
        assert (outs[0][0][12:] == mw.MISS).all() and (outs[0][0][:12] != mw.MISS).all()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("case", ["readback17", "readback40"])
def test_device_hash_readback_vs_oracle(gpu, env, variant, case):
    """past 16 stores read back into a hashtable's values: the spilled overlay on the portable
    interpreter, the stores replayed into the table after the batch — results, faults and the
    table against the oracle"""
    mk, vs, _ = mw.READBACK[case]
    lay = mk()
    n = (1 << 14) + 13
    pk = mw.packets(n, 33)
    items = _hash_items(vs, 34)
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [pyoracle.HashSpec(4, vs, items=items, capacity=16)])
    want, wf, _, _ = op.run(pk.reshape(-1), n, 64, nthreads=8)
    wtab = dict(op.hash_models[0].items())
    m = gpu.HashMap(env, 4, vs, 16)
    for k, v in items:
        assert m.update(k, v) == 0
    p = gpu.Prog(env, lay.patched([m.handle]))
    try:
        gpu.set_variant(variant)
        ret, flt, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1).copy()), n, 64)
        tab = {k: m.lookup(k)[1] for k, _ in items}
    finally:
        gpu.set_variant(0)
        p.destroy()
        m.destroy()
    np.testing.assert_array_equal(flt, wf)
    np.testing.assert_array_equal(ret, want)
    assert tab == {k: wtab[k] for k, _ in items}


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_device_readback_spilled_other_entry_points(gpu, env, variant):
    """the spilled overlay through the other batch entry points: sharded over [0, 0]
    (ebpf_prog_run_batch_multi: each shard's chunks at its own packet base, the shards' logs
    merged in global order), as (start, end) extents of ragged packets, and asynchronously —
    each against the oracle"""
    mk, vs, me = mw.READBACK["readback40"]
    lay = mk()
    n = (1 << 13) + 7
    pk = mw.packets(n, 41)
    init = _init(vs, me, 42)
    want, wf, wafter = _oracle(lay, vs, me, init, pk.reshape(-1), n, 64)
    (rdata, roffs) = _ragged(pk, 43)
    rwant, rwf, rwafter = _oracle(lay, vs, me, init, rdata, n, 0, roffs)
    ext = np.stack([roffs[:-1], roffs[1:]], axis=1).reshape(-1).astype(np.uint64)

    def run(how):
        m = gpu.Map(env, me, vs)
        m.fill(init)
        p = gpu.Prog(env, lay.patched([m.handle]))
        try:
            gpu.set_variant(variant)
            if how == "multi":
                ret, flt, _ = p.run_batch_multi([0, 0], np.ascontiguousarray(pk.reshape(-1).copy()), n, 64)
            elif how == "extents":
                ret, flt, _ = p.run_batch(np.ascontiguousarray(rdata.copy()), n, 0, ext, extents=True)
            else:
                data = np.ascontiguousarray(pk.reshape(-1).copy())
                ret, flt, _ = p.run_batch_async(data, n, 64).wait()
            return ret, flt, b"".join(m.lookup(k)[1] for k in range(me))
        finally:
            gpu.set_variant(0)
            p.destroy()
            m.destroy()

    for how in ("multi", "extents", "async"):
        ret, flt, after = run(how)
        w, f, a = (rwant, rwf, rwafter) if how == "extents" else (want, wf, wafter)
        np.testing.assert_array_equal(flt, f, err_msg=how)
        np.testing.assert_array_equal(ret, w, err_msg=how)
        assert after == a, how
