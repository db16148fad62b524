"""Hashtable writes in a device batch (include/ebpf_gpu.h "Map writes in a device batch"):
map_update_elem / map_delete_elem on hashtable maps called by the program.

Semantics (oracle/ebpf_oracle.h): every packet sees the table as it was when the batch started.
update's return code is the reference's against that table — EINVAL for NULL key / value or
flags > EBPF_EXIST (ebpf_map.c:101-108), EEXIST / ENOENT by the key's presence
(ebpf_map_hashtable.c:87-100), EBUSY for a new key when the table is full (:371-377), else 0;
delete returns 0 (:475-502, EINVAL for a NULL key).  The successful calls are replayed after the
batch in (packet, call) order through the map's own update / delete, so the table the host API
and the next batch see is the reference's after running those calls in that order; a replay
that fails against the table as it then is (two packets inserting one key with EBPF_NOEXIST, a
table filling up) leaves it unchanged.  A packet that faults leaves no write.

CPU tests pin the oracle mode against a pure-Python restatement (HashtableModel); GPU tests
compare every device variant with the oracle: results, faults, the table walked with
get_next_key in the reference's order (values included) and a second batch over that table."""
import copy

import numpy as np
import pytest

import pyoracle

R0, R1, R2, R3, R4, R5, R6, R7, R8, R9, R10 = range(11)
NKEYS = 64
KEY_PAD = 0x5a5a5a5a


def _nodes():
    from generic_ebpf_amd import isa, layout
    return isa.Insn, layout.LdDw, layout.MapRef, layout.Branch


def prog_hash_writes(ks):
    """key = u32 pkt[0] & 63 at r10 - 24 (ks 12: then 8 bytes 0x5a), value = pkt[8..16) at
    r10 - 8; op = pkt[1] & 7: bit 2 set -> map_delete_elem(key), else map_update_elem(key, value,
    flags = op & 3) (3: EINVAL); sel = pkt[2] & 3: 3 -> the write's key pointer is r1 + 60 (ks 4:
    the packet's last 4 bytes; ks 12: runs past the packet -> MEM fault), 2 -> the value pointer
    is NULL (update: EINVAL).  Then a lookup of the stack key (the batch-start table):
    r0 = rc | (u16 value << 8, or 0xffff << 8 when absent)."""
    from generic_ebpf_amd import layout
    I, LdDw, MapRef, Branch = _nodes()

    def result():
        return [I("mov_imm", R6, imm=0), I("mov64_reg", R6, R0),
                LdDw(R1, MapRef(0)),
                I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-24),
                I("call", imm=0),
                Branch(I("jeq_imm", R0, imm=0), [I("mov_imm", R0, imm=0xffff), I("lsh64_imm", R0, imm=8),
                                                 I("or64_reg", R0, R6), I("exit")]),
                I("ldxh", R0, R0, 0), I("lsh64_imm", R0, imm=8), I("or64_reg", R0, R6), I("exit")]

    def write(sel):
        key = ([I("mov_imm", R2, imm=0), I("mov64_reg", R2, R9)] if sel == 3 else
               [I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-24)])
        val = ([I("mov_imm", R3, imm=0)] if sel == 2 else
               [I("mov_imm", R3, imm=0), I("mov64_reg", R3, R10), I("add64_imm", R3, imm=-8)])
        return [LdDw(R1, MapRef(0))] + key + [
            Branch(I("jset_imm", R7, imm=4), [I("call", imm=2)] + result()),
        ] + val + [I("mov_imm", R4, imm=0), I("mov64_reg", R4, R7), I("and_imm", R4, imm=3),
                   I("call", imm=1)] + result()

    n = [I("mov_imm", R9, imm=0), I("mov64_reg", R9, R1), I("add64_imm", R9, imm=60),
         I("ldxw", R6, R1, 0), I("and_imm", R6, imm=NKEYS - 1), I("stxw", R10, R6, -24)]
    if ks == 12:
        n += [I("mov_imm", R6, imm=KEY_PAD), I("stxw", R10, R6, -20), I("stxw", R10, R6, -16)]
    n += [I("ldxdw", R8, R1, 8), I("stxdw", R10, R8, -8),
          I("ldxb", R7, R1, 1), I("and_imm", R7, imm=7),
          I("ldxb", R5, R1, 2), I("and_imm", R5, imm=3),
          Branch(I("jeq_imm", R5, imm=3), write(3)),
          Branch(I("jeq_imm", R5, imm=2), write(2))] + write(0)
    return layout.assemble(n)


def _key(k, ks):
    b = int(k).to_bytes(4, "little")
    return b if ks == 4 else b + KEY_PAD.to_bytes(4, "little") * 2


def _packets(n, seed):
    from generic_ebpf_amd import workloads
    return workloads.packets_random(n, 64, seed=seed)


def _table(ks, seed, nlive, cap):
    """nlive distinct keys out of NKEYS with random 8-byte values."""
    g = np.random.default_rng(seed)
    keys = g.choice(NKEYS, nlive, replace=False)
    return pyoracle.HashSpec(ks, 8, items=[(_key(k, ks), g.bytes(8)) for k in keys], capacity=cap)


def _expect(pk, spec):
    """Pure-Python restatement: per packet against the batch-start model, then the replay."""
    ks = spec.key_size
    snap = spec.model()
    live = copy.deepcopy(snap)
    ret, faults, log = [], [], []
    for p in pk:
        k = _key(int.from_bytes(p[0:4].tobytes(), "little") & (NKEYS - 1), ks)
        op, sel = int(p[1]) & 7, int(p[2]) & 3
        wkey = k
        if sel == 3:
            if ks == 12 and (op & 4 or (op & 3) != 3):
                ret.append(0)
                faults.append(3)    # MEM: the key runs past the packet (flags 3: EINVAL first)
                continue
            wkey = p[60:64].tobytes()
        if op & 4:
            rc = 0
            log.append(("d", wkey, None, 0))
        elif sel == 2 or (op & 3) == 3:
            rc = 22
        else:
            flags = op & 3
            exists = snap.lookup(wkey) is not None
            rc = 17 if exists and flags & 1 else 2 if not exists and flags & 2 else \
                16 if not exists and len(snap) >= snap.cap else 0
            if rc == 0:
                log.append(("u", wkey, p[8:16].tobytes(), flags))
        v = snap.lookup(k)
        ret.append(rc | ((0xffff if v is None else int.from_bytes(v[:2], "little")) << 8))
        faults.append(0)
    for kind, key, val, flags in log:
        if kind == "d":
            live.delete(key)
        else:
            live.update(key, val, flags)
    return np.array(ret, dtype=np.uint64), np.array(faults, dtype=np.uint8), live


@pytest.mark.parametrize("ks", [4, 12])
@pytest.mark.parametrize("room", ["room", "full"])
def test_oracle_hash_writes_known_answers(ks, room):
    n = 4000
    pk = _packets(n, 61)
    spec = _table(ks, 62, 30, 40 if room == "room" else 30)
    lay = prog_hash_writes(ks)
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [spec])
    ret, faults, _, _ = op.run(pk, n, 64, nthreads=4)
    want, wf, live = _expect(pk, spec)
    np.testing.assert_array_equal(faults, wf)
    np.testing.assert_array_equal(ret, want)
    assert op.hash_models[0].items() == live.items()
    assert {16} <= set((ret & 0xff).tolist()) if room == "full" else True


def test_oracle_hash_delete_null_key_and_unreadable_key():
    """delete(NULL) is EINVAL with nothing logged; a key the program cannot read faults MEM
    (the reference hashes it first, ebpf_map_hashtable.c:478)."""
    from generic_ebpf_amd import layout
    I, LdDw, MapRef, Branch = _nodes()
    lay = layout.assemble([
        I("ldxb", R6, R1, 0), I("and_imm", R6, imm=1),
        LdDw(R1, MapRef(0)),
        Branch(I("jeq_imm", R6, imm=0), [I("mov_imm", R2, imm=0), I("call", imm=2), I("exit")]),
        I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-2),
        I("call", imm=2), I("exit")])
    spec = _table(4, 63, 10, 20)
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [spec])
    pk = _packets(200, 64)
    ret, faults, _, _ = op.run(pk, 200, 64)
    odd = (pk[:, 0] & 1).astype(bool)
    assert (faults[odd] == 3).all() and (faults[~odd] == 0).all()
    assert (ret[~odd] == 22).all()
    assert op.last_hlog == []


def test_translation_of_hash_writes(native, env):
    """The translator resolves update / delete on a hashtable known at translation time (device
    code builds for every layout)."""
    for ks in (4, 12):
        lay = prog_hash_writes(ks)
        m = native.HashMap(env, ks, 8, 40)
        p = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [m.handle]))
        try:
            p.info()
            assert len(p.device_code(1)) > 0 and len(p.device_code(0)) > 0
        finally:
            p.destroy()
            m.destroy()


# ---------------------------------------------------------------- GPU


def _walk(gpu, hm):
    """The table through the host API: get_next_key's walk with each key's value."""
    import ctypes
    L = gpu.lib()
    out, prev = [], None
    while True:
        nk = ctypes.create_string_buffer(hm.key_size)
        k = None if prev is None else ctypes.create_string_buffer(prev, hm.key_size)
        if L.ebpf_map_get_next_key_from_user(hm.ptr, k, nk) != 0:
            return out
        prev = nk.raw
        err, v = hm.lookup(prev)
        assert err == 0
        out.append((prev, v))


def _device_map(gpu, env, spec):
    hm = gpu.HashMap(env, spec.key_size, spec.value_size, spec.capacity)
    for k, v in spec.items:
        assert hm.update(k, v) == 0
    return hm


def _run(gpu, p, pk, resident):
    import torch
    n = len(pk)
    if not resident:
        ret, faults, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), n, 64)
        return ret, faults
    dev = torch.device("cuda:0")
    d_pk = torch.from_numpy(np.ascontiguousarray(pk.reshape(-1))).to(dev)
    d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
    d_flt = torch.zeros(n, dtype=torch.uint8, device=dev)
    p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), None, d_flt.data_ptr(), None,
                    torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return d_ret.cpu().numpy().view(np.uint64), d_flt.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("resident", [False, True])
@pytest.mark.parametrize("ks", [4, 12])
@pytest.mark.parametrize("room", ["room", "full"])
def test_device_hash_writes_vs_oracle(gpu, env, variant, resident, ks, room):
    """Two batches: results and faults of each against the oracle, the table after each through
    get_next_key (the reference's bucket order) against the oracle's replayed model."""
    n = (1 << 16) + 29
    spec = _table(ks, 71, 30, 40 if room == "room" else 30)
    lay = prog_hash_writes(ks)
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [spec])
    hm = _device_map(gpu, env, spec)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [hm.handle]))
    try:
        gpu.set_variant(variant)
        for seed in (72, 73):
            pk = _packets(n, seed)
            want, wf, _, _ = op.run(pk, n, 64, nthreads=16)
            ret, faults = _run(gpu, p, pk, resident)
            np.testing.assert_array_equal(faults, wf)
            np.testing.assert_array_equal(ret, want)
            assert _walk(gpu, hm) == op.hash_models[0].items()
            # the next batch starts from the replayed table
            op = pyoracle.OracleProgram(lay.code, lay.relocs, [
                pyoracle.HashSpec.from_model(op.hash_models[0], ks, 8)])
    finally:
        gpu.set_variant(0)
        p.destroy()
        hm.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("ndev", [2, 3])
def test_device_hash_writes_multi_device(gpu, env, ndev):
    """Sharded over several devices (one GPU listed ndev times): the shards' logs replay in
    global packet order, so the table equals ONE batch's (the oracle)."""
    n = (1 << 17) + 3
    spec = _table(12, 81, 30, 40)
    lay = prog_hash_writes(12)
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [spec])
    pk = _packets(n, 82)
    want, wf, _, _ = op.run(pk, n, 64, nthreads=16)
    hm = _device_map(gpu, env, spec)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [hm.handle]))
    try:
        ret, faults, _ = p.run_batch_multi([0] * ndev, np.ascontiguousarray(pk.reshape(-1)), n, 64)
        np.testing.assert_array_equal(faults, wf)
        np.testing.assert_array_equal(ret, want)
        assert _walk(gpu, hm) == op.hash_models[0].items()
    finally:
        p.destroy()
        hm.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2])
def test_device_hash_writes_host_update_between_batches(gpu, env, variant):
    """A host update / delete between two batches is what the second batch sees."""
    n = 1 << 15
    spec = _table(4, 91, 20, 48)
    lay = prog_hash_writes(4)
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [spec])
    hm = _device_map(gpu, env, spec)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [hm.handle]))
    try:
        gpu.set_variant(variant)
        pk1, pk2 = _packets(n, 92), _packets(n, 93)
        op.run(pk1, n, 64, nthreads=16)
        ret, faults = _run(gpu, p, pk1, False)
        model = op.hash_models[0]
        k_new, k_old = _key(63, 4), model.items()[0][0]
        for m in (model, hm):
            m.update(k_new, b"\x11" * 8, 0)
            m.delete(k_old)
        op2 = pyoracle.OracleProgram(lay.code, lay.relocs, [pyoracle.HashSpec.from_model(model, 4, 8)])
        want, wf, _, _ = op2.run(pk2, n, 64, nthreads=16)
        ret, faults = _run(gpu, p, pk2, True)
        np.testing.assert_array_equal(faults, wf)
        np.testing.assert_array_equal(ret, want)
        assert _walk(gpu, hm) == op2.hash_models[0].items()
    finally:
        gpu.set_variant(0)
        p.destroy()
        hm.destroy()
