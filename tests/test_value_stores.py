"""Stores into map values through a lookup result, in a device batch (include/ebpf_gpu.h
"Stores into map values"; the reference writes in place: ebpf_interpreter.c:343-366 through the
pointer array_map_lookup_elem returns, ebpf_map_array.c:115-124).

CPU: the oracle's batch mode against the hand restatement in valueprogs.py (read-your-writes,
byte-wise last writer, counter updates as additions, faults), and against the oracle's
sequential mode — the reference's own one-packet-after-the-other run — where the rules promise
equality (maps touched only by counter updates; one-packet batches).
GPU: every device variant against the oracle, host-buffer and device-resident."""
import os

import numpy as np
import pytest

import pyoracle
import valueprogs as vp

N = 3000


def _init(vs, seed):
    return np.random.default_rng(seed).integers(0, 256, vp.NKEYS * vs, dtype=np.uint8).tobytes()


def _oracle(lay, maps, pk, semantics=0, sequential=False, nthreads=4):
    op = pyoracle.OracleProgram(lay[0] if isinstance(lay, tuple) else lay.code,
                                lay[1] if isinstance(lay, tuple) else lay.relocs, maps,
                                semantics=semantics, sequential=sequential)
    ret, faults, _, _ = op.run(pk, len(pk), 64, nthreads=nthreads)
    return ret, faults, op


@pytest.mark.parametrize("width,off,vs,alu", [
    (8, 0, 8, "add64_reg"), (4, 0, 8, "add32_reg"), (4, 4, 8, "add64_reg"), (8, 0, 8, "sub64_reg"),
    (8, 0, 8, "add64_imm"), (8, 0, 8, "mov64_reg"), (8, 4, 12, "add64_reg"), (4, 2, 12, "add32_reg")])
@pytest.mark.parametrize("reload", [False, True])
def test_oracle_counter_known_answers(width, off, vs, alu, reload):
    pk = vp.packets(N, 81)
    init = _init(vs, 82)
    lay = vp.prog_counter(width, off, alu, reload)
    ret, faults, op = _oracle(lay, [(vs, vp.NKEYS, init)], pk)
    want, wf, after = vp.expect_counter(pk, init, vs, width, off, alu, reload)
    np.testing.assert_array_equal(faults, wf)
    np.testing.assert_array_equal(ret, want)
    assert op.map_bytes(0) == after
    if all((k * vs + off) % width == 0 for k in range(vp.NKEYS)):
        # only counter updates touch the map: it ends as the reference's sequential run leaves it
        assert after == vp.sequential_counter_map(pk, init, vs, width, off, alu)
        _, _, seq = _oracle(lay, [(vs, vp.NKEYS, init)], pk, sequential=True)
        assert seq.map_bytes(0) == after


def test_oracle_sequential_mode_is_the_reference_run():
    """sequential=True: every update at once — a packet sees the earlier packets' counts."""
    pk = vp.packets(500, 83)
    init = _init(8, 84)
    lay = vp.prog_counter(8, 0, "add64_reg")
    ret, faults, op = _oracle(lay, [(8, vp.NKEYS, init)], pk, sequential=True)
    m = bytearray(init)
    for i, p in enumerate(pk):
        k = int(p[0]) & (vp.NKEYS - 1)
        x = (int.from_bytes(m[8 * k:8 * k + 8], "little") + int(p[1])) & vp.MASK[8]
        m[8 * k:8 * k + 8] = x.to_bytes(8, "little")
        assert int(ret[i]) == x
    assert op.map_bytes(0) == bytes(m)


@pytest.mark.parametrize("width,off", [(4, 2), (8, 0), (1, 7), (2, 3)])
def test_oracle_plain_store_known_answers(width, off):
    pk = vp.packets(N, 85)
    init = _init(8, 86)
    lay = vp.prog_store(width, off)
    ret, faults, op = _oracle(lay, [(8, vp.NKEYS, init)], pk)
    want, wf, after = vp.expect_store(pk, init, 8, width, off)
    np.testing.assert_array_equal(faults, wf)
    np.testing.assert_array_equal(ret, want)
    assert op.map_bytes(0) == after


def test_oracle_faults_keep_counter_updates_only():
    pk = vp.packets(N, 87)
    init = _init(8, 88)
    lay = vp.prog_counter(8, 0, "add64_reg", fault=True)
    ret, faults, op = _oracle(lay, [(8, vp.NKEYS, init)], pk)
    want, wf, after = vp.expect_counter(pk, init, 8, fault=True)
    assert (wf == 2).any() and (wf == 0).any()
    np.testing.assert_array_equal(faults, wf)
    np.testing.assert_array_equal(ret, want)
    assert op.map_bytes(0) == after
    lay = vp.prog_store(4, 2, fault=True)
    ret, faults, op = _oracle(lay, [(8, vp.NKEYS, init)], pk)
    want, wf, after = vp.expect_store(pk, init, 8, 4, 2, fault=True)
    np.testing.assert_array_equal(faults, wf)
    np.testing.assert_array_equal(ret, want)
    assert op.map_bytes(0) == after


def test_oracle_mixed_counter_and_store_in_packet_order():
    pk = vp.packets(N, 89)
    init = _init(8, 90)
    _, faults, op = _oracle(vp.prog_mixed(), [(8, vp.NKEYS, init)], pk)
    assert not faults.any()
    assert op.map_bytes(0) == vp.expect_mixed(pk, init)


@pytest.mark.parametrize("width", [4, 8])
@pytest.mark.parametrize("fetch", [False, True])
def test_oracle_xadd(width, fetch):
    pk = vp.packets(N, 91)
    init = _init(8, 92)
    code, rel = vp.prog_xadd(width, fetch)
    ret, faults, op = _oracle((code, rel), [(8, vp.NKEYS, init)], pk, semantics=1)
    want, after = vp.expect_xadd(pk, init, width, fetch)
    assert not faults.any()
    np.testing.assert_array_equal(ret, want)
    assert op.map_bytes(0) == after
    # the reference has no XADD (ebpf_interpreter.c:367-369: an invalid opcode)
    from generic_ebpf_amd import isa
    bare = isa.encode(0xdb if width == 8 else 0xc3, 10, 1, -8, 0) + isa.encode(isa.OPS["exit"])
    _, f2, _ = _oracle((bare, []), [], pk[:10], semantics=0)
    assert (f2 == 1).all()


def test_oracle_hash_value_counters():
    """A hashtable's values: the counter updates go to the replay (op 4), in place."""
    rng = np.random.default_rng(93)
    keys = [int(k).to_bytes(4, "little") for k in range(0, vp.NKEYS, 2)]
    items = [(k, rng.bytes(8)) for k in keys]
    spec = pyoracle.HashSpec(4, 8, items=items, capacity=32)
    lay = vp.prog_counter(8, 0, "add64_reg")
    pk = vp.packets(N, 94)
    ret, faults, op = _oracle(lay, [spec], pk)
    assert not faults.any()
    model = dict(items)
    for p in pk:
        k = (int(p[0]) & (vp.NKEYS - 1)).to_bytes(4, "little")
        if k in model:
            v = (int.from_bytes(model[k], "little") + int(p[1])) & vp.MASK[8]
            model[k] = v.to_bytes(8, "little")
    assert dict(op.hash_models[0].items()) == model
    assert (ret == vp.MISS).sum() == sum(1 for p in pk if (int(p[0]) & 15) % 2)


# ---------------------------------------------------------------- GPU: every variant vs the oracle

VARIANTS = [int(v) for v in os.environ.get("EBPF_TEST_VARIANTS", "0,1,2").split(",")]


def _device(gpu, env, lay, maps_spec, pk, variant, resident, semantics=0):
    """Run on the device; returns (ret, faults, the maps' bytes after: arrays through lookup,
    hashtables through get_next_key's walk)."""
    import torch
    n = len(pk)
    maps = []
    for spec in maps_spec:
        if isinstance(spec, pyoracle.HashSpec):
            m = gpu.HashMap(env, spec.key_size, spec.value_size, spec.capacity or len(spec))
            for k, v in spec.items:
                assert m.update(k, v) == 0
        else:
            vs, me, d = spec
            m = gpu.Map(env, me, vs)
            m.fill(d)
        maps.append(m)
    code, rel = (lay if isinstance(lay, tuple) else (lay.code, lay.relocs))
    p = gpu.Prog(env, gpu.patch_relocs(code, rel, [m.handle for m in maps]))
    try:
        if semantics:
            p.set_semantics(gpu.SEM_STANDARD)
        gpu.set_variant(variant)
        if resident:
            dev = torch.device("cuda:0")
            d_pk = torch.from_numpy(np.ascontiguousarray(pk.reshape(-1))).to(dev)
            d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
            d_flt = torch.zeros(n, dtype=torch.uint8, device=dev)
            p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), None, d_flt.data_ptr(),
                            None, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            ret, faults = d_ret.cpu().numpy().view(np.uint64), d_flt.cpu().numpy()
        else:
            ret, faults, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), n, 64)
        after = []
        for m, spec in zip(maps, maps_spec):
            if isinstance(spec, pyoracle.HashSpec):
                after.append(_walk(gpu, m))
            else:
                after.append(b"".join(m.lookup(k)[1] for k in range(m.max_entries)))
        return ret, faults, after
    finally:
        gpu.set_variant(0)
        p.destroy()
        for m in maps:
            m.destroy()


def _walk(gpu, hm):
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


def _vs_oracle(gpu, env, lay, maps_spec, pk, variant, resident, semantics=0):
    op = pyoracle.OracleProgram(*(lay if isinstance(lay, tuple) else (lay.code, lay.relocs)),
                                maps_spec, semantics=semantics)
    want, wf, _, _ = op.run(pk, len(pk), 64, nthreads=16)
    ret, faults, after = _device(gpu, env, lay, maps_spec, pk, variant, resident, semantics)
    np.testing.assert_array_equal(faults, wf)
    np.testing.assert_array_equal(ret, want)
    for k, spec in enumerate(maps_spec):
        if isinstance(spec, pyoracle.HashSpec):
            assert after[k] == op.hash_models[k].items()
        else:
            assert after[k] == op.map_bytes(k), k
    return op


CASES = {
    "counter64": (lambda: vp.prog_counter(8, 0, "add64_reg"), 8),
    "counter32": (lambda: vp.prog_counter(4, 4, "add32_reg"), 8),
    "counter_sub_reload": (lambda: vp.prog_counter(8, 0, "sub64_reg", reload=True), 8),
    "counter_unaligned": (lambda: vp.prog_counter(8, 4, "add64_reg"), 12),
    "counter_fault": (lambda: vp.prog_counter(8, 0, "add64_reg", fault=True), 8),
    "store": (lambda: vp.prog_store(4, 2), 8),
    "store_fault": (lambda: vp.prog_store(8, 0, fault=True), 8),
    "mixed": (lambda: vp.prog_mixed(), 8),
}


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("resident", [False, True])
@pytest.mark.parametrize("case", sorted(CASES))
def test_device_value_stores_vs_oracle(gpu, env, variant, resident, case):
    mk, vs = CASES[case]
    pk = vp.packets((1 << 16) + 17, 101)
    _vs_oracle(gpu, env, mk(), [(vs, vp.NKEYS, _init(vs, 102))], pk, variant, resident)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("width", [4, 8])
@pytest.mark.parametrize("fetch", [False, True])
def test_device_xadd_vs_oracle(gpu, env, variant, width, fetch):
    pk = vp.packets((1 << 16) + 5, 103)
    _vs_oracle(gpu, env, vp.prog_xadd(width, fetch), [(8, vp.NKEYS, _init(8, 104))], pk, variant,
               False, semantics=1)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_device_hash_value_counters(gpu, env, variant):
    rng = np.random.default_rng(105)
    items = [(int(k).to_bytes(4, "little"), rng.bytes(8)) for k in range(0, vp.NKEYS, 2)]
    spec = pyoracle.HashSpec(4, 8, items=items, capacity=32)
    pk = vp.packets((1 << 14) + 3, 106)
    _vs_oracle(gpu, env, vp.prog_counter(8, 0, "add64_reg", reload=True), [spec], pk, variant, False)
    _vs_oracle(gpu, env, vp.prog_store(4, 2), [spec], pk, variant, True)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("case", ["counter_sub_reload", "store", "mixed"])
def test_one_packet_batch_equals_cpu_run(gpu, env, variant, case):
    """A one-packet batch of a store-then-load program is the reference's own run: results and
    the map equal the CPU ebpf_prog_run (which writes in place, ebpf_interpreter.c:343-366)."""
    mk, vs = CASES[case]
    lay = mk()
    init = _init(vs, 107)
    for seed in range(6):
        pk = vp.packets(1, 200 + seed)
        ret, faults, after = _device(gpu, env, lay, [(vs, vp.NKEYS, init)], pk, variant, seed % 2 == 1)
        m = gpu.Map(env, vp.NKEYS, vs)
        m.fill(init)
        p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle]))
        try:
            r = p.run_cpu(np.ascontiguousarray(pk[0]))[0]
            cpu_after = b"".join(m.lookup(k)[1] for k in range(vp.NKEYS))
        finally:
            p.destroy()
            m.destroy()
        assert not faults.any()
        assert int(ret[0]) == r
        assert after[0] == cpu_after


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_counter_full_size_equals_sequential_reference(gpu, env, variant):
    """64M packets of the counter idiom: the final map equals the reference's sequential run
    (the oracle in sequential mode over the distinct packets, times the tiling)."""
    import torch
    D = 1 << 20
    n = 1 << 26 if variant != 1 else 1 << 22
    pk = vp.packets(D, 108)
    init = _init(8, 109)
    lay = vp.prog_counter(8, 0, "add64_reg")
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, vp.NKEYS, init)], sequential=True)
    op.run(pk, D, 64, nthreads=1)
    once = np.frombuffer(op.map_bytes(0), dtype=np.uint64) - np.frombuffer(init, dtype=np.uint64)
    want = (np.frombuffer(init, dtype=np.uint64) + once * np.uint64(n // D)).tobytes()
    m = gpu.Map(env, vp.NKEYS, 8)
    m.fill(init)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle]))
    dev = torch.device("cuda:0")
    try:
        gpu.set_variant(variant)
        d_pk = torch.from_numpy(pk.reshape(-1)).to(dev).repeat(n // D)
        d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
        p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), None, None, None,
                        torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        after = b"".join(m.lookup(k)[1] for k in range(vp.NKEYS))
        assert after == want
    finally:
        gpu.set_variant(0)
        p.destroy()
        m.destroy()


# ---------------------------------------------------------------- random programs


def _random_case(k):
    from generic_ebpf_amd import randprog
    g = np.random.default_rng(9000 + k)
    vs = int(g.choice([4, 8, 12, 16]))
    me = int(g.choice([8, 256]))
    lay = randprog.random_program(7000 + k, length=int(g.integers(10, 60)), nmaps=2,
                                  map_value_size=vs, writes=k % 3 == 0, vstores=True)
    maps = [(vs, me, g.integers(0, 256, vs * me, dtype=np.uint8).tobytes()) for _ in range(2)]
    return lay, maps


def test_oracle_one_packet_batches_are_the_reference_run():
    """For random programs with value stores: a one-packet batch (overlay, records applied after
    the batch) leaves the same results, faults, packet bytes and maps as the sequential run that
    writes in place — the rules reduce to the reference's behaviour for one packet."""
    from generic_ebpf_amd import workloads
    for k in range(40):
        lay, maps = _random_case(k)
        pk = workloads.packets_random(8, 64, seed=k)
        for i in range(len(pk)):
            a = pyoracle.OracleProgram(lay.code, lay.relocs, maps)
            b = pyoracle.OracleProgram(lay.code, lay.relocs, maps, sequential=True)
            ra, fa, da, _ = a.run(pk[i:i + 1], 1, 64)
            rb, fb, db, _ = b.run(pk[i:i + 1], 1, 64)
            assert (ra == rb).all() and (fa == fb).all() and (da == db).all(), (k, i)
            if not fa.any():
                assert a.map_bytes(0) == b.map_bytes(0) and a.map_bytes(1) == b.map_bytes(1), (k, i)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_random_value_store_programs_vs_oracle(gpu, env, variant):
    """Random programs whose lookups store into the values (plain stores, counter updates,
    read back), a third with map_update_elem / delete too: results, faults, packet bytes and
    both maps against the oracle's batch mode."""
    import goldens
    from helpers import device_run
    from generic_ebpf_amd import workloads
    bad = []
    for k in range(60):
        lay, maps = _random_case(k)
        n = 2048
        pk = workloads.packets_random(n, 64, seed=300 + k)
        op = pyoracle.OracleProgram(lay.code, lay.relocs, maps)
        want, wf, wdata, _ = op.run(pk.reshape(-1), n, 64, nthreads=8)
        ret, faults, after = _device(gpu, env, lay, maps, pk, variant, False)
        if not (np.array_equal(want, ret) and np.array_equal(wf, faults) and
                after[0] == op.map_bytes(0) and after[1] == op.map_bytes(1)):
            bad.append(k)
    assert not bad, bad
