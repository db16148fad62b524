"""Map writes inside loops (include/ebpf_gpu.h "Map writes in a device
batch", "Stores into map values"; the reference writes anywhere: ebpf_interpreter.c:343-366,
282-284, ebpf_map_array.c:198-211).  Option walks over a TLV area (tests/loopwrites.py) that
count with XADD and with the LDX / ADD / STX idiom, call map_update_elem and store into map
values inside the loop.

CPU: the oracle's batch mode against the step-by-step restatement in loopwrites.py (16 logged
writes per packet, the 17th faulting EBPF_FAULT_WRITES; counter updates uncapped additions), the
oracle's sequential mode for the counters (additions commute: the reference's own run), and the
translation rules for loops (counter updates only into atomic arrays, never read back).
GPU: every device variant, host-buffer and device-resident, results + faults + the map against
the oracle."""
import ctypes
import errno
import os

import numpy as np
import pytest

import loopwrites as lw
import pyoracle

VARIANTS = [int(v) for v in os.environ.get("EBPF_TEST_VARIANTS", "0,1,2").split(",")]


def _init(vs, seed):
    return np.random.default_rng(seed).integers(0, 256, lw.NKEYS * vs, dtype=np.uint8).tobytes()


def _nkeys(kind):
    return lw.MAP_KEYS.get(kind, lw.NKEYS)


def _oracle(kind, pk, init, sequential=False):
    code, rel = lw.PROGS[kind]()
    op = pyoracle.OracleProgram(code, rel, [(lw.VALUE_SIZE[kind], _nkeys(kind), init)], semantics=1,
                                sequential=sequential)
    ret, flt, _, _ = op.run(pk.reshape(-1), len(pk), 64, nthreads=1 if sequential else 4)
    return ret, flt, op.map_bytes(0)


@pytest.mark.parametrize("kind", sorted(lw.PROGS))
def test_oracle_loop_writes_known_answers(kind):
    pk = lw.packets(4000, 11)
    init = lw.initial_map(kind, 12)
    ret, flt, after = _oracle(kind, pk, init)
    want, wf, wafter = lw.expect(kind, pk, init, lw.VALUE_SIZE[kind])
    np.testing.assert_array_equal(flt, wf)
    np.testing.assert_array_equal(ret, want)
    assert after == wafter
    assert (wf == 0).any() and (wf == lw.FAULT_MEM).any()
    if kind in ("updates", "stores", "xadd_fetch"):
        assert (wf == lw.FAULT_WRITES).any()       # some walks pass 16 logged writes / 32 words
    if kind == "limiter":
        assert (want >= 0x1000).any() and (want < 0x1000).any()   # some walks are cut short
    if kind in ("xadd", "idiom"):
        # counters: the batch ends where the reference's sequential run ends
        _, _, seq = _oracle(kind, pk, init, sequential=True)
        assert seq == after
    if kind == "xadd_fetch":
        # ... over the walks that keep within the 32 words (the reference has no such limit)
        sel = pk[wf != lw.FAULT_WRITES]
        _, _, seq = _oracle(kind, sel, init, sequential=True)
        assert seq == _oracle(kind, sel, init)[2]


def test_oracle_write_cap_is_batch_only():
    """The reference's own run (sequential mode) has no limit: a 20-update walk succeeds."""
    pk = lw.packets(2000, 13)
    opts = np.array([len(lw.walk_options(p)) for p in pk])
    init = _init(8, 14)
    ret, flt, _ = _oracle("updates", pk, init, sequential=True)
    assert ((opts > 16) & (flt == 0)).any()


def limiter_packets(n, seed):
    """limiter walks whose options all carry type n_i (packet i's own key, 0 < n_i < 256: no
    two packets count the same key)"""
    pk = lw.packets(n, seed)
    for i, p in enumerate(pk):
        for at in lw.walk_options(p):
            p[at] = i + 1
    return pk


def test_oracle_limiter_distinct_keys_equal_sequential_reference():
    """packets that count distinct keys: the batch (each packet's view = batch start + its own
    additions) is the reference's one-after-the-other run, results and map"""
    pk = limiter_packets(255, 15)
    code, rel = lw.prog_limiter(nkeys=256)
    init = np.random.default_rng(16).integers(0, 3, 256, dtype=np.uint64).tobytes()
    outs = []
    for seq in (False, True):
        op = pyoracle.OracleProgram(code, rel, [(8, 256, init)], semantics=1, sequential=seq)
        ret, flt, _, _ = op.run(pk.reshape(-1), len(pk), 64, nthreads=1 if seq else 4)
        outs.append((ret, flt, op.map_bytes(0)))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2]
    assert (outs[0][0] >= 0x1000).any()


def _translate_error(native, env, code, rel, maps):
    p = native.Prog(env, native.patch_relocs(code, rel, [m.handle for m in maps]))
    try:
        p.set_semantics(native.SEM_STANDARD)

        class Info(ctypes.Structure):
            _fields_ = [("nslots", ctypes.c_uint32), ("nentries", ctypes.c_uint32),
                        ("nmaps", ctypes.c_uint32), ("max_stack", ctypes.c_uint32)]
        i = Info()
        return native.lib().ebpf_prog_device_info(p.ptr, ctypes.byref(i))
    finally:
        p.destroy()


def test_loop_translation_rules(native, env):
    """Counter updates in a loop go into an atomic array: XADD, the idiom with a dead register,
    and (round 6) the idiom whose register is read afterwards and XADD with BPF_FETCH, read back
    through the packet's view, translate; a plain load of a counter's word after its update, and
    a counter update into a map that stores also change, return EOPNOTSUPP.  Updates and stores
    in loops translate (capped)."""
    m = native.Map(env, lw.NKEYS, 16)
    m8 = native.Map(env, lw.NKEYS, 8)
    m64 = native.Map(env, lw.FETCH_KEYS, 16)
    try:
        assert _translate_error(native, env, *lw.prog_xadd_counters(), [m]) == 0
        assert _translate_error(native, env, *lw.prog_idiom_counters(), [m8]) == 0
        assert _translate_error(native, env, *lw.prog_idiom_counters(live=True), [m8]) == 0
        assert _translate_error(native, env, *lw.prog_limiter(), [m8]) == 0
        assert _translate_error(native, env, *lw.prog_xadd_fetch(), [m64]) == 0
        assert _translate_error(native, env, *lw.prog_xadd_then_load(), [m8]) == errno.EOPNOTSUPP
        assert _translate_error(native, env, *lw.prog_updates(), [m8]) == 0
        assert _translate_error(native, env, *lw.prog_stores(), [m8]) == 0
        code, rel = lw.prog_mixed_counter_store()
        assert _translate_error(native, env, code, rel, [m8]) == errno.EOPNOTSUPP
    finally:
        m.destroy()
        m8.destroy()
        m64.destroy()


# ---- counter updates into a hashtable inside loops (round 6): records, counted writes ----

def _hash_oracle(kind, pk, init, sequential=False):
    """(ret, faults, array image of the table after the batch) on the oracle"""
    code, rel = lw.HASH_PROGS[kind]()
    vs = lw.VALUE_SIZE[kind]
    items = lw.hash_items(init, vs)
    spec = pyoracle.HashSpec(4, vs, items=items, capacity=lw.NKEYS)
    op = pyoracle.OracleProgram(code, rel, [spec], semantics=1, sequential=sequential)
    ret, flt, _, _ = op.run(pk.reshape(-1), len(pk), 64, nthreads=1 if sequential else 4)
    if sequential:   # (the values written in place, in the spec's order)
        vals = op.map_bytes(0)
        after = [(k, vals[i * vs:(i + 1) * vs]) for i, (k, _) in enumerate(items)]
    else:
        after = op.hash_models[0].items()
    return ret, flt, lw.hash_image(after, vs)


def _hash_init(kind, seed):
    vs = lw.VALUE_SIZE[kind]
    return lw.hash_image(lw.hash_items(lw.initial_map(kind, seed), vs), vs)


@pytest.mark.parametrize("kind", sorted(lw.HASH_PROGS))
def test_oracle_hash_loop_counters_known_answers(kind):
    """the oracle's batch mode against the step-by-step restatement: hashtable counter updates
    are counted records (the 17th logged write faults WRITES, the additions before it land);
    over the walks that keep within 16, the map is the reference's sequential run's (the
    limiter's additions depend on what it reads, so only its batch is checked)"""
    pk = lw.packets(4000, 41)
    vs = lw.VALUE_SIZE[kind]
    init = _hash_init(kind, 42)
    ret, flt, after = _hash_oracle(kind, pk, init)
    want, wf, wafter = lw.expect(kind, pk, init, vs, present=lw.HASH_PRESENT)
    np.testing.assert_array_equal(flt, wf)
    np.testing.assert_array_equal(ret, want)
    assert after == wafter
    assert (wf == 0).any() and (wf == lw.FAULT_MEM).any()
    if kind == "xadd":
        assert (wf == lw.FAULT_WRITES).any()    # two records an option
    if kind != "limiter":
        sel = pk[wf != lw.FAULT_WRITES]
        assert _hash_oracle(kind, sel, init, sequential=True)[2] == _hash_oracle(kind, sel, init)[2]


def test_hash_loop_translation_rules(native, env):
    """Counter updates into a hashtable inside a loop translate (XADD, the idiom with a dead and
    a live register, the limiter, XADD then a plain load of the word, a counter and a store into
    one hashtable); the plain load after an array counter's XADD stays EOPNOTSUPP."""
    h16 = native.HashMap(env, 4, 16, lw.NKEYS)
    h8 = native.HashMap(env, 4, 8, lw.NKEYS)
    m8 = native.Map(env, lw.NKEYS, 8)
    try:
        assert _translate_error(native, env, *lw.prog_xadd_counters(), [h16]) == 0
        assert _translate_error(native, env, *lw.prog_idiom_counters(), [h8]) == 0
        assert _translate_error(native, env, *lw.prog_idiom_counters(live=True), [h8]) == 0
        assert _translate_error(native, env, *lw.prog_limiter(), [h8]) == 0
        assert _translate_error(native, env, *lw.prog_xadd_then_load(), [h8]) == 0
        assert _translate_error(native, env, *lw.prog_mixed_counter_store(), [h8]) == 0
        assert _translate_error(native, env, *lw.prog_xadd_then_load(), [m8]) == errno.EOPNOTSUPP
    finally:
        h16.destroy()
        h8.destroy()
        m8.destroy()


def _hash_device(gpu, env, kind, pk, init, variant, resident):
    code, rel = lw.HASH_PROGS[kind]()
    vs = lw.VALUE_SIZE[kind]
    items = lw.hash_items(init, vs)
    m = gpu.HashMap(env, 4, vs, lw.NKEYS)
    try:
        m.fill(np.frombuffer(b"".join(k for k, _ in items), np.uint8),
               np.frombuffer(b"".join(v for _, v in items), np.uint8))
        ret, flt, ex = _run(gpu, env, code, rel, m, pk, variant, resident)
        after = []
        for k, _ in items:
            err, v = m.lookup(k)
            assert err == 0
            after.append((k, v))
        return ret, flt, lw.hash_image(after, vs), ex
    finally:
        m.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("kind", sorted(lw.HASH_PROGS))
@pytest.mark.parametrize("resident", [False, True])
def test_device_hash_loop_counters_vs_oracle(gpu, env, variant, kind, resident):
    """hashtable counter walks on every variant: results, faults and the table against the
    oracle's batch mode"""
    pk = lw.packets((1 << 15) + 11, 43)
    init = _hash_init(kind, 44)
    want, wf, wafter = _hash_oracle(kind, pk, init)
    ret, flt, after, _ = _hash_device(gpu, env, kind, pk, init, variant, resident)
    np.testing.assert_array_equal(flt, wf)
    np.testing.assert_array_equal(ret, want)
    assert after == wafter


def _run(gpu, env, code, rel, m, pk, variant, resident):
    """(ret, faults, exec path) of one batch of the program over map m, host buffers or
    device-resident"""
    import torch
    p = gpu.Prog(env, gpu.patch_relocs(code, rel, [m.handle]))
    n = len(pk)
    try:
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
            ret, flt = d_ret.cpu().numpy().view(np.uint64), d_flt.cpu().numpy()
        else:
            ret, flt, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), n, 64)
        return ret, flt, p.exec_info(0)[0]
    finally:
        gpu.set_variant(0)
        p.destroy()


def _device(gpu, env, kind, pk, init, variant, resident):
    code, rel = lw.PROGS[kind]()
    m = gpu.Map(env, _nkeys(kind), lw.VALUE_SIZE[kind])
    try:
        m.fill(init)
        ret, flt, ex = _run(gpu, env, code, rel, m, pk, variant, resident)
        after = b"".join(m.lookup(k)[1] for k in range(_nkeys(kind)))
        return ret, flt, after, ex
    finally:
        m.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("kind", sorted(lw.PROGS))
@pytest.mark.parametrize("resident", [False, True])
def test_device_loop_writes_vs_oracle(gpu, env, variant, kind, resident):
    pk = lw.packets((1 << 15) + 11, 21)
    init = lw.initial_map(kind, 22)
    want, wf, wafter = _oracle(kind, pk, init)
    ret, flt, after, ex = _device(gpu, env, kind, pk, init, variant, resident)
    np.testing.assert_array_equal(flt, wf)
    np.testing.assert_array_equal(ret, want)
    assert after == wafter
    if variant in (0, 2):
        # (a loop program that reads map values back keeps 32 overlay words per lane, and a
        # load through a map value the generic handler serves reserves the whole 512-B frame:
        # 256 lanes' slices leave the assembly kernels no room, so it runs on the portable HIP
        # interpreter, DESIGN.md "Out of scope".  xadd_fetch has no such load: it runs on the
        # assembly paths, whose overlay fills and faults WRITES, round 6)
        want_ex = "compiled" if variant == 0 else "interpreter"
        assert ex == ("hip" if kind in ("stores", "limiter") else want_ex)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_device_limiter_distinct_keys_equal_sequential_reference(gpu, env, variant):
    """the rate limiter over packets that count distinct keys: results and the map equal the
    reference's one-after-the-other run (the oracle's sequential mode)"""
    pk = limiter_packets(255, 17)
    code, rel = lw.prog_limiter(nkeys=256)
    init = np.random.default_rng(18).integers(0, 3, 256, dtype=np.uint64).tobytes()
    op = pyoracle.OracleProgram(code, rel, [(8, 256, init)], semantics=1, sequential=True)
    want, wf, _, _ = op.run(pk.reshape(-1), len(pk), 64, nthreads=1)
    m = gpu.Map(env, 256, 8)
    m.fill(init)
    p = gpu.Prog(env, gpu.patch_relocs(code, rel, [m.handle]))
    try:
        p.set_semantics(gpu.SEM_STANDARD)
        gpu.set_variant(variant)
        ret, flt, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), len(pk), 64)
        after = b"".join(m.lookup(k)[1] for k in range(256))
    finally:
        gpu.set_variant(0)
        p.destroy()
        m.destroy()
    np.testing.assert_array_equal(flt, wf)
    np.testing.assert_array_equal(ret, want)
    assert after == op.map_bytes(0)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_device_xadd_walk_full_size_equals_sequential_reference(gpu, env, variant):
    """1M packets of the per-option XADD counter walk: the counters equal the reference's
    sequential run (oracle, sequential mode) bit-exact."""
    pk = lw.packets(1 << 20 if variant != 1 else 1 << 18, 23)
    init = _init(16, 24)
    _, _, seq = _oracle("xadd", pk, init, sequential=True)
    ret, flt, after, _ = _device(gpu, env, "xadd", pk, init, variant, True)
    assert after == seq


def _random_maps(k):
    g = np.random.default_rng(500 + k)
    return [(16, 16, g.integers(0, 256, 256, dtype=np.uint8).tobytes()),
            (8, 16, g.integers(0, 256, 128, dtype=np.uint8).tobytes())]


def test_oracle_random_loop_write_programs_fault_writes_somewhere():
    """The generator's programs exercise the cap: over 40 programs some packets fault WRITES,
    some finish, and a one-packet batch equals the sequential run (no cap for the reference)
    whenever the packet made at most 16 logged writes."""
    import stdprogs
    from generic_ebpf_amd import workloads
    seen = set()
    for k in range(40):
        code, rel = stdprogs.gen_loop_write_program(800 + k, counters=k % 3 == 2)
        pk = workloads.packets_random(256, 64, seed=900 + k)
        op = pyoracle.OracleProgram(code, rel, _random_maps(k), semantics=1)
        ret, flt, _, _ = op.run(pk.reshape(-1), len(pk), 64, nthreads=4)
        seen |= set(int(x) for x in np.unique(flt))
    assert {0, lw.FAULT_WRITES} <= seen


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_device_random_loop_write_programs_vs_oracle(gpu, env, variant):
    """Random loop programs with stores, loads back, updates (and, every third, counter
    updates) inside the loops: results, faults and both maps against the oracle's batch mode."""
    import stdprogs
    from generic_ebpf_amd import workloads
    bad = []
    for k in range(30):
        code, rel = stdprogs.gen_loop_write_program(800 + k, counters=k % 3 == 2)
        maps = _random_maps(k)
        n = 4096 + k
        pk = workloads.packets_random(n, 64, seed=900 + k)
        op = pyoracle.OracleProgram(code, rel, maps, semantics=1)
        want, wf, _, _ = op.run(pk.reshape(-1), n, 64, nthreads=8)
        ms = []
        for vs, me, d in maps:
            m = gpu.Map(env, me, vs)
            m.fill(d)
            ms.append(m)
        p = gpu.Prog(env, gpu.patch_relocs(code, rel, [m.handle for m in ms]))
        try:
            p.set_semantics(gpu.SEM_STANDARD)
            gpu.set_variant(variant)
            ret, flt, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), n, 64)
            after = [b"".join(m.lookup(key)[1] for key in range(m.max_entries)) for m in ms]
        finally:
            gpu.set_variant(0)
            p.destroy()
            for m in ms:
                m.destroy()
        if not (np.array_equal(ret, want) and np.array_equal(flt, wf) and
                after[0] == op.map_bytes(0) and after[1] == op.map_bytes(1)):
            bad.append((k, int((ret != want).sum()), int((flt != wf).sum()),
                        after[0] == op.map_bytes(0), after[1] == op.map_bytes(1)))
    assert not bad, bad


def prog_spilled_packet_stores():
    """A loop that stores through a packet pointer reloaded from a stack spill (the translator
    cannot prove it is the packet: a possible store into a map value): trip k
    writes byte k + 20 of the packet, then r0 = the packet's bytes 20..28 read back."""
    import stdprogs
    I = stdprogs.I
    return stdprogs.asm([
        I("stxdw", 10, 1, -8), I("ldxb", 8, 1, 3), I("and64_imm", 8, imm=7), I("add64_imm", 8, imm=1),
        ("label", "L"), I("ldxdw", 7, 10, -8), I("add64_reg", 7, 8), I("stxb", 7, 8, 19),
        I("sub64_imm", 8, imm=1), I("jne_imm", 8, imm=0, off="L"),
        I("ldxdw", 0, 1, 20), I("exit")])


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("stride", [64, 72])
def test_device_loop_stores_through_spilled_packet_pointer(gpu, env, variant, stride):
    from generic_ebpf_amd import workloads
    code, rel = prog_spilled_packet_stores()
    n = 20011
    pk = workloads.packets_random(n, stride, seed=31)
    want, wf, wdata, _ = pyoracle.OracleProgram(code, rel, [], semantics=1).run(pk.reshape(-1), n, stride)
    assert not wf.any()
    p = gpu.Prog(env, code)
    try:
        p.set_semantics(gpu.SEM_STANDARD)
        gpu.set_variant(variant)
        data = np.ascontiguousarray(pk.reshape(-1).copy())
        ret, flt, _ = p.run_batch(data, n, stride)
    finally:
        gpu.set_variant(0)
        p.destroy()
    assert not flt.any()
    np.testing.assert_array_equal(ret, want)
    np.testing.assert_array_equal(data, wdata)


def test_spilled_packet_pointer_store_loop_translates(native, env):
    code, rel = prog_spilled_packet_stores()
    assert _translate_error(native, env, code, rel, []) == 0


# ---- random loop programs over a hashtable: counters, stores, loads and updates mixed ----

def _random_hash_maps(k):
    """map 0: a hashtable of u32 keys holding 12 of the 16 the programs look up (16-B values);
    map 1: an array of 16 8-B values (as _random_maps)"""
    g = np.random.default_rng(700 + k)
    items = [(key.to_bytes(4, "little"), g.integers(0, 256, 16, dtype=np.uint8).tobytes())
             for key in sorted(lw.HASH_PRESENT)]
    return items, (8, 16, g.integers(0, 256, 128, dtype=np.uint8).tobytes())


def _hash_oracle_random(code, rel, k, pk):
    items, arr = _random_hash_maps(k)
    spec = pyoracle.HashSpec(4, 16, items=items, capacity=lw.NKEYS)
    op = pyoracle.OracleProgram(code, rel, [spec, arr], semantics=1)
    ret, flt, _, _ = op.run(pk.reshape(-1), len(pk), 64, nthreads=8)
    table = dict(op.hash_models[0].items())
    return ret, flt, [table[key] for key, _ in items], op.map_bytes(1)


def test_oracle_random_hash_loop_programs_fault_writes_somewhere():
    """the mixed generator's programs translate, and over 30 of them some packets fault WRITES
    (their counter records count) and some finish"""
    import stdprogs
    from generic_ebpf_amd import workloads
    seen = set()
    for k in range(30):
        code, rel = stdprogs.gen_loop_write_program(1200 + k, mixed=True)
        pk = workloads.packets_random(256, 64, seed=1300 + k)
        _, flt, _, _ = _hash_oracle_random(code, rel, k, pk)
        seen |= set(int(x) for x in np.unique(flt))
    assert {0, lw.FAULT_WRITES} <= seen


def test_random_hash_loop_programs_translate(native, env):
    import stdprogs
    h = native.HashMap(env, 4, 16, lw.NKEYS)
    a = native.Map(env, 16, 8)
    try:
        for k in range(30):
            code, rel = stdprogs.gen_loop_write_program(1200 + k, mixed=True)
            p = native.Prog(env, native.patch_relocs(code, rel, [h.handle, a.handle]))
            try:
                p.set_semantics(native.SEM_STANDARD)

                class Info(ctypes.Structure):
                    _fields_ = [("nslots", ctypes.c_uint32), ("nentries", ctypes.c_uint32),
                                ("nmaps", ctypes.c_uint32), ("max_stack", ctypes.c_uint32)]
                i = Info()
                assert native.lib().ebpf_prog_device_info(p.ptr, ctypes.byref(i)) == 0, k
            finally:
                p.destroy()
    finally:
        h.destroy()
        a.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_device_random_hash_loop_programs_vs_oracle(gpu, env, variant):
    """30 random loop programs mixing counter updates (fetched or not), stores, loads back and
    updates in one hashtable's values: results, faults, the table and the array against the
    oracle's batch mode"""
    import stdprogs
    from generic_ebpf_amd import workloads
    bad = []
    for k in range(30):
        code, rel = stdprogs.gen_loop_write_program(1200 + k, mixed=True)
        n = 4096 + k
        pk = workloads.packets_random(n, 64, seed=1300 + k)
        want, wf, wtab, warr = _hash_oracle_random(code, rel, k, pk)
        items, (avs, ame, ad) = _random_hash_maps(k)
        h = gpu.HashMap(env, 4, 16, lw.NKEYS)
        a = gpu.Map(env, ame, avs)
        h.fill(np.frombuffer(b"".join(key for key, _ in items), np.uint8),
               np.frombuffer(b"".join(v for _, v in items), np.uint8))
        a.fill(ad)
        p = gpu.Prog(env, gpu.patch_relocs(code, rel, [h.handle, a.handle]))
        try:
            p.set_semantics(gpu.SEM_STANDARD)
            gpu.set_variant(variant)
            ret, flt, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), n, 64)
            tab = [h.lookup(key)[1] for key, _ in items]
            arr = b"".join(a.lookup(key)[1] for key in range(ame))
        finally:
            gpu.set_variant(0)
            p.destroy()
            h.destroy()
            a.destroy()
        if not (np.array_equal(ret, want) and np.array_equal(flt, wf) and tab == wtab and arr == warr):
            bad.append((k, int((ret != want).sum()), int((flt != wf).sum()), tab == wtab, arr == warr))
    assert not bad, bad


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_device_hash_loop_counters_other_entry_points(gpu, env, variant):
    """the hashtable rate limiter and XADD walk sharded over [0, 0] (the shards' counted records
    merged in global packet order on the host) and asynchronously: as one batch, against the
    oracle"""
    for kind in ("limiter", "xadd"):
        code, rel = lw.HASH_PROGS[kind]()
        vs = lw.VALUE_SIZE[kind]
        pk = lw.packets((1 << 13) + 5, 51)
        init = _hash_init(kind, 52)
        want, wf, wafter = _hash_oracle(kind, pk, init)
        items = lw.hash_items(init, vs)
        for how in ("multi", "async"):
            m = gpu.HashMap(env, 4, vs, lw.NKEYS)
            m.fill(np.frombuffer(b"".join(k for k, _ in items), np.uint8),
                   np.frombuffer(b"".join(v for _, v in items), np.uint8))
            p = gpu.Prog(env, gpu.patch_relocs(code, rel, [m.handle]))
            try:
                p.set_semantics(gpu.SEM_STANDARD)
                gpu.set_variant(variant)
                data = np.ascontiguousarray(pk.reshape(-1).copy())
                if how == "multi":
                    ret, flt, _ = p.run_batch_multi([0, 0], data, len(pk), 64)
                else:
                    ret, flt, _ = p.run_batch_async(data, len(pk), 64).wait()
                after = lw.hash_image([(k, m.lookup(k)[1]) for k, _ in items], vs)
            finally:
                gpu.set_variant(0)
                p.destroy()
                m.destroy()
            np.testing.assert_array_equal(flt, wf, err_msg="%s %s" % (kind, how))
            np.testing.assert_array_equal(ret, want, err_msg="%s %s" % (kind, how))
            assert after == wafter, (kind, how)
