"""Map writes in a device batch (§8(f) rank 4, write side; include/ebpf_gpu.h "Map writes in a
device batch"): map_update_elem / map_delete_elem called by the program.

Semantics (the oracle's ORACLE_HELPER_MAP_UPDATE mode, oracle/ebpf_oracle.h): every packet reads
the maps as they were when the batch started; an update returns the reference's code
(ebpf_map.c:101-108 -> ebpf_map_array.c:185-211: EINVAL for a NULL key / value or flags >
EBPF_EXIST, EEXIST for EBPF_NOEXIST, EINVAL for a key >= max_entries, else 0) and its write
lands after the batch in packet order (within a packet in call order); delete on an array map
is EINVAL (ebpf_map_array.c:246-250).  Hashtable maps: tests/test_hash_writes.py.

CPU tests pin the oracle mode with hand-computed answers and check the translator; GPU tests
compare every device variant (results, faults and the map's contents after the batch, read back
through the host API) with the oracle."""
import errno

import numpy as np
import pytest

import goldens
import pyoracle
from helpers import make_maps

R0, R1, R2, R3, R4, R5, R6, R7, R8, R9, R10 = range(11)
NKEYS = 16


def _nodes():
    from generic_ebpf_amd import isa, layout
    return isa.Insn, layout.LdDw, layout.MapRef, layout.Branch


def prog_static(second_update=False):
    """key = pkt[0] & 31 (half the keys out of range), flags = pkt[1] & 3 (3: EINVAL),
    value = pkt[8..16) — key and value on the stack at known offsets; then a lookup of the same
    key (the batch's snapshot) and r0 = value ^ rc (or 1000 + rc when the key is out of range).
    ``second_update``: a second update of the same key in the packet (value + 1, flags 0)."""
    from generic_ebpf_amd import layout
    I, LdDw, MapRef, Branch = _nodes()
    n = [I("ldxb", R6, R1, 0), I("ldxb", R7, R1, 1), I("ldxdw", R8, R1, 8),
         I("and_imm", R6, imm=31), I("and_imm", R7, imm=3),
         I("stxw", R10, R6, -4), I("stxdw", R10, R8, -16),
         LdDw(R1, MapRef(0)),
         I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
         I("mov_imm", R3, imm=0), I("mov64_reg", R3, R10), I("add64_imm", R3, imm=-16),
         I("mov_imm", R4, imm=0), I("mov64_reg", R4, R7),
         I("call", imm=1),
         I("mov_imm", R9, imm=0), I("mov64_reg", R9, R0)]
    if second_update:
        n += [I("add64_imm", R8, imm=1), I("stxdw", R10, R8, -16), I("mov_imm", R4, imm=0),
              I("call", imm=1), I("lsh64_imm", R0, imm=8), I("or64_reg", R9, R0)]
    n += [LdDw(R1, MapRef(0)),
          I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
          I("call", imm=0),
          Branch(I("jeq_imm", R0, imm=0), [I("mov_imm", R0, imm=1000), I("add64_reg", R0, R9),
                                           I("exit")]),
          I("ldxdw", R0, R0, 0), I("xor64_reg", R0, R9), I("exit")]
    return layout.assemble(n)


def prog_generic():
    """The key pointer is r10 - 4 times (pkt[2] & 1) — NULL for even bytes (EINVAL, nothing
    read), a stack pointer of unknown provenance otherwise — and the value is read straight from
    the packet (r3 = r1 + 16); then delete (EINVAL on an array) and r0 = rc | delete << 8."""
    from generic_ebpf_amd import layout
    I, LdDw, MapRef, Branch = _nodes()
    n = [I("ldxb", R6, R1, 0), I("and_imm", R6, imm=15), I("stxw", R10, R6, -4),
         I("ldxb", R5, R1, 2), I("and_imm", R5, imm=1),
         I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
         I("mul64_reg", R2, R5),
         I("mov_imm", R3, imm=0), I("mov64_reg", R3, R1), I("add64_imm", R3, imm=16),
         LdDw(R1, MapRef(0)), I("mov_imm", R4, imm=0),
         I("call", imm=1), I("mov_imm", R9, imm=0), I("mov64_reg", R9, R0),
         LdDw(R1, MapRef(0)),
         I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
         I("call", imm=2), I("lsh64_imm", R0, imm=8), I("or64_reg", R0, R9), I("exit")]
    return layout.assemble(n)


def prog_fault_after_write():
    """key = pkt[0] & 15, value = pkt[8..16): an update (always in range, flags 0), then
    r0 = 7 / (pkt[1] & 1): a packet with an even pkt[1] faults DIV_ZERO after its write."""
    from generic_ebpf_amd import layout
    I, LdDw, MapRef, Branch = _nodes()
    n = [I("ldxb", R6, R1, 0), I("ldxb", R7, R1, 1), I("ldxdw", R8, R1, 8),
         I("and_imm", R6, imm=15), I("and_imm", R7, imm=1),
         I("stxw", R10, R6, -4), I("stxdw", R10, R8, -16),
         LdDw(R1, MapRef(0)),
         I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
         I("mov_imm", R3, imm=0), I("mov64_reg", R3, R10), I("add64_imm", R3, imm=-16),
         I("mov_imm", R4, imm=0), I("call", imm=1),
         I("mov_imm", R0, imm=7), I("div64_reg", R0, R7), I("exit")]
    return layout.assemble(n)


def _expect_fault_after_write(pk, init):
    vals = np.frombuffer(init, dtype=np.uint64).copy()
    ret, faults = [], []
    for p in pk:
        if int(p[1]) & 1:
            vals[int(p[0]) & 15] = np.frombuffer(p[8:16].tobytes(), dtype=np.uint64)[0]
            ret.append(7)
            faults.append(0)
        else:
            ret.append(0)
            faults.append(2)
    return np.array(ret, dtype=np.uint64), np.array(faults, dtype=np.uint8), vals.tobytes()


def test_oracle_faulting_packet_leaves_no_write():
    """A packet that faults after its map_update_elem leaves no write behind (include/ebpf_gpu.h,
    "Map writes in a device batch")."""
    n = 3000
    pk = _packets(n, 13)
    init = _map_init(8)
    lay = prog_fault_after_write()
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, NKEYS, init)])
    ret, faults, _, _ = op.run(pk, n, 64, nthreads=4)
    want, wf, after = _expect_fault_after_write(pk, init)
    np.testing.assert_array_equal(ret, want)
    np.testing.assert_array_equal(faults, wf)
    assert op.map_bytes(0) == after


def _map_init(seed=5):
    return np.random.default_rng(seed).integers(0, 2**63, NKEYS, dtype=np.uint64).tobytes()


def _packets(n, seed):
    from generic_ebpf_amd import workloads
    return workloads.packets_random(n, 64, seed=seed)


def _expect_static(pk, init, second=False):
    """Hand computation of prog_static over packets pk (n x 64) on a map holding ``init``."""
    vals = np.frombuffer(init, dtype=np.uint64).copy()
    snap = vals.copy()
    ret = []
    for p in pk:
        key, flags = int(p[0]) & 31, int(p[1]) & 3
        value = int(np.frombuffer(p[8:16].tobytes(), dtype=np.uint64)[0])
        rc = 22 if flags == 3 else 17 if flags & 1 else (22 if key >= NKEYS else 0)
        if rc == 0:
            vals[key] = value
        if second:
            rc2 = 22 if key >= NKEYS else 0
            if rc2 == 0:
                vals[key] = (value + 1) & 0xffffffffffffffff
            rc |= rc2 << 8
        ret.append(1000 + rc if key >= NKEYS else int(snap[key]) ^ rc)
    return np.array(ret, dtype=np.uint64), vals.tobytes()


@pytest.mark.parametrize("second", [False, True])
def test_oracle_deferred_update_known_answers(second):
    """The oracle's batch mode against the hand computation: return codes, the snapshot seen by
    the lookup, and the map after the batch (last writer in packet order wins)."""
    n = 3000
    pk = _packets(n, 11)
    init = _map_init()
    lay = prog_static(second)
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, NKEYS, init)])
    ret, faults, _, _ = op.run(pk, n, 64, nthreads=4)
    want, after = _expect_static(pk, init, second)
    assert not faults.any()
    np.testing.assert_array_equal(ret, want)
    assert op.map_bytes(0) == after


def test_oracle_generic_pointers_and_delete():
    n = 2000
    pk = _packets(n, 12)
    init = _map_init(6)
    lay = prog_generic()
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, NKEYS, init)])
    ret, faults, _, _ = op.run(pk, n, 64, nthreads=4)
    assert not faults.any()
    vals = np.frombuffer(init, dtype=np.uint64).copy()
    for i, p in enumerate(pk):
        rc = 0 if p[2] & 1 else 22
        assert int(ret[i]) == (22 << 8) | rc
        if rc == 0:
            vals[int(p[0]) & 15] = np.frombuffer(p[16:24].tobytes(), dtype=np.uint64)[0]
    assert op.map_bytes(0) == vals.tobytes()


def prog_runtime_map():
    """The map of the update and of the delete is chosen at run time (pkt[1] & 3: map 0, map 1,
    NULL, or r10 — a pointer that is no map); key = pkt[0] & 15, value = pkt[8..16);
    r0 = delete rc << 8 | update rc.  (The reference's stepping needs a tree: every branch
    carries its own copy of the tail.)"""
    from generic_ebpf_amd import layout
    I, LdDw, MapRef, Branch = _nodes()

    def tail():
        # (the pointer goes through the stack: the translator no longer knows which map it is,
        # so the helpers run through the run-time compare chain)
        return [I("stxdw", R10, R1, -24), I("ldxdw", R1, R10, -24),
                I("mov_imm", R9, imm=0), I("mov64_reg", R9, R1),          # r9 = the map pointer
                I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
                I("mov_imm", R3, imm=0), I("mov64_reg", R3, R10), I("add64_imm", R3, imm=-16),
                I("mov_imm", R4, imm=0), I("call", imm=1),
                I("mov_imm", R1, imm=0), I("mov64_reg", R1, R9), I("mov_imm", R9, imm=0),
                I("mov64_reg", R9, R0),
                I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
                I("call", imm=2), I("lsh64_imm", R0, imm=8), I("or64_reg", R0, R9), I("exit")]

    n = [I("ldxb", R6, R1, 0), I("ldxdw", R8, R1, 8), I("and_imm", R6, imm=15),
         I("stxw", R10, R6, -4), I("stxdw", R10, R8, -16),
         I("ldxb", R7, R1, 1), I("and_imm", R7, imm=3),
         Branch(I("jeq_imm", R7, imm=0), [LdDw(R1, MapRef(0))] + tail()),
         Branch(I("jeq_imm", R7, imm=1), [LdDw(R1, MapRef(1))] + tail()),
         Branch(I("jeq_imm", R7, imm=2), [I("mov_imm", R1, imm=0)] + tail()),
         I("mov_imm", R1, imm=0), I("mov64_reg", R1, R10)] + tail()
    return layout.assemble(n)


def _expect_runtime_map(pk, inits):
    vals = [np.frombuffer(x, dtype=np.uint64).copy() for x in inits]
    ret, faults = [], []
    for p in pk:
        key, sel = int(p[0]) & 15, int(p[1]) & 3
        if sel == 3:
            ret.append(0)
            faults.append(10)       # BAD_MAP: the update dereferences r10 as a map
            continue
        if sel == 2:
            ret.append((22 << 8) | 22)
        else:
            vals[sel][key] = np.frombuffer(p[8:16].tobytes(), dtype=np.uint64)[0]
            ret.append(22 << 8)
        faults.append(0)
    return (np.array(ret, dtype=np.uint64), np.array(faults, dtype=np.uint8),
            [v.tobytes() for v in vals])


def test_oracle_runtime_map_known_answers():
    n = 3000
    pk = _packets(n, 15)
    inits = [_map_init(30), _map_init(31)]
    lay = prog_runtime_map()
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, NKEYS, inits[0]), (8, NKEYS, inits[1])])
    ret, faults, _, _ = op.run(pk, n, 64, nthreads=4)
    want, wf, after = _expect_runtime_map(pk, inits)
    np.testing.assert_array_equal(faults, wf)
    np.testing.assert_array_equal(ret, want)
    assert op.map_bytes(0) == after[0] and op.map_bytes(1) == after[1]


def test_translation_of_map_writes(native, env):
    """The translator accepts update / delete with an LDDW-known map (device info works, the
    compiled code builds), and with a map known only at run time (a compare chain on r1)."""
    from generic_ebpf_amd import isa
    for lay in (prog_static(), prog_static(True), prog_generic()):
        m = native.Map(env, NKEYS, 8)
        p = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [m.handle]))
        try:
            p.info()
            assert len(p.device_code(1)) > 0 and len(p.device_code(0)) > 0
        finally:
            p.destroy()
            m.destroy()
    e, O = isa.encode, isa.OPS
    p = native.Prog(env, e(O["call"], imm=1) + e(O["exit"]))   # r1 = the packet, not a map
    try:
        p.info()
        assert len(p.device_code(0)) > 0
    finally:
        p.destroy()
    lay = prog_runtime_map()
    maps = [native.Map(env, NKEYS, 8), native.Map(env, NKEYS, 8)]
    p = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    try:
        assert p.info().nmaps == 2
        assert len(p.device_code(1)) > 0 and len(p.device_code(0)) > 0
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


def _run_device(gpu, env, lay, maps_spec, pk, variant, resident):
    import torch
    n = len(pk)
    case = goldens.Case("w", lay.code, lay.relocs, maps_spec, pk.reshape(-1), n, 64, None)
    maps = make_maps(gpu, env, case)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    try:
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
        after = b"".join(maps[0].lookup(k)[1] for k in range(maps[0].max_entries))
        return ret, faults, after
    finally:
        gpu.set_variant(0)
        p.destroy()
        for m in maps:
            m.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("resident", [False, True])
@pytest.mark.parametrize("which", ["static", "static2", "generic"])
def test_device_map_writes_vs_oracle(gpu, env, variant, resident, which):
    n = (1 << 18) + 77
    pk = _packets(n, 21)
    init = _map_init(7)
    lay = {"static": prog_static, "static2": lambda: prog_static(True),
           "generic": prog_generic}[which]()
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, NKEYS, init)])
    want, wf, _, _ = op.run(pk, n, 64, nthreads=16)
    ret, faults, after = _run_device(gpu, env, lay, [(8, NKEYS, init)], pk, variant, resident)
    np.testing.assert_array_equal(faults, wf)
    np.testing.assert_array_equal(ret, want)
    assert after == op.map_bytes(0)


@pytest.mark.gpu
def test_device_map_writes_across_batches(gpu, env):
    """Batch 2 reads what batch 1 wrote (on the device, without a host round trip); a host
    update between batches wins over the device's earlier write."""
    import torch
    n = 1 << 16
    lay = prog_static()
    init = _map_init(8)
    pk1, pk2 = _packets(n, 31), _packets(n, 32)
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, NKEYS, init)])
    w1, _, _, _ = op.run(pk1, n, 64, nthreads=16)
    op.maps_arr[0].data  # (the oracle's map now holds batch 1's writes)
    mid = bytearray(op.map_bytes(0))
    mid[3 * 8:4 * 8] = (12345).to_bytes(8, "little")          # host write between the batches
    op2 = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, NKEYS, bytes(mid))])
    w2, _, _, _ = op2.run(pk2, n, 64, nthreads=16)
    case = goldens.Case("w", lay.code, lay.relocs, [(8, NKEYS, init)], pk1.reshape(-1), n, 64, None)
    maps = make_maps(gpu, env, case)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    try:
        dev = torch.device("cuda:0")
        st = torch.cuda.current_stream().cuda_stream
        d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
        for pk, want, host_write in ((pk1, w1, True), (pk2, w2, False)):
            d_pk = torch.from_numpy(np.ascontiguousarray(pk.reshape(-1))).to(dev)
            p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), stream=st)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(d_ret.cpu().numpy().view(np.uint64), want)
            if host_write:
                assert maps[0].update(3, (12345).to_bytes(8, "little")) == 0
        after = b"".join(maps[0].lookup(k)[1] for k in range(NKEYS))
        assert after == op2.map_bytes(0)
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("resident", [False, True])
def test_device_faulting_packet_leaves_no_write(gpu, env, variant, resident):
    n = (1 << 17) + 5
    pk = _packets(n, 14)
    init = _map_init(9)
    ret, faults, after = _run_device(gpu, env, prog_fault_after_write(), [(8, NKEYS, init)], pk,
                                     variant, resident)
    want, wf, want_after = _expect_fault_after_write(pk, init)
    np.testing.assert_array_equal(faults, wf)
    np.testing.assert_array_equal(ret, want)
    assert after == want_after


def _percpu_copies(gpu, m, ncpu):
    """lookup_from_user on a percpu array: every CPU's value of every key
    (ebpf_map_array.c:153-170) -> {cpu: bytes of the whole array as that CPU sees it}."""
    import ctypes
    L = gpu.lib()
    per = {c: bytearray() for c in range(ncpu)}
    for k in range(NKEYS):
        kk = ctypes.c_uint32(k)
        buf = ctypes.create_string_buffer(8 * ncpu)
        assert L.ebpf_map_lookup_elem_from_user(m.ptr, ctypes.byref(kk), buf) == 0
        for c in range(ncpu):
            per[c] += buf.raw[8 * c: 8 * c + 8]
    return {c: bytes(v) for c, v in per.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("resident", [False, True])
def test_device_percpu_array_writes(gpu, env, variant, resident):
    """Program-side map_update_elem on a percpu array lands in the copy of the CPU the batch is
    submitted from (ebpf_map_array.c:213-226: ma + ebpf_curcpu()).  Batches from two pinned CPUs:
    each CPU's copy holds exactly its own batch's writes (the others keep the initial values), the
    host's lookup_from_user sees them, and a third batch from the first CPU reads the first
    batch's writes — which a batch from the second CPU on the same device must not discard."""
    import os
    import torch
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < 2:
        pytest.skip("needs two CPUs")
    c1, c2 = cpus[0], cpus[-1]
    ncpu = os.sysconf("SC_NPROCESSORS_ONLN")
    saved = os.sched_getaffinity(0)
    n = (1 << 16) + 9
    lay = prog_static()
    init = _map_init(10)
    pks = [_packets(n, 41), _packets(n, 42), _packets(n, 43)]
    # the oracle: per CPU, a plain array map that only that CPU's batches touch
    state = {c1: init, c2: init}
    expect = []
    for pk, c in zip(pks, (c1, c2, c1)):
        op = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, NKEYS, state[c])])
        want, wf, _, _ = op.run(pk, n, 64, nthreads=16)
        state[c] = op.map_bytes(0)
        expect.append((want, wf, dict(state)))
    m = gpu.Map(env, NKEYS, 8, type=gpu.MAP_TYPE_PERCPU_ARRAY)
    for k in range(NKEYS):   # from user: every CPU's copy
        assert m.update(k, init[8 * k: 8 * k + 8]) == 0
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle]))
    dev = torch.device("cuda:0")
    try:
        gpu.set_variant(variant)
        for (pk, c), (want, wf, st) in zip(zip(pks, (c1, c2, c1)), expect):
            os.sched_setaffinity(0, {c})
            if resident:
                d_pk = torch.from_numpy(np.ascontiguousarray(pk.reshape(-1))).to(dev)
                d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
                d_flt = torch.zeros(n, dtype=torch.uint8, device=dev)
                p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), None,
                                d_flt.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                ret, faults = d_ret.cpu().numpy().view(np.uint64), d_flt.cpu().numpy()
            else:
                ret, faults, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), n, 64)
            np.testing.assert_array_equal(faults, wf)
            np.testing.assert_array_equal(ret, want)
        os.sched_setaffinity(0, saved)
        copies = _percpu_copies(gpu, m, ncpu)
        final = expect[-1][2]
        assert copies[c1] == final[c1]
        assert copies[c2] == final[c2]
        for c in range(ncpu):
            if c not in (c1, c2):
                assert copies[c] == init, c
    finally:
        os.sched_setaffinity(0, saved)
        gpu.set_variant(0)
        p.destroy()
        m.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("resident", [False, True])
def test_device_runtime_map_writes(gpu, env, variant, resident):
    """map_update_elem / map_delete_elem whose map is chosen at run time (ebpf_map.c:101-108,
    :130-136): two array maps, NULL (EINVAL) and a pointer that is no map (BAD_MAP), against the
    oracle and the hand computation; both maps' contents after the batch."""
    import torch
    n = (1 << 16) + 3
    pk = _packets(n, 16)
    inits = [_map_init(32), _map_init(33)]
    lay = prog_runtime_map()
    want, wf, after = _expect_runtime_map(pk, inits)
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, NKEYS, inits[0]), (8, NKEYS, inits[1])])
    ow, owf, _, _ = op.run(pk, n, 64, nthreads=16)
    np.testing.assert_array_equal(ow, want)
    np.testing.assert_array_equal(owf, wf)
    case = goldens.Case("w", lay.code, lay.relocs, [(8, NKEYS, inits[0]), (8, NKEYS, inits[1])],
                        pk.reshape(-1), n, 64, None)
    maps = make_maps(gpu, env, case)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    try:
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
        np.testing.assert_array_equal(faults, wf)
        np.testing.assert_array_equal(ret, want)
        for k in range(2):
            got = b"".join(maps[k].lookup(i)[1] for i in range(NKEYS))
            assert got == after[k], k
    finally:
        gpu.set_variant(0)
        p.destroy()
        for m in maps:
            m.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("ndev", [2, 3])
@pytest.mark.parametrize("which", ["static2", "runtime"])
def test_multi_device_writers_host_buffers(gpu, env, ndev, which):
    """A map-writing program sharded over several devices (here one GPU listed `ndev` times, so
    each shard has its own staging set and log): the shards' logs merge on the host in global
    packet order, so the results and the maps equal ONE batch over the whole input (the
    oracle)."""
    n = (1 << 18) + 7
    pk = _packets(n, 51)
    if which == "static2":
        lay, specs = prog_static(True), [(8, NKEYS, _map_init(52))]
    else:
        lay, specs = prog_runtime_map(), [(8, NKEYS, _map_init(53)), (8, NKEYS, _map_init(54))]
    op = pyoracle.OracleProgram(lay.code, lay.relocs, specs)
    want, wf, _, _ = op.run(pk, n, 64, nthreads=16)
    case = goldens.Case("w", lay.code, lay.relocs, specs, pk.reshape(-1), n, 64, None)
    maps = make_maps(gpu, env, case)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    try:
        ret, faults, st = p.run_batch_multi([0] * ndev, np.ascontiguousarray(pk.reshape(-1)), n, 64)
        np.testing.assert_array_equal(faults, wf)
        np.testing.assert_array_equal(ret, want)
        for k in range(len(maps)):
            assert b"".join(maps[k].lookup(i)[1] for i in range(NKEYS)) == op.map_bytes(k), k
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("same_stream", [False, True])
def test_multi_device_writers_device_resident(gpu, env, same_stream):
    """ebpf_prog_run_batch_multi_dev with a map-writing program: two shards (one GPU listed
    twice), histogram summed; the logs merge in shard order = one batch; a second call reads the
    first one's writes."""
    import torch
    n = (1 << 17) + 11
    half = n // 2
    lay, init = prog_static(), _map_init(55)
    pk1, pk2 = _packets(n, 56), _packets(n, 57)
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, NKEYS, init)])
    w1, _, _, _ = op.run(pk1, n, 64, nthreads=16)
    op2 = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, NKEYS, op.map_bytes(0))])
    w2, _, _, _ = op2.run(pk2, n, 64, nthreads=16)
    case = goldens.Case("w", lay.code, lay.relocs, [(8, NKEYS, init)], pk1.reshape(-1), n, 64, None)
    maps = make_maps(gpu, env, case)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    try:
        dev = torch.device("cuda:0")
        s0 = torch.cuda.Stream()
        s1 = s0 if same_stream else torch.cuda.Stream()
        d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
        hists = [torch.zeros(257, dtype=torch.int64, device=dev) for _ in range(2)]
        for pk, want in ((pk1, w1), (pk2, w2)):
            d_pk = torch.from_numpy(np.ascontiguousarray(pk.reshape(-1))).to(dev)
            torch.cuda.synchronize()
            p.run_batch_multi_dev([0, 0], [(d_pk.data_ptr(), half, 64, None),
                                           (d_pk.data_ptr() + half * 64, n - half, 64, None)],
                                  [d_ret.data_ptr(), d_ret.data_ptr() + half * 8],
                                  hists=[h.data_ptr() for h in hists],
                                  streams=[s0.cuda_stream, s1.cuda_stream], hist_overwrite=True)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(d_ret.cpu().numpy().view(np.uint64), want)
            hw = np.bincount(np.minimum(want, 255).astype(np.int64), minlength=257)
            for h in hists:
                np.testing.assert_array_equal(h.cpu().numpy(), hw)
        assert b"".join(maps[0].lookup(i)[1] for i in range(NKEYS)) == op2.map_bytes(0)
    finally:
        p.destroy()
        for m in maps:
            m.destroy()
