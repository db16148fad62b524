"""Order of map writes and map state (include/ebpf_gpu.h "Map writes in a device batch").

* Within a packet, the writes land in call order.  The device orders a packet's log records by
  the order its lane took the log slots (one call after the other), not by the state-tree entry
  that made them: the entries of a run-time-map compare chain, and merge points under standard
  semantics, are numbered after entries that a path reaches later.
* A map's device mirror is ordered across streams: an upload (after a host update) waits for
  launches still reading the old contents on other streams, and a launch waits for an upload
  made on another stream.
* Asynchronous jobs of a map-writing program run as if one after the other in submission order,
  each from its submitting thread's CPU (percpu maps).

The expected values come from the oracle (oracle/ebpf_oracle.c batch mode), which orders a
packet's writes by its own call sequence."""
import os

import numpy as np
import pytest

import pyoracle
import stdprogs

pytestmark = pytest.mark.gpu

R0, R1, R2, R3, R4, R5, R6, R7, R8, R9, R10 = range(11)
NKEYS = 16


def _nodes():
    from generic_ebpf_amd import isa, layout
    return isa.Insn, layout.LdDw, layout.MapRef, layout.Branch


def _packets(n, seed):
    from generic_ebpf_amd import workloads
    return workloads.packets_random(n, 64, seed=seed)


def prog_chain_then_const():
    """key = pkt[0] & 15 (4 B at r10 - 8), value = pkt[8..16) (r10 - 16).  pkt[1] odd: update
    through a map pointer reloaded from the stack (the translator cannot name the map: a run-time
    compare chain, whose entries come after the rest), then delete through the LDDW constant —
    the key ends absent; pkt[1] even: the same two calls the other way round — present."""
    from generic_ebpf_amd import layout
    I, LdDw, MapRef, Branch = _nodes()

    def upd_chain():
        return [LdDw(R1, MapRef(0)), I("stxdw", R10, R1, -24), I("ldxdw", R1, R10, -24),
                I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-8),
                I("mov_imm", R3, imm=0), I("mov64_reg", R3, R10), I("add64_imm", R3, imm=-16),
                I("mov_imm", R4, imm=0), I("call", imm=1)]

    def del_const():
        return [LdDw(R1, MapRef(0)),
                I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-8),
                I("call", imm=2)]

    n = [I("ldxb", R6, R1, 0), I("and_imm", R6, imm=NKEYS - 1), I("stxw", R10, R6, -8),
         I("ldxdw", R7, R1, 8), I("stxdw", R10, R7, -16),
         I("ldxb", R8, R1, 1), I("and_imm", R8, imm=1),
         Branch(I("jeq_imm", R8, imm=0), del_const() + upd_chain() + [I("mov_imm", R0, imm=2),
                                                                      I("exit")])]
    n += upd_chain() + del_const() + [I("mov_imm", R0, imm=1), I("exit")]
    return layout.assemble(n)


def prog_std_merge():
    """Standard semantics, array map: key = pkt[0] & 15; pkt[1] odd: update(key, pkt[8..16)) at
    L, then both sides meet at M: update(key, pkt[16..24)).  The translator reaches M through the
    fall-through side first, so M's entry is numbered before L's; on the L path M's write is the
    later one and must win."""
    I = stdprogs.I

    def update(voff):
        return [("lddw_map", 1, 0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4),
                I("mov64_reg", 3, 10), I("add64_imm", 3, imm=voff), I("mov64_imm", 4, imm=0),
                I("call", imm=1)]

    items = [I("ldxb", 6, 1, 0), I("and_imm", 6, imm=NKEYS - 1), I("stxw", 10, 6, -4),
             I("ldxdw", 7, 1, 8), I("stxdw", 10, 7, -16),
             I("ldxdw", 9, 1, 16), I("stxdw", 10, 9, -24),
             I("ldxb", 8, 1, 1),
             I("jset_imm", 8, off="L", imm=1),
             I("ja", off="M"),
             ("label", "L")] + update(-16) + [("label", "M")] + update(-24) + [I("exit")]
    return stdprogs.asm(items)


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


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_chain_update_then_const_delete(gpu, env, variant):
    lay = prog_chain_then_const()
    g = np.random.default_rng(5)
    items = [(int(k).to_bytes(4, "little"), g.bytes(8)) for k in range(0, NKEYS, 2)]
    spec = pyoracle.HashSpec(4, 8, items=items, capacity=2 * NKEYS)
    n = (1 << 15) + 3
    pk = _packets(n, 51)
    op = pyoracle.OracleProgram(lay.code, lay.relocs, [spec])
    want, wf, _, _ = op.run(pk, n, 64, nthreads=16)
    hm = gpu.HashMap(env, 4, 8, 2 * NKEYS)
    for k, v in items:
        assert hm.update(k, v) == 0
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [hm.handle]))
    try:
        gpu.set_variant(variant)
        ret, faults, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), n, 64)
        np.testing.assert_array_equal(faults, wf)
        np.testing.assert_array_equal(ret, want)
        assert _walk(gpu, hm) == op.hash_models[0].items()
        # both orders occur, and the table ends with both kinds of key
        odd = (pk[:, 1] & 1).astype(bool)
        assert odd.any() and (~odd).any()
    finally:
        gpu.set_variant(0)
        p.destroy()
        hm.destroy()


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("resident", [False, True])
def test_std_merge_two_writes_one_key(gpu, env, variant, resident):
    import torch
    code, rel = prog_std_merge()
    init = np.random.default_rng(6).integers(0, 2**63, NKEYS, dtype=np.uint64).tobytes()
    n = (1 << 16) + 11
    pk = _packets(n, 52)
    op = pyoracle.OracleProgram(code, rel, [(8, NKEYS, init)], semantics=1)
    want, wf, _, _ = op.run(pk, n, 64, nthreads=16)
    m = gpu.Map(env, NKEYS, 8)
    m.fill(init)
    p = gpu.Prog(env, gpu.patch_relocs(code, rel, [m.handle]))
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
            ret, faults = d_ret.cpu().numpy().view(np.uint64), d_flt.cpu().numpy()
        else:
            ret, faults, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), n, 64)
        np.testing.assert_array_equal(faults, wf)
        np.testing.assert_array_equal(ret, want)
        after = b"".join(m.lookup(k)[1] for k in range(NKEYS))
        assert after == op.map_bytes(0)
        # the last packet of every key decides it; keys whose last packet took L hold
        # pkt[16..24) (M's write), never pkt[8..16)
        last = {}
        for i, row in enumerate(pk):
            last[int(row[0]) & (NKEYS - 1)] = i
        for k, i in last.items():
            assert after[8 * k: 8 * k + 8] == pk[i, 16:24].tobytes()
    finally:
        gpu.set_variant(0)
        p.destroy()
        m.destroy()


# ---------------------------------------------------------------- mirror order across streams


def _lookup_prog():
    """r0 = map[pkt[0] & 15] (8 B), through an array-map lookup."""
    from generic_ebpf_amd import layout
    I, LdDw, MapRef, Branch = _nodes()
    return layout.assemble([
        I("ldxb", R6, R1, 0), I("and_imm", R6, imm=NKEYS - 1), I("stxw", R10, R6, -4),
        LdDw(R1, MapRef(0)),
        I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
        I("call", imm=0),
        Branch(I("jeq_imm", R0, imm=0), [I("mov_imm", R0, imm=0), I("exit")]),
        I("ldxdw", R0, R0, 0), I("exit")])


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_host_update_between_launches_on_two_streams(gpu, env, variant):
    """A long launch on stream A reads the map; the host updates it; a launch on stream B (whose
    mirror upload must wait for A) reads the new contents, A the old.  Then the other way round:
    the upload happens on A's next launch, and B's launch right after must wait for it."""
    import torch
    lay = _lookup_prog()
    v1 = np.arange(NKEYS, dtype=np.uint64) + 1000
    v2 = np.arange(NKEYS, dtype=np.uint64) + 2000
    v3 = np.arange(NKEYS, dtype=np.uint64) + 3000
    n = (1 << 22) if variant != 1 else (1 << 20)
    pk = _packets(n, 53)
    key = (pk[:, 0] & (NKEYS - 1)).astype(np.int64)
    m = gpu.Map(env, NKEYS, 8)
    m.fill(v1.tobytes())
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle]))
    dev = torch.device("cuda:0")
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    d_pk = torch.from_numpy(np.ascontiguousarray(pk.reshape(-1))).to(dev)
    rets = [torch.zeros(n, dtype=torch.int64, device=dev) for _ in range(4)]
    torch.cuda.synchronize()
    try:
        gpu.set_variant(variant)

        def run(r, s):
            p.run_batch_dev(0, d_pk.data_ptr(), n, 64, r.data_ptr(), None, None, None, s.cuda_stream)

        run(rets[0], sa)                     # reads v1 (uploaded on A)
        m.fill(v2.tobytes())                 # host update while A may still run
        run(rets[1], sb)                     # uploads v2 on B: after A's launch
        m.fill(v3.tobytes())
        run(rets[2], sa)                     # uploads v3 on A: after B's launch
        run(rets[3], sb)                     # no upload: must wait for A's
        torch.cuda.synchronize()
        for r, vals in zip(rets, (v1, v2, v3, v3)):
            np.testing.assert_array_equal(r.cpu().numpy().view(np.uint64), vals[key])
    finally:
        gpu.set_variant(0)
        p.destroy()
        m.destroy()


# ---------------------------------------------------------------- asynchronous writing jobs


def _writer_prog():
    """key = pkt[0] & 15, value = pkt[8..16): update(key, value); r0 = the batch-start value of
    the key (a lookup before the update), so each job's results show which writes it saw."""
    from generic_ebpf_amd import layout
    I, LdDw, MapRef, Branch = _nodes()
    return layout.assemble([
        I("ldxb", R6, R1, 0), I("and_imm", R6, imm=NKEYS - 1), I("stxw", R10, R6, -4),
        I("ldxdw", R7, R1, 8), I("stxdw", R10, R7, -16),
        LdDw(R1, MapRef(0)),
        I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
        I("call", imm=0),
        I("ldxdw", R9, R0, 0),
        LdDw(R1, MapRef(0)),
        I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
        I("mov_imm", R3, imm=0), I("mov64_reg", R3, R10), I("add64_imm", R3, imm=-16),
        I("mov_imm", R4, imm=0), I("call", imm=1),
        I("mov_imm", R0, imm=0), I("mov64_reg", R0, R9), I("exit")])


@pytest.mark.parametrize("variant", [0, 2])
def test_async_writing_jobs_in_submission_order(gpu, env, variant):
    """8 jobs of a map-writing program in flight at once: each job's results and the final map
    equal the oracle running the 8 batches one after the other in submission order."""
    lay = _writer_prog()
    init = np.random.default_rng(7).integers(0, 2**63, NKEYS, dtype=np.uint64).tobytes()
    sizes = [(1 << 18) + 13 * k for k in range(8)]
    pks = [_packets(s, 60 + k) for k, s in enumerate(sizes)]
    state, expect = init, []
    for pk, s in zip(pks, sizes):
        op = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, NKEYS, state)])
        want, wf, _, _ = op.run(pk, s, 64, nthreads=16)
        state = op.map_bytes(0)
        expect.append(want)
    m = gpu.Map(env, NKEYS, 8)
    m.fill(init)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle]))
    try:
        gpu.set_variant(variant)
        data = [np.ascontiguousarray(pk.reshape(-1)) for pk in pks]
        jobs = [p.run_batch_async(d, s, 64) for d, s in zip(data, sizes)]
        for j, want in zip(jobs, expect):
            ret, faults, _ = j.wait()
            assert not faults.any()
            np.testing.assert_array_equal(ret, want)
        after = b"".join(m.lookup(k)[1] for k in range(NKEYS))
        assert after == state
    finally:
        gpu.set_variant(0)
        p.destroy()
        m.destroy()


def test_async_percpu_writes_land_in_the_submitting_cpus_copy(gpu, env):
    """Jobs submitted from a thread pinned to CPU c1, then to CPU c2 (the pool's workers were
    started by the first): each job's writes land in its submitter's copy of a percpu array."""
    import ctypes
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < 2:
        pytest.skip("needs two CPUs")
    c1, c2 = cpus[0], cpus[-1]
    ncpu = os.sysconf("SC_NPROCESSORS_ONLN")
    saved = os.sched_getaffinity(0)
    lay = _writer_prog()
    init = np.random.default_rng(8).integers(0, 2**63, NKEYS, dtype=np.uint64).tobytes()
    n = (1 << 16) + 5
    pks = [_packets(n, 70), _packets(n, 71)]
    state = {c1: init, c2: init}
    for pk, c in zip(pks, (c1, c2)):
        op = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, NKEYS, state[c])])
        op.run(pk, n, 64, nthreads=16)
        state[c] = op.map_bytes(0)
    m = gpu.Map(env, NKEYS, 8, type=gpu.MAP_TYPE_PERCPU_ARRAY)
    for k in range(NKEYS):
        assert m.update(k, init[8 * k: 8 * k + 8]) == 0
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle]))
    try:
        for pk, c in zip(pks, (c1, c2)):
            os.sched_setaffinity(0, {c})
            j = p.run_batch_async(np.ascontiguousarray(pk.reshape(-1)), n, 64)
            j.wait()
        os.sched_setaffinity(0, saved)
        L = gpu.lib()
        for c in (c1, c2):
            got = bytearray()
            for k in range(NKEYS):
                kk = ctypes.c_uint32(k)
                buf = ctypes.create_string_buffer(8 * ncpu)
                assert L.ebpf_map_lookup_elem_from_user(m.ptr, ctypes.byref(kk), buf) == 0
                got += buf.raw[8 * c: 8 * c + 8]
            assert bytes(got) == state[c], c
    finally:
        os.sched_setaffinity(0, saved)
        p.destroy()
        m.destroy()
