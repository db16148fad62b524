"""Parity of the device interpreters with the genuine reference (golden vectors) and with the
oracle (fresh random programs, full-size workloads, faults).  Every test calls the engine
through the C-ABI (lib/libebpf.so): host-buffer batches (ebpf_prog_run_batch) and
device-resident batches (ebpf_prog_run_batch_dev on torch-allocated memory)."""
import numpy as np
import pytest

import goldens
from helpers import device_run, make_maps, oracle_run

pytestmark = pytest.mark.gpu

CASES = [c for f in goldens.all_golden_files() for c in goldens.load(f)]
VARIANTS = [0, 1, 2]  # 0 = compiled (default), 1 = portable HIP baseline, 2 = asm interpreter


@pytest.mark.parametrize("variant", VARIANTS)
def test_goldens_on_device(gpu, env, variant):
    bad = []
    for c in CASES:
        ret, faults, after = device_run(gpu, env, c, variant)
        if not (np.array_equal(ret, c.expect_r0) and not faults.any()
                and np.array_equal(after, c.expect_data)):
            bad.append((c.name, int(np.count_nonzero(ret != c.expect_r0)),
                        int(np.count_nonzero(faults))))
    assert not bad, bad[:10]


@pytest.mark.parametrize("variant", VARIANTS)
def test_random_programs_vs_oracle(gpu, env, variant):
    from generic_ebpf_amd import randprog, workloads
    g = np.random.default_rng(77)
    bad = []
    for k in range(120):
        vs = int(g.choice([8, 16]))
        me = int(g.choice([16, 256]))
        lay = randprog.random_program(50000 + k, length=int(g.integers(10, 80)), nmaps=2,
                                      map_value_size=vs)
        maps = [(vs, me, g.integers(0, 256, vs * me, dtype=np.uint8).tobytes()) for _ in range(2)]
        n = 2048
        c = goldens.Case("r%d" % k, lay.code, lay.relocs, maps,
                         workloads.packets_random(n, 64, seed=k), n, 64, None)
        want, wf, wdata, _ = oracle_run(c)
        got, gf, gdata = device_run(gpu, env, c, variant)
        if not (np.array_equal(want, got) and np.array_equal(wf, gf)
                and np.array_equal(wdata, gdata)):
            bad.append(k)
    assert not bad, bad


FAULT_PROGS = None


def _fault_programs():
    from generic_ebpf_amd import isa, layout
    O, e, I = isa.OPS, isa.encode, isa.Insn
    return {
        "div0_imm": e(O["mov_imm"], 0, imm=1) + e(O["div_imm"], 0, imm=0),
        "div0_reg": layout.assemble([I("mov_imm", 0, imm=5), I("ldxb", 2, 1, 0),
                                     I("and_imm", 2, imm=1), I("mod64_reg", 0, 2),
                                     I("exit")]).code,
        "bad_opcode": e(0x06) + e(O["exit"]),
        "oob_load": layout.assemble([I("ldxb", 2, 1, 0), I("and_imm", 2, imm=3),
                                     I("add64_imm", 2, imm=61), I("mov_imm", 3, imm=0),
                                     I("mov64_reg", 3, 1), I("add64_reg", 3, 2),
                                     I("ldxw", 0, 3, 0), I("exit")]).code,
        "slot": e(O["mov_imm"], 0, imm=1) + e(O["mov_imm"], 0, imm=2),
        "helper_unset": e(O["call"], imm=9) + e(O["exit"]),
        "helper_unsupported": e(O["call"], imm=3) + e(O["exit"]),
        "bad_reg": e(O["mov_imm"], 11, imm=1) + e(O["exit"]),
        "loop": e(O["ja"], off=-1) + e(O["exit"]),
        "bad_map": layout.assemble([layout.LdDw(1, 0x1234), I("mov_imm", 2, imm=8),
                                    I("call", imm=0), I("exit")]).code,
        "stack_oob": layout.assemble([I("stb", 10, 0, -513, 1), I("exit")]).code,
        # the only reachable spin under reference stepping: a jump of -1 taken at state (0, 1)
        "cond_loop": e(O["jeq_imm"], 2, 0, -1, 0) + e(O["exit"]) * 4,
    }


@pytest.mark.parametrize("variant", VARIANTS)
def test_fault_codes_match_oracle(gpu, env, variant):
    from generic_ebpf_amd import workloads
    bad = {}
    for name, code in _fault_programs().items():
        n = 256
        c = goldens.Case(name, code, [], [], workloads.packets_random(n, 64, seed=9), n, 64, None)
        want, wf, _, _ = oracle_run(c)
        got, gf, _ = device_run(gpu, env, c, variant)
        if not (np.array_equal(want, got) and np.array_equal(wf, gf)):
            bad[name] = (np.unique(wf).tolist(), np.unique(gf).tolist())
        assert wf.any(), name  # every program here faults on some packet
    assert not bad, bad


def _tiled_case(name, base, tiles):
    data = np.tile(base.data, tiles)
    return goldens.Case(name, base.code, base.relocs, base.maps, data, base.count * tiles,
                        base.stride, None)


@pytest.mark.parametrize("variant", [0, 2])
@pytest.mark.parametrize("cfg,distinct,tiles", [("c2", 1 << 20, 1), ("c3", 1 << 20, 16),
                                                 ("c4", 1 << 20, 64)])
def test_full_size_workloads(gpu, env, cfg, distinct, tiles, variant):
    """BASELINE.json sizes (C2 1M, C3 16M, C4 64M packets): the device result for packet i must
    equal the oracle's for the distinct packet it tiles (size-independent property)."""
    from generic_ebpf_amd import workloads
    lay = workloads.CONFIGS[cfg]["prog"]()
    pk = (workloads.packets_random if cfg == "c2" else workloads.packets_l2l3)(distinct, 64)
    maps = []
    if cfg == "c4":
        vals = workloads.c4_map_values()
        maps = [(8, 256, vals.tobytes())]
    base = goldens.Case(cfg, lay.code, lay.relocs, maps, pk, distinct, 64, None)
    want, wf, _, _ = oracle_run(base, nthreads=8)
    assert not wf.any()
    full = _tiled_case(cfg, base, tiles)
    got, gf, _ = device_run(gpu, env, full, variant)
    assert not gf.any()
    np.testing.assert_array_equal(got.reshape(tiles, distinct), np.broadcast_to(want, (tiles, distinct)))


@pytest.mark.parametrize("variant", [0, 2])
def test_c5_imix_vs_oracle(gpu, env, variant):
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c5()
    n = 1 << 18
    data, offs, _ = workloads.packets_imix(n)
    c = goldens.Case("c5", lay.code, [], [], data, n, 0, offs)
    want, wf, _, _ = oracle_run(c, nthreads=8)
    got, gf, _ = device_run(gpu, env, c, variant)
    np.testing.assert_array_equal(wf, gf)
    np.testing.assert_array_equal(want, got)


@pytest.mark.parametrize("variant,runmask", [(0, True), (0, False), (2, True)])
def test_c5_truncated_packets_vs_oracle(gpu, env, variant, runmask, monkeypatch):
    """C5 on IMIX packets whose lengths are cut at random and stored unpadded (CSR packets at
    any byte offset): lanes of one group now end inside a leaf's straight run, so the compiled
    code's run mask (asm_cc.cpp: one extent compare per run) misses them and the per-load path
    must fault those past their end at the right load and load directly for the others.
    EBPF_CC_NORUNMASK=1 compiles the per-load compares instead; the assembly interpreter
    (variant 2) runs the same packets through its general handlers.  All must equal the oracle."""
    from generic_ebpf_amd import native, workloads
    if not runmask:
        monkeypatch.setenv("EBPF_CC_NORUNMASK", "1")
    lay = workloads.prog_c5()
    n = 1 << 16
    data, offs, sizes = workloads.packets_imix(n, seed=21)
    g = np.random.default_rng(22)
    cut = g.random(n) < 0.3
    lens = sizes.astype(np.int64)
    lens[cut] = g.integers(18, lens[cut] + 1)
    # the kept bytes of every packet, back to back (CSR offsets, no padding)
    starts = offs[:-1].astype(np.int64)
    parts = [data[s:s + L] for s, L in zip(starts, lens)]
    new_offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=new_offs[1:])
    new_data = np.concatenate(parts)
    c = goldens.Case("c5cut", lay.code, [], [], new_data, n, 0, new_offs)
    want, wf, _, _ = oracle_run(c, nthreads=8)
    assert wf.any() and (~wf.astype(bool)).any()
    got, gf, _ = device_run(gpu, env, c, variant)
    np.testing.assert_array_equal(wf, gf)
    np.testing.assert_array_equal(want, got)


def test_device_resident_api_and_histogram(gpu, env):
    """ebpf_prog_run_batch_dev on torch device memory, verdict histogram included."""
    import torch
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c4()
    n = 1 << 20
    pk = workloads.packets_l2l3(n, 64)
    vals = workloads.c4_map_values()
    case = goldens.Case("c4", lay.code, lay.relocs, [(8, 256, vals.tobytes())], pk, n, 64, None)
    want, _, _, _ = oracle_run(case, nthreads=8)
    maps = make_maps(gpu, env, case)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    try:
        dev = torch.device("cuda:0")
        d_pk = torch.from_numpy(pk.reshape(-1)).to(dev)
        d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
        d_flt = torch.zeros(n, dtype=torch.uint8, device=dev)
        d_hist = torch.zeros(257, dtype=torch.int64, device=dev)
        st = torch.cuda.current_stream()
        p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), None, d_flt.data_ptr(),
                        d_hist.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        got = d_ret.cpu().numpy().view(np.uint64)
        np.testing.assert_array_equal(got, want)
        h = np.zeros(257, dtype=np.int64)
        np.add.at(h, np.minimum(want, 255).astype(np.int64), 1)
        np.testing.assert_array_equal(d_hist.cpu().numpy(), h)
        assert int(d_flt.sum()) == 0
        # a host-side map update must reach the device mirror before the next launch
        m = maps[0]
        m.fill(np.zeros(256, dtype=np.uint64).tobytes())
        case2 = goldens.Case("c4z", lay.code, lay.relocs, [(8, 256, bytes(2048))], pk, n, 64, None)
        want2, _, _, _ = oracle_run(case2, nthreads=8)
        p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), stream=st.cuda_stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_ret.cpu().numpy().view(np.uint64), want2)
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


def test_deep_async_queue_with_histogram(gpu, env):
    """More queued launches than the 64 histogram row buffers, with no synchronisation in
    between (a bench loop of many steps): every launch succeeds and the accumulated histogram
    counts every packet of every launch."""
    import torch
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c4()
    n = 1 << 20
    pk = workloads.packets_l2l3(n, 64)
    vals = workloads.c4_map_values()
    case = goldens.Case("c4", lay.code, lay.relocs, [(8, 256, vals.tobytes())], pk, n, 64, None)
    want, _, _, _ = oracle_run(case, nthreads=8)
    maps = make_maps(gpu, env, case)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    try:
        dev = torch.device("cuda:0")
        d_pk = torch.from_numpy(pk.reshape(-1)).to(dev)
        d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
        d_hist = torch.zeros(257, dtype=torch.int64, device=dev)
        st = torch.cuda.current_stream()
        launches = 200
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(launches)]
        for e0, e1 in evs:  # created at their first record
            e0.record(st)
            e1.record(st)
        for e0, e1 in evs:  # every launch timed by the library's kernel events
            gpu.time_next_launch(e0.cuda_event, e1.cuda_event)
            p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), None, None,
                            d_hist.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        ms = [e0.elapsed_time(e1) for e0, e1 in evs]
        assert all(0.0 < m < 100.0 for m in ms), ms[:4]
        np.testing.assert_array_equal(d_ret.cpu().numpy().view(np.uint64), want)
        h = np.zeros(257, dtype=np.int64)
        np.add.at(h, np.minimum(want, 255).astype(np.int64), launches)
        np.testing.assert_array_equal(d_hist.cpu().numpy(), h)
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_histogram_overwrite_with_faults(gpu, env, variant):
    """EBPF_BATCH_HIST_OVERWRITE: the histogram (faulted bin 256 included) is set to each
    launch's counts over a garbage-filled buffer, launch after launch (the fault count's scratch
    is left zero for the next launch), in add mode the counts accumulate, and an empty batch
    zeroes it."""
    import torch
    from generic_ebpf_amd import isa, layout, workloads
    I = isa.Insn
    # r0 = pkt[0]; faults (division by zero) where pkt[1] & 3 == 0
    code = layout.assemble([I("ldxb", 0, 1, 0), I("ldxb", 2, 1, 1), I("and_imm", 2, imm=3),
                            I("div64_reg", 0, 2), I("exit")]).code
    n = 64 * 4096 + 77
    pk = workloads.packets_random(n, 64, seed=31)
    c = goldens.Case("ovw", code, [], [], pk.reshape(-1), n, 64, None)
    want, wf, _, _ = oracle_run(c, nthreads=8)
    h = np.zeros(257, dtype=np.int64)
    ok = wf == 0
    np.add.at(h, np.minimum(want[ok], 255).astype(np.int64), 1)
    h[256] = int((~ok).sum())
    assert h[256] > 0
    gpu.set_variant(variant)
    p = gpu.Prog(env, code)
    try:
        dev = torch.device("cuda:0")
        d_pk = torch.from_numpy(pk.reshape(-1)).to(dev)
        d_ret = torch.zeros(n, dtype=torch.int64, device=dev)
        d_hist = torch.full((257,), 12345, dtype=torch.int64, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(3):
            p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), None, None,
                            d_hist.data_ptr(), st, hist_overwrite=True)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(d_hist.cpu().numpy(), h)
        for _ in range(2):  # add mode on top
            p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), None, None,
                            d_hist.data_ptr(), st)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_hist.cpu().numpy(), 3 * h)
        p.run_batch_dev(0, d_pk.data_ptr(), 0, 64, d_ret.data_ptr(), None, None,
                        d_hist.data_ptr(), st, hist_overwrite=True)
        torch.cuda.synchronize()
        assert not d_hist.cpu().numpy().any()
    finally:
        gpu.set_variant(0)
        p.destroy()


@pytest.mark.parametrize("variant", [0, 2])
def test_empty_and_ragged_batches(gpu, env, variant):
    """Empty, sub-group and ragged batches; the last size gives every wave of the persistent
    grid several groups and ends in a partial group."""
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c3()
    for n in (0, 1, 63, 65, 255, 257, 1000, 64 * 8192 * 2 + 37):
        pk = workloads.packets_l2l3(max(n, 1), 64)[:n]
        c = goldens.Case("c3", lay.code, [], [], pk.reshape(-1) if n else np.zeros(1, np.uint8),
                         n, 64, None)
        got, gf, _ = device_run(gpu, env, c, variant)
        if n:
            want, wf, _, _ = oracle_run(c, nthreads=8)
            np.testing.assert_array_equal(want, got)
        else:
            assert got.size == 0


@pytest.mark.parametrize("superblock", [1, 2, 4, 8])
def test_superblock_sizes(gpu, env, superblock, monkeypatch):
    """Staged kernels walk superblocks of K' groups whose results go out as one burst; the host
    picks K' per launch (small batches: shorter superblocks).  Every K' on ragged batches that
    end inside a superblock and inside a group, with the histogram."""
    from generic_ebpf_amd import workloads
    monkeypatch.setenv("EBPF_SUPERBLOCK", str(superblock))
    lay = workloads.prog_c3()
    for n in (1, 64 * 5 + 3, 64 * 6144 * superblock + 64 * 3 + 17):
        pk = workloads.packets_l2l3(n, 64)
        c = goldens.Case("c3", lay.code, [], [], pk.reshape(-1), n, 64, None)
        got, gf, _ = device_run(gpu, env, c, 0)
        want, wf, _, _ = oracle_run(c, nthreads=8)
        np.testing.assert_array_equal(want, got)
        np.testing.assert_array_equal(wf, gf)


@pytest.mark.parametrize("wphase", ["6,20", "20,1", "4,15", "6,20,16", "20,1,16", "4,15,16"])
@pytest.mark.parametrize("superblock", [2, 4, 8])
def test_write_phasing(gpu, env, superblock, wphase, monkeypatch):
    """Write phasing (gen_interp.py store_phased, dp_launch.wphase) forced on every staged launch:
    a wave writes its unwritten result slots when the clock is in the window, when the next
    group's slot is taken, and at the end.  "6,20": windows every 640 ns (both kinds of writes
    mixed); "20,1": a window once per 10 ms (nearly every write is a full-slot one, so the slots
    span two superblocks); "4,15": almost always in the window (a write after every group);
    ",16": the wide kernel's 16 slots (superblocks alternating between two halves, so the
    unwritten slots span three superblocks).
    Ragged batches that end inside a superblock and inside a group, faults included, against
    the oracle, the fault codes and the histogram."""
    import torch
    from generic_ebpf_amd import isa, layout, workloads
    monkeypatch.setenv("EBPF_SUPERBLOCK", str(superblock))
    monkeypatch.setenv("EBPF_WPHASE", wphase)
    lay = workloads.prog_c3()
    for n in (1, 64 * 5 + 3, 64 * 4096 * superblock * 3 + 64 * 3 + 17):
        pk = workloads.packets_l2l3(n, 64)
        c = goldens.Case("c3", lay.code, [], [], pk.reshape(-1), n, 64, None)
        got, gf, _ = device_run(gpu, env, c, 0)
        want, wf, _, _ = oracle_run(c, nthreads=8)
        np.testing.assert_array_equal(want, got)
        np.testing.assert_array_equal(wf, gf)
    # faults and the histogram (r0 = pkt[0] / (pkt[1] & 3))
    I = isa.Insn
    code = layout.assemble([I("ldxb", 0, 1, 0), I("ldxb", 2, 1, 1), I("and_imm", 2, imm=3),
                            I("div64_reg", 0, 2), I("exit")]).code
    n = 64 * 4096 * superblock * 2 + 77
    pk = workloads.packets_random(n, 64, seed=41)
    c = goldens.Case("wph", code, [], [], pk.reshape(-1), n, 64, None)
    want, wf, _, _ = oracle_run(c, nthreads=8)
    h = np.zeros(257, dtype=np.int64)
    ok = wf == 0
    np.add.at(h, np.minimum(want[ok], 255).astype(np.int64), 1)
    h[256] = int((~ok).sum())
    p = gpu.Prog(env, code)
    try:
        dev = torch.device("cuda:0")
        d_pk = torch.from_numpy(pk.reshape(-1)).to(dev)
        d_ret = torch.full((n,), -1, dtype=torch.int64, device=dev)
        d_flt = torch.zeros(n, dtype=torch.uint8, device=dev)
        d_hist = torch.zeros(257, dtype=torch.int64, device=dev)
        p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), None, d_flt.data_ptr(),
                        d_hist.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = d_ret.cpu().numpy().view(np.uint64)
        np.testing.assert_array_equal(got[ok], want[ok])
        np.testing.assert_array_equal(d_flt.cpu().numpy(), wf)
        np.testing.assert_array_equal(d_hist.cpu().numpy(), h)
    finally:
        p.destroy()


@pytest.mark.parametrize("variant", VARIANTS)
def test_general_kernels_header_staging(gpu, env, variant):
    """General kernels stage the first 64 bytes of each packet for constant-offset loads: ragged
    packets of 1..140 bytes (CSR offsets) and a 40-byte stride, so some lanes are unstaged
    (shorter than 64 B) and some loads run past the packet (MEM faults).  C3 and random
    programs against the oracle."""
    from generic_ebpf_amd import randprog, workloads
    g = np.random.default_rng(31)
    progs = [(workloads.prog_c3(), [])]
    for k in range(30):
        vs = 8
        lay = randprog.random_program(70000 + k, length=int(g.integers(10, 60)), nmaps=1,
                                      map_value_size=vs)
        progs.append((lay, [(vs, 16, g.integers(0, 256, vs * 16, dtype=np.uint8).tobytes())]))
    n = 3000
    lens = g.integers(1, 141, n)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    base = workloads.packets_l2l3(n, 160)
    data = np.concatenate([base[i, :lens[i]] for i in range(n)])
    bad = []
    for i, (lay, maps) in enumerate(progs):
        for stride, o in ((0, offs), (40, None)):
            d = data if o is not None else base[:, :40].reshape(-1).copy()
            c = goldens.Case("gs%d" % i, lay.code, lay.relocs, maps, d, n, stride, o)
            want, wf, wd, _ = oracle_run(c)
            got, gf, gd = device_run(gpu, env, c, variant)
            if not (np.array_equal(want, got) and np.array_equal(wf, gf) and np.array_equal(wd, gd)):
                bad.append((i, stride, int(np.count_nonzero(want != got)), int(np.count_nonzero(wf != gf))))
    assert not bad, bad


@pytest.mark.parametrize("cfg", ["c4", "c3"])
def test_one_launch_full_size_overwrite(gpu, env, cfg):
    """The launch bench.py times: ONE device-resident ebpf_prog_run_batch_dev over the full
    BASELINE batch (C4: 64M x 64 B = 4 GiB; C3: 16M) with EBPF_BATCH_HIST_OVERWRITE on a
    garbage-filled histogram.  Every packet's result must equal the oracle's for the distinct
    packet it tiles (4M distinct packets, the bench's tiling), and the histogram the tiled
    oracle histogram."""
    import torch
    from generic_ebpf_amd import workloads
    D = 1 << 22
    n = {"c4": 1 << 26, "c3": 1 << 24}[cfg]
    lay = workloads.CONFIGS[cfg]["prog"]()
    pk = workloads.packets_l2l3(D, 64)
    maps_spec = [(8, 256, workloads.c4_map_values().tobytes())] if cfg == "c4" else []
    base = goldens.Case(cfg, lay.code, lay.relocs, maps_spec, pk, D, 64, None)
    want, wf, _, _ = oracle_run(base, nthreads=16)
    assert not wf.any()
    maps = make_maps(gpu, env, base)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    try:
        dev = torch.device("cuda:0")
        d_pk = torch.from_numpy(pk.reshape(-1)).to(dev).repeat(n // D)
        d_ret = torch.full((n,), -1, dtype=torch.int64, device=dev)
        d_hist = torch.full((257,), 987654321, dtype=torch.int64, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), None, None,
                        d_hist.data_ptr(), st, hist_overwrite=True)
        torch.cuda.synchronize()
        wt = torch.from_numpy(want.view(np.int64)).to(dev)
        bad = int((d_ret.view(n // D, D) != wt.unsqueeze(0)).sum())
        assert bad == 0, "%d of %d packets differ from the oracle" % (bad, n)
        h = np.bincount(np.minimum(want, 255).astype(np.int64), minlength=257) * (n // D)
        np.testing.assert_array_equal(d_hist.cpu().numpy(), h)
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


def test_many_streams_separate_histograms(gpu, env):
    """More concurrent streams (8) than the library's 4 pooled histogram row buffers, each
    launching into its own histogram with no synchronisation between launches: the row buffers
    are handed across streams with GPU-side waits, and every histogram must come out exact."""
    import torch
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c4()
    n = 1 << 20
    pk = workloads.packets_l2l3(n, 64, seed=41)
    vals = workloads.c4_map_values()
    case = goldens.Case("c4", lay.code, lay.relocs, [(8, 256, vals.tobytes())], pk, n, 64, None)
    want, _, _, _ = oracle_run(case, nthreads=8)
    maps = make_maps(gpu, env, case)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    try:
        dev = torch.device("cuda:0")
        d_pk = torch.from_numpy(pk.reshape(-1)).to(dev)
        nst, rounds = 8, 6
        streams = [torch.cuda.Stream() for _ in range(nst)]
        rets = [torch.zeros(n, dtype=torch.int64, device=dev) for _ in range(nst)]
        hists = [torch.zeros(257, dtype=torch.int64, device=dev) for _ in range(nst)]
        torch.cuda.synchronize()
        for r in range(rounds):
            for s, d_ret, h in zip(streams, rets, hists):
                p.run_batch_dev(0, d_pk.data_ptr(), n, 64, d_ret.data_ptr(), None, None,
                                h.data_ptr(), s.cuda_stream, hist_overwrite=(r == 0))
        torch.cuda.synchronize()
        exp = np.bincount(np.minimum(want, 255).astype(np.int64), minlength=257) * rounds
        for d_ret, h in zip(rets, hists):
            np.testing.assert_array_equal(d_ret.cpu().numpy().view(np.uint64), want)
            np.testing.assert_array_equal(h.cpu().numpy(), exp)
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


@pytest.mark.parametrize("variant", VARIANTS)
def test_literal_slot_programs(gpu, env, variant):
    """The literal 64- and 256-slot variants (bench c3lit / c5lit) on 64-B and IMIX packets."""
    from generic_ebpf_amd import workloads
    for n_slots in (64, 256):
        lay = workloads.prog_literal(n_slots)
        n = 50000
        data, offs, _ = workloads.packets_imix(n)
        for c in (goldens.Case("lit", lay.code, [], [], workloads.packets_l2l3(n, 64), n, 64, None),
                  goldens.Case("lit", lay.code, [], [], data, n, 0, offs)):
            want, wf, _, _ = oracle_run(c, nthreads=8)
            got, gf, _ = device_run(gpu, env, c, variant)
            np.testing.assert_array_equal(want, got)
            np.testing.assert_array_equal(wf, gf)


def test_per_thread_stream_histograms(gpu, env):
    """hipStreamPerThread is one handle naming a different stream in each thread: two threads
    launching on it concurrently, each into its own histogram, must each get exact counts (the
    library keys its per-stream verdict partials by (handle, thread) for that handle)."""
    import threading
    import torch
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c4()
    n = 1 << 20
    pk = workloads.packets_l2l3(n, 64, seed=43)
    vals = workloads.c4_map_values()
    case = goldens.Case("c4", lay.code, lay.relocs, [(8, 256, vals.tobytes())], pk, n, 64, None)
    want, _, _, _ = oracle_run(case, nthreads=8)
    maps = make_maps(gpu, env, case)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]))
    per_thread = 2  # hipStreamPerThread
    try:
        dev = torch.device("cuda:0")
        d_pk = torch.from_numpy(pk.reshape(-1)).to(dev)
        rounds, nthr = 20, 2
        rets = [torch.zeros(n, dtype=torch.int64, device=dev) for _ in range(nthr)]
        hists = [torch.zeros(257, dtype=torch.int64, device=dev) for _ in range(nthr)]
        torch.cuda.synchronize()
        errors = []

        def worker(t):
            try:
                gpu.lib().ebpf_gpu_set_device(0)
                for r in range(rounds):
                    p.run_batch_dev(0, d_pk.data_ptr(), n, 64, rets[t].data_ptr(), None, None,
                                    hists[t].data_ptr(), per_thread, hist_overwrite=(r == 0))
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        ths = [threading.Thread(target=worker, args=(t,)) for t in range(nthr)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        torch.cuda.synchronize()
        assert not errors, errors
        exp = np.bincount(np.minimum(want, 255).astype(np.int64), minlength=257) * rounds
        for d_ret, h in zip(rets, hists):
            np.testing.assert_array_equal(d_ret.cpu().numpy().view(np.uint64), want)
            np.testing.assert_array_equal(h.cpu().numpy(), exp)
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


@pytest.mark.parametrize("variant", VARIANTS)
def test_taken_jump_pc_wrap_leaves_program(gpu, env, variant):
    """A taken jump that wraps the reference's u32 pc (ebpf_interpreter.c:26, pc += off) lands
    2^32 slots on, past the program: SLOT for every packet.  Slot 1 (JNE r0, 0, -2) at pc 2 goes
    to (1, 1), then at pc 1 to pc 0xffffffff (fuzz_gpu.py --mutate found the translator folding
    that target back onto slot 0: a state key kept 32 bits of the slot)."""
    from generic_ebpf_amd import isa
    E = isa.encode
    code = b"".join([E(0xb4, 0, 0, 0, 1), E(0x55, 0, 0, -2, 0), E(0xb4, 9, 0, 0, 1), E(0x95)])
    pk = np.zeros((130, 64), dtype=np.uint8)
    p = gpu.Prog(env, code)
    try:
        gpu.set_variant(variant)
        ret, faults, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), 130, 64)
    finally:
        gpu.set_variant(0)
        p.destroy()
    assert (faults == 4).all() and (ret == 0).all()


def _fused_swap_programs():
    """A packet load fused with the BE16 / BE32 after it (asm_cc.cpp ldxpkc): the loaded bytes
    land at the top of the swapped word, so a later shift or 64-bit multiply must see all 16 / 32
    bits (fuzz_gpu.py seed 91 found the compiled code taking the load's own width: a carry into
    the high word dropped by the multiply that followed)."""
    from generic_ebpf_amd import isa, layout
    I = isa.Insn
    progs = []
    for ld, be, sh in (("ldxb", 16, 8), ("ldxb", 32, 24), ("ldxh", 32, 16), ("ldxb", 32, 0)):
        body = [I(ld, 0, 1, 13), I("be", 0, imm=be)]
        if sh:
            body.append(I("rsh64_imm", 0, imm=sh))
        else:   # the seed-91 shape: a carry past bit 32, then a 64-bit multiply
            body += [I("add64_imm", 0, imm=301528363), I("mul64_imm", 0, imm=625341585)]
        progs.append(layout.assemble(body + [I("exit")]))
    return progs


@pytest.mark.parametrize("variant", VARIANTS)
def test_fused_load_swap_value_range(gpu, env, variant):
    from generic_ebpf_amd import workloads
    pk = workloads.packets_random(4099, 64, seed=61)
    for lay in _fused_swap_programs():
        c = goldens.Case("fused", lay.code, lay.relocs, [], pk.reshape(-1), len(pk), 64, None)
        want, wf, _, _ = oracle_run(c)
        ret, faults, _ = device_run(gpu, env, c, variant)
        np.testing.assert_array_equal(faults, wf)
        np.testing.assert_array_equal(ret, want)
        assert len(np.unique(want)) > 100
