"""Standard-eBPF semantics on the device (every variant, staged and general kernels) against the
oracle's standard restatement: the hand-computed known answers, random loop-free programs with
every ALU op / JMP32 / stack / packet access / array lookup, and one program at full size."""
import numpy as np
import pytest

import pyoracle
import stdprogs

pytestmark = pytest.mark.gpu

VARIANTS = [0, 1, 2]


def run_device(native, env, code, rel, specs, data, count, stride, variant, offsets=None,
               want_exec=None):
    maps = []
    for vs, me, d in specs:
        m = native.Map(env, me, vs)
        m.fill(d)
        maps.append(m)
    p = native.Prog(env, native.patch_relocs(code, rel, [m.handle for m in maps]))
    try:
        p.set_semantics(native.SEM_STANDARD)
        native.set_variant(variant)
        d = np.ascontiguousarray(data.copy())
        ret, faults, _ = p.run_batch(d, count, stride, offsets)
        if want_exec is not None:  # what the launch ran (variant 0: the compiled program)
            assert p.exec_info(0)[0] == want_exec
        return ret, faults
    finally:
        native.set_variant(0)
        p.destroy()
        for m in maps:
            m.destroy()


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("stride", [64, 96])
def test_known_answers_on_device(gpu, env, variant, stride):
    bad = []
    for name, items, want in stdprogs.KATS:
        code, rel = stdprogs.asm(items)
        pk = np.zeros((256, stride), dtype=np.uint8)
        pk[:, :64] = np.frombuffer(stdprogs.PKT, dtype=np.uint8)
        got, gf = run_device(gpu, env, code, rel, [], pk.reshape(-1), 256, stride, variant)
        if gf.any() or not (got == want).all():
            bad.append((name, hex(int(got[0])), hex(want), int(gf[0])))
    assert not bad, bad


@pytest.mark.parametrize("variant", VARIANTS)
def test_random_programs_vs_oracle(gpu, env, variant):
    bad = []
    for seed in range(80):
        g = np.random.default_rng(seed)
        with_map = seed % 3 == 0
        code, rel = stdprogs.gen_program(5000 + seed, length=20 + seed % 60, with_map=with_map)
        specs = []
        if with_map:
            specs = [(8, 16, g.integers(0, 256, 128, dtype=np.uint8).tobytes())]
        stride = 64 if seed % 2 == 0 else 72
        n = 2048
        pk = g.integers(0, 256, (n, stride), dtype=np.uint8)
        want, wf, _, _ = pyoracle.OracleProgram(code, rel, specs, semantics=1).run(
            pk.reshape(-1), n, stride)
        got, gf = run_device(gpu, env, code, rel, specs, pk.reshape(-1), n, stride, variant)
        if not (np.array_equal(want, got) and np.array_equal(wf, gf)):
            bad.append((seed, int(np.count_nonzero(want != got)), int(np.count_nonzero(wf != gf))))
    assert not bad, bad


@pytest.mark.parametrize("variant", [0, 2])
def test_full_size_random_program(gpu, env, variant):
    """16M packets tiled from 256k distinct: result i equals the oracle's for its distinct packet."""
    code, rel = stdprogs.gen_program(777, length=60)
    distinct, tiles = 1 << 18, 64
    pk = np.random.default_rng(4).integers(0, 256, (distinct, 64), dtype=np.uint8)
    want, wf, _, _ = pyoracle.OracleProgram(code, rel, [], semantics=1).run(
        pk.reshape(-1), distinct, 64, nthreads=8)
    assert not wf.any()
    got, gf = run_device(gpu, env, code, rel, [], np.tile(pk.reshape(-1), tiles), distinct * tiles,
                         64, variant)
    assert not gf.any()
    np.testing.assert_array_equal(got.reshape(tiles, distinct), np.broadcast_to(want, (tiles, distinct)))


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("extra,fault", [(0, 0), (1, 8)])
def test_loop_budget_on_device(gpu, env, variant, extra, fault):
    """2^20 taken backward jumps run to EXIT, the next one faults LOOP (dprog.h DP_LOOP_BUDGET;
    oracle run_std; the same hand count as tests/test_standard.py)."""
    n = stdprogs.LOOP_BUDGET + 1 + extra
    code, rel = stdprogs.countdown(n)
    pk = np.zeros((64, 64), dtype=np.uint8)
    got, gf = run_device(gpu, env, code, rel, [], pk.reshape(-1), 64, 64, variant,
                         want_exec="compiled" if variant == 0 else None)
    assert (gf == fault).all()
    assert (got == (0 if fault else n * (n + 1) // 2)).all()


@pytest.mark.parametrize("variant", VARIANTS)
def test_loop_programs_vs_oracle(gpu, env, variant):
    """Random programs with counted loops (data-dependent trip counts, nested loops, JA and
    conditional back edges, forward branches inside the bodies); every 8th also has packets that
    loop forever and fault LOOP at the budget.  Staged (64 B) and general (72 B) kernels."""
    bad = []
    for seed in range(24):
        forever = 97 if seed % 8 == 0 else 0
        code, rel = stdprogs.gen_loop_program(9000 + seed, forever_every=forever)
        g = np.random.default_rng(seed)
        stride = 64 if seed % 2 == 0 else 72
        n = 2048
        pk = g.integers(0, 256, (n, stride), dtype=np.uint8)
        want, wf, _, _ = pyoracle.OracleProgram(code, rel, [], semantics=1).run(
            pk.reshape(-1), n, stride, nthreads=8)
        if forever:
            assert (wf == 8).any()
        got, gf = run_device(gpu, env, code, rel, [], pk.reshape(-1), n, stride, variant,
                             want_exec="compiled" if variant == 0 else None)
        if not (np.array_equal(want, got) and np.array_equal(wf, gf)):
            bad.append((seed, int(np.count_nonzero(want != got)), int(np.count_nonzero(wf != gf))))
    assert not bad, bad


@pytest.mark.parametrize("variant", VARIANTS)
def test_cursor_loops_vs_oracle(gpu, env, variant):
    """Packet walks with a cursor in a loop (LDXPKTV: loads at run-time offsets, any alignment,
    cursors running off the end fault MEM) against the oracle.  Staged 64-B batches of 600,001
    packets (many groups per wave: the compiled program reads the LDS packet buffer, whose next
    DMA waits for the group's end; a partial last group) and general 72-B batches."""
    bad, outcomes = [], set()
    for seed in range(12):
        code, rel = stdprogs.gen_cursor_program(7000 + seed)
        g = np.random.default_rng(seed)
        stride = 64 if seed % 3 else 72
        n = 600001 if stride == 64 else 20011
        pk = g.integers(0, 256, (n, stride), dtype=np.uint8)
        want, wf, _, _ = pyoracle.OracleProgram(code, rel, [], semantics=1).run(
            pk.reshape(-1), n, stride, nthreads=8)
        got, gf = run_device(gpu, env, code, rel, [], pk.reshape(-1), n, stride, variant,
                             want_exec="compiled" if variant == 0 else None)
        if not (np.array_equal(want, got) and np.array_equal(wf, gf)):
            bad.append((seed, int(np.count_nonzero(want != got)), int(np.count_nonzero(wf != gf))))
        outcomes |= set(int(x) for x in np.unique(wf))
    assert not bad, bad
    assert {0, 3} <= outcomes


def test_keep_mode_refill_on_interpreter(gpu, env):
    """Keep mode on the assembly interpreter's staged kernel (one result slot per group, the
    RETK = 1 image): every group of the interpreter ends with no live lane (.Lr_schedule reaches
    .Lgroup_done with exec = 0), and only then is the wave's next group DMA'd into the LDS
    packet buffer the program's run-time-offset loads read.  That DMA's lane mask must not
    depend on the arriving exec (round 4: with it, refilled groups read the previous group's
    bytes or a mix).  4M + 37 distinct packets (8 groups per wave and a partial last group), a
    walk whose every load is at a run-time offset, against the oracle
    (ebpf_interpreter.c:327-338: each packet reads its own bytes)."""
    I = stdprogs.I
    code, rel = stdprogs.asm([
        I("mov64_reg", 6, 1), I("ldxb", 8, 6, 0), I("and64_imm", 8, imm=7), I("add64_imm", 8, imm=1),
        I("mov64_imm", 0, imm=1), ("label", "L"),
        I("ldxw", 2, 6, 3), I("mul64_imm", 0, imm=0x1e3779b1), I("xor64_reg", 0, 2),
        I("add64_imm", 6, imm=5), I("sub64_imm", 8, imm=1), I("jne_imm", 8, imm=0, off="L"),
        I("exit")])
    n = (1 << 22) + 37
    pk = np.random.default_rng(91).integers(0, 256, (n, 64), dtype=np.uint8)
    want, wf, _, _ = pyoracle.OracleProgram(code, rel, [], semantics=1).run(pk.reshape(-1), n, 64,
                                                                            nthreads=16)
    assert not wf.any()
    p = gpu.Prog(env, code)
    try:
        p.set_semantics(gpu.SEM_STANDARD)
        gpu.set_variant(2)
        got, gf, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), n, 64)
        ex, layout = p.exec_info(0)[:2]
    finally:
        gpu.set_variant(0)
        p.destroy()
    assert (ex, layout) == ("interpreter", 1)
    assert not gf.any()
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (bad.size, bad[:8])


@pytest.mark.parametrize("variant", [0, 2])
def test_cursor_walk_then_hash_probe(gpu, env, variant):
    """A cursor walk (packet loads at run-time offsets: keep mode, the LDS packet buffer held
    until the group ends) followed by a hashtable probe keyed by the walk's result (the probe's
    routine and the group-end DMA on one wave), 200,001 staged packets against the oracle."""
    I = stdprogs.I
    code, rel = stdprogs.asm([
        I("mov64_reg", 6, 1), I("mov64_imm", 0, imm=7), I("mov64_reg", 7, 6),
        I("add64_imm", 7, imm=2), I("ldxb", 8, 6, 40), I("and64_imm", 8, imm=7),
        I("add64_imm", 8, imm=1), ("label", "L"),
        I("ldxh", 2, 7, 1), I("mul64_imm", 0, imm=31), I("add64_reg", 0, 2),
        I("ldxb", 3, 7, 0), I("and64_imm", 3, imm=3), I("add64_reg", 7, 3), I("add64_imm", 7, imm=2),
        I("sub64_imm", 8, imm=1), I("jne_imm", 8, imm=0, off="L"),
        I("mov64_reg", 9, 0), I("and64_imm", 0, imm=63), I("stxw", 10, 0, -4),
        ("lddw_map", 1, 0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4),
        I("call", imm=0), I("jeq_imm", 0, imm=0, off="M"),
        I("ldxdw", 0, 0, 0), I("xor64_reg", 9, 0), ("label", "M"),
        I("mov64_reg", 0, 9), I("exit")])
    g = np.random.default_rng(77)
    keys = np.arange(0, 64, 2, dtype=np.uint32)   # every other key present
    vals = g.integers(0, 256, (len(keys), 8), dtype=np.uint8)
    spec = pyoracle.HashSpec(4, 8, keys=keys.view(np.uint8).reshape(-1, 4), values=vals, capacity=64)
    n = 200001
    pk = g.integers(0, 256, (n, 64), dtype=np.uint8)
    want, wf, _, _ = pyoracle.OracleProgram(code, rel, [spec], semantics=1).run(pk.reshape(-1), n, 64,
                                                                                nthreads=8)
    assert not wf.any()
    m = gpu.HashMap(env, 4, 8, 64)
    try:
        m.fill(keys.view(np.uint8).reshape(-1, 4), vals)
        p = gpu.Prog(env, gpu.patch_relocs(code, rel, [m.handle]))
        try:
            p.set_semantics(gpu.SEM_STANDARD)
            gpu.set_variant(variant)
            got, gf, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1).copy()), n, 64)
            if variant == 0:
                assert p.exec_info(0)[0] == "compiled"
        finally:
            gpu.set_variant(0)
            p.destroy()
    finally:
        m.destroy()
    assert not gf.any()
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("variant", VARIANTS)
def test_c3l_full_size(gpu, env, variant):
    """The bench's loop workload (C3L: IPv4 header checksum over IHL words, 5-12 trips) over 16M
    packets tiled from 256k distinct: result i equals the oracle's for its distinct packet (and
    the numpy restatement of the rule); variant 0 runs it compiled."""
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c3l()
    distinct, tiles = 1 << 18, 64
    pk = workloads.packets_ipv4opt(distinct)
    want, wf, _, _ = pyoracle.OracleProgram(lay.code, [], [], semantics=1).run(
        pk.reshape(-1), distinct, 64, nthreads=8)
    assert not wf.any()
    np.testing.assert_array_equal(want, workloads.c3l_expected(pk))
    got, gf = run_device(gpu, env, lay.code, [], [], np.tile(pk.reshape(-1), tiles), distinct * tiles,
                         64, variant, want_exec="compiled" if variant == 0 else None)
    assert not gf.any()
    np.testing.assert_array_equal(got.reshape(tiles, distinct), np.broadcast_to(want, (tiles, distinct)))


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("stride", [64, 72])
def test_zero_offset_conditionals(gpu, env, variant, stride):
    """Conditional jumps of offset 0 (64- and 32-bit) go to the next slot taken or not: r0 = 6
    for every packet (fuzz_gpu.py --standard found the compiled staged path losing such groups'
    results before the translator turned these compares into no-ops)."""
    code, rel = stdprogs.asm([
        stdprogs.I("mov64_imm", 0, imm=5), (stdprogs.JMP64["jeq"], 0, 0, 0, 5),
        stdprogs.I("add64_imm", 0, imm=1),
        (stdprogs.JMP32["jset"], 0, 0, 0, 7), (stdprogs.JMP64["jgt"] + 8, 1, 0, 0, 0),
        (stdprogs.JMP64["jne"], 1, 0, 0, 0), stdprogs.I("exit")])
    n = 777
    pk = np.random.default_rng(1).integers(0, 256, (n, stride), dtype=np.uint8)
    got, gf = run_device(gpu, env, code, rel, [], pk.reshape(-1), n, stride, variant)
    assert not gf.any()
    assert (got == 6).all()


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("stride", [64, 72])
def test_zero_offset_conditionals_reference(gpu, env, variant, stride):
    """The same under the reference's cumulative stepping (ebpf_interpreter.c:209-211: pc += 0
    leaves the next state unchanged): slots 0 (r0 = 5), 1 (JEQ r0, 5, +0), 3 (r0 += 1), 6 (EXIT)."""
    from generic_ebpf_amd import isa
    E = isa.encode
    filler = E(0xb4, 9, 0, 0, 77)
    code = b"".join([E(0xb4, 0, 0, 0, 5), E(0x15, 0, 0, 0, 5), filler, E(0x04, 0, 0, 0, 1), filler,
                     filler, E(0x95, 0, 0, 0, 0)])
    n = 777
    pk = np.random.default_rng(2).integers(0, 256, (n, stride), dtype=np.uint8)
    want, wf, _, _ = pyoracle.OracleProgram(code, [], []).run(pk.reshape(-1), n, stride)
    assert not wf.any() and (want == 6).all()
    p = gpu.Prog(env, code)
    try:
        gpu.set_variant(variant)
        got, gf, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1).copy()), n, stride)
    finally:
        gpu.set_variant(0)
        p.destroy()
    assert not gf.any()
    assert (got == 6).all()
