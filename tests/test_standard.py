"""EBPF_SEM_STANDARD (standard eBPF semantics) on the CPU: the oracle's
restatement against hand-computed known answers, the product's ebpf_prog_run against both, the
API contract of ebpf_prog_set_semantics, and random loop-free programs (oracle vs ebpf_prog_run).
No reference implementation of these semantics exists (the reference interpreter has its own);
the known answers in tests/stdprogs.py are derived by hand from the ISA rules."""
import errno

import numpy as np
import pytest

import pyoracle
import stdprogs

PKT = np.frombuffer(stdprogs.PKT, dtype=np.uint8)


@pytest.mark.parametrize("kat", stdprogs.KATS, ids=[k[0] for k in stdprogs.KATS])
def test_oracle_known_answers(kat):
    name, items, want = kat
    code, rel = stdprogs.asm(items)
    r, f, _, _ = pyoracle.OracleProgram(code, rel, [], semantics=1).run(PKT, 1, 64)
    assert not f[0] and int(r[0]) == want


@pytest.mark.parametrize("kat", stdprogs.KATS, ids=[k[0] for k in stdprogs.KATS])
def test_cpu_path_known_answers(native, env, kat):
    name, items, want = kat
    code, _ = stdprogs.asm(items)
    p = native.Prog(env, code)
    try:
        p.set_semantics(native.SEM_STANDARD)
        r, _ = p.run_cpu(stdprogs.PKT)
        assert r == want
    finally:
        p.destroy()


def test_semantics_select_the_interpreter(native, env):
    """The same bytecode under both semantics: the reference visits slots 0, 1, 3 (cumulative
    stepping) and its MOV64 adds (5 + 7 = 12); standard eBPF runs slots 0..3 and moves (100)."""
    I = stdprogs.I
    code, _ = stdprogs.asm([I("mov64_imm", 0, imm=5), I("mov64_imm", 0, imm=7),
                            I("mov64_imm", 0, imm=100), I("exit")])
    p = native.Prog(env, code)
    try:
        r_ref, _ = p.run_cpu(stdprogs.PKT)
        p.set_semantics(native.SEM_STANDARD)
        r_std, _ = p.run_cpu(stdprogs.PKT)
        want_ref, f, _, _ = pyoracle.OracleProgram(code).run(PKT, 1, 64)
        assert r_std == 100 and r_ref == int(want_ref[0]) == 12
    finally:
        p.destroy()


def test_set_semantics_contract(native, env):
    code, _ = stdprogs.asm([stdprogs.I("mov64_imm", 0, imm=1), stdprogs.I("exit")])
    p = native.Prog(env, code)
    L = native.lib()
    try:
        assert L.ebpf_prog_set_semantics(None, 1) == errno.EINVAL
        assert L.ebpf_prog_set_semantics(p.ptr, 2) == errno.EINVAL
        assert L.ebpf_prog_set_semantics(p.ptr, 1) == 0
        assert L.ebpf_prog_set_semantics(p.ptr, 1) == 0
        p.info()                                    # translated (device form) ...
        assert L.ebpf_prog_set_semantics(p.ptr, 0) == errno.EBUSY   # ... so now fixed
        assert L.ebpf_prog_set_semantics(p.ptr, 1) == 0
    finally:
        p.destroy()


@pytest.mark.parametrize("seed", range(60))
def test_random_programs_oracle_vs_cpu_path(native, env, seed):
    with_map = seed % 3 == 0
    code, rel = stdprogs.gen_program(1000 + seed, length=30 + seed % 40, with_map=with_map)
    g = np.random.default_rng(seed)
    pk = g.integers(0, 256, (24, 64), dtype=np.uint8)
    maps, specs = [], []
    if with_map:
        vals = g.integers(0, 256, 16 * 8, dtype=np.uint8).tobytes()
        m = native.Map(env, 16, 8)
        m.fill(vals)
        maps.append(m)
        specs.append((8, 16, vals))
    want, wf, _, _ = pyoracle.OracleProgram(code, rel, specs, semantics=1).run(pk.reshape(-1), len(pk), 64)
    assert not wf.any()
    p = native.Prog(env, native.patch_relocs(code, rel, [m.handle for m in maps]))
    try:
        p.set_semantics(native.SEM_STANDARD)
        for i in range(len(pk)):
            r, _ = p.run_cpu(pk[i].tobytes())
            assert r == int(want[i]), i
    finally:
        p.destroy()
        for m in maps:
            m.destroy()


@pytest.mark.parametrize("seed", range(0, 60, 7))
def test_device_translation_compiles(native, env, seed):
    """Standard programs translate for the device and compile in both packet layouts."""
    code, rel = stdprogs.gen_program(1000 + seed, length=30 + seed % 40)
    p = native.Prog(env, code)
    try:
        p.set_semantics(native.SEM_STANDARD)
        p.info()
        for layout in (0, 1):
            assert len(p.device_code(layout)) > 0
    finally:
        p.destroy()


def test_device_accepts_loops_cpu_runs_them(native, env):
    """A bounded loop (r0 = 0; r2 = 5; do r0 += r2 while --r2 != 0): 15 on the CPU path; the
    device translation accepts it (its backward jump is counted: dprog.h DK_LOOPCNT)."""
    I = stdprogs.I
    code, _ = stdprogs.asm([I("mov64_imm", 0, imm=0), I("mov64_imm", 2, imm=5), ("label", "L"),
                            I("add64_reg", 0, 2), I("sub64_imm", 2, imm=1),
                            I("jne_imm", 2, imm=0, off="L"), I("exit")])
    p = native.Prog(env, code)
    try:
        p.set_semantics(native.SEM_STANDARD)
        assert p.run_cpu(stdprogs.PKT)[0] == 15
        p.info()
    finally:
        p.destroy()


@pytest.mark.parametrize("extra,fault", [(0, 0), (1, 8)])
def test_oracle_loop_budget(extra, fault):
    """The budget: 2^20 taken backward jumps run, the next one faults LOOP (hand count: the
    countdown from n takes n - 1 backward jumps and sums 1..n)."""
    n = stdprogs.LOOP_BUDGET + 1 + extra
    code, rel = stdprogs.countdown(n)
    want, wf, _, _ = pyoracle.OracleProgram(code, rel, [], semantics=1).run(
        np.zeros(64, np.uint8), 1, 64)
    assert int(wf[0]) == fault
    assert int(want[0]) == (0 if fault else n * (n + 1) // 2)


@pytest.mark.parametrize("seed", range(12))
def test_loop_programs_oracle_vs_cpu_path(native, env, seed):
    """Random counted-loop programs (no packet loops forever): the oracle's run_std and the CPU
    ebpf_prog_run agree."""
    code, rel = stdprogs.gen_loop_program(7000 + seed)
    pk = np.random.default_rng(seed).integers(0, 256, (32, 64), dtype=np.uint8)
    want, wf, _, _ = pyoracle.OracleProgram(code, rel, [], semantics=1).run(pk.reshape(-1), 32, 64)
    assert not wf.any()
    p = native.Prog(env, code)
    try:
        p.set_semantics(native.SEM_STANDARD)
        for i in range(len(pk)):
            assert p.run_cpu(pk[i].tobytes())[0] == int(want[i]), i
        p.info()
    finally:
        p.destroy()


@pytest.mark.parametrize("seed", range(24))
def test_loop_programs_compile(native, env, seed):
    """Programs with loops compile for variant 0 (both layouts): the code generator's facts and
    liveness cross only single-predecessor edges, so a loop head starts from nothing known."""
    code, rel = stdprogs.gen_loop_program(9000 + seed, forever_every=97 if seed % 8 == 0 else 0)
    p = native.Prog(env, code)
    try:
        p.set_semantics(native.SEM_STANDARD)
        for layout in (0, 1):
            assert len(p.device_code(layout)) > 0
    finally:
        p.destroy()


def test_c3l_workload_oracle_and_cpu_path(native, env):
    """C3L (workloads.prog_c3l, the bench's loop workload): the oracle's standard restatement,
    a numpy restatement of the header checksum rule and the CPU ebpf_prog_run agree; every
    verdict class occurs."""
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c3l()
    pk = workloads.packets_ipv4opt(1 << 14)
    want = workloads.c3l_expected(pk)
    got, gf, _, _ = pyoracle.OracleProgram(lay.code, [], [], semantics=1).run(pk.reshape(-1), len(pk), 64)
    assert not gf.any()
    np.testing.assert_array_equal(got, want)
    assert {0, 2, 4} <= set(int(x) for x in np.unique(want)) and (want >= 16).mean() > 0.5
    p = native.Prog(env, lay.code)
    try:
        p.set_semantics(native.SEM_STANDARD)
        for i in range(0, len(pk), 37):
            assert p.run_cpu(pk[i].tobytes())[0] == int(want[i]), i
        for layout in (0, 1):
            assert len(p.device_code(layout)) > 0
    finally:
        p.destroy()


def test_cursor_programs_cpu_and_code(native, env):
    """Cursor walks (stdprogs.gen_cursor_program, the GPU test's programs): the CPU
    ebpf_prog_run equals the oracle on every packet the oracle does not fault MEM; both layouts
    compile.  (Keep mode — the staged kernel double-buffering its packets so that the loads at
    run-time offsets read LDS — is the host's choice per launch, dp_launch.vflags DP_VF_KEEP, and
    is exercised by the GPU cursor tests.)"""
    for seed in range(4):
        code, rel = stdprogs.gen_cursor_program(7000 + seed)
        g = np.random.default_rng(seed)
        pk = g.integers(0, 256, (64, 64), dtype=np.uint8)
        want, wf, _, _ = pyoracle.OracleProgram(code, rel, [], semantics=1).run(pk.reshape(-1), 64, 64)
        p = native.Prog(env, code)
        try:
            p.set_semantics(native.SEM_STANDARD)
            for i in np.nonzero(wf == 0)[0]:   # (ebpf_prog_run has no packet bound to check)
                assert p.run_cpu(pk[i].tobytes())[0] == int(want[i]), (seed, i)
            for layout in (0, 1):
                assert len(p.device_code(layout)) > 0
        finally:
            p.destroy()


def _keeps_loop_count(native, env, code):
    import subprocess
    p = native.Prog(env, code)
    try:
        p.set_semantics(native.SEM_STANDARD)
        c = p.device_code(1)
    finally:
        p.destroy()
    r = subprocess.run(["/opt/rocm/llvm/bin/llvm-mc", "--disassemble", "-triple=amdgcn-amd-amdhsa",
                        "-mcpu=gfx950"], input=" ".join("0x%02x" % b for b in c),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0
    return "ds_add_rtn_u32" in r.stdout   # (the LOOPCNT body: one LDS add per back edge)


def _disasm(code):
    """(byte offset, instruction text) pairs of gfx950 machine code (llvm-mc)."""
    import subprocess
    r = subprocess.run(["/opt/rocm/llvm/bin/llvm-mc", "--disassemble", "-triple=amdgcn-amd-amdhsa",
                        "-mcpu=gfx950", "-show-encoding"], input=" ".join("0x%02x" % b for b in code),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0
    out, off = [], 0
    for line in r.stdout.splitlines():
        if "encoding:" not in line:
            continue
        ins, enc = line.split("encoding:", 1)
        out.append((off, ins.strip().rstrip(";/").strip()))
        off += enc.count("0x")
    return out


def test_loop_back_edge_code_shape(native, env):
    """C3L's staged compiled code (asm_jit.cpp, the reversed split): both branches of a back edge
    that keeps the looping lanes go to the loop block itself, never to an s_branch; the staged
    packet load at a run-time offset checks the offset with one unsigned 64-bit compare
    (gen_interp.py h_ldx_pktv)."""
    import os
    from generic_ebpf_amd import workloads
    if not os.path.exists("/opt/rocm/llvm/bin/llvm-mc"):
        pytest.skip("llvm-mc not available")
    p = native.Prog(env, workloads.prog_c3l().code)
    try:
        p.set_semantics(native.SEM_STANDARD)
        ins = _disasm(p.device_code(1))
    finally:
        p.destroy()
    at = dict(ins)
    back = 0
    for off, text in ins:
        op = text.split()[0]
        if op not in ("s_cbranch_execnz", "s_cbranch_scc0"):
            continue
        simm = int(text.split()[1])
        tgt = off + 4 + 4 * (simm - 65536 if simm >= 32768 else simm)
        if tgt < off:   # a back edge
            back += 1
            assert not at[tgt].startswith("s_branch"), (hex(off), at[tgt])
    assert back == 2
    assert any(t.startswith("v_cmp_ge_u64") for _, t in ins)


def test_counted_loop_needs_no_count(native, env):
    """translate.cpp elide_loop_count: a single counted loop whose counter enters in [1, K] with
    K - 1 <= 2^20 drops its per-lane count (C3L: IHL in [5, 12]; countdown(n) for n <= 2^20 + 1,
    which takes exactly the budget); one more trip than the budget keeps it (the GPU budget test
    then faults LOOP), and so do programs with two loops."""
    import os
    from generic_ebpf_amd import workloads
    if not os.path.exists("/opt/rocm/llvm/bin/llvm-mc"):
        pytest.skip("llvm-mc not available")
    assert not _keeps_loop_count(native, env, workloads.prog_c3l().code)
    assert not _keeps_loop_count(native, env, stdprogs.countdown(100)[0])
    assert not _keeps_loop_count(native, env, stdprogs.countdown(stdprogs.LOOP_BUDGET + 1)[0])
    assert _keeps_loop_count(native, env, stdprogs.countdown(stdprogs.LOOP_BUDGET + 2)[0])
    # the counter may enter at 0 (r2 = packet byte & 15, no lower bound): 2^64 - 1 trips
    code, _ = stdprogs.asm([stdprogs.I("ldxb", 2, 1, 5), stdprogs.I("and64_imm", 2, imm=15),
                            ("label", "L"), stdprogs.I("add64_imm", 0, imm=1),
                            stdprogs.I("sub64_imm", 2, imm=1), stdprogs.I("jne_imm", 2, imm=0, off="L"),
                            stdprogs.I("exit")])
    assert _keeps_loop_count(native, env, code)
    # ... with the +1 the cursor/loop generators use it cannot
    code, _ = stdprogs.asm([stdprogs.I("ldxb", 2, 1, 5), stdprogs.I("and64_imm", 2, imm=15),
                            stdprogs.I("add64_imm", 2, imm=1),
                            ("label", "L"), stdprogs.I("add64_imm", 0, imm=1),
                            stdprogs.I("sub64_imm", 2, imm=1), stdprogs.I("jne_imm", 2, imm=0, off="L"),
                            stdprogs.I("exit")])
    assert not _keeps_loop_count(native, env, code)
    # a second write of the counter in the body keeps the count
    code, _ = stdprogs.asm([stdprogs.I("mov64_imm", 2, imm=9), ("label", "L"),
                            stdprogs.I("sub64_imm", 2, imm=1), stdprogs.I("add64_imm", 2, imm=1),
                            stdprogs.I("sub64_imm", 2, imm=1), stdprogs.I("jne_imm", 2, imm=0, off="L"),
                            stdprogs.I("exit")])
    assert _keeps_loop_count(native, env, code)
    assert sum(_keeps_loop_count(native, env, stdprogs.gen_cursor_program(7000 + s)[0])
               for s in range(6)) == 0
