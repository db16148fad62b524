"""Compiled programs (variant 0) on the CPU: ebpf_prog_device_code must produce code for both
packet layouts, within the code area, that decodes completely as gfx950 instructions (no GPU
needed; the GPU parity tests check what it computes)."""
import os
import subprocess

import numpy as np
import pytest

import goldens

LLVM_MC = "/opt/rocm/llvm/bin/llvm-mc"


def _decode(code):
    hexs = " ".join("0x%02x" % b for b in code)
    r = subprocess.run([LLVM_MC, "--disassemble", "-triple=amdgcn-amd-amdhsa", "-mcpu=gfx950"],
                       input=hexs, capture_output=True, text=True, timeout=60)
    return r.stdout, r.stderr


def _encodings(code):
    """Re-encode the disassembly: llvm-mc's encoding of every decoded instruction, concatenated
    (must reproduce `code` exactly when every instruction decodes as what was encoded)."""
    hexs = " ".join("0x%02x" % b for b in code)
    r = subprocess.run([LLVM_MC, "--disassemble", "-show-encoding", "-triple=amdgcn-amd-amdhsa",
                        "-mcpu=gfx950"], input=hexs, capture_output=True, text=True, timeout=60)
    out = bytearray()
    for ln in r.stdout.splitlines():
        if "encoding: [" in ln:
            enc = ln.split("encoding: [")[1].split("]")[0]
            out += bytes(int(x, 16) for x in enc.split(","))
    return bytes(out), r.stdout


def _progs(native, env):
    from generic_ebpf_amd import workloads
    out = []
    for cfg in ("c0", "c2", "c3", "c4", "c5"):
        lay = workloads.CONFIGS[cfg]["prog"]()
        maps = [native.Map(env, 256, 8)] if cfg == "c4" else []
        out.append((cfg, native.patch_relocs(lay.code, lay.relocs, [m.handle for m in maps]), maps))
    for c in goldens.load(os.path.join(goldens.GOLDEN_DIR, "rand.npz"))[:24]:
        maps = [native.Map(env, me, vs) for vs, me, _ in c.maps]
        out.append((c.name, native.patch_relocs(c.code, c.relocs, [m.handle for m in maps]), maps))
    return out


def test_compiled_code_decodes(native, env):
    have_mc = os.path.exists(LLVM_MC)
    progs = _progs(native, env)
    try:
        for name, code, _ in progs:
            p = native.Prog(env, code)
            try:
                for layout in (1, 0):
                    dc = p.device_code(layout)
                    assert 0 < len(dc) <= 512 * 1024 and len(dc) % 4 == 0, name
                    if have_mc:
                        out, err = _decode(dc)
                        assert "invalid" not in err, (name, layout, err[:400])
                        assert out.count("\n") >= len(dc) // 8, (name, layout)
            finally:
                p.destroy()
    finally:
        for _, _, maps in progs:
            for m in maps:
                m.destroy()


def test_compiled_code_without_gpu_is_deterministic(native, env):
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c3()
    p = native.Prog(env, lay.code)
    try:
        a, b = p.device_code(1), p.device_code(1)
        assert a == b
        assert p.device_code(0) != a   # general layout: bounds-checked packet loads
    finally:
        p.destroy()


def test_device_code_rejects_bad_layout(native, env):
    from generic_ebpf_amd import workloads
    p = native.Prog(env, workloads.prog_c2().code)
    try:
        with pytest.raises(native.EbpfError):
            native._check(native.lib().ebpf_prog_device_code(p.ptr, 7, None,
                                                              native.ctypes.byref(native.ctypes.c_size_t(0))),
                          "device_code")
    finally:
        p.destroy()


@pytest.mark.skipif(not os.path.exists(LLVM_MC), reason="llvm-mc not available")
def test_optimised_c4_instruction_forms(native, env):
    """Spot-check the encodings of the optimising code generator (asm_cc.cpp) on the classifier:
    the decoded instructions are exactly the forms it means to emit."""
    from generic_ebpf_amd import workloads
    m = native.Map(env, 256, 8)
    try:
        lay = workloads.prog_c4()
        p = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [m.handle]))
        try:
            text, err = _decode(p.device_code(1))
        finally:
            p.destroy()
    finally:
        m.destroy()
    lines = [ln.strip() for ln in text.splitlines() if ln.strip() and not ln.strip().startswith(".")]
    want = [
        # LDXH r2, [r1+12]; BE16 r2  ->  one byte-select from the staged packet dwords 3/4
        "s_mov_b32 s13, 0xc0c0001", "v_perm_b32 v4, v26, v25, s13",
        # JEQ r2, 0x86dd with r2 < 2^16: one 32-bit compare, constant as a literal
        "v_cmp_eq_u32_e32 vcc, 0x86dd, v4",
        # LDXB r3, [r1+23]
        "v_bfe_u32 v6, v27, 24, 8",
        # LDXW r4, [r1+26]; BE32 r4
        "s_mov_b32 s13, 0x2030405", "v_perm_b32 v8, v29, v28, s13",
        # r8 = 0; r8 |= r4; r8 <<= 32; r8 |= r5  ->  moves
        "v_mov_b32_e32 v16, v8", "v_mov_b32_e32 v17, v16", "v_mov_b32_e32 v16, 0",
        "v_or_b32_e32 v16, v10, v16",
        # MUL64 r8, 0x1e3779b1: the cross term into the addend {0, hi*K}, one in-place
        # v_mad_u64_u32 (v48 = 0 is kept for the rest of the path)
        "s_mov_b32 s13, 0x1e3779b1", "v_mov_b32_e32 v48, 0", "v_mul_lo_u32 v49, v17, s13",
        "v_mad_u64_u32 v[16:17], s[60:61], v16, s13, v[48:49]",
        # XOR64 r8, imm with a zero high word: low half only
        "v_xor_b32_e32 v16, 0x5bd1e995, v16",
        # lookup(map, key = r6 < 256 = max_entries) cannot fail: its NULL check is gone and the
        # value load reads the LDS copy of the map at lds_off + key * 8
        "v_mad_u32_u24 v46, v12, 8, s13", "ds_read2_b32 v[12:13], v46 offset1:1",
    ]
    for w in want:
        assert w in lines, (w, "\n".join(lines[:80]))
    # STXW [r10-4] = r6 (the key): nothing reads the frame afterwards (the lookup takes the key
    # from r6), so the store is dead and emits nothing (round 5)
    assert not any(ln.startswith("ds_write") for ln in lines), "\n".join(lines)
    # dead code: r1 = map handle (LDDW) and r2 = r10 - 4 are only the statically resolved
    # lookup's arguments
    assert "v_mov_b64_e32 v[4:5], v[20:21]" not in lines
    assert not any(ln.startswith("v_mov_b32_e32 v2,") or ln.startswith("v_mov_b32_e32 v3,")
                   for ln in lines)


def _count_valu(native, env, code, layout, nocc):
    if nocc:
        os.environ["EBPF_JIT_NOCC"] = "1"
    try:
        p = native.Prog(env, code)
        try:
            dc = p.device_code(layout)
        finally:
            p.destroy()
    finally:
        os.environ.pop("EBPF_JIT_NOCC", None)
    out, _ = _decode(dc)
    return sum(1 for ln in out.splitlines() if ln.strip().startswith("v_")), len(dc)


@pytest.mark.skipif(not os.path.exists(LLVM_MC), reason="llvm-mc not available")
def test_optimised_code_is_smaller(native, env):
    """The known-bits code generator must not emit more vector instructions than the
    handler-copy baseline, and must remove a good share of them on the classifier (C4)."""
    from generic_ebpf_amd import workloads
    m = native.Map(env, 256, 8)
    try:
        for cfg in ("c2", "c3", "c4", "c5"):
            lay = workloads.CONFIGS[cfg]["prog"]()
            code = native.patch_relocs(lay.code, lay.relocs, [m.handle] if cfg == "c4" else [])
            for layout in (1, 0):
                opt, _ = _count_valu(native, env, code, layout, False)
                base, _ = _count_valu(native, env, code, layout, True)
                assert opt <= base, (cfg, layout, opt, base)
                if cfg == "c4" and layout == 1:
                    assert opt <= 0.8 * base, (opt, base)
    finally:
        m.destroy()


def test_hash_value_loads_forwarded(native, env):
    """C4H: the hashtable probe routine also loads the slot's first value bytes; the code
    generator keeps them in a dead register so the load through the non-NULL lookup result is a
    register move (EBPF_CC_NOHFWD=1 turns it off: one more global load)."""
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c4h()
    m = native.HashMap(env, 4, 8, 64)
    try:
        code = native.patch_relocs(lay.code, lay.relocs, [m.handle])
        p = native.Prog(env, code)
        dc = p.device_code(1)
        p.destroy()
        os.environ["EBPF_CC_NOHFWD"] = "1"
        try:
            p = native.Prog(env, code)
            dc_off = p.device_code(1)
            p.destroy()
        finally:
            os.environ.pop("EBPF_CC_NOHFWD", None)
        assert dc != dc_off
        if os.path.exists(LLVM_MC):
            out, err = _decode(dc)
            out_off, _ = _decode(dc_off)
            assert "invalid" not in err.lower()
            loads = lambda s: sum(1 for ln in s.splitlines() if "global_load" in ln)
            assert loads(out) == loads(out_off) - 1
    finally:
        m.destroy()


@pytest.mark.skipif(not os.path.exists(LLVM_MC), reason="llvm-mc not available")
def test_run_mask_code_shape(native, env):
    """General layout (C5): every straight run of hoisted packet loads starts with ONE extent
    compare into s[76:77] and issues its loads under it with no per-load compare; each use tests
    s[76:77] with a scalar AND-NOT before any vector compare.  EBPF_CC_NORUNMASK=1 restores the
    per-load compares (two per hoisted load), so that build has more VALU compares."""
    from generic_ebpf_amd import workloads
    lay = workloads.prog_c5()

    def decode(off):
        if off:
            os.environ["EBPF_CC_NORUNMASK"] = "1"
        try:
            p = native.Prog(env, lay.code)
            try:
                dc = p.device_code(0)
            finally:
                p.destroy()
        finally:
            os.environ.pop("EBPF_CC_NORUNMASK", None)
        out, err = _decode(dc)
        assert "invalid" not in err.lower(), err[:500]
        return [ln.strip() for ln in out.splitlines() if ln.strip()]

    on, off = decode(False), decode(True)
    assert "s_mov_b64 s[76:77], vcc" in on and "s_mov_b64 s[76:77], vcc" not in off
    assert "s_andn2_b64 s[48:49], exec, s[76:77]" in on
    # the run head: compare, mask, one saveexec, the hoisted loads back to back, restore
    k = on.index("s_mov_b64 s[76:77], vcc")
    assert on[k - 1].startswith("v_cmp_le_u32_e32 vcc,") and on[k + 1] == "s_and_saveexec_b64 s[60:61], vcc"
    j = k + 2
    while on[j].startswith("global_load_"):
        j += 1
    assert j - (k + 2) >= 2 and on[j] == "s_mov_b64 exec, s[60:61]", on[k:j + 1]
    cmps_on = sum(ln.startswith("v_cmp_") for ln in on)
    cmps_off = sum(ln.startswith("v_cmp_") for ln in off)
    assert cmps_on < cmps_off, (cmps_on, cmps_off)


@pytest.mark.skipif(not os.path.exists(LLVM_MC), reason="llvm-mc not available")
def test_hash_forwarding_register_alias_code(native, env):
    """The register that receives a hashtable probe's value bytes is not one a stack word was
    stored from: the fall-through exit of test_gpu_hash._forward_alias_program stays the
    constant the liveness pass proved (0x5bd1e995 + 3), so no code it removed is read."""
    import hashprogs
    from test_gpu_hash import _forward_alias_program
    lay = _forward_alias_program()
    m = hashprogs.NativeHash(native, env, 4, 8, 16, [])
    try:
        p = native.Prog(env, native.patch_relocs(lay.code, lay.relocs, [m.handle]))
        try:
            out, _ = _decode(p.device_code(1))
        finally:
            p.destroy()
    finally:
        m.destroy()
    assert "v_mov_b32_e32 v44, 0x5bd1e998" in out
    assert "v_mov_b64_e32 v[14:15], v[50:51]" not in out   # (r7: the key was stored from it)


def test_device_code_layouts(native, env):
    """ebpf_prog_device_code compiles layouts 0 (general kernels) and 1 (staged 64-B packets);
    2 (the window kernels, removed in round 5) and 3 (the path-sorted prefix, removed in round
    4) are rejected."""
    from generic_ebpf_amd import workloads
    p = native.Prog(env, workloads.prog_c5().code)
    try:
        for layout in (0, 1):
            assert len(p.device_code(layout)) > 0
        for layout in (2, 3, -1):
            with pytest.raises(native.EbpfError):
                p.device_code(layout)
    finally:
        p.destroy()


def test_no_vop3_reads_two_sgprs(native, env):
    """gfx950's VOP3 reads at most one SGPR; the encoder counts violations and the build fails
    on one (asm_cc.cpp enc::vop3).  Array maps whose value size is no inline constant (> 64)
    were the round-5 case: the compiled lookup (map base pair + value size) and LDS loads (LDS
    base + value size).  Both layouts compile, and the value size goes through a VGPR."""
    import stdprogs
    I = stdprogs.I
    code, rel = stdprogs.asm([
        I("ldxb", 5, 1, 3), I("and64_imm", 5, imm=15), I("stxw", 10, 5, -4),
        ("lddw_map", 1, 0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4), I("call", imm=0),
        I("ldxw", 4, 0, 100), I("mov64_reg", 3, 0), I("add64_reg", 3, 4), I("mov64_reg", 0, 3),
        I("exit")])
    for vs in (8, 200, 288):
        m = native.Map(env, 16, vs)
        p = native.Prog(env, native.patch_relocs(code, rel, [m.handle]))
        try:
            p.set_semantics(native.SEM_STANDARD)
            for layout in (0, 1):
                text, _ = _decode(p.device_code(layout))
                if vs > 64 and os.path.exists(LLVM_MC):
                    assert "v_mov_b32_e32 v46, 0x%x" % vs in text or \
                        "v_mov_b32_e32 v47, 0x%x" % vs in text, text
        finally:
            p.destroy()
            m.destroy()


def test_write_phasing_code(tmp_path):
    """Write phasing (gen_interp.py store_phased) is generated into the staged image with result
    slots only (m1): its shared group code reads the constant clock once (the window check) and
    marks slots in s98; the general (m0) and interpreter-staged (m3) images have none of it.  The
    kernels stay within the 102 addressable SGPRs, and the generator's dp_launch.wphase offset
    matches dprog.h."""
    import re
    root = os.path.join(os.path.dirname(__file__), "..", "generic-ebpf_amd", "csrc")
    out = [str(tmp_path / n) for n in ("m1.s", "m0.s", "m3.s", "h.h")]
    subprocess.run(["python3", os.path.join(root, "asm", "gen_interp.py")] + out, check=True)
    m1, m0, m3 = (open(p).read() for p in out[:3])
    assert m1.count("s_memrealtime") == 1
    assert "s_bitset1_b32 s98" in m1 and ".Lph_write_g:" in m1
    for img in (m0, m3):
        assert "s_memrealtime" not in img and "s98" not in img
    for img in (m1, m0, m3):
        assert all(int(x) <= 102 for x in re.findall(r"amdhsa_next_free_sgpr (\d+)", img))
    # the wide kernel: the staged compiled kernel's code with 96 VGPRs (16 result slots)
    assert "ebpf_jit_s64w:" in m1 and "ebpf_jit_s64w" not in m0 + m3
    kds = dict(re.findall(r"\.amdhsa_kernel (\w+)\n(?:.*\n)*?\s*\.amdhsa_next_free_vgpr (\d+)", m1))
    assert kds["ebpf_jit_s64w"] == "96" and kds["ebpf_jit_s64"] == "80"
    gen = open(os.path.join(root, "asm", "gen_interp.py")).read()
    off = int(re.search(r"WPHASE_OFF = (0x[0-9a-f]+)", gen).group(1), 16)
    hdr = open(os.path.join(root, "dprog.h")).read()
    assert "offsetof(dp_launch, wphase) == 0x%x" % off in hdr
