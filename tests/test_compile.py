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
