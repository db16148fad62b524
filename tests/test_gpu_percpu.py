"""Percpu array and percpu hashtable maps in device batches.  A batch behaves like the caller's
own loop over ebpf_prog_run on the CPU it is submitted from, so lookups see that CPU's copy
(ebpf_map_array.c percpu lookup -> ebpf_curcpu(); ebpf_map_hashtable.c HASH_ELEM_CURCPU_VALUE).
The test pins the submitting thread to two different CPUs, writes per-CPU values with the
program-side update API (which writes the current CPU's copy), and checks each batch against the
oracle given that CPU's values, and against ebpf_prog_run on the same CPU."""
import ctypes
import os
import struct

import numpy as np
import pytest

import hashprogs
import pyoracle

pytestmark = pytest.mark.gpu


def _two_cpus():
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < 2:
        pytest.skip("needs two CPUs")
    return cpus[0], cpus[-1]


def _array_prog():
    from generic_ebpf_amd import isa
    from generic_ebpf_amd.layout import Branch, LdDw, MapRef, assemble
    I = isa.Insn
    # key = packet byte 0 & 15; r0 = value or 0xdead
    return assemble([I("ldxb", 6, 1, 0), I("and_imm", 6, imm=15), I("stxw", 10, 6, -4),
                     LdDw(1, MapRef(0)), I("mov_imm", 2, imm=0), I("mov64_reg", 2, 10),
                     I("add64_imm", 2, imm=-4), I("call", imm=0),
                     Branch(I("jeq_imm", 0, imm=0), [I("mov_imm", 0, imm=0xdead), I("exit")]),
                     I("ldxdw", 0, 0, 0), I("exit")])


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_percpu_array_uses_the_submitting_cpu(gpu, env, variant):
    c1, c2 = _two_cpus()
    saved = os.sched_getaffinity(0)
    m = gpu.Map(env, 16, 8, type=gpu.MAP_TYPE_PERCPU_ARRAY)
    lay = _array_prog()
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle]))
    L = gpu.lib()
    pk = np.random.default_rng(1).integers(0, 256, (4096, 64), dtype=np.uint8)
    try:
        gpu.set_variant(variant)
        vals = {}
        for c in (c1, c2):
            os.sched_setaffinity(0, {c})
            v = np.arange(16, dtype=np.uint64) * 1000 + c
            for k in range(16):   # ebpf_map_update_elem: this CPU's copy only
                kk, vv = ctypes.c_uint32(k), ctypes.c_uint64(int(v[k]))
                assert L.ebpf_map_update_elem(m.ptr, ctypes.byref(kk), ctypes.byref(vv), 0) == 0
            vals[c] = v
        for c in (c1, c2, c1):
            os.sched_setaffinity(0, {c})
            got, gf, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1).copy()), len(pk), 64)
            want, wf, _, _ = pyoracle.OracleProgram(
                lay.code, lay.relocs, [(8, 16, vals[c].tobytes())]).run(pk.reshape(-1), len(pk), 64)
            assert not gf.any() and np.array_equal(want, got), c
            assert p.run_cpu(pk[0].tobytes())[0] == int(got[0])
    finally:
        os.sched_setaffinity(0, saved)
        gpu.set_variant(0)
        p.destroy()
        m.destroy()


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_percpu_hashtable_uses_the_submitting_cpu(gpu, env, variant):
    c1, c2 = _two_cpus()
    saved = os.sched_getaffinity(0)
    rng = np.random.default_rng(2)
    items, keys = hashprogs.make_table(rng, 4, 8, 40)
    m = hashprogs.NativeHash(gpu, env, 4, 8, 64, items, type=3)   # from user: every CPU
    lay = hashprogs.lookup_program(4, "stack", 0)
    p = gpu.Prog(env, gpu.patch_relocs(lay.code, lay.relocs, [m.handle]))
    L = gpu.lib()
    pk = hashprogs.packets_with_keys(rng, 4096, 64, keys, 0, 4)
    try:
        gpu.set_variant(variant)
        per = {}
        for c in (c1, c2):
            os.sched_setaffinity(0, {c})
            cur = dict(items)
            for k, _ in items[:20]:   # program-side update: this CPU's copy
                v = struct.pack("<Q", c * 7919 + k[0])
                assert L.ebpf_map_update_elem(m.ptr, ctypes.create_string_buffer(k, 4),
                                              ctypes.create_string_buffer(v, 8), 0) == 0
                cur[k] = v
            per[c] = cur
        for c in (c2, c1):
            os.sched_setaffinity(0, {c})
            got, gf, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1).copy()), len(pk), 64)
            want, wf, _ = hashprogs.oracle(lay, [pyoracle.HashSpec(4, 8, list(per[c].items()))],
                                           pk.reshape(-1), len(pk), 64)
            assert not gf.any() and np.array_equal(want, got), c
    finally:
        os.sched_setaffinity(0, saved)
        gpu.set_variant(0)
        p.destroy()
        m.destroy()
