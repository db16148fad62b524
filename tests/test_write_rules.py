"""Edge cases of the round-6 write rules (include/ebpf_gpu.h, oracle/ebpf_oracle.h), each decided
from the program's own bytecode in the translator and, independently, in the oracle:

* a program "loops" when a backward jump is reachable from slot 0 — an unreachable one does not
  count, nor does JA -1 (it spins: EBPF_FAULT_LOOP), nor a conditional jump whose target lies
  before slot 0 (EBPF_FAULT_SLOT);
* a loop "reads its counters back" when a counter idiom's register is live after its STX on the
  slot graph, where a CALL reads only its helper's arguments (lookup r1-r2, update r1-r4);
* a loop-free program with more than 16 stores it reads back needs more overlay words than the
  lanes keep on chip: it runs on the portable interpreter with the overlay spilled to memory, up
  to 2,048 stores on one path (EOPNOTSUPP, honestly, at 2,049).

CPU: the oracle against hand-derived expectations.  GPU: the device against the oracle on every
variant (it must reach the same decisions)."""
import ctypes
import errno
import os

import numpy as np
import pytest

import pyoracle
import stdprogs

I = stdprogs.I
VARIANTS = [int(v) for v in os.environ.get("EBPF_TEST_VARIANTS", "0,1,2").split(",")]
F_SLOT, F_LOOP, F_MEM, F_WRITES = 4, 8, 3, 11
START = 14


def _hit_then(tail, nstores=20):
    """r0 = lookup(map 0, pkt[0] & 15); a miss exits 1; a hit stores nstores bytes into the value,
    then `tail` (items)"""
    return [I("ldxb", 6, 1, 0), I("and64_imm", 6, imm=15), I("stxw", 10, 6, -4), ("lddw_map", 1, 0),
            I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4), I("call", imm=0),
            I("jne_imm", 0, off="hit", imm=0), I("mov64_imm", 0, imm=1), I("exit"), ("label", "hit")] + \
        [I("stb", 0, 0, j % 8, j) for j in range(nstores)] + tail


def prog_unreachable_back():
    """20 stores, r0 = 7, exit; then a backward JA nothing reaches"""
    return stdprogs.asm(_hit_then([I("mov64_imm", 0, imm=7), I("exit"), ("label", "dead"),
                                   I("ja", off="dead")]))


def prog_ja_self():
    """20 stores, then JA -1 (spins)"""
    return stdprogs.asm(_hit_then([("label", "spin"), I("ja", off="spin")]))


def prog_cond_before_start():
    """20 stores, then a taken conditional jump to before slot 0"""
    code, rel = stdprogs.asm(_hit_then([I("jeq_reg", 0, 0, off=0), I("exit")]))
    b = bytearray(code)
    at = len(b) // 8 - 2
    b[8 * at + 2:8 * at + 4] = (-(at + 5) & 0xffff).to_bytes(2, "little")
    return bytes(b), rel


def prog_walk_counters(call):
    """A TLV walk from byte 14 ({type, len}, type 0 ends, next at + 2 + (len & 3)): per option,
    v = lookup(map 0, type & 63) (16-B values); counter idioms v[0] += len (register r4) and
    v[8] += 1 (register r5); then call == "update": map_update_elem(map 1, &key, &stack, r4) —
    the update reads r4 (its flags: EINVAL for a counter's size, no write), so r4 is live after its
    STX and the loop reads its counters back; call == "lookup": lookup(map 1, &key), which reads
    only r1-r2, so r4 is dead.  r0 = options seen."""
    items = [I("mov64_reg", 6, 1), I("mov64_reg", 7, 6), I("add64_imm", 7, imm=START),
             I("mov64_imm", 8, imm=0), I("stdw", 10, 0, -16, 0), ("label", "L"),
             I("ldxb", 2, 7, 0), I("jeq_imm", 2, imm=0, off="E"),
             I("mov64_reg", 4, 2), I("and64_imm", 4, imm=63), I("stxw", 10, 4, -4),
             ("lddw_map", 1, 0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4), I("call", imm=0),
             I("ldxb", 3, 7, 1), I("jeq_imm", 0, imm=0, off="N"),
             I("ldxdw", 4, 0, 0), I("add64_reg", 4, 3), I("stxdw", 0, 4, 0),
             I("ldxdw", 5, 0, 8), I("add64_imm", 5, imm=1), I("stxdw", 0, 5, 8),
             ("lddw_map", 1, 1), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4)]
    if call == "update":
        items += [I("mov64_reg", 3, 10), I("add64_imm", 3, imm=-16), I("call", imm=1)]
    else:
        items += [I("call", imm=0)]
    items += [I("ldxb", 3, 7, 1), ("label", "N"), I("add64_imm", 8, imm=1), I("and64_imm", 3, imm=3),
              I("add64_imm", 3, imm=2), I("add64_reg", 7, 3), I("ja", off="L"),
              ("label", "E"), I("mov64_reg", 0, 8), I("exit")]
    return stdprogs.asm(items)


def walk_packets(n, seed):
    """64-B packets whose TLV area holds 0..24 options of random types (1..255), short ones
    mostly"""
    g = np.random.default_rng(seed)
    pk = g.integers(0, 256, (n, 64), dtype=np.uint8)
    for i in range(n):
        at = START
        for _ in range(int(g.integers(0, 25))):
            if at + 1 >= 64:
                break
            pk[i, at] = int(g.integers(1, 256))
            ln = int(g.choice([0, 1, 2, 3], p=[0.7, 0.1, 0.1, 0.1]))
            pk[i, at + 1] = (int(pk[i, at + 1]) & ~3) | ln
            at += 2 + ln
        if at < 64:
            pk[i, at] = 0
    return pk


def expect_walk(pk, words_limited):
    """(r0, fault) per packet: options until type 0 (MEM when the walk runs off the packet); with
    the 32-word view, the option that brings a 17th distinct type (33rd and 34th words) faults
    WRITES at its first counter update"""
    ret, flt = [], []
    for p in pk:
        at, n, types, fault = START, 0, set(), 0
        while True:
            if at >= 64:
                fault = F_MEM
                break
            t = int(p[at])
            if t == 0:
                break
            if at + 1 >= 64:
                fault = F_MEM
                break
            if words_limited and (t & 63) not in types and len(types) == 16:
                fault = F_WRITES
                break
            types.add(t & 63)
            n += 1
            at += 2 + (int(p[at + 1]) & 3)
        ret.append(0 if fault else n)
        flt.append(fault)
    return np.array(ret, dtype=np.uint64), np.array(flt, dtype=np.uint8)


def _maps(seed, walk=False):
    g = np.random.default_rng(seed)
    if walk:
        return [(16, 64, g.integers(0, 256, 16 * 64, dtype=np.uint8).tobytes()),
                (8, 64, g.integers(0, 256, 8 * 64, dtype=np.uint8).tobytes())]
    return [(8, 16, g.integers(0, 256, 128, dtype=np.uint8).tobytes())]


def _oracle(code, rel, maps, pk, nthreads=4):
    op = pyoracle.OracleProgram(code, rel, maps, semantics=1)
    ret, flt, _, _ = op.run(pk.reshape(-1), len(pk), 64, nthreads=nthreads)
    return ret, flt, [op.map_bytes(k) for k in range(len(maps))]


def test_oracle_unreachable_backward_jump_is_no_loop():
    pk = walk_packets(200, 1)
    ret, flt, after = _oracle(*prog_unreachable_back(), _maps(2), pk)
    assert not flt.any() and (ret == 7).all()
    init = bytearray(_maps(2)[0][2])
    for p in pk:   # every key's value (map 0 holds them all): byte b last stored by the j < 20
        k = int(p[0]) & 15   # with j % 8 == b
        init[8 * k:8 * k + 8] = bytes([16, 17, 18, 19, 12, 13, 14, 15])
    assert after[0] == bytes(init)


def test_oracle_ja_self_is_a_spin_not_a_loop():
    """JA -1 after 20 stores: EBPF_FAULT_LOOP (the budget), not WRITES at the 17th store"""
    pk = walk_packets(16, 3)
    ret, flt, after = _oracle(*prog_ja_self(), _maps(4), pk, nthreads=8)
    assert (flt == F_LOOP).all() and after[0] == _maps(4)[0][2]


def test_oracle_jump_before_slot_0_is_no_loop():
    pk = walk_packets(100, 5)
    ret, flt, after = _oracle(*prog_cond_before_start(), _maps(6), pk)
    assert (flt == F_SLOT).all() and after[0] == _maps(6)[0][2]


@pytest.mark.parametrize("call,limited", [("update", True), ("lookup", False)])
def test_oracle_helper_arguments_decide_read_back(call, limited):
    pk = walk_packets(3000, 7)
    want, wf = expect_walk(pk, limited)
    ret, flt, _ = _oracle(*prog_walk_counters(call), _maps(8, walk=True), pk)
    np.testing.assert_array_equal(flt, wf)
    np.testing.assert_array_equal(ret, want)
    assert ((wf == F_WRITES).any()) == limited


class _Info(ctypes.Structure):
    _fields_ = [("nslots", ctypes.c_uint32), ("nentries", ctypes.c_uint32),
                ("nmaps", ctypes.c_uint32), ("max_stack", ctypes.c_uint32)]


def _readback_stores(n):
    """reference semantics, loop-free: a hit stores n bytes into the value, then reads it back"""
    import valueprogs as vp
    from generic_ebpf_amd import isa, layout
    nodes = vp._lookup(isa.Insn, layout.LdDw, layout.MapRef, layout.Branch)
    nodes += [isa.Insn("stb", 0, 0, j % 8, j) for j in range(n)]
    nodes += [isa.Insn("ldxdw", 8, 0, 0), isa.Insn("mov_imm", 0, imm=0), isa.Insn("mov64_reg", 0, 8),
              isa.Insn("exit")]
    return layout.assemble(nodes)


@pytest.mark.parametrize("n,err", [(16, 0), (17, 0), (2048, 0), (2049, errno.EOPNOTSUPP)])
def test_loop_free_read_back_overlay_bound(native, env, n, err):
    lay = _readback_stores(n)
    m = native.Map(env, 16, 8)
    p = native.Prog(env, lay.patched([m.handle]))
    try:
        assert native.lib().ebpf_prog_device_info(p.ptr, ctypes.byref(_Info())) == err
    finally:
        p.destroy()
        m.destroy()


def test_oracle_loop_free_read_back_of_16_stores():
    import valueprogs as vp
    lay = _readback_stores(16)
    pk = vp.packets(500, 9)
    init = _maps(10)[0][2]
    ret, flt, _, _ = pyoracle.OracleProgram(lay.code, lay.relocs, [(8, 16, init)]).run(pk, 500, 64)
    assert not flt.any()
    assert (ret == int.from_bytes(bytes([8, 9, 10, 11, 12, 13, 14, 15]), "little")).all()


# ---------------------------------------------------------------- GPU: the same decisions


def _device(gpu, env, code, rel, maps, pk, variant, std=True):
    ms = []
    for vs, me, d in maps:
        m = gpu.Map(env, me, vs)
        m.fill(d)
        ms.append(m)
    p = gpu.Prog(env, gpu.patch_relocs(code, rel, [m.handle for m in ms]))
    try:
        if std:
            p.set_semantics(gpu.SEM_STANDARD)
        gpu.set_variant(variant)
        ret, flt, _ = p.run_batch(np.ascontiguousarray(pk.reshape(-1)), len(pk), 64)
        after = [b"".join(m.lookup(k)[1] for k in range(m.max_entries)) for m in ms]
        return ret, flt, after
    finally:
        gpu.set_variant(0)
        p.destroy()
        for m in ms:
            m.destroy()


CASES = {
    "unreachable_back": (prog_unreachable_back, False),
    "ja_self": (prog_ja_self, False),
    "cond_before_start": (prog_cond_before_start, False),
    "walk_update": (lambda: prog_walk_counters("update"), True),
    "walk_lookup": (lambda: prog_walk_counters("lookup"), True),
}


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("case", sorted(CASES))
def test_device_write_rules_vs_oracle(gpu, env, variant, case):
    mk, walk = CASES[case]
    code, rel = mk()
    pk = walk_packets(64 if case == "ja_self" else 4099, 11)
    maps = _maps(12, walk=walk)
    want, wf, wafter = _oracle(code, rel, maps, pk, nthreads=8)
    ret, flt, after = _device(gpu, env, code, rel, maps, pk, variant)
    np.testing.assert_array_equal(flt, wf)
    np.testing.assert_array_equal(ret, want)
    assert after == wafter
