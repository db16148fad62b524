"""Programs that store into map values through a lookup result (ebpf_interpreter.c:343-366
writing through the pointer array_map_lookup_elem returns, ebpf_map_array.c:115-124), and pure
Python restatements of the batch semantics for them (oracle/ebpf_oracle.h "Stores into map
values in a batch"):

* a packet's loads see its own stores; other packets see the batch-start maps;
* stores land after the batch in packet order, byte by byte (last writer wins);
* counter updates (LDX; ADD/SUB; STX on one address, and XADD under standard semantics) land as
  additions when aligned to their width within the values;
* a packet that faults leaves no write behind but its counter updates.

Every expectation here is worked out from those rules by hand, not by the implementations under
test."""
import numpy as np

import stdprogs

R0, R1, R2, R3, R4, R5, R6, R7, R8, R9, R10 = range(11)
NKEYS = 16
MISS = 0xdead
LDX = {1: "ldxb", 2: "ldxh", 4: "ldxw", 8: "ldxdw"}
STX = {1: "stxb", 2: "stxh", 4: "stxw", 8: "stxdw"}
MASK = {1: 0xff, 2: 0xffff, 4: 0xffffffff, 8: 0xffffffffffffffff}


def _nodes():
    from generic_ebpf_amd import isa, layout
    return isa.Insn, layout.LdDw, layout.MapRef, layout.Branch, layout.assemble


def _lookup(I, LdDw, MapRef, Branch):
    """r6 = pkt[0] & 15 as the key at r10 - 4, r7 = pkt[1] (the addend), r0 = lookup, miss:
    r0 = MISS and exit."""
    return [I("ldxb", R6, R1, 0), I("and_imm", R6, imm=NKEYS - 1), I("stxw", R10, R6, -4),
            I("ldxb", R7, R1, 1),
            I("mov_imm", R9, imm=0), I("mov64_reg", R9, R1),               # r9 = the packet
            LdDw(R1, MapRef(0)),
            I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
            I("call", imm=0),
            Branch(I("jeq_imm", R0, imm=0), [I("mov_imm", R0, imm=MISS), I("exit")])]


def prog_counter(width=8, off=0, alu="add64_reg", reload=False, fault=False):
    """The counter idiom on map[key] at byte `off`: X = [v + off]; X (alu) r7; [v + off] = X.
    r0 = X, or (reload) a fresh load of the value's first 8 bytes after the store (the packet's
    own update read back).  fault: then r0 = 7 / (pkt[2] & 1) (even pkt[2]: DIV_ZERO after the
    update, which still lands)."""
    I, LdDw, MapRef, Branch, assemble = _nodes()
    n = _lookup(I, LdDw, MapRef, Branch)
    a = {"add64_reg": I("add64_reg", R8, R7), "add32_reg": I("add_reg", R8, R7),
         "sub64_reg": I("sub64_reg", R8, R7), "add64_imm": I("add64_imm", R8, imm=-3),
         "mov64_reg": I("mov64_reg", R8, R7)}[alu]
    n += [I(LDX[width], R8, R0, off), a, I(STX[width], R0, R8, off)]
    if reload:
        n += [I("ldxdw", R8, R0, 0)]
    if fault:
        n += [I("ldxb", R5, R9, 2), I("and_imm", R5, imm=1), I("mov_imm", R4, imm=7),
              I("div64_reg", R4, R5)]
    n += [I("mov_imm", R0, imm=0), I("mov64_reg", R0, R8), I("exit")]
    return assemble(n)


def prog_store(width=4, off=2, fault=False):
    """A plain store of pkt[8 .. 8 + width) into map[key] at byte `off`, then r0 = the value's
    first 8 bytes (read back: the snapshot with the packet's own bytes over it)."""
    I, LdDw, MapRef, Branch, assemble = _nodes()
    n = _lookup(I, LdDw, MapRef, Branch)
    n += [I(LDX[width], R8, R9, 8), I(STX[width], R0, R8, off), I("ldxdw", R8, R0, 0)]
    if fault:
        n += [I("ldxb", R5, R9, 2), I("and_imm", R5, imm=1), I("mov_imm", R4, imm=7),
              I("div64_reg", R4, R5)]
    n += [I("mov_imm", R0, imm=0), I("mov64_reg", R0, R8), I("exit")]
    return assemble(n)


def prog_mixed():
    """pkt[3] odd: the counter idiom (+pkt[1]) on the value's first 8 bytes; even: a plain store
    of pkt[8..16) there.  r0 = 0."""
    I, LdDw, MapRef, Branch, assemble = _nodes()
    n = _lookup(I, LdDw, MapRef, Branch)
    n += [I("ldxb", R5, R9, 3),
          Branch(I("jset_imm", R5, imm=1), [I("ldxdw", R8, R0, 0), I("add64_reg", R8, R7),
                                            I("stxdw", R0, R8, 0), I("mov_imm", R0, imm=0),
                                            I("exit")]),
          I("ldxdw", R8, R9, 8), I("stxdw", R0, R8, 0), I("mov_imm", R0, imm=0), I("exit")]
    return assemble(n)


def prog_xadd(width=8, fetch=False):
    """Standard semantics: *(u64 / u32 *)(v + 0) += pkt[1] by XADD (imm 1: fetch the old value
    into r7).  r0 = r7 (the addend, or the old value)."""
    I = stdprogs.I
    op = 0xdb if width == 8 else 0xc3
    items = [I("ldxb", 6, 1, 0), I("and_imm", 6, imm=NKEYS - 1), I("stxw", 10, 6, -4),
             I("ldxb", 7, 1, 1),
             ("lddw_map", 1, 0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4), I("call", imm=0),
             I("jne_imm", 0, off="hit", imm=0), I("mov64_imm", 0, imm=MISS), I("exit"),
             ("label", "hit"),
             (op, 0, 7, 0, 1 if fetch else 0),
             I("mov64_reg", 0, 7), I("exit")]
    return stdprogs.asm(items)


# ---------------------------------------------------------------- the rules, in Python


def packets(n, seed):
    from generic_ebpf_amd import workloads
    return workloads.packets_random(n, 64, seed=seed)


def _get(buf, at, w):
    return int.from_bytes(bytes(buf[at:at + w]), "little")


def _put(buf, at, w, v):
    buf[at:at + w] = (v & MASK[w]).to_bytes(w, "little")


def expect_counter(pk, init, vs, width=8, off=0, alu="add64_reg", reload=False, fault=False):
    """(r0 per packet, faults, map bytes after the batch) of prog_counter.  The counter update is
    an addition when off + key * vs is a multiple of the width, else a plain store of the value
    the packet computed."""
    snap = bytearray(init)
    final = bytearray(init)
    ret, flt, last_plain = [], [], {}
    for i, p in enumerate(pk):
        k, y = int(p[0]) & (NKEYS - 1), int(p[1])
        at = k * vs + off
        L = _get(snap, at, width)
        if alu == "add64_reg":
            X = L + y
        elif alu == "add32_reg":
            X = (L + y) & 0xffffffff
        elif alu == "sub64_reg":
            X = L - y
        elif alu == "add64_imm":
            X = L - 3
        else:                       # the reference's MOV64 adds
            X = L + y
        X &= MASK[8]
        delta = (X - L) & MASK[width]
        aligned = at % width == 0
        faulted = fault and not (int(p[2]) & 1)
        if aligned:
            _put(final, at, width, _get(final, at, width) + delta)
        elif not faulted:
            last_plain[at] = (i, X)
        own = bytearray(snap)
        _put(own, at, width, X)
        r = _get(own, k * vs, 8) if reload else X
        ret.append(0 if faulted else r)
        flt.append(2 if faulted else 0)
    for at, (i, X) in sorted(last_plain.items()):
        _put(final, at, width, X)
    return np.array(ret, dtype=np.uint64), np.array(flt, dtype=np.uint8), bytes(final)


def expect_store(pk, init, vs, width=4, off=2, fault=False):
    snap = bytearray(init)
    final = bytearray(init)
    ret, flt = [], []
    for p in pk:
        k = int(p[0]) & (NKEYS - 1)
        faulted = fault and not (int(p[2]) & 1)
        own = bytearray(snap)
        own[k * vs + off:k * vs + off + width] = p[8:8 + width].tobytes()
        if not faulted:
            final[k * vs + off:k * vs + off + width] = p[8:8 + width].tobytes()
        ret.append(0 if faulted else _get(own, k * vs, 8))
        flt.append(2 if faulted else 0)
    return np.array(ret, dtype=np.uint64), np.array(flt, dtype=np.uint8), bytes(final)


def expect_mixed(pk, init):
    """Packet order decides: a plain store replaces the word, a counter update adds to it."""
    final = bytearray(init)
    for p in pk:
        at = (int(p[0]) & (NKEYS - 1)) * 8
        if int(p[3]) & 1:
            _put(final, at, 8, _get(final, at, 8) + int(p[1]))
        else:
            final[at:at + 8] = p[8:16].tobytes()
    return bytes(final)


def expect_xadd(pk, init, width=8, fetch=False):
    snap = bytearray(init)
    final = bytearray(init)
    ret = []
    for p in pk:
        k, y = int(p[0]) & (NKEYS - 1), int(p[1])
        _put(final, 8 * k, width, _get(final, 8 * k, width) + y)
        ret.append(_get(snap, 8 * k, width) if fetch else y)
    return np.array(ret, dtype=np.uint64), bytes(final)


def sequential_counter_map(pk, init, vs, width=8, off=0, alu="add64_reg"):
    """The reference's own run, one packet after the other (every update at once)."""
    m = bytearray(init)
    for p in pk:
        k, y = int(p[0]) & (NKEYS - 1), int(p[1])
        at = k * vs + off
        L = _get(m, at, width)
        X = {"add64_reg": L + y, "add32_reg": (L + y) & 0xffffffff, "sub64_reg": L - y,
             "add64_imm": L - 3, "mov64_reg": L + y}[alu]
        _put(m, at, width, X)
    return bytes(m)
