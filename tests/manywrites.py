"""Loop-free programs under the reference's semantics that make many map writes on one path
(VERDICT round 5, item 1): the reference runs every store and every map_update_elem a program
reaches (ebpf_interpreter.c:343-366 stores, :282-284 CALL -> ebpf_map.c:101-108 ->
ebpf_map_array.c:198-211), so a loop-free program has no write limit on the device either
(include/ebpf_gpu.h "Map writes in a device batch": the log is sized by the longest path).

Every program here is laid out by the stepping-aware assembler (generic-ebpf_amd/layout.py), keeps
its results value-derived (never a pointer) and reads no map value after its first write, so the
packet never needs its own stores back (no overlay: the count of stores is not bounded by it).

* prog_probe(): one lookup, 20 STDW into the value, r0 = 7 (the round-5 probe);
* prog_stores(n, vs): one lookup of key pkt[0] & kmask, n ST / STX of 1..8 bytes at offsets that
  walk the value, r0 = the packet-derived register the stores used;
* prog_updates(n, kmask): n map_update_elem calls, key (pkt[1] & kmask) * 64 + j, value from an
  evolving register, flags EBPF_NOEXIST on every seventh call (EEXIST: not a write), r0 = the
  return codes folded together;
* prog_mixed(n_st, n_up): both on one path."""
import numpy as np

MISS = 0x5a5a
KEYS_PER_PKT = 64


def _nodes():
    from generic_ebpf_amd import isa, layout
    return isa.Insn, layout.LdDw, layout.MapRef, layout.Branch, layout.assemble


def _ptr(I, r, base, off):
    """r = base + off (the reference's MOV64 adds: clear with a 32-bit MOV first)"""
    return [I("mov_imm", r, imm=0), I("mov64_reg", r, base), I("add64_imm", r, imm=off)]


def _lookup(I, LdDw, MapRef, Branch, kmask):
    """r9 = packet; key pkt[0] & kmask at r10 - 4; r0 = lookup(map 0); a miss exits with MISS"""
    return [I("mov_imm", 9, imm=0), I("mov64_reg", 9, 1),
            I("ldxb", 6, 1, 0), I("and_imm", 6, imm=kmask), I("stxw", 10, 6, -4),
            LdDw(1, MapRef(0))] + _ptr(I, 2, 10, -4) + [
            I("call", imm=0),
            Branch(I("jeq_imm", 0, imm=0), [I("mov_imm", 0, imm=MISS), I("exit")])]


def _stores(I, n, vs):
    """n stores through r0 (the lookup result); r8 (from the packet) evolves between them"""
    out = [I("ldxdw", 8, 9, 8)]
    widths = [8, 4, 2, 1, 8, 1, 4, 2]
    for j in range(n):
        w = min(widths[j % len(widths)], vs)
        off = (j * 7) % (vs - w + 1)
        if j % 5 == 3:
            out.append(I({1: "stb", 2: "sth", 4: "stw", 8: "stdw"}[w], 0, 0, off,
                         (0x1234567 * (j + 1)) & 0x7fffffff if j % 2 else -(j + 2)))
        else:
            out.append(I({1: "stxb", 2: "stxh", 4: "stxw", 8: "stxdw"}[w], 0, 8, off))
        out += [I("mul64_imm", 8, imm=5), I("add64_imm", 8, imm=j + 1)]
    return out


def _updates(I, LdDw, MapRef, n, kmask):
    """n map_update_elem(map 0, &key, &value, flags) calls; r7 folds the return codes"""
    out = [I("mov_imm", 7, imm=0), I("ldxdw", 8, 9, 16),
           I("ldxb", 6, 9, 1), I("and_imm", 6, imm=kmask), I("lsh64_imm", 6, imm=6)]
    for j in range(n):
        out += [I("mov_imm", 5, imm=0), I("mov64_reg", 5, 6), I("add64_imm", 5, imm=j % KEYS_PER_PKT),
                I("stxw", 10, 5, -4), I("stxdw", 10, 8, -16),
                LdDw(1, MapRef(0))] + _ptr(I, 2, 10, -4) + _ptr(I, 3, 10, -16) + [
                I("mov_imm", 4, imm=1 if j % 7 == 6 else 0),
                I("call", imm=1),
                I("lsh64_imm", 0, imm=j % 56), I("xor64_reg", 7, 0),
                I("mul64_imm", 8, imm=3), I("add64_imm", 8, imm=j + 11)]
    return out


def _exit_with(I, r):
    return [I("mov_imm", 0, imm=0), I("mov64_reg", 0, r), I("exit")]


def prog_probe():
    """The round-5 probe: one lookup, 20 STDW into the value, r0 = 7."""
    I, LdDw, MapRef, Branch, assemble = _nodes()
    n = _lookup(I, LdDw, MapRef, Branch, 15)
    n += [I("stdw", 0, 0, 0, 100 + j) for j in range(20)]
    n += [I("mov_imm", 0, imm=7), I("exit")]
    return assemble(n)


def prog_stores(count, vs, kmask=15):
    I, LdDw, MapRef, Branch, assemble = _nodes()
    return assemble(_lookup(I, LdDw, MapRef, Branch, kmask) + _stores(I, count, vs) + _exit_with(I, 8))


def prog_readback(count, vs, kmask=15):
    """prog_stores, then the value read back (its first 8 bytes, and its last 8): the packet sees
    its own stores, so the device keeps an overlay of 2 words per store on the path — past
    DP_OVL_MAX (16 stores) spilled to memory on the portable interpreter.  r0 = the two words
    xor the evolving register."""
    I, LdDw, MapRef, Branch, assemble = _nodes()
    n = _lookup(I, LdDw, MapRef, Branch, kmask) + _stores(I, count, vs)
    n += [I("ldxdw", 7, 0, 0), I("xor64_reg", 8, 7), I("ldxdw", 7, 0, vs - 8), I("xor64_reg", 8, 7)]
    return assemble(n + _exit_with(I, 8))


def prog_updates(count, kmask=3):
    """map 0: (kmask + 1) * 64 entries of 8 bytes"""
    I, LdDw, MapRef, Branch, assemble = _nodes()
    n = [I("mov_imm", 9, imm=0), I("mov64_reg", 9, 1)] + _updates(I, LdDw, MapRef, count, kmask)
    return assemble(n + _exit_with(I, 7))


def prog_mixed(n_stores, n_updates, vs=8, kmask=3):
    """a lookup's n_stores stores, then n_updates calls on the same map (keys from pkt[1])"""
    I, LdDw, MapRef, Branch, assemble = _nodes()
    n = _lookup(I, LdDw, MapRef, Branch, kmask) + _stores(I, n_stores, vs)
    n += [I("mov_imm", 4, imm=0), I("mov64_reg", 4, 8)]   # (r8 is reused by the updates)
    n += _updates(I, LdDw, MapRef, n_updates, kmask)
    n += [I("xor64_reg", 7, 4)]
    return assemble(n + _exit_with(I, 7))


def packets(n, seed):
    from generic_ebpf_amd import workloads
    return workloads.packets_random(n, 64, seed=seed)


def distinct_key_packets(n, seed):
    """packets whose key bytes (0 and 1) are distinct: no two packets write the same key (the
    batch then equals the reference's one-after-the-other run)"""
    pk = packets(n, seed)
    assert n <= 256
    pk[:, 0] = np.arange(n, dtype=np.uint8)
    pk[:, 1] = np.arange(n, dtype=np.uint8)
    return pk


# name -> (builder, value_size, map entries)
CASES = {
    "probe20": (prog_probe, 8, 16),
    "stores17": (lambda: prog_stores(17, 16), 16, 16),
    "stores40": (lambda: prog_stores(40, 72), 72, 16),
    "stores120": (lambda: prog_stores(120, 200), 200, 16),
    "updates17": (lambda: prog_updates(17), 8, 4 * KEYS_PER_PKT),
    "updates40": (lambda: prog_updates(40), 8, 4 * KEYS_PER_PKT),
    "mixed17_17": (lambda: prog_mixed(17, 17), 8, 4 * KEYS_PER_PKT),
}

# stores read back (the overlay past DP_OVL_MAX: spilled, portable interpreter)
READBACK = {
    "readback16": (lambda: prog_readback(16, 16), 16, 16),
    "readback17": (lambda: prog_readback(17, 16), 16, 16),
    "readback40": (lambda: prog_readback(40, 72), 72, 16),
    "readback120": (lambda: prog_readback(120, 200), 200, 16),
}


def distinct_case(name, n):
    """the case with a key space wide enough for n packets of distinct keys"""
    if name.startswith("probe"):
        return prog_probe(), 8, 16            # (the probe masks its key to 15)
    if name.startswith("stores"):
        cnt, vs = {"stores17": (17, 16), "stores40": (40, 72), "stores120": (120, 200)}[name]
        return prog_stores(cnt, vs, kmask=255), vs, 256
    if name.startswith("updates"):
        return prog_updates(int(name[7:]), kmask=255), 8, 256 * KEYS_PER_PKT
    return prog_mixed(17, 17, kmask=255), 8, 256 * KEYS_PER_PKT
