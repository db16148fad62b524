"""Map writes inside loops (standard semantics; include/ebpf_gpu.h "Map writes in a device
batch", "Stores into map values"): option walks over a TLV area of the packet — the shape
§8(f)'s standard-semantics row exists for — that count, update and store per option, and the
Python restatement of the batch rules each is checked against:

* counter updates (XADD, or the LDX / ADD / STX idiom whose register is dead afterwards) into an
  array only counter updates change are additions, uncapped;
* successful map_update_elem / map_delete_elem calls and plain stores into map values are
  logged writes: 16 per packet, the 17th faults EBPF_FAULT_WRITES (11) and the packet's logged
  writes do not land;
* every packet reads the batch-start maps plus its own stores.

The TLV area: options from byte 14 on, {u8 type, u8 len, data...}, type 0 ends the walk, the next
option at + 2 + (len & 3); an option that runs past the packet's end faults MEM on its load, as
the reference's bounds check would (here: the oracle's checked mode).  Every expectation below is
worked out from those rules, not by the implementations under test."""
import numpy as np

import stdprogs

I = stdprogs.I
NKEYS = 16
START = 14
FAULT_MEM, FAULT_WRITES = 3, 11


def _walk_head():
    """r6 = packet, r7 = cursor (packet + START), r8 = options seen; loop head "L": r2 = type, r3
    = len (the walk ends at type 0)."""
    return [I("mov64_reg", 6, 1), I("mov64_reg", 7, 6), I("add64_imm", 7, imm=START),
            I("mov64_imm", 8, imm=0), ("label", "L"),
            I("ldxb", 2, 7, 0), I("jeq_imm", 2, imm=0, off="E"), I("ldxb", 3, 7, 1)]


def _walk_tail(extra_exit=()):
    """r8 += 1; cursor += 2 + (len & 3); back to L.  "E": r0 = r8 (+ extra), exit."""
    return [I("add64_imm", 8, imm=1), I("and64_imm", 3, imm=3), I("add64_imm", 3, imm=2),
            I("add64_reg", 7, 3), I("ja", off="L"), ("label", "E"), I("mov64_reg", 0, 8)] + \
        list(extra_exit) + [I("exit")]


def _key_lookup(k=0, nkeys=NKEYS):
    """stack[-4] = type & (nkeys - 1); r0 = lookup(map k, &stack[-4]); a miss skips to "N"."""
    return [I("mov64_reg", 4, 2), I("and64_imm", 4, imm=nkeys - 1), I("stxw", 10, 4, -4),
            ("lddw_map", 1, k), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4),
            I("call", imm=0), I("ldxb", 3, 7, 1), I("jeq_imm", 0, imm=0, off="N")]


def prog_xadd_counters():
    """Per option: counters[type & 15].packets += 1 and .bytes += len (XADD, 8-byte words of a
    16-B value).  r0 = options."""
    return stdprogs.asm(_walk_head() + _key_lookup() + [
        I("mov64_imm", 9, imm=1), (0xdb, 0, 9, 0, 0), (0xdb, 0, 3, 8, 0), ("label", "N")] +
        _walk_tail())


def prog_idiom_counters(live=False):
    """Per option: counters[type & 15] += len through LDX / ADD / STX.  live=True: the loaded
    register feeds r0 afterwards (the packet reads its own additions back: refused in a loop)."""
    body = [I("ldxdw", 5, 0, 0), I("add64_reg", 5, 3), I("stxdw", 0, 5, 0)]
    if live:
        body.append(I("xor64_reg", 8, 5))
    return stdprogs.asm(_walk_head() + _key_lookup() + body + [("label", "N")] + _walk_tail())


def prog_updates():
    """Per option: map_update_elem(map 0, &(type & 15), &option data (8 bytes at cursor + 2),
    ANY); r9 ^= its return code << option number.  r0 = options | r9 << 8."""
    return stdprogs.asm(_walk_head() + [
        I("mov64_reg", 4, 2), I("and64_imm", 4, imm=NKEYS - 1), I("stxw", 10, 4, -4),
        ("lddw_map", 1, 0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4),
        I("mov64_reg", 3, 7), I("add64_imm", 3, imm=2), I("mov64_imm", 4, imm=0),
        I("call", imm=1), I("lsh64_reg", 0, 8), I("xor64_reg", 9, 0), I("ldxb", 3, 7, 1)] +
        _walk_tail([I("lsh64_imm", 9, imm=8), I("or64_reg", 0, 9)]))


def prog_stores():
    """Per option: values[type & 15] bytes 4..8 = the option's 4 data bytes (a plain store), then
    r9 += the value's first 8 bytes as the packet sees them (its own stores over the batch-start
    map).  r0 = options ^ r9."""
    return stdprogs.asm(_walk_head() + _key_lookup() + [
        I("ldxw", 5, 7, 2), I("stxw", 0, 5, 4), I("ldxdw", 5, 0, 0), I("add64_reg", 9, 5),
        ("label", "N")] + _walk_tail([I("xor64_reg", 0, 9)]))


def prog_limiter(thresh=3, nkeys=NKEYS):
    """The per-option rate limiter (round 6): c = counters[type & (nkeys - 1)] (8-B values); c += 1;
    counters[type & 15] = c; c > thresh: r0 = 0x1000 + the options before this one, exit — the
    idiom's register read back, so the packet sees the batch-start count plus its own additions.
    A walk that ends: r0 = options."""
    return stdprogs.asm(_walk_head() + _key_lookup(nkeys=nkeys) + [
        I("ldxdw", 5, 0, 0), I("add64_imm", 5, imm=1), I("stxdw", 0, 5, 0),
        I("jgt_imm", 5, imm=thresh, off="D"), ("label", "N")] + _walk_tail() +
        [("label", "D"), I("mov64_imm", 0, imm=0x1000), I("add64_reg", 0, 8), I("exit")])


FETCH_KEYS = 64


def prog_xadd_fetch():
    """Per option, on counters[type & 63] (16-B values): old0 = XADD | FETCH word 0 += len,
    r9 ^= old0; old1 = XADD | FETCH word 1 += 1, r9 += old1 (values as the packet sees them:
    the batch start plus its own additions).  r0 = options ^ r9.  Two words an option: a walk
    over more than 16 distinct types passes the 32 words of the packet's view and faults WRITES
    at the counter update that needs one more (the additions before it land)."""
    return stdprogs.asm(_walk_head() + _key_lookup(nkeys=FETCH_KEYS) + [
        I("mov64_reg", 5, 3), (0xdb, 0, 5, 0, 1), I("xor64_reg", 9, 5),
        I("mov64_imm", 5, imm=1), (0xdb, 0, 5, 8, 1), I("add64_reg", 9, 5), ("label", "N")] +
        _walk_tail([I("xor64_reg", 0, 9)]))


def prog_xadd_then_load():
    """XADD (no fetch) into counters[type & 15], then a plain load of the same word, r9 ^= it.
    r0 = options ^ r9.  Into an array (device atomics): a read-back the device does not provide
    for in a loop (EOPNOTSUPP); into a hashtable (counted records): allowed."""
    return stdprogs.asm(_walk_head() + _key_lookup() + [
        I("mov64_imm", 5, imm=1), (0xdb, 0, 5, 0, 0), I("ldxdw", 5, 0, 0), I("xor64_reg", 9, 5),
        ("label", "N")] + _walk_tail([I("xor64_reg", 0, 9)]))


def packets(n, seed, max_opts=24):
    """64-B packets whose TLV area holds 0..max_opts options, short ones mostly (len & 3 = 0 in
    70 %): most walks end at a type-0 option, some run off the end of the packet (MEM)."""
    g = np.random.default_rng(seed)
    pk = g.integers(0, 256, (n, 64), dtype=np.uint8)
    for i in range(n):
        k = int(g.integers(0, max_opts + 1))
        at = START
        for _ in range(k):
            if at + 1 >= 64:
                break
            pk[i, at] = int(g.integers(1, 256))
            ln = int(g.choice([0, 1, 2, 3], p=[0.7, 0.1, 0.1, 0.1]))
            pk[i, at + 1] = (int(pk[i, at + 1]) & ~3) | ln
            at += 2 + ln
        if at < 64:
            pk[i, at] = 0
    return pk


def _u(b, at, w):
    return int.from_bytes(bytes(b[at:at + w]), "little")


def expect(kind, pk, init, vs, present=None):
    """(r0, fault, map bytes after the batch) of prog_<kind> over pk, step by step in each
    program's own order of loads, checks and writes.  present: the map is a hashtable holding
    only these keys (a lookup of another misses and skips the option's body), and its counter
    updates are records, counted with the logged writes (16 a packet, the 17th faults WRITES
    before it happens; the additions before it land)."""
    m = bytearray(init)
    M64 = 2**64 - 1
    counted = present is not None
    ret, flt = [], []
    for p in pk:
        own = bytearray(init)   # the packet's view (its own stores over the batch start)
        adds, writes, fault = [], [], 0
        words = set()           # (limiter, xadd_fetch) the 8-byte words of the packet's view

        def full():             # the next logged write would be the 17th
            return len(writes) + (len(adds) if counted else 0) == 16
        n, r9, at, r0 = 0, 0, START, None
        while True:
            if at >= 64:                      # ldxb type
                fault = FAULT_MEM
                break
            t = int(p[at])
            if t == 0:
                break
            k = (t & (NKEYS - 1)) * vs
            if kind == "updates":
                if at + 2 + vs > 64:          # the value, region-checked before the call counts
                    fault = FAULT_MEM
                    break
                if len(writes) == 16:
                    fault = FAULT_WRITES
                    break
                writes.append((k, bytes(p[at + 2:at + 2 + vs])))
            if at + 1 >= 64:                  # ldxb len
                fault = FAULT_MEM
                break
            ln = int(p[at + 1])
            if present is not None and (t & (NKEYS - 1)) not in present:
                n += 1                        # the lookup missed: on to the next option
                at += 2 + (ln & 3)
                continue
            if kind in ("limiter", "xadd_fetch"):
                k = (t & (FETCH_KEYS - 1 if kind == "xadd_fetch" else NKEYS - 1)) * vs
                ups = [(k, 1)] if kind == "limiter" else [(k, ln), (k + 8, 1)]
                for j, (w, add) in enumerate(ups):
                    if (w not in words and len(words) == 32) or (counted and full()):
                        fault = FAULT_WRITES
                        break
                    words.add(w)
                    old = _u(own, w, 8)
                    own[w:w + 8] = ((old + add) & M64).to_bytes(8, "little")
                    adds.append((w, add))
                    r9 = r9 ^ old if j == 0 else (r9 + old) & M64
                if fault:
                    break
                if kind == "limiter" and (_u(own, k, 8)) > 3:
                    r0 = 0x1000 + n
                    break
            if kind in ("xadd", "idiom", "xadd_load"):
                ups = {"xadd": [(k, 1), (k + 8, ln)], "idiom": [(k, ln)], "xadd_load": [(k, 1)]}[kind]
                for w, add in ups:
                    if counted and full():
                        fault = FAULT_WRITES
                        break
                    own[w:w + 8] = ((_u(own, w, 8) + add) & M64).to_bytes(8, "little")
                    adds.append((w, add))
                if fault:
                    break
                if kind == "xadd_load":
                    r9 ^= _u(own, k, 8)
            elif kind == "stores":
                if at + 6 > 64:               # ldxw data
                    fault = FAULT_MEM
                    break
                if len(writes) == 16:
                    fault = FAULT_WRITES
                    break
                writes.append((k + 4, bytes(p[at + 2:at + 6])))
                own[k + 4:k + 8] = bytes(p[at + 2:at + 6])
                r9 = (r9 + _u(own, k, 8)) & M64
            n += 1
            at += 2 + (ln & 3)
        for k, a in adds:                     # atomic additions land even when the packet faults
            m[k:k + 8] = ((_u(m, k, 8) + a) & M64).to_bytes(8, "little")
        if not fault:
            for k, b in writes:
                m[k:k + len(b)] = b
        if r0 is None:
            r0 = n ^ r9 if kind in ("stores", "xadd_fetch", "xadd_load") else n
        ret.append(0 if fault else r0)
        flt.append(fault)
    return np.array(ret, dtype=np.uint64), np.array(flt, dtype=np.uint8), bytes(m)


def walk_options(p):
    """The options a walk of packet p visits before it ends (or runs off the packet)."""
    out, at = [], START
    while at + 1 < 64 and int(p[at]) != 0:
        out.append(at)
        at += 2 + (int(p[at + 1]) & 3)
    return out


def prog_mixed_counter_store():
    """A counter update and a plain store into the same array inside the loop (refused: the
    counter would need the ordered host replay, whose log a loop cannot bound)."""
    return stdprogs.asm(_walk_head() + _key_lookup() + [
        I("mov64_imm", 9, imm=1), (0xdb, 0, 9, 0, 0), I("stxb", 0, 3, 4), ("label", "N")] +
        _walk_tail())


VALUE_SIZE = {"xadd": 16, "idiom": 8, "updates": 8, "stores": 8, "limiter": 8, "xadd_fetch": 16,
              "xadd_load": 8}
MAP_KEYS = {"xadd_fetch": FETCH_KEYS}
PROGS = {"xadd": prog_xadd_counters, "idiom": prog_idiom_counters, "updates": prog_updates,
         "stores": prog_stores, "limiter": prog_limiter, "xadd_fetch": prog_xadd_fetch}


def initial_map(kind, seed):
    """the batch-start map of a kind: random bytes; the limiter's counts 0..2"""
    g = np.random.default_rng(seed)
    keys = MAP_KEYS.get(kind, NKEYS)
    if kind == "limiter":
        return g.integers(0, 3, keys, dtype=np.uint64).tobytes()
    return g.integers(0, 256, keys * VALUE_SIZE[kind], dtype=np.uint8).tobytes()


# Counter updates into a hashtable inside loops (round 6): the same walks over a hashtable of u32
# keys that holds 12 of the 16 types (the other 4 miss); every counter update is a record, counted
# with the logged writes
HASH_PRESENT = frozenset(range(12))
HASH_PROGS = {"xadd": prog_xadd_counters, "idiom": prog_idiom_counters, "limiter": prog_limiter,
              "xadd_load": prog_xadd_then_load}


def hash_items(init, vs):
    """[(u32 key bytes, value bytes)] of the present keys, values from the array image init"""
    return [(k.to_bytes(4, "little"), bytes(init[k * vs:(k + 1) * vs])) for k in sorted(HASH_PRESENT)]


def hash_image(items, vs):
    """the array image (NKEYS * vs bytes, absent keys zero) of [(key, value)]"""
    m = bytearray(NKEYS * vs)
    for key, val in items:
        k = int.from_bytes(key, "little")
        m[k * vs:(k + 1) * vs] = val
    return bytes(m)
