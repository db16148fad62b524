"""Synthetic workloads for the BASELINE.json configs.

  C2  8-insn ALU-only program over 64-B random packets
  C3  64-insn L2/L3 parse + classify (VALE-BPF style) over structured 64-B packets
  C4  C3 + one array-map lookup per packet (array map, 256 x 8 B)
  C5  256-insn branch-heavy filter over mixed 64-1500 B packets (offsets array)
  C4H C3 + one hashtable lookup per packet keyed by the IPv4 destination address (a 1M-entry
      route/flow table, half the packets' addresses present) — the §8(f) hashtable row

Programs are laid out with the stepping-aware assembler (layout.py) so the reference
interpreter executes them as written; "N-insn" = N executed instructions on the main path,
JA stride resets included.  Packets come from a seeded generator, so every config is
reproducible bit for bit.  Everything here is input generation; nothing executes eBPF.
"""
import numpy as np

from . import isa
from .layout import Branch, LdDw, MapRef, assemble

I = isa.Insn
R0, R1, R2, R3, R4, R5, R6, R7, R8, R9, R10 = range(11)


def _exit_with(v):
    return [I("mov_imm", R0, imm=v), I("exit")]


# --------------------------------------------------------------------------- packets

def _rng(seed):
    return np.random.default_rng(seed)


def packets_random(n, size=64, seed=2):
    """Uniform random bytes, fixed stride (C2)."""
    return _rng(seed).integers(0, 256, size=(n, size), dtype=np.uint8)


def packets_l2l3(n, size=64, seed=3):
    """Structured Ethernet/IPv4/IPv6/ARP frames (C3/C4), fixed stride ``size`` bytes.
    ethertype 0x0800 80 %, 0x86DD 10 %, 0x0806 10 %; IPv4 proto TCP/UDP/ICMP 60/30/10 %."""
    g = _rng(seed)
    p = g.integers(0, 256, size=(n, size), dtype=np.uint8)
    u = g.random(n)
    et = np.where(u < 0.8, 0x0800, np.where(u < 0.9, 0x86DD, 0x0806)).astype(np.uint16)
    p[:, 12] = et >> 8
    p[:, 13] = et & 0xff
    v4 = et == 0x0800
    p[v4, 14] = 0x45
    tot = size - 14
    p[v4, 16] = tot >> 8
    p[v4, 17] = tot & 0xff
    pu = g.random(n)
    proto = np.where(pu < 0.6, 6, np.where(pu < 0.9, 17, 1)).astype(np.uint8)
    p[v4, 23] = proto[v4]
    ttl = g.integers(0, 256, n).astype(np.uint8)
    ttl[g.random(n) < 0.02] = 1
    p[v4, 22] = ttl[v4]
    ports = np.array([80, 443, 53, 22, 8080, 123], dtype=np.uint16)
    dp = np.where(g.random(n) < 0.7, ports[g.integers(0, len(ports), n)],
                  g.integers(0, 65536, n)).astype(np.uint16)
    p[v4, 36] = dp[v4] >> 8
    p[v4, 37] = dp[v4] & 0xff
    ten = g.random(n) < 0.1            # 10.0.0.0/16 destinations
    sel = v4 & ten
    p[sel, 30] = 10
    p[sel, 31] = 0
    v6 = et == 0x86DD
    p[v6, 14] = 0x60
    p[v6, 20] = np.where(g.random(int(v6.sum())) < 0.7, 6, 17)
    return p


IMIX = ((64, 7), (576, 4), (1500, 1))


def packets_imix(n, seed=5):
    """Mixed-size IPv4 frames (C5): sizes 64/576/1500 in IMIX 7:4:1, each packet starts on a
    64-B boundary.  Returns (data uint8[total], offsets uint64[n+1], sizes uint32[n])."""
    g = _rng(seed)
    sizes_tab = np.array([s for s, _ in IMIX], dtype=np.uint32)
    w = np.array([c for _, c in IMIX], dtype=np.float64)
    sizes = sizes_tab[g.choice(len(IMIX), size=n, p=w / w.sum())]
    padded = ((sizes.astype(np.uint64) + 63) // 64) * 64
    offsets = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(padded, out=offsets[1:])
    data = g.integers(0, 256, size=int(offsets[-1]), dtype=np.uint8)
    base = offsets[:-1].astype(np.int64)
    data[base + 12] = 0x08
    data[base + 13] = 0x00
    data[base + 14] = 0x45
    tot = sizes - 14
    data[base + 16] = (tot >> 8).astype(np.uint8)
    data[base + 17] = (tot & 0xff).astype(np.uint8)
    return data, offsets, sizes


IMIX_BLOCK = 1 << 16


def packets_imix_range(lo, hi, seed=5):
    """Packets [lo, hi) of an endless IMIX stream generated in blocks of IMIX_BLOCK packets
    (block b from seed (seed, b)), so that any shard of a batch is reproducible on its own:
    the shards of [0, n) concatenate to the packets of [0, n) whatever the shard count.
    Returns (data, offsets rebased to 0, sizes) as packets_imix."""
    parts, sizes = [], []
    for b in range(lo // IMIX_BLOCK, (hi + IMIX_BLOCK - 1) // IMIX_BLOCK):
        d, o, s = packets_imix(IMIX_BLOCK, seed=(seed, b))
        a = max(lo, b * IMIX_BLOCK) - b * IMIX_BLOCK
        e = min(hi, (b + 1) * IMIX_BLOCK) - b * IMIX_BLOCK
        parts.append(d[int(o[a]):int(o[e])])
        sizes.append(s[a:e])
    sizes = np.concatenate(sizes) if sizes else np.zeros(0, np.uint32)
    padded = ((sizes.astype(np.uint64) + 63) // 64) * 64
    offsets = np.zeros(len(sizes) + 1, dtype=np.uint64)
    np.cumsum(padded, out=offsets[1:])
    data = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return data, offsets, sizes


# --------------------------------------------------------------------------- programs

def prog_c2():
    """8 executed instructions: two 8-byte loads, ALU mixing, EXIT (29 slots)."""
    nodes = [
        I("ldxdw", R0, R1, 0), I("ldxdw", R2, R1, 8), I("xor64_reg", R0, R2),
        I("mul64_imm", R0, imm=0x1E3779B1), I("rsh64_imm", R0, imm=29),
        I("xor64_reg", R0, R2), I("and64_imm", R0, imm=0xff), I("exit"),
    ]
    return assemble(nodes)


def _classify_program(with_lookup, pad, reset, hash_key=False, counter=False):
    """Ethernet → IPv4 (TCP/UDP main path) | IPv6 | ICMP | other.  The flow hash and the
    verdict arithmetic run first and the ACL decisions sit at the end of the path, so nearly
    every IPv4 packet executes the full main path (no early-exit shortcut)."""
    ipv6 = [I("ldxb", R3, R1, 20), I("ldxb", R7, R1, 21),
            I("ldxw", R4, R1, 22), I("ldxw", R5, R1, 38), I("ldxw", R6, R1, 54),
            I("xor64_reg", R4, R5), I("xor64_reg", R4, R6), I("mul64_imm", R4, imm=0x1E3779B1)]
    ipv6 += [I("xor64_imm", R4, imm=0x3c6ef372 + 97 * k) if k % 2 else
             I("mul64_imm", R4, imm=0x27d4eb2d) for k in range(24)]
    ipv6 += [Branch(I("jle_imm", R7, imm=1), _exit_with(1)),
             I("rsh64_imm", R4, imm=17), I("and_imm", R4, imm=7), I("add_imm", R4, imm=8),
             I("mov_reg", R0, R4), I("exit")]
    icmp = [I("ldxb", R6, R1, 34), I("mov_imm", R0, imm=4),
            Branch(I("jne_imm", R6, imm=8), [I("exit")]), I("mov_imm", R0, imm=5), I("exit")]
    head = [
        I("ldxh", R2, R1, 12), I("be", R2, imm=16),
        Branch(I("jeq_imm", R2, imm=0x86DD), ipv6),
        Branch(I("jne_imm", R2, imm=0x0800), _exit_with(2)),
        I("ldxb", R3, R1, 23),
        Branch(I("jeq_imm", R3, imm=1), icmp),
        I("ldxw", R4, R1, 26), I("be", R4, imm=32),
        I("ldxw", R5, R1, 30), I("be", R5, imm=32),
        I("ldxh", R7, R1, 34), I("be", R7, imm=16),
        I("ldxh", R9, R1, 36), I("be", R9, imm=16),
        # flow hash over (src, dst, sport, dport, proto)
        I("mov_imm", R8, imm=0), I("or64_reg", R8, R4), I("lsh64_imm", R8, imm=32),
        I("or64_reg", R8, R5), I("mul64_imm", R8, imm=0x1E3779B1),
        I("mov_reg", R6, R9), I("lsh64_imm", R6, imm=16), I("or64_reg", R6, R7),
        I("lsh64_imm", R6, imm=8), I("or64_reg", R6, R3),
        I("xor64_reg", R8, R6), I("mov_reg", R6, R8), I("rsh64_imm", R6, imm=31),
        I("xor64_reg", R8, R6), I("mul64_imm", R8, imm=0x2545F491),
        I("mov_reg", R6, R8), I("rsh64_imm", R6, imm=29), I("xor64_reg", R8, R6),
    ]
    pads = [I("xor64_imm", R8, imm=0x5bd1e995 ^ (k * 0x1f1f)) if k % 2 == 0 else
            I("mul64_imm", R8, imm=0x27d4eb2d) for k in range(pad)]
    lookup = []
    if with_lookup and hash_key:   # key: the destination address (r5, host order)
        lookup = [
            I("stxw", R10, R5, -4),
            LdDw(R1, MapRef(0)),
            I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
            I("call", imm=0),
            Branch(I("jeq_imm", R0, imm=0), _exit_with(2)),
            I("ldxdw", R6, R0, 0), I("xor64_reg", R8, R6),
        ]
    elif with_lookup:
        lookup = [
            I("mov_reg", R6, R9), I("and_imm", R6, imm=0xff),
            I("stxw", R10, R6, -4),
            LdDw(R1, MapRef(0)),
            I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
            I("call", imm=0),
            Branch(I("jeq_imm", R0, imm=0), _exit_with(2)),
            I("ldxdw", R6, R0, 0), I("xor64_reg", R8, R6),
        ]
        if counter:   # counters[key] += 1: the per-port packet counter (map 1)
            lookup += [
                LdDw(R1, MapRef(1)),
                I("mov_imm", R2, imm=0), I("mov64_reg", R2, R10), I("add64_imm", R2, imm=-4),
                I("call", imm=0),
                Branch(I("jeq_imm", R0, imm=0), _exit_with(2)),
                I("ldxdw", R6, R0, 0), I("add64_imm", R6, imm=1), I("stxdw", R0, R6, 0),
            ]
    verdict = [
        I("mov_reg", R0, R8), I("rsh_imm", R0, imm=13), I("and_imm", R0, imm=7),
        I("add_imm", R0, imm=8),
        # ACL at the end of the path: ssh → drop, 10.0/16 → redirect,
        # ephemeral destination port → pass, else the hash-derived class 8..15
        I("mov_reg", R6, R5),
        I("and_imm", R6, imm=isa.s32(0xffff0000)),
        Branch(I("jeq_imm", R9, imm=22), _exit_with(1)),
        Branch(I("jeq_imm", R6, imm=0x0a000000), _exit_with(3)),
        Branch(I("jgt_imm", R9, imm=49151), _exit_with(2)),
        I("exit"),
    ]
    return assemble(head + pads + lookup + verdict, reset_stride=reset)


def _fit(with_lookup, target, exact=True, hash_key=False, counter=False):
    """Smallest padding whose main path executes ``target`` instructions (JA resets included)."""
    for reset in (8, 7, 9, 6, 10):
        for pad in range(0, 64):
            lay = _classify_program(with_lookup, pad, reset, hash_key, counter)
            if lay.main_path_steps == target or (not exact and lay.main_path_steps >= target):
                return lay
            if lay.main_path_steps > target:
                break
    raise ValueError("cannot hit %d executed instructions" % target)


def prog_c3():
    """L2/L3 parse + classify; exactly 64 executed instructions on the IPv4 TCP/UDP path."""
    return _fit(False, 64)


def prog_c4():
    """C3 + one array-map lookup keyed by the low byte of the destination port: the C3 main
    path (64) plus STXW key, LDDW map, r2 = r10-4 (3 insns), CALL, NULL check, LDXDW value and
    XOR into the hash — 75 executed instructions on the main path."""
    return _fit(True, 75, exact=False)


def prog_c4c():
    """C4 + a per-key packet counter: after the array lookup, counters[key] += 1 through a second
    array map's lookup result (LDDW, r2 = r10-4, CALL, NULL check, LDXDW / ADD64 1 / STXDW — the
    counter update the device runs as an atomic addition, ebpf_gpu.h "Stores into map values")."""
    return _fit(True, 84, exact=False, counter=True)


def prog_c4h():
    """C3 + one hashtable lookup keyed by the IPv4 destination address (STXW key, LDDW map,
    r2 = r10-4, CALL, NULL check, LDXDW value, XOR): the C4 path shape on a hashtable."""
    return _fit(True, 73, exact=False, hash_key=True)


C4H_ENTRIES = 1 << 20


def c4h_table(seed=12, entries=C4H_ENTRIES):
    """(universe u32[2*entries] distinct addresses, keys u8[entries,4], values u8[entries,8]):
    the map holds the first half of the universe; keys are the addresses in host order (the
    program's BE32 of the packet bytes), stored little-endian like the STXW that builds them."""
    g = _rng(seed)
    u = np.unique(g.integers(0, 2**32, int(entries * 2.2), dtype=np.uint64))
    u = u[g.permutation(len(u))][:2 * entries].astype(np.uint32)
    keys = u[:entries].view(np.uint8).reshape(-1, 4)
    values = g.integers(0, 2**63, entries, dtype=np.uint64).view(np.uint8).reshape(-1, 8)
    return u, keys, values


def packets_c4h(n, universe, seed=4):
    """C3/C4 packets whose IPv4 destination address is drawn from ``universe``."""
    p = packets_l2l3(n, 64, seed)
    a = universe[_rng(seed + 100).integers(0, len(universe), n)]
    for b in range(4):
        p[:, 30 + b] = (a >> (24 - 8 * b)) & 0xff
    return p


def c4_map_values(seed=11, entries=256):
    return _rng(seed).integers(0, 2**63, size=entries, dtype=np.uint64)


def _c5_nodes(seed, body, depth=2):
    g = _rng(seed)

    def leaf(limit):
        n = []
        acc = R8
        for k in range(body):
            if k % 4 == 0:
                off = int(g.integers(18, limit - 8))
                op = ("ldxb", "ldxh", "ldxw", "ldxdw")[int(g.integers(0, 4))]
                n += [I(op, R6, R1, off), I("xor64_reg", acc, R6)]
            elif k % 24 == 23:
                # rare data-dependent early exit (byte == 0x5a): more divergence, no duplication
                off = int(g.integers(18, limit - 1))
                n += [I("ldxb", R6, R1, off),
                      Branch(I("jeq_imm", R6, imm=0x5a), _exit_with(int(g.integers(0, 16))))]
            else:
                c = int(g.integers(1, 1 << 30))
                n.append(I(("mul64_imm", "add64_imm", "xor64_imm")[k % 3], acc, imm=c))
        n += [I("mov_reg", R0, acc), I("rsh_imm", R0, imm=7), I("and_imm", R0, imm=15),
              I("exit")]
        return n

    def tree(limit, depth):
        if depth == 0:
            return leaf(limit)
        off = int(g.integers(18, limit - 1))
        bit = int(g.integers(0, 8))
        test = [I("ldxb", R6, R1, off), I("rsh_imm", R6, imm=bit), I("and_imm", R6, imm=1),
                I("xor64_reg", R8, R6)]
        taken = tree(limit, depth - 1)
        return test + [Branch(I("jne_imm", R6, imm=0), taken)] + tree(limit, depth - 1)

    head = [I("ldxh", R7, R1, 16), I("be", R7, imm=16), I("mov_imm", R8, imm=0x1234)]
    return head + [Branch(I("jgt_imm", R7, imm=1000), tree(1500, depth)),
                   Branch(I("jgt_imm", R7, imm=100), tree(576, depth))] + tree(64, depth)


def _meldsim_nodes(seed, body, exits=True, table_alu=True, ops=("mul64_reg", "add64_reg", "xor64_reg"),
                   tests=2, split=True):
    """Probe (round 5): what melding C5's isomorphic leaves could gain, as an optimistic bound.
    C5's shape — the 3-way size split, then per class two data-dependent bit tests — but the
    tests do not branch: they pick a per-lane row of an LDS-resident operand table (array map 0,
    16 rows of 4-B words, row = class * 4 + the two test bits), and ONE leaf per class runs for
    all its lanes with every ALU immediate and early-exit verdict read from the lane's row
    (LDXMAP: an LDS read, then the register form of the operation), as a melding compiler would
    emit them.  Packet loads stay at the class's constant offsets and widths (a melded load
    would add a per-lane offset and a width mask: a few VALU each, not counted here)."""
    g = _rng(seed)
    limits = (64, 576, 1500)
    cols = []   # per word: values[class][variant]

    def col(draw):
        cols.append([[draw(c) for _ in range(4)] for c in range(3)])
        return 4 * (len(cols) - 1)

    plan = []
    for k in range(body):
        if k % 4 == 0:
            offs = [int(g.integers(18, limits[c] - 8)) for c in range(3)]
            op = ("ldxb", "ldxh", "ldxw", "ldxdw")[int(g.integers(0, 4))]
            plan.append(("ld", op, offs))
        elif k % 24 == 23 and exits:
            offs = [int(g.integers(18, limits[c] - 1)) for c in range(3)]
            plan.append(("exit", offs, col(lambda c: int(g.integers(0, 16)))))
        else:
            plan.append(("alu", ops[k % len(ops)], col(lambda c: int(g.integers(1, 1 << 30)))))

    def leaf(cls):
        n, acc = [], R8
        for k, x in enumerate(plan):
            if x[0] == "ld":
                n += [I(x[1], R6, R7, x[2][cls]), I("xor64_reg", acc, R6)]
            elif x[0] == "exit":
                n += [I("ldxb", R6, R7, x[1][cls]), I("jne_imm", R6, imm=0x5a, off="c%dk%d" % (cls, k)),
                      I("ldxw", R0, R0, x[2]), I("exit"), ("label", "c%dk%d" % (cls, k))]
            elif table_alu:
                n += [I("ldxw", R4, R0, x[2]), I(x[1], acc, R4)]
            else:
                n += [I(x[1].replace("_reg", "_imm"), acc, imm=cols[x[2] // 4][cls][0])]
        n += [I("mov_reg", R0, acc), I("rsh_imm", R0, imm=7), I("and_imm", R0, imm=15), I("exit")]
        return n

    def cls_tree(cls):
        t = [I("mov64_reg", R7, R1), I("mov64_imm", R5, imm=4 * cls)]
        for j in range(tests):   # two tests: bit j of the row
            t += [I("ldxb", R6, R7, int(g.integers(18, limits[cls] - 1))),
                  I("rsh_imm", R6, imm=int(g.integers(0, 8))), I("and_imm", R6, imm=1),
                  I("xor64_reg", R8, R6), I("lsh64_imm", R6, imm=j), I("or64_reg", R5, R6)]
        t += [I("stxw", R10, R5, -4), LdDw(R1, MapRef(0)), I("mov64_reg", R2, R10),
              I("add64_imm", R2, imm=-4), I("call", imm=0)]
        return t + leaf(cls)

    head = [I("ldxh", R7, R1, 16), I("be", R7, imm=16), I("mov64_imm", R8, imm=0x1234)]
    if not split:
        return head + cls_tree(0), cols
    out = head + [I("jgt_imm", R7, imm=1000, off="C2"), I("jgt_imm", R7, imm=100, off="C1")] + \
        cls_tree(0) + [("label", "C1")] + cls_tree(1) + [("label", "C2")] + cls_tree(2)
    return out, cols


def prog_c5meldsim(seed=7, body=96):
    return _asm_std(_meldsim_nodes(seed, body)[0])


def c5meldsim_table(seed=7, body=96):
    """prog_c5meldsim's operand table: 16 rows x one 4-B word per column (row class * 4 + v)."""
    cols = _meldsim_nodes(seed, body)[1]
    t = np.zeros((16, len(cols)), dtype=np.uint32)
    for ci, vals in enumerate(cols):
        for c in range(3):
            for v in range(4):
                t[4 * c + v, ci] = vals[c][v]
    return t


def prog_c5d(depth, body=96, seed=7):
    """C5's generator with a given leaf body and tree depth (the probes' same-size baselines)."""
    return assemble(_c5_nodes(seed, body, depth))


def prog_c5(seed=7, target=256, depth=2):
    """Branch-heavy filter over IMIX packets: a 3-way split on the IPv4 total length, then a
    depth-2 tree of data-dependent tests on payload bytes (within the size class) whose leaves
    are straight segments of loads + mixing with rare data-dependent early exits.  The leaf
    length is fitted so the main (all-not-taken) path executes ``target`` instructions."""
    for body in range(target // 2, target):
        lay = assemble(_c5_nodes(seed, body, depth))
        if lay.main_path_steps >= target:
            return lay
    raise ValueError("cannot fit C5")


_LIT_BODY = [I("ldxh", R2, R1, 12), I("be", R2, imm=16), I("ldxw", R3, R1, 26),
             I("be", R3, imm=32), I("xor64_reg", R2, R3), I("mul64_imm", R2, imm=0x1E3779B1),
             I("ldxw", R4, R1, 30), I("xor64_reg", R2, R4)]
_LIT_MORE = [I("ldxh", R5, R1, 34), I("xor64_reg", R2, R5), I("ldxh", R5, R1, 36),
             I("add64_reg", R2, R5), I("mul64_imm", R2, imm=0x27D4EB2D), I("ldxb", R5, R1, 23),
             I("xor64_reg", R2, R5), I("ldxw", R5, R1, 40), I("xor64_reg", R2, R5),
             I("rsh64_imm", R2, imm=7), I("ldxdw", R5, R1, 48), I("add64_reg", R2, R5)]
_LIT_TAIL = [I("and64_imm", R2, imm=0xff), I("mov_reg", R0, R2)]


def prog_literal(nslots):
    """The literal N-slot variant of a classifier: the program written as N
    consecutive slots, of which the reference's cumulative stepping (slot i at step p goes to
    i + p) executes only slots 0, 1, 3, 6, 10, ... — 11 of 64, 23 of 256.  The executed slots
    hold header loads (offsets < 64) and mixing ending in EXIT; the others a never-executed
    filler."""
    execd = []
    i, p = 0, 1
    while i < nslots:
        execd.append(i)
        i, p = i + p, p + 1
    body = _LIT_BODY + (_LIT_MORE if len(execd) > 11 else [])
    n = len(execd) - 1 - len(_LIT_TAIL)
    body = (body * ((n + len(body) - 1) // len(body)))[:n] + _LIT_TAIL + [I("exit")]
    filler = I("mov_imm", R9, imm=0x5eed).encode()
    code = [filler] * nslots
    for s_, ins in zip(execd, body):
        code[s_] = ins.encode()
    from .layout import Layout
    return Layout(b"".join(code), [], len(execd), nslots)


def _asm_std(items):
    """Standard-semantics code (pc += off + 1) from Insn, LdDw (two slots; a MapRef value is a
    relocation) and ("label", name) items; a jump's ``off`` may name a label."""
    at, k = {}, 0
    for it in items:
        if isinstance(it, tuple):
            at[it[1]] = k
        else:
            k += 2 if isinstance(it, LdDw) else 1
    code, relocs, k = [], [], 0
    for it in items:
        if isinstance(it, tuple):
            continue
        if isinstance(it, LdDw):
            v = 0 if isinstance(it.value, MapRef) else it.value & 0xffffffffffffffff
            if isinstance(it.value, MapRef):
                relocs.append((k, it.value.index))
            code += [isa.encode(0x18, it.dst, 0, 0, isa.s32(v)), isa.encode(0, 0, 0, 0, isa.s32(v >> 32))]
            k += 2
            continue
        off = at[it.off] - (k + 1) if isinstance(it.off, str) else it.off
        code.append(isa.encode(it.op, it.dst, it.src, off, it.imm))
        k += 1
    from .layout import Layout
    return Layout(b"".join(code), relocs, None, len(code))


def packets_ipv4opt(n, seed=6):
    """C3L packets: the C3 frames (packets_l2l3) with IPv4 header lengths of 5 words (half) or
    6-12 (options, the rest of the header random bytes), and a correct header checksum on 90 %
    of the IPv4 frames (the others keep random checksum bytes)."""
    p = packets_l2l3(n, 64, seed)
    g = _rng(seed + 1)
    v4 = (p[:, 12] == 0x08) & (p[:, 13] == 0x00)
    ihl = np.where(g.random(n) < 0.5, 5, g.integers(6, 13, n)).astype(np.uint8)
    p[v4, 14] = 0x40 | ihl[v4]
    fix = v4 & (g.random(n) < 0.9)
    for h in range(5, 13):
        sel = np.nonzero(fix & (ihl == h))[0]
        if len(sel) == 0:
            continue
        hdr = p[sel, 14:14 + 4 * h].astype(np.uint32)
        hdr[:, 10:12] = 0
        s = ((hdr[:, 0::2] << 8) | hdr[:, 1::2]).sum(axis=1)
        while (s >> 16).any():
            s = (s & 0xffff) + (s >> 16)
        c = (~s) & 0xffff
        p[sel, 24] = (c >> 8).astype(np.uint8)
        p[sel, 25] = (c & 0xff).astype(np.uint8)
    return p


def prog_c3l():
    """IPv4 header check with a bounded loop (standard semantics, ebpf_prog_set_semantics): not
    IPv4 -> 0; IHL outside 5..12 -> 3; a loop over the IHL 32-bit header words (LDXW through a
    cursor, 5 instructions per word, one backward jump per word) sums them, four folds reduce the
    sum to the 16-bit one's-complement sum; != 0xffff (bad checksum) -> 2; TTL <= 1 -> 4; else
    16 + (protocol & 15).  Accepted frames execute 34 + 5 x IHL instructions (59-94)."""
    L = "label"
    items = [I("mov64_reg", R6, R1), I("mov64_imm", R0, imm=0), I("ldxh", R2, R6, 12),
             I("jne_imm", R2, imm=0x0008, off="out"), I("ldxb", R3, R6, 14),
             I("and64_imm", R3, imm=15), I("jlt_imm", R3, imm=5, off="mal"),
             I("jgt_imm", R3, imm=12, off="mal"), I("mov64_imm", R4, imm=0),
             I("mov64_reg", R5, R6), I("add64_imm", R5, imm=14), (L, "word"),
             I("ldxw", R7, R5, 0), I("add64_reg", R4, R7), I("add64_imm", R5, imm=4),
             I("sub64_imm", R3, imm=1), I("jne_imm", R3, imm=0, off="word"),
             I("mov64_reg", R7, R4), I("rsh64_imm", R7, imm=32), I("mov_reg", R4, R4),
             I("add64_reg", R4, R7)]
    for _ in range(3):
        items += [I("mov64_reg", R7, R4), I("rsh64_imm", R7, imm=16), I("and64_imm", R4, imm=0xffff),
                  I("add64_reg", R4, R7)]
    items += [I("jne_imm", R4, imm=0xffff, off="bad"), I("ldxb", R2, R6, 22),
              I("jle_imm", R2, imm=1, off="ttl"), I("ldxb", R0, R6, 23), I("and64_imm", R0, imm=15),
              I("add64_imm", R0, imm=16), I("exit"),
              (L, "out"), I("exit"),
              (L, "mal"), I("mov64_imm", R0, imm=3), I("exit"),
              (L, "bad"), I("mov64_imm", R0, imm=2), I("exit"),
              (L, "ttl"), I("mov64_imm", R0, imm=4), I("exit")]
    return _asm_std(items)


def c3l_expected(p):
    """numpy restatement of prog_c3l's verdict per packet (tests; input generation aside,
    nothing here executes eBPF)."""
    v4 = (p[:, 12] == 0x08) & (p[:, 13] == 0x00)
    ihl = (p[:, 14] & 15).astype(np.int64)
    out = np.zeros(len(p), dtype=np.uint64)
    mal = v4 & ((ihl < 5) | (ihl > 12))
    out[mal] = 3
    ok = v4 & ~mal
    for h in range(5, 13):
        sel = np.nonzero(ok & (ihl == h))[0]
        hdr = p[sel, 14:14 + 4 * h].astype(np.uint64)
        s = ((hdr[:, 0::2] << 8) | hdr[:, 1::2]).sum(axis=1)
        while (s >> 16).any():
            s = (s & 0xffff) + (s >> 16)
        good = s == 0xffff
        ttl = p[sel, 22]
        v = np.where(~good, 2, np.where(ttl <= 1, 4, 16 + (p[sel, 23] & 15).astype(np.uint64)))
        out[sel] = v
    return out


def prog_c0():
    """Floor: MOV r0, 2; EXIT (2 executed instructions) — measures staging + retirement."""
    return assemble([I("mov_imm", R0, imm=2), I("exit")])


def prog_chain(kind, n=200):
    """Microbenchmarks: n straight-line instructions of one kind, then EXIT.
    kind "nop": LE r0, 64 (a no-op in the reference); "alu": ADD64 r0, imm."""
    body = [I("mov_imm", R0, imm=1)]
    for k in range(n):
        body.append(I("le", R0, imm=64) if kind == "nop" else I("add64_imm", R0, imm=k))
    return assemble(body + [I("exit")])


CONFIGS = {
    "nop200": dict(desc="microbench: 200 no-op dispatches", prog=lambda: prog_chain("nop"),
                   pkt="random"),
    "alu200": dict(desc="microbench: 200 ADD64 dispatches", prog=lambda: prog_chain("alu"),
                   pkt="random"),
    "c0": dict(desc="2-insn floor (MOV r0; EXIT), 64 B packets", prog=prog_c0, pkt="random"),
    "c2": dict(desc="8-insn ALU-only, 64 B random packets", prog=prog_c2, pkt="random"),
    "c3": dict(desc="64-insn L2/L3 parse+classify, 64 B packets", prog=prog_c3, pkt="l2l3"),
    "c4": dict(desc="64-insn classify + array-map lookup, 64 B packets", prog=prog_c4,
               pkt="l2l3"),
    "c5": dict(desc="256-insn branch-heavy filter, IMIX 64-1500 B packets", prog=prog_c5,
               pkt="imix"),
    # (probes: C5's shape with shallower trees, fewer leaves per group)
    "c5d0": dict(desc="probe: C5 with depth-0 trees (3 leaves)", prog=lambda: prog_c5(depth=0),
                 pkt="imix"),
    "c5d1": dict(desc="probe: C5 with depth-1 trees (6 leaves)", prog=lambda: prog_c5(depth=1),
                 pkt="imix"),
    "c5ms": dict(desc="probe: C5's shape melded by hand (per-lane operands from an LDS table)",
                 prog=prog_c5meldsim, pkt="imix", semantics=1),
    "c5b2": dict(desc="probe: C5, body 96, depth 2", prog=lambda: prog_c5d(2), pkt="imix"),
    "c5b0": dict(desc="probe: C5, body 96, depth 0", prog=lambda: prog_c5d(0), pkt="imix"),
    "c4c": dict(desc="64-insn classify + array-map lookup + per-key packet counter "
                     "(counters[key] += 1 through a lookup result), 64 B packets", prog=prog_c4c,
                pkt="l2l3"),
    "c3l": dict(desc="IPv4 header checksum over IHL words in a bounded loop (standard "
                     "semantics; 59-94 executed insns), 64 B packets", prog=prog_c3l,
                pkt="ipv4opt", semantics=1),
    "c4h": dict(desc="64-insn classify + hashtable lookup (1M-entry table keyed by IPv4 dst), "
                     "64 B packets", prog=prog_c4h, pkt="c4h"),
    "c3lit": dict(desc="literal 64-slot classify (11 executed), 64 B packets",
                  prog=lambda: prog_literal(64), pkt="l2l3"),
    "c5lit": dict(desc="literal 256-slot filter (23 executed), IMIX 64-1500 B packets",
                  prog=lambda: prog_literal(256), pkt="imix", extent=64),
}
