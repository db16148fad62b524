"""Standard-eBPF test programs (EBPF_SEM_STANDARD): a sequential assembler with labels, the
hand-computed known-answer programs, and a seeded generator of loop-free programs."""
import numpy as np

from generic_ebpf_amd import isa

E = isa.encode
O = isa.OPS
JMP32 = {"jeq": 0x16, "jgt": 0x26, "jge": 0x36, "jset": 0x46, "jne": 0x56, "jsgt": 0x66,
         "jsge": 0x76, "jlt": 0xa6, "jle": 0xb6, "jslt": 0xc6, "jsle": 0xd6}
JMP64 = {k: v - 1 for k, v in JMP32.items()}   # class 5 twins


def asm(items):
    """items: (op, dst, src, off, imm) tuples (op a name or byte; off may be a label name),
    ("label", name), ("lddw", dst, value) or ("lddw_map", dst, k).  Returns (code, relocs)."""
    slots, labels, fix = [], {}, []
    relocs = []
    for it in items:
        if it[0] == "label":
            labels[it[1]] = len(slots)
        elif it[0] == "lddw":
            v = it[2] & 0xffffffffffffffff
            slots += [E(0x18, it[1], 0, 0, isa.s32(v)), E(0, 0, 0, 0, isa.s32(v >> 32))]
        elif it[0] == "lddw_map":
            relocs.append((len(slots), it[2]))
            slots += [E(0x18, it[1], 0, 0, 0), E(0, 0, 0, 0, 0)]
        else:
            op, d, s, off, imm = it
            op = O[op] if isinstance(op, str) else op
            if isinstance(off, str):
                fix.append((len(slots), off))
                off = 0
            slots.append([op, d, s, off, imm])
    out = []
    for i, x in enumerate(slots):
        if isinstance(x, list):
            for at, lab in fix:
                if at == i:
                    x[3] = labels[lab] - (i + 1)
            out.append(E(*x))
        else:
            out.append(x)
    return b"".join(out), relocs


def I(op, d=0, s=0, off=0, imm=0):
    return (op, d, s, off, imm)


# (name, items, packet bytes (64), expected r0) — every expectation worked out by hand from the
# standard semantics (comments), not computed by any of the implementations under test
PKT = bytes(range(64))
KATS = [
    ("mov64_imm_moves", [I("mov64_imm", 0, imm=5), I("mov64_imm", 0, imm=7), I("exit")], 7),
    ("mov64_imm_sign_extends", [I("mov64_imm", 0, imm=-1), I("exit")], 0xffffffffffffffff),
    ("mov64_reg_moves", [I("mov64_imm", 2, imm=3), I("mov64_imm", 0, imm=100),
                         I("mov64_reg", 0, 2), I("exit")], 3),
    ("neg64", [I("mov64_imm", 0, imm=5), I("neg64", 0), I("exit")], (-5) & (2**64 - 1)),
    ("neg32", [I("mov64_imm", 0, imm=5), I("neg", 0), I("exit")], 0xfffffffb),
    ("neg32_of_big", [("lddw", 0, 0x1_0000_0001), I("neg", 0), I("exit")], 0xffffffff),
    ("arsh64_imm", [I("mov64_imm", 0, imm=-16), I("arsh64_imm", 0, imm=2), I("exit")],
     (-4) & (2**64 - 1)),
    ("arsh64_reg_63", [I("mov64_imm", 0, imm=-2), I("mov64_imm", 2, imm=63),
                       I("arsh64_reg", 0, 2), I("exit")], 2**64 - 1),
    ("arsh32_imm", [I("mov_imm", 0, imm=isa.s32(0x80000000)), I("arsh_imm", 0, imm=4), I("exit")],
     0xf8000000),
    ("arsh32_reg_positive", [I("mov_imm", 0, imm=0x40000000), I("mov64_imm", 3, imm=30),
                             I("arsh_reg", 0, 3), I("exit")], 1),
    ("arsh32_truncates_upper", [("lddw", 0, 0xffff_ffff_0000_0100), I("arsh_imm", 0, imm=4),
                                I("exit")], 0x10),
    ("div64_reg_by_zero_is_zero", [I("mov64_imm", 0, imm=10), I("mov64_imm", 2, imm=0),
                                   I("div64_reg", 0, 2), I("exit")], 0),
    ("mod64_reg_by_zero_keeps_dst", [I("mov64_imm", 0, imm=10), I("mov64_imm", 2, imm=0),
                                     I("mod64_reg", 0, 2), I("exit")], 10),
    ("mod32_reg_by_zero_truncates", [("lddw", 0, 0x1_0000_0007), I("mov64_imm", 2, imm=0),
                                     I("mod_reg", 0, 2), I("exit")], 7),
    ("div32_imm_zero", [I("mov64_imm", 0, imm=9), I("div_imm", 0, imm=0), I("exit")], 0),
    ("mod64_imm_zero", [I("mov64_imm", 0, imm=9), I("mod64_imm", 0, imm=0), I("exit")], 9),
    ("div32_reg_by_upper_only_is_zero", [I("mov64_imm", 0, imm=9), ("lddw", 2, 0x1_0000_0000),
                                         I("div_reg", 0, 2), I("exit")], 0),
    ("div64_normal", [I("mov64_imm", 0, imm=100), I("mov64_imm", 2, imm=7),
                      I("div64_reg", 0, 2), I("exit")], 14),
    ("ja_sequential", [I("mov64_imm", 0, imm=1), I("ja", off="L"), I("mov64_imm", 0, imm=2),
                       ("label", "L"), I("exit")], 1),
    ("jeq_taken_skips", [I("mov64_imm", 0, imm=0), I("mov64_imm", 2, imm=5),
                         I("jeq_imm", 2, imm=5, off="L"), I("mov64_imm", 0, imm=9),
                         ("label", "L"), I("exit")], 0),
    ("jeq_not_taken", [I("mov64_imm", 0, imm=0), I("mov64_imm", 2, imm=4),
                       I("jeq_imm", 2, imm=5, off="L"), I("mov64_imm", 0, imm=9),
                       ("label", "L"), I("exit")], 9),
    ("jmp32_eq_low_word", [I("mov64_imm", 0, imm=0), ("lddw", 2, 0x1_0000_0005),
                           I(JMP32["jeq"], 2, imm=5, off="A"), I("add64_imm", 0, imm=1),
                           ("label", "A"), I("jeq_imm", 2, imm=5, off="B"),
                           I("add64_imm", 0, imm=2), ("label", "B"), I("exit")], 2),
    ("jmp32_signed", [I("mov64_imm", 0, imm=0), I("mov_imm", 2, imm=-1),
                      I(JMP32["jsgt"], 2, imm=0, off="A"), I("add64_imm", 0, imm=1),
                      ("label", "A"), I(JMP32["jgt"], 2, imm=0, off="B"),
                      I("add64_imm", 0, imm=2), ("label", "B"), I("exit")], 1),
    ("jmp32_reg_unsigned", [I("mov64_imm", 0, imm=0), ("lddw", 2, 0x5_0000_0003),
                            ("lddw", 3, 0x1_0000_0004), I(JMP32["jlt"] | 8, 2, 3, off="A"),
                            I("add64_imm", 0, imm=1), ("label", "A"),
                            I(JMP64["jlt"] | 8, 2, 3, off="B"), I("add64_imm", 0, imm=2),
                            ("label", "B"), I("exit")], 2),
    ("jmp32_jset", [I("mov64_imm", 0, imm=0), ("lddw", 2, 0x1_0000_0000),
                    I(JMP32["jset"], 2, imm=-1, off="A"), I("add64_imm", 0, imm=1),
                    ("label", "A"), I("exit")], 1),
    ("lddw_full", [("lddw", 0, 0x1122334455667788), I("exit")], 0x1122334455667788),
    ("stack_roundtrip", [("lddw", 2, 0x1122334455667788), I("stxdw", 10, 2, -8),
                         I("ldxw", 0, 10, -8), I("exit")], 0x55667788),
    ("ctx_copy_and_load", [I("mov64_reg", 6, 1), I("mov64_imm", 1, imm=0),
                           I("ldxb", 0, 6, 3), I("exit")], 3),
    ("packet_be16", [I("ldxh", 0, 1, 12), I("be", 0, imm=16), I("exit")], 0x0c0d),
    ("pointer_arith_clang_style", [I("mov64_reg", 2, 1), I("add64_imm", 2, imm=8),
                                   I("ldxdw", 0, 2, 0), I("exit")], 0x0f0e0d0c0b0a0908),
    ("shift_masks", [I("mov64_imm", 0, imm=1), I("mov64_imm", 2, imm=65),
                     I("lsh64_reg", 0, 2), I("exit")], 2),
    ("alu32_zero_extends", [I("mov64_imm", 0, imm=-1), I("add_imm", 0, imm=1), I("exit")], 0),
    ("loop_free_diamond", [I("ldxb", 2, 1, 5), I("mov64_imm", 0, imm=10),
                           I("jgt_imm", 2, imm=4, off="T"), I("mov64_imm", 0, imm=20),
                           I("ja", off="J"), ("label", "T"), I("mov64_imm", 0, imm=30),
                           ("label", "J"), I("add64_imm", 0, imm=1), I("exit")], 31),
]


def gen_program(seed, length=40, with_map=False):
    """A loop-free standard program: r6 = ctx, r0-r5/r7-r9 seeded with immediates, then
    `length` random ALU32/ALU64 ops (every opcode, divisors possibly zero), byte swaps, packet
    loads in range, stack stores/loads, forward JMP/JMP32 branches, an optional hashless array
    lookup; EXIT with r0."""
    g = np.random.default_rng(seed)
    regs = [0, 1, 2, 3, 4, 5, 7, 8, 9]
    items = [I("mov64_reg", 6, 1)]
    for r in regs:
        items.append(I("mov64_imm", r, imm=int(g.integers(-2**31, 2**31))))
    for k in range(1, 9):      # every stack slot the program may read is defined on all paths
        items.append(I("stxdw", 10, regs[k], -8 * k))
    alu = ["add", "sub", "mul", "div", "or", "and", "lsh", "rsh", "mod", "xor", "mov", "arsh"]
    pending = []   # (label, position to place it)
    nlab = 0
    stored = []
    for k in range(length):
        for lab, at in list(pending):
            if at == k:
                items.append(("label", lab))
                pending.remove((lab, at))
        c = g.random()
        d = int(g.choice(regs))
        if c < 0.55:
            name = alu[int(g.integers(0, len(alu)))]
            w64 = g.random() < 0.6
            if g.random() < 0.5:
                imm = int(g.integers(-40, 40)) if g.random() < 0.5 else int(g.integers(-2**31, 2**31))
                items.append(I(name + ("64_imm" if w64 else "_imm"), d, imm=imm))
            else:
                items.append(I(name + ("64_reg" if w64 else "_reg"), d, int(g.choice(regs))))
        elif c < 0.6:
            items.append(I("neg64" if g.random() < 0.5 else "neg", d))
        elif c < 0.65:
            items.append(I("be" if g.random() < 0.5 else "le", d, imm=int(g.choice([16, 32, 64]))))
        elif c < 0.75:
            z = int(g.choice([1, 2, 4, 8]))
            op = {1: "ldxb", 2: "ldxh", 4: "ldxw", 8: "ldxdw"}[z]
            items.append(I(op, d, 6, int(g.integers(0, 64 - z + 1))))
        elif c < 0.82:
            so = -8 * int(g.integers(1, 9))
            items.append(I("stxdw", 10, int(g.choice(regs)), so))
            stored.append(so)
        elif c < 0.86:
            items.append(I("ldxdw", d, 10, -8 * int(g.integers(1, 9))))
        elif k < length - 2:
            lab = "L%d" % nlab
            nlab += 1
            conds = list(JMP32)
            cn = conds[int(g.integers(0, len(conds)))]
            tab = JMP32 if g.random() < 0.5 else JMP64
            op = tab[cn] + (8 if g.random() < 0.5 else 0)
            if op & 8:
                items.append(I(op, d, int(g.choice(regs)), lab))
            else:
                items.append(I(op, d, 0, lab, int(g.integers(-50, 50))))
            pending.append((lab, int(g.integers(k + 1, length + 1))))
    if with_map:
        items += [I("mov64_reg", 7, 0), I("and64_imm", 7, imm=15), I("stxw", 10, 7, -4),
                  ("lddw_map", 1, 0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4),
                  I("call", imm=0), I("jeq_imm", 0, imm=0, off="M"),
                  I("ldxdw", 0, 0, 0), ("label", "M")]
    for lab, at in pending:
        items.append(("label", lab))
    items.append(I("exit"))
    return asm(items)


# Loops (standard semantics): every taken backward jump counts against the lane's budget of
# 2^20 (dprog.h DP_LOOP_BUDGET, oracle run_std); the next one faults LOOP (8).
LOOP_BUDGET = 1 << 20


def countdown(n):
    """r2 = n; do { r0 += r2; r2 -= 1 } while (r2 != 0): n - 1 taken backward jumps, r0 = the
    sum 1..n."""
    return asm([I("mov64_imm", 0, imm=0), ("lddw", 2, n), ("label", "L"),
                I("add64_reg", 0, 2), I("sub64_imm", 2, imm=1),
                I("jne_imm", 2, imm=0, off="L"), I("exit")])


def gen_loop_program(seed, length=30, forever_every=0):
    """A standard program with counted loops: a loop-free prefix (gen_program's ops), then 1-2
    loops (one nested sometimes) whose trip counts come from packet bytes (1-16: lanes diverge),
    with random ALU ops and a forward branch inside the bodies; one loop's exit is a JA back
    edge variant.  forever_every = k > 0: packets whose byte 3 is a multiple of k loop forever
    (a JA back edge that nothing breaks) and fault LOOP at the budget."""
    g = np.random.default_rng(seed)
    regs = [0, 3, 4, 7, 8, 9]
    items = [I("mov64_reg", 6, 1)]
    for r in regs:
        items.append(I("mov64_imm", r, imm=int(g.integers(-2**31, 2**31))))
    alu = ["add", "sub", "mul", "or", "and", "lsh", "rsh", "xor", "arsh"]

    def body(k, tag):
        out = []
        for j in range(k):
            d = int(g.choice(regs))
            name = alu[int(g.integers(0, len(alu)))]
            w = "64" if g.random() < 0.6 else ""
            if g.random() < 0.5:
                out.append(I(name + w + "_imm", d, imm=int(g.integers(-40, 40))))
            else:
                out.append(I(name + w + "_reg", d, int(g.choice(regs))))
            if j == k // 2:    # a forward branch inside the body
                out += [I("jgt_imm", d, imm=int(g.integers(0, 2**20)), off="S" + tag),
                        I("xor64_imm", 0, imm=int(g.integers(1, 1000))), ("label", "S" + tag)]
        return out

    nloops = 1 + int(g.random() < 0.6)
    for li in range(nloops):
        tag = "%d" % li
        off = int(g.integers(0, 60))
        items += [I("ldxb", 5, 6, off), I("and64_imm", 5, imm=15), I("add64_imm", 5, imm=1),
                  ("label", "L" + tag)]
        items += body(int(g.integers(2, 8)), tag + "a")
        if li == 0 and nloops == 2 and g.random() < 0.5:   # nested inner loop on r2
            items += [I("ldxb", 2, 6, int(g.integers(0, 60))), I("and64_imm", 2, imm=3),
                      I("add64_imm", 2, imm=1), ("label", "N"),
                      I("add64_reg", 0, 2), I("sub64_imm", 2, imm=1),
                      I("jne_imm", 2, imm=0, off="N")]
        items += [I("add64_reg", 0, 5), I("sub64_imm", 5, imm=1)]
        if g.random() < 0.5:
            items.append(I("jne_imm", 5, imm=0, off="L" + tag))
        else:   # exit test forward, JA back
            items += [I("jeq_imm", 5, imm=0, off="E" + tag), I("ja", off="L" + tag),
                      ("label", "E" + tag)]
    if forever_every:
        items += [I("ldxb", 2, 6, 3), I("mod64_imm", 2, imm=forever_every),
                  I("jne_imm", 2, imm=0, off="F"), ("label", "H"), I("add64_imm", 0, imm=1),
                  I("ja", off="H"), ("label", "F")]
    items += [I("xor64_reg", 0, int(g.choice(regs))), I("exit")]
    return asm(items)


def gen_cursor_program(seed):
    """A standard program that walks the packet with a cursor in a loop (the C3L / TLV shape:
    packet loads at run-time offsets): r7 = ctx + a start offset, a trip count of 1-16 from a
    packet byte, and per trip 1-3 loads of 1/2/4/8 bytes at small offsets from the cursor (any
    alignment) mixed into r0, then the cursor advances by a constant or by a packet byte (0-7).
    Cursors that run past the packet end fault MEM, as in the reference's bounds check."""
    g = np.random.default_rng(seed)
    items = [I("mov64_reg", 6, 1), I("mov64_imm", 0, imm=int(g.integers(0, 2**31))),
             I("mov64_reg", 7, 6), I("add64_imm", 7, imm=int(g.integers(0, 9))),
             I("ldxb", 8, 6, int(g.integers(0, 64))), I("and64_imm", 8, imm=15),
             I("add64_imm", 8, imm=1), ("label", "L")]
    for _ in range(int(g.integers(1, 4))):
        z = int(g.choice([1, 2, 4, 8]))
        op = {1: "ldxb", 2: "ldxh", 4: "ldxw", 8: "ldxdw"}[z]
        items += [I(op, 2, 7, int(g.integers(0, 4))), I("mul64_imm", 0, imm=31),
                  I("add64_reg", 0, 2)]
    if g.random() < 0.5:
        items.append(I("add64_imm", 7, imm=int(g.integers(3, 8))))
    else:
        items += [I("ldxb", 3, 7, 0), I("and64_imm", 3, imm=7), I("add64_reg", 7, 3)]
    items.append(I("sub64_imm", 8, imm=1))
    if g.random() < 0.7:
        items.append(I("jne_imm", 8, imm=0, off="L"))
    else:   # exit test forward, JA back
        items += [I("jeq_imm", 8, imm=0, off="E"), I("ja", off="L"), ("label", "E")]
    items += [I("ldxb", 2, 6, 1), I("xor64_reg", 0, 2), I("exit")]
    return asm(items)


def gen_loop_write_program(seed, counters=False, fetched=False, mixed=False):
    """A standard program that writes maps inside loops (include/ebpf_gpu.h "Map writes in a
    device batch"): 1-2 counted loops (trip counts 1-24 from packet bytes, so some packets pass
    the 16 logged writes a packet may make and fault EBPF_FAULT_WRITES), each trip looking up
    map 0 (16 entries, 16-B values; the key from the trip counter and a packet byte) and then,
    at random:
      counters=False: plain stores of 1/2/4/8 bytes of a register into the value at any
        offset, loads back from the value (the packet reads its own stores), and
        map_update_elem of map 1 (8-B values) with a stack value (flags ANY or, rarely,
        NOEXIST: EEXIST, not logged);
      counters=True: XADD (W or DW, aligned, no fetch) into map 0's value, and the LDX / ADD /
        STX idiom on another word whose register is overwritten right after (a dead counter
        register), no loads back;
      fetched=True (round 6; map 0 then has 32-B values, 4 words a key): the counters read
        back — XADD with BPF_FETCH whose old value r9 mixes in, and the idiom whose register r9
        mixes in after the STX — so that a packet sees the batch start plus its own additions
        and a long walk over many keys passes the 32 words of its view (EBPF_FAULT_WRITES);
      mixed=True (round 6; map 0 a hashtable, 16-B values): everything into the same values —
        XADD with and without BPF_FETCH, the idiom with a live or a dead register, plain stores
        and loads back — and map_update_elem of map 1: every one of them a record, counted.
    r0 mixes the trip count, loaded values and helper return codes."""
    counters = counters or fetched
    vs0 = 32 if fetched else 16
    g = np.random.default_rng(seed)
    items = [I("mov64_reg", 6, 1), I("mov64_imm", 0, imm=int(g.integers(0, 2**31))),
             I("mov64_imm", 9, imm=0)]
    cw = int(g.choice([4, 8]))   # counters: one width per program (a device-atomic array)
    nloops = 1 + int(g.random() < 0.4)
    for li in range(nloops):
        t = "%d" % li
        items += [I("ldxb", 8, 6, int(g.integers(0, 64))), I("mod64_imm", 8, imm=24),
                  I("add64_imm", 8, imm=1), ("label", "L" + t),
                  # key = (trip + pkt byte) & 15
                  I("ldxb", 4, 6, int(g.integers(0, 64))), I("add64_reg", 4, 8),
                  I("and64_imm", 4, imm=15), I("stxw", 10, 4, -4),
                  ("lddw_map", 1, 0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4),
                  I("call", imm=0), I("jeq_imm", 0, imm=0, off="M" + t)]
        for j in range(int(g.integers(1, 4))):
            r = g.random()
            if mixed and r < 0.5:
                off = int(g.integers(0, vs0 // cw)) * cw
                fetch = g.random() < 0.5
                if r < 0.25:
                    items += [I("mov64_reg", 3, 8), I("add64_imm", 3, imm=int(g.integers(0, 9))),
                              (0xdb if cw == 8 else 0xc3, 0, 3, off, 1 if fetch else 0),
                              I("mul64_imm", 9, imm=31), I("add64_reg", 9, 3)]
                else:
                    ld, st = ("ldxdw", "stxdw") if cw == 8 else ("ldxw", "stxw")
                    items += [I(ld, 5, 0, off), I("add64_imm", 5, imm=int(g.integers(1, 100))),
                              I(st, 0, 5, off)]
                    items += [I("xor64_reg", 9, 5)] if fetch else [I("mov64_imm", 5, imm=0)]
                continue
            if mixed:
                r = (r - 0.5) * 2           # stores, loads, updates as below
            if counters and not mixed:
                off = int(g.integers(0, vs0 // cw)) * cw
                if r < 0.6:
                    items += [I("mov64_reg", 3, 8), I("add64_imm", 3, imm=int(g.integers(0, 9))),
                              (0xdb if cw == 8 else 0xc3, 0, 3, off, 1 if fetched else 0)]
                    if fetched:
                        items += [I("mul64_imm", 9, imm=31), I("add64_reg", 9, 3)]
                else:
                    ld, st = ("ldxdw", "stxdw") if cw == 8 else ("ldxw", "stxw")
                    items += [I(ld, 5, 0, off), I("add64_imm", 5, imm=int(g.integers(1, 100))),
                              I(st, 0, 5, off)]
                    items += [I("xor64_reg", 9, 5)] if fetched else [I("mov64_imm", 5, imm=0)]
            elif r < 0.45:
                z = int(g.choice([1, 2, 4, 8]))
                op = {1: "stxb", 2: "stxh", 4: "stxw", 8: "stxdw"}[z]
                items += [I("mov64_reg", 3, 8), I("mul64_imm", 3, imm=int(g.integers(1, 2**20))),
                          I(op, 0, 3, int(g.integers(0, 17 - z)))]
            elif r < 0.75:
                z = int(g.choice([1, 2, 4, 8]))
                op = {1: "ldxb", 2: "ldxh", 4: "ldxw", 8: "ldxdw"}[z]
                items += [I(op, 3, 0, int(g.integers(0, 17 - z))), I("mul64_imm", 9, imm=33),
                          I("add64_reg", 9, 3)]
            else:   # map_update_elem(map 1, &key, &stack value, flags); r9 += the code
                items += [I("stxdw", 10, 8, -16), I("mov64_reg", 7, 0),
                          ("lddw_map", 1, 1), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4),
                          I("mov64_reg", 3, 10), I("add64_imm", 3, imm=-16),
                          I("mov64_imm", 4, imm=1 if g.random() < 0.15 else 0),
                          I("call", imm=1), I("add64_reg", 9, 0), I("mov64_reg", 0, 7)]
        items += [("label", "M" + t), I("sub64_imm", 8, imm=1)]
        if g.random() < 0.5:
            items.append(I("jne_imm", 8, imm=0, off="L" + t))
        else:
            items += [I("jeq_imm", 8, imm=0, off="E" + t), I("ja", off="L" + t), ("label", "E" + t)]
    items += [I("mov64_reg", 0, 9), I("exit")]
    return asm(items)
