"""Seeded random eBPF programs for opcode-coverage parity testing.

Every program is well-defined under the reference interpreter (so the genuine reference, the
oracle and the device must agree bit for bit): no undefined register or stack reads, no
division by zero, every load/store inside the 64-B packet, the 512-B stack or a looked-up map
value, and r0 at EXIT never derived from a pointer.  The generator covers all 90 opcodes and the
reference quirks (MOV64 adds, NEG ignores dst, logical ARSH, masked shift counts, LE/BE with odd
widths, cumulative pc stepping — via the stepping-aware assembler).
"""
import numpy as np

from . import isa
from .layout import Branch, LdDw, MapRef, assemble

I = isa.Insn
PKT = 64

_ALU_BIN = ["add", "sub", "mul", "div", "or", "and", "lsh", "rsh", "mod", "xor", "mov", "arsh"]
_JMP = ["jeq", "jgt", "jge", "jset", "jne", "jsgt", "jsge", "jlt", "jle", "jslt", "jsle"]
_SPECIAL_IMM = [0, 1, -1, 2, 7, 8, 15, 16, 31, 32, 33, 48, 63, 64, 65, 127, 255, 0x7fffffff,
                -0x80000000, 0x12345678, -0x12345678, 0xffff, -2]


class _Gen:
    def __init__(self, seed, nmaps, map_value_size, writes=False, vstores=False):
        self.g = np.random.default_rng(seed)
        self.nmaps = nmaps
        self.vs = map_value_size
        self.writes = writes
        self.vstores = vstores
        self.scalars = [0, 2, 3, 4, 5, 6, 7, 8, 9]
        self.ctx = 1
        self.stack_ok = set()   # initialised stack byte offsets (negative, relative to r10)

    def r(self, n):
        return int(self.g.integers(0, n))

    def pick(self, seq):
        return seq[self.r(len(seq))]

    def imm(self):
        if self.r(3) == 0:
            return self.pick(_SPECIAL_IMM)
        return int(self.g.integers(-(1 << 31), 1 << 31))

    def scalar(self):
        return self.pick(self.scalars)

    # -- instruction groups --------------------------------------------------------------
    def alu(self):
        bits = self.pick(["", "64"])
        name = self.pick(_ALU_BIN)
        d = self.scalar()
        out = []
        if self.r(2) == 0:
            imm = self.imm()
            if name in ("div", "mod") and (imm & 0xffffffff if bits == "" else imm) == 0:
                imm = 3
            out.append(I("%s%s_imm" % (name, bits), d, imm=imm))
        else:
            s = self.scalar()
            if name in ("div", "mod"):
                out.append(I("or64_imm", s, imm=1 + 2 * self.r(8)))
            out.append(I("%s%s_reg" % (name, bits), d, s))
        return out

    def unary(self):
        d = self.scalar()
        k = self.r(4)
        if k == 0:
            return [I("neg", d, imm=self.imm())]
        if k == 1:
            return [I("neg64", d, imm=self.imm())]
        return [I(self.pick(["le", "be"]), d, imm=self.pick([16, 32, 64, 16, 32, 64, 8, 0, 48]))]

    def lddw(self):
        v = int(self.g.integers(0, 1 << 63)) * 2 + self.r(2)
        return [LdDw(self.scalar(), v)]

    def ldx_pkt(self):
        size = self.pick([1, 2, 4, 8])
        off = self.r(PKT - size + 1)
        name = {1: "ldxb", 2: "ldxh", 4: "ldxw", 8: "ldxdw"}[size]
        if self.r(4) == 0:
            # through a derived pointer: t = ctx + k; load [t + off - k]; t back to a scalar
            t = self.scalar()
            k = self.r(PKT)
            return [I("mov_imm", t, imm=0), I("mov64_reg", t, self.ctx), I("add64_imm", t, imm=k),
                    I(name, self.scalar() if False else t, t, off - k)]
        return [I(name, self.scalar(), self.ctx, off)]

    def stack_store(self):
        size = self.pick([1, 2, 4, 8])
        off = -self.r(64 - size + 1) - size   # within the top 64 bytes (plus deeper below)
        if self.r(5) == 0:
            off = -int(self.g.integers(size, 512 - 0)) // size * size
            off = max(off, -512)
        out = []
        if self.r(2) == 0:
            out.append(I({1: "stb", 2: "sth", 4: "stw", 8: "stdw"}[size], 10, 0, off, self.imm()))
        else:
            out.append(I({1: "stxb", 2: "stxh", 4: "stxw", 8: "stxdw"}[size], 10, self.scalar(),
                         off))
        for b in range(size):
            self.stack_ok.add(off + b)
        return out

    def stack_load(self):
        cands = []
        for size in (1, 2, 4, 8):
            for off in sorted(self.stack_ok):
                if all((off + b) in self.stack_ok for b in range(size)):
                    cands.append((size, off))
        if not cands:
            return self.stack_store()
        size, off = self.pick(cands)
        return [I({1: "ldxb", 2: "ldxh", 4: "ldxw", 8: "ldxdw"}[size], self.scalar(), 10, off)]

    def pkt_store(self):
        size = self.pick([1, 2, 4, 8])
        off = self.r(PKT - size + 1)
        if self.r(2) == 0:
            return [I({1: "stb", 2: "sth", 4: "stw", 8: "stdw"}[size], self.ctx, 0, off,
                      self.imm())]
        return [I({1: "stxb", 2: "stxh", 4: "stxw", 8: "stxdw"}[size], self.ctx, self.scalar(),
                  off)]

    def lookup(self):
        """ctx moves to r6 (r1 is needed for the map); key from a scalar, hit or miss."""
        if self.nmaps == 0:
            return self.alu()
        out = []
        if self.ctx != 6:
            out += [I("mov_imm", 6, imm=0), I("mov64_reg", 6, self.ctx)]
            self.ctx = 6
            self.scalars = [0, 2, 3, 4, 5, 7, 8, 9]
        k = self.scalar()
        key_mask = self.pick([0x7, 0xff, 0x1ff, 0xffffffff])
        out += [I("mov_reg", 7, k), I("and64_imm", 7, imm=isa.s32(key_mask)),
                I("stxw", 10, 7, -4)]
        for b in range(-4, 0):
            self.stack_ok.add(b)
        out += [LdDw(1, MapRef(self.r(self.nmaps))),
                I("mov_imm", 2, imm=0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4),
                I("call", imm=0)]
        miss = [I("mov_imm", 0, imm=0x77), I("xor64_reg", 0, 7), I("exit")]
        vsz = self.pick([s for s in (1, 2, 4, 8) if s <= self.vs])
        voff = self.r(self.vs - vsz + 1)
        dst = self.pick([3, 4, 5, 8, 9])
        out += [Branch(I("jeq_imm", 0, imm=0), miss)]
        if self.vstores:
            out += self.value_stores()
        out += [I({1: "ldxb", 2: "ldxh", 4: "ldxw", 8: "ldxdw"}[vsz], dst, 0, voff),
                I("mov_imm", 0, imm=self.imm()), I("mov_imm", 1, imm=self.imm()),
                I("mov_imm", 2, imm=self.imm())]
        return out

    def value_stores(self):
        """Stores through the lookup result in r0 (ebpf_gpu.h "Stores into map values"): plain
        STX / ST of 1-8 bytes anywhere in the value, and counter updates (LDX{W,DW} X; ADD/SUB
        (32- or 64-bit, immediate or register; the reference's MOV64, which adds); STX back),
        aligned or not.  The lookup's own load follows (the packet reads its stores back)."""
        out = []
        safe = [3, 4, 5, 7, 8, 9]   # (r0 holds the value's address, r1 the map, r2 the key's)
        for _ in range(self.r(3) + 1):
            k = self.r(4)
            if k < 2 or self.vs < 4:
                size = self.pick([z for z in (1, 2, 4, 8) if z <= self.vs])
                off = self.r(self.vs - size + 1)
                if k == 0:
                    out.append(I({1: "stb", 2: "sth", 4: "stw", 8: "stdw"}[size], 0, 0, off, self.imm()))
                else:
                    out.append(I({1: "stxb", 2: "stxh", 4: "stxw", 8: "stxdw"}[size], 0,
                                 self.pick(safe), off))
                continue
            size = self.pick([z for z in (4, 8) if z <= self.vs])
            off = self.r(self.vs - size + 1)
            x = self.pick([3, 4, 5, 8, 9])
            y = self.pick([s for s in safe if s != x])
            alu = self.pick(["add64_imm", "sub64_imm", "add64_reg", "sub64_reg", "mov64_reg"] +
                            (["add_imm", "sub_imm", "add_reg"] if size == 4 else []))
            a = I(alu, x, imm=self.imm()) if alu.endswith("imm") else I(alu, x, y)
            out += [I({4: "ldxw", 8: "ldxdw"}[size], x, 0, off), a,
                    I({4: "stxw", 8: "stxdw"}[size], 0, x, off)]
        return out

    def value_base(self):
        """stack offset of an update's value: below the key at r10 - 4, inside the stack"""
        return -8 - (self.vs + 7) // 8 * 8

    def update(self):
        """map_update_elem (helper 1) or map_delete_elem (helper 2, EINVAL on an array): key and
        value from the stack, flags 0..3 (3: EINVAL); the return code mixed into a scalar; the
        pointer-holding argument registers reset to scalars afterwards (the test environment's
        helper slots, oracle/pyoracle.py DEFAULT_HELPER_KINDS)."""
        if self.nmaps == 0:
            return self.alu()
        out = []
        if self.ctx != 6:
            out += [I("mov_imm", 6, imm=0), I("mov64_reg", 6, self.ctx)]
            self.ctx = 6
            self.scalars = [0, 2, 3, 4, 5, 7, 8, 9]
        k = self.scalar()
        key_mask = self.pick([0x7, 0xff, 0xffffffff])
        out += [I("mov_reg", 7, k), I("and64_imm", 7, imm=isa.s32(key_mask)),
                I("stxw", 10, 7, -4)]
        vb = self.value_base()
        for off in range(0, self.vs, 8):
            out.append(I("stxdw", 10, self.scalar(), vb + off))
        for b in list(range(-4, 0)) + list(range(vb, vb + self.vs)):
            self.stack_ok.add(b)
        out += [LdDw(1, MapRef(self.r(self.nmaps))),
                I("mov_imm", 2, imm=0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4)]
        if self.r(4) == 0:
            out += [I("call", imm=2)]
        else:
            out += [I("mov_imm", 3, imm=0), I("mov64_reg", 3, 10), I("add64_imm", 3, imm=vb),
                    I("mov_imm", 4, imm=self.r(4)), I("call", imm=1)]
        dst = self.pick([3, 4, 5, 8, 9])
        out += [I("mov_imm", dst, imm=self.imm()), I("xor64_reg", dst, 0)]
        for r in (1, 2, 3, 4):
            if r != dst:
                out.append(I("mov_imm", r, imm=self.imm()))
        return out

    def bulk_writes(self):
        """More than 16 map writes on one path (a loop-free program has no write limit, as in
        the reference: ebpf_gpu.h "Map writes in a device batch"): a lookup hit followed by
        17..60 ST / STX into the value, or 17..40 map_update_elem calls.  Placed last on the
        main path, after every load of a map value (no read-back: the overlay does not bound
        the count); the pointer registers become scalars again afterwards."""
        if self.nmaps == 0:
            return self.alu()
        out = []
        if self.ctx != 6:
            out += [I("mov_imm", 6, imm=0), I("mov64_reg", 6, self.ctx)]
            self.ctx = 6
            self.scalars = [0, 2, 3, 4, 5, 7, 8, 9]
        src = [3, 4, 5, 8, 9]
        if self.r(2) == 0:
            k = self.scalar()
            out += [I("mov_reg", 7, k), I("and64_imm", 7, imm=self.pick([0x7, 0xff, 0x1ff])),
                    I("stxw", 10, 7, -4), LdDw(1, MapRef(self.r(self.nmaps))),
                    I("mov_imm", 2, imm=0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4),
                    I("call", imm=0),
                    Branch(I("jeq_imm", 0, imm=0), [I("mov_imm", 0, imm=0x55), I("xor64_reg", 0, 7),
                                                    I("exit")])]
            for b in range(-4, 0):
                self.stack_ok.add(b)
            for _ in range(17 + self.r(44)):
                size = self.pick([z for z in (1, 2, 4, 8) if z <= self.vs])
                off = self.r(self.vs - size + 1)
                if self.r(3) == 0:
                    out.append(I({1: "stb", 2: "sth", 4: "stw", 8: "stdw"}[size], 0, 0, off, self.imm()))
                else:
                    out.append(I({1: "stxb", 2: "stxh", 4: "stxw", 8: "stxdw"}[size], 0,
                                 self.pick(src), off))
                if self.r(2) == 0:
                    out.append(I("add64_imm", self.pick(src), imm=self.imm()))
            out += [I("mov_imm", 0, imm=self.imm()), I("mov_imm", 1, imm=self.imm()),
                    I("mov_imm", 2, imm=self.imm())]
            return out
        m = self.r(self.nmaps)
        vb = self.value_base()
        for b in list(range(-4, 0)) + list(range(vb, vb + self.vs)):
            self.stack_ok.add(b)
        for off in range(0, self.vs, 8):
            out.append(I("stxdw", 10, self.scalar(), vb + off))
        acc = self.pick([5, 8, 9])   # (r1..r4 are the call's arguments)
        out += [I("mov_imm", acc, imm=self.imm())]
        keyreg = self.pick([s for s in src if s != acc])
        out += [I("mov_reg", 7, keyreg)]
        for j in range(17 + self.r(24)):
            out += [I("add_imm", 7, imm=1 + self.r(3)), I("and64_imm", 7, imm=self.pick([0x7, 0x7, 0xf, 0xff])),
                    I("stxw", 10, 7, -4), I("stxw", 10, acc, vb),
                    LdDw(1, MapRef(m)),
                    I("mov_imm", 2, imm=0), I("mov64_reg", 2, 10), I("add64_imm", 2, imm=-4),
                    I("mov_imm", 3, imm=0), I("mov64_reg", 3, 10), I("add64_imm", 3, imm=vb),
                    I("mov_imm", 4, imm=self.pick([0, 0, 0, 2, 1])), I("call", imm=1),
                    I("xor64_reg", acc, 0), I("mul64_imm", acc, imm=0x2545F491)]
        for r in (0, 1, 2, 3, 4):
            if r != acc:
                out.append(I("mov_imm", r, imm=self.imm()))
        return out

    def branch(self, depth):
        name = self.pick(_JMP)
        d = self.scalar()
        if self.r(2) == 0:
            ins = I(name + "_imm", d, imm=self.imm())
        else:
            ins = I(name + "_reg", d, self.scalar())
        saved = (list(self.scalars), self.ctx, set(self.stack_ok))
        taken = self.block(self.r(4) + 1, depth + 1) + self.epilogue()
        self.scalars, self.ctx, self.stack_ok = saved
        return [Branch(ins, taken)]

    def block(self, n, depth=0):
        out = []
        for _ in range(n):
            k = self.r(20)
            if k < 7:
                out += self.alu()
            elif k < 9:
                out += self.unary()
            elif k < 10:
                out += self.lddw()
            elif k < 13:
                out += self.ldx_pkt()
            elif k < 14:
                out += self.stack_store()
            elif k < 15:
                out += self.stack_load()
            elif k < 16:
                out += self.pkt_store()
            elif k < 17:
                out += self.update() if (self.writes and self.r(2) == 0) else self.lookup()
            elif depth < 3:
                out += self.branch(depth)
            else:
                out += self.alu()
        return out

    def prologue(self):
        out = []
        for r in self.scalars:
            if self.r(3) == 0:
                out += [LdDw(r, int(self.g.integers(0, 1 << 63)))]
            else:
                out += [I("mov_imm", r, imm=self.imm())]
        return out

    def epilogue(self):
        out = []
        for r in self.scalars:
            if r != 0:
                out += [I("xor64_reg", 0, r), I("mul64_imm", 0, imm=0x2545F491)]
        for off in sorted(self.stack_ok)[:4]:
            out += [I("ldxb", 3, 10, off), I("add64_reg", 0, 3)]
        return out + [I("exit")]


def random_program(seed, length=40, nmaps=1, map_value_size=8, reset_stride=None, writes=False,
                   vstores=False, pkt_stores=True, many_writes=False):
    """writes: half the map helper calls are map_update_elem / map_delete_elem (the device
    batch semantics: ebpf_gpu.h "Map writes in a device batch"); vstores: every lookup hit
    stores into the value first (ebpf_gpu.h "Stores into map values"); pkt_stores=False: packet
    loads where stores into the packet would be (programs that leave the packet unchanged);
    many_writes: the main path ends with more than 16 map writes (bulk_writes)."""
    gen = _Gen(seed, nmaps, map_value_size, writes, vstores)
    if not pkt_stores:
        gen.pkt_store = gen.ldx_pkt
    body = gen.block(length)
    if many_writes:
        body += gen.bulk_writes()
    nodes = gen.prologue() + body + gen.epilogue()
    rs = reset_stride if reset_stride is not None else int(gen.g.integers(3, 12))
    return assemble(nodes, reset_stride=rs)
