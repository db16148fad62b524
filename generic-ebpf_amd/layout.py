"""Stepping-aware assembler: lays a logical eBPF program out in slots so that the REFERENCE
interpreter executes it in the intended order.

The reference does not step pc by one.  ebpf_interpreter.c:39 is ``inst = inst + pc++`` with
``pc`` a u32 counter, so execution state is (slot i, pc p) and

    plain instruction : (i, p) -> (i + p,       p + 1)
    LDDW (:339-342)   : (i, p) -> (i + p + 1,   p + 2)
    taken jump (:210) : (i, p) -> (i + p + off, p + off + 1)

starting from (0, 1).  A straight-line program therefore visits slots 0, 1, 3, 6, 10, ...
(SURVEY.md §0).  The assembler places each logical instruction at the slot the reference will
fetch it from, inserts a stride-reset ``JA 1-p`` (next state (i+1, 2)) whenever the stride
grows past ``reset_stride``, and places the taken side of every conditional branch in a fresh
region after everything placed so far, patching the branch offset.  Holes stay zero (opcode
0x00 is not dispatched by the reference: executing one is a BAD_OPCODE fault).

Control flow is tree-shaped: under this stepping rule two different (slot, pc) states can never
merge again (a state (j, q) has the unique predecessor slot j - q + 1), so a join is expressed by
duplicating the tail into both arms (``if_else``).
"""
from . import isa


class LdDw:
    """LDDW dst, imm64.  ``value`` is an int or ``MapRef(k)`` (patched with map k's handle)."""
    __slots__ = ("dst", "value")

    def __init__(self, dst, value):
        self.dst, self.value = dst, value


class MapRef:
    __slots__ = ("index",)

    def __init__(self, index):
        self.index = index


class Branch:
    """Conditional jump; ``taken`` is a node list that must end in EXIT on every path."""
    __slots__ = ("insn", "taken")

    def __init__(self, insn, taken):
        self.insn, self.taken = insn, taken


def if_else(cond_insn, then_nodes, else_nodes, tail_nodes):
    """if (cond) {then} else {else}; tail — with the tail duplicated into both arms."""
    return [Branch(cond_insn, list(then_nodes) + list(tail_nodes))] + list(else_nodes) + \
        list(tail_nodes)


class Layout:
    """Result of assembling: ``code`` (bytes), map relocations, per-path execution counts."""

    def __init__(self, code, relocs, main_path_steps, nslots):
        self.code = code
        self.relocs = relocs                 # [(slot, map_index)]: LDDW at slot, hi imm at slot+1
        self.main_path_steps = main_path_steps  # executed insns when no branch is taken
        self.nslots = nslots

    def patched(self, handles):
        """Code with every MapRef LDDW patched to handles[map_index] (a u64)."""
        b = bytearray(self.code)
        for slot, k in self.relocs:
            h = handles[k] & 0xffffffffffffffff
            b[slot * 8 + 4: slot * 8 + 8] = (h & 0xffffffff).to_bytes(4, "little")
            b[slot * 8 + 12: slot * 8 + 16] = (h >> 32).to_bytes(4, "little")
        return bytes(b)


def assemble(nodes, reset_stride=8):
    slots = {}
    relocs = []
    queue = []
    state = {"hi": 0}

    def emit(i, b):
        if i in slots:
            raise ValueError("slot %d placed twice" % i)
        if i < 0:
            raise ValueError("negative slot")
        slots[i] = b
        state["hi"] = max(state["hi"], i + 1)

    def place(nodes, i, p):
        steps = 0
        for node in nodes:
            if p > reset_stride:
                emit(i, isa.encode(isa.OPS["ja"], off=1 - p))
                i, p = i + 1, 2
                steps += 1
            steps += 1
            if isinstance(node, LdDw):
                v = node.value
                if isinstance(v, MapRef):
                    relocs.append((i, v.index))
                    v = 0
                v &= 0xffffffffffffffff
                emit(i, isa.encode(isa.OPS["lddw"], node.dst, 0, 0, isa.s32(v)))
                emit(i + 1, isa.encode(0, 0, 0, 0, isa.s32(v >> 32)))
                i, p = i + p + 1, p + 2
            elif isinstance(node, Branch):
                ins = node.insn
                emit(i, ins.encode())  # offset patched when the taken side is placed
                queue.append((node.taken, i, p, ins))
                i, p = i + p, p + 1
            else:
                emit(i, node.encode())
                if node.op == isa.OPS["exit"]:
                    return steps
                if node.op == isa.OPS["ja"]:
                    raise ValueError("use Branch/if_else for control flow, not raw JA")
                if node.op in isa.COND_JUMPS:
                    raise ValueError("conditional jump must be a Branch node")
                i, p = i + p, p + 1
        raise ValueError("block does not end in EXIT")

    main_steps = place(nodes, 0, 1)
    while queue:
        taken, bi, bp, ins = queue.pop(0)
        t = state["hi"]
        off = t - bi - bp
        if not -32768 <= off <= 32767:
            raise ValueError("program too large for a 16-bit branch offset")
        slots[bi] = isa.encode(ins.op, ins.dst, ins.src, off, ins.imm)
        place(taken, t, t - bi + 1)

    n = state["hi"]
    code = bytearray(8 * n)
    for i, b in slots.items():
        code[8 * i: 8 * i + 8] = b
    return Layout(bytes(code), relocs, main_steps, n)


def simulate_slots(code, max_steps=100000):
    """Slot sequence the reference visits when no conditional jump is taken (JA always is).
    Pure bookkeeping for tests of the assembler; it does not evaluate instructions."""
    n = len(code) // 8
    i, p, out = 0, 1, []
    for _ in range(max_steps):
        if i >= n:
            return out, "slot"
        op, d, s, off, imm = isa.decode(code[8 * i: 8 * i + 8])
        out.append(i)
        if op == isa.OPS["exit"]:
            return out, "exit"
        if op == isa.OPS["lddw"]:
            i, p = i + p + 1, p + 2
        elif op == isa.OPS["ja"]:
            np_ = (p + off) & 0xffffffff
            i, p = i + np_, np_ + 1
        else:
            i, p = i + p, p + 1
    return out, "limit"
