"""eBPF instruction encoding (mirror of include/ebpf_vm_isa.h).

Reference: generic-ebpf sys/sys/ebpf_vm_isa.h:21-27 (struct ebpf_inst, dst = low nibble of byte 1)
and :145-238 (the 90 opcodes dispatched by sys/dev/ebpf/ebpf_interpreter.c:40-369).
"""
import struct

# name -> opcode byte
OPS = {
    # ALU32
    "add_imm": 0x04, "add_reg": 0x0c, "sub_imm": 0x14, "sub_reg": 0x1c,
    "mul_imm": 0x24, "mul_reg": 0x2c, "div_imm": 0x34, "div_reg": 0x3c,
    "or_imm": 0x44, "or_reg": 0x4c, "and_imm": 0x54, "and_reg": 0x5c,
    "lsh_imm": 0x64, "lsh_reg": 0x6c, "rsh_imm": 0x74, "rsh_reg": 0x7c,
    "neg": 0x84, "mod_imm": 0x94, "mod_reg": 0x9c, "xor_imm": 0xa4, "xor_reg": 0xac,
    "mov_imm": 0xb4, "mov_reg": 0xbc, "arsh_imm": 0xc4, "arsh_reg": 0xcc,
    "le": 0xd4, "be": 0xdc,
    # ALU64
    "add64_imm": 0x07, "add64_reg": 0x0f, "sub64_imm": 0x17, "sub64_reg": 0x1f,
    "mul64_imm": 0x27, "mul64_reg": 0x2f, "div64_imm": 0x37, "div64_reg": 0x3f,
    "or64_imm": 0x47, "or64_reg": 0x4f, "and64_imm": 0x57, "and64_reg": 0x5f,
    "lsh64_imm": 0x67, "lsh64_reg": 0x6f, "rsh64_imm": 0x77, "rsh64_reg": 0x7f,
    "neg64": 0x87, "mod64_imm": 0x97, "mod64_reg": 0x9f, "xor64_imm": 0xa7, "xor64_reg": 0xaf,
    "mov64_imm": 0xb7, "mov64_reg": 0xbf, "arsh64_imm": 0xc7, "arsh64_reg": 0xcf,
    # memory
    "ldxw": 0x61, "ldxh": 0x69, "ldxb": 0x71, "ldxdw": 0x79,
    "stw": 0x62, "sth": 0x6a, "stb": 0x72, "stdw": 0x7a,
    "stxw": 0x63, "stxh": 0x6b, "stxb": 0x73, "stxdw": 0x7b,
    "lddw": 0x18,
    # jumps
    "ja": 0x05, "jeq_imm": 0x15, "jeq_reg": 0x1d, "jgt_imm": 0x25, "jgt_reg": 0x2d,
    "jge_imm": 0x35, "jge_reg": 0x3d, "jset_imm": 0x45, "jset_reg": 0x4d,
    "jne_imm": 0x55, "jne_reg": 0x5d, "jsgt_imm": 0x65, "jsgt_reg": 0x6d,
    "jsge_imm": 0x75, "jsge_reg": 0x7d, "call": 0x85, "exit": 0x95,
    "jlt_imm": 0xa5, "jlt_reg": 0xad, "jle_imm": 0xb5, "jle_reg": 0xbd,
    "jslt_imm": 0xc5, "jslt_reg": 0xcd, "jsle_imm": 0xd5, "jsle_reg": 0xdd,
}
NAMES = {v: k for k, v in OPS.items()}
assert len(OPS) == 90 and len(NAMES) == 90

COND_JUMPS = {v for k, v in OPS.items() if k.startswith("j") and k != "ja"}
ALU32 = {v for v in OPS.values() if v & 7 == 4}
ALU64 = {v for v in OPS.values() if v & 7 == 7}
LDX = {0x61, 0x69, 0x71, 0x79}
ST = {0x62, 0x6a, 0x72, 0x7a}
STX = {0x63, 0x6b, 0x73, 0x7b}
MEM_SIZE = {0x61: 4, 0x69: 2, 0x71: 1, 0x79: 8, 0x62: 4, 0x6a: 2, 0x72: 1, 0x7a: 8,
            0x63: 4, 0x6b: 2, 0x73: 1, 0x7b: 8}


def uses_dst(op):
    return op not in (0x05, 0x85, 0x95)


def uses_src(op):
    cls = op & 7
    if cls in (1, 3):
        return True
    if cls in (4, 5, 7) and (op & 0x08):
        return op not in (0xdc, 0x85, 0x95)
    return False


def encode(op, dst=0, src=0, off=0, imm=0):
    """One 8-byte struct ebpf_inst."""
    return struct.pack("<BBhi", op & 0xff, (dst & 0xf) | ((src & 0xf) << 4),
                       int(off), int(imm))


def decode(b):
    op, regs, off, imm = struct.unpack("<BBhi", bytes(b[:8]))
    return op, regs & 0xf, regs >> 4, off, imm


class Insn:
    """A single (non-LDDW) instruction.  ``op`` may be a name from OPS or a byte."""
    __slots__ = ("op", "dst", "src", "off", "imm")

    def __init__(self, op, dst=0, src=0, off=0, imm=0):
        self.op = OPS[op] if isinstance(op, str) else op
        self.dst, self.src, self.off, self.imm = dst, src, off, imm

    def encode(self):
        return encode(self.op, self.dst, self.src, self.off, self.imm)

    def __repr__(self):
        return "%s d=%d s=%d off=%d imm=%d" % (NAMES.get(self.op, hex(self.op)), self.dst,
                                               self.src, self.off, self.imm)


def s32(x):
    x &= 0xffffffff
    return x - (1 << 32) if x & 0x80000000 else x
