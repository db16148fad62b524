/*
 * ebpf_vm_isa.h — eBPF instruction encoding understood by the MI355X engine.
 *
 * Drop-in for the reference's sys/sys/ebpf_vm_isa.h (generic-ebpf @ v0):
 *   - struct ebpf_inst          ↔ sys/sys/ebpf_vm_isa.h:21-27  (8 bytes, dst = low nibble of byte 1)
 *   - enum ebpf_registers       ↔ sys/sys/ebpf_vm_isa.h:29-42
 *   - class / source / size / mode / ALU-op / JMP-op fields ↔ :46-105
 *   - EBPF_OP_* opcode values   ↔ :145-238 (90 opcodes dispatched by ebpf_interpreter.c:40-369)
 *
 *   - construction macros       ↔ :107-143, bug for bug (see the block comment there)
 *
 * Every opcode below is spelled out as its final byte value so the table doubles as the
 * device decoder's reference.
 */
#ifndef EBPF_AMD_VM_ISA_H
#define EBPF_AMD_VM_ISA_H

#include <stdint.h>

struct ebpf_inst {
	uint8_t opcode;
	uint8_t dst : 4; /* low nibble of byte 1 */
	uint8_t src : 4; /* high nibble of byte 1 */
	int16_t offset;
	int32_t imm;
};

#ifdef __cplusplus
static_assert(sizeof(struct ebpf_inst) == 8, "ebpf_inst must stay 8 bytes (ABI)");
#else
_Static_assert(sizeof(struct ebpf_inst) == 8, "ebpf_inst must stay 8 bytes (ABI)");
#endif

enum ebpf_registers {
	EBPF_R0 = 0, EBPF_R1, EBPF_R2, EBPF_R3, EBPF_R4, EBPF_R5,
	EBPF_R6, EBPF_R7, EBPF_R8, EBPF_R9, EBPF_R10,
	EBPF_REG_MAX /* 11 */
};

#define EBPF_PSEUDO_MAP_DESC 1

/* opcode byte = | op (4 bits) | source (1 bit) | class (3 bits) |  (ALU / JMP)
 *             = | mode (3)    | size (2)       | class (3)       |  (LD / LDX / ST / STX) */
#define EBPF_CLS(op)     ((op) & 0x07)
#define EBPF_SRC(op)     ((op) & 0x08)
#define EBPF_SIZE(op)    ((op) & 0x18)
#define EBPF_MODE(op)    ((op) & 0xe0)
#define EBPF_ALU_OP(op)  ((op) & 0xf0)
#define EBPF_JMP_OP(op)  ((op) & 0xf0)

#define EBPF_CLS_LD    0x00
#define EBPF_CLS_LDX   0x01
#define EBPF_CLS_ST    0x02
#define EBPF_CLS_STX   0x03
#define EBPF_CLS_ALU   0x04
#define EBPF_CLS_JMP   0x05
#define EBPF_CLS_ALU64 0x07

#define EBPF_SRC_IMM 0x00
#define EBPF_SRC_REG 0x08
#define EBPF_TO_LE   0x00
#define EBPF_TO_BE   0x08

#define EBPF_SIZE_W  0x00
#define EBPF_SIZE_H  0x08
#define EBPF_SIZE_B  0x10
#define EBPF_SIZE_DW 0x18

#define EBPF_MODE_IMM 0x00
#define EBPF_MODE_MEM 0x60

#define EBPF_ADD  0x00
#define EBPF_SUB  0x10
#define EBPF_MUL  0x20
#define EBPF_DIV  0x30
#define EBPF_OR   0x40
#define EBPF_AND  0x50
#define EBPF_LSH  0x60
#define EBPF_RSH  0x70
#define EBPF_NEG  0x80
#define EBPF_MOD  0x90
#define EBPF_XOR  0xa0
#define EBPF_MOV  0xb0
#define EBPF_ARSH 0xc0
#define EBPF_END  0xd0

#define EBPF_JA   0x00
#define EBPF_JEQ  0x10
#define EBPF_JGT  0x20
#define EBPF_JGE  0x30
#define EBPF_JSET 0x40
#define EBPF_JNE  0x50
#define EBPF_JSGT 0x60
#define EBPF_JSGE 0x70
#define EBPF_CALL 0x80
#define EBPF_EXIT 0x90
#define EBPF_JLT  0xa0
#define EBPF_JLE  0xb0
#define EBPF_JSLT 0xc0
#define EBPF_JSLE 0xd0

/* ---- instruction construction macros (sys/sys/ebpf_vm_isa.h:107-143) ----
 * Brace initializers for struct ebpf_inst {opcode, dst, src, offset, imm}.  They reproduce the
 * reference's encodings exactly, defects included, so that a program built with them means the
 * same bytes against either header:
 *   - EBPF_ALU_REG / EBPF_ALU64_REG set the IMMEDIATE source bit (SRC_IMM, :109-110, :113-114):
 *     the instruction executes as "dst op imm" with imm = 0, src only recorded in the byte;
 *   - EBPF_LD / EBPF_LDX / EBPF_ST / EBPF_STX name EBPF_SRC_MEM, which neither header defines,
 *     and EBPF_STX would encode class ST (:119-126);
 *   - EBPF_LDDW names the undefined EBPF_DW (:127-129);
 *   - EBPF_PSEUDO_MAP_LD has no comma between its two initializers (:130-133);
 *   - EBPF_JMP_JA puts a variable named `imm` into the offset field and ignores `ofs` (:134-135).
 * The ones the reference can compile compile here to the same bytes
 * (tests/test_isa_macros.py builds a program with them and runs it). */
#define EBPF_ALU_IMM(op, dst, imm) \
	{ (EBPF_CLS_ALU | EBPF_SRC_IMM | op), dst, 0, 0, imm }
#define EBPF_ALU_REG(op, dst, src) \
	{ (EBPF_CLS_ALU | EBPF_SRC_IMM | op), dst, src, 0, 0 }
#define EBPF_ALU64_IMM(op, dst, imm) \
	{ (EBPF_CLS_ALU64 | EBPF_SRC_IMM | op), dst, 0, 0, imm }
#define EBPF_ALU64_REG(op, dst, src) \
	{ (EBPF_CLS_ALU64 | EBPF_SRC_IMM | op), dst, src, 0, 0 }
#define EBPF_LE(dst, size) \
	{ (EBPF_CLS_ALU | EBPF_TO_LE | EBPF_END), dst, 0, 0, size }
#define EBPF_BE(dst, size) \
	{ (EBPF_CLS_ALU | EBPF_TO_BE | EBPF_END), dst, 0, 0, size }
#define EBPF_LD(size, dst, src, ofs) \
	{ (EBPF_CLS_LD | EBPF_SRC_MEM | size), dst, src, ofs, 0 }
#define EBPF_LDX(size, dst, src, ofs) \
	{ (EBPF_CLS_LDX | EBPF_SRC_MEM | size), dst, src, ofs, 0 }
#define EBPF_ST(size, dst, src, ofs) \
	{ (EBPF_CLS_ST | EBPF_SRC_MEM | size), dst, src, ofs, 0 }
#define EBPF_STX(size, dst, src, ofs) \
	{ (EBPF_CLS_ST | EBPF_SRC_MEM | size), dst, src, ofs, 0 }
#define EBPF_LDDW(dst, imm) \
	{ (EBPF_CLS_LD | EBPF_SRC_IMM | EBPF_DW), dst, 0, 0, (uint32_t)imm }, \
	{ 0, 0, 0, 0, ((uint64_t)imm) >> 32 }
#define EBPF_PSEUDO_MAP_LD(dst, imm) \
	{ (EBPF_CLS_LD | EBPF_SRC_IMM | EBPF_DW), dst, \
		EBPF_PSEUDO_MAP_DESC, 0, (uint32_t)imm } \
	{ 0, 0, 0, 0, 0 }
#define EBPF_JMP_JA(ofs) \
	{ (EBPF_CLS_JMP | EBPF_JA ), 0, 0, imm, 0 }
#define EBPF_JMP_IMM(op, dst, ofs, imm) \
	{ (EBPF_CLS_JMP | EBPF_SRC_IMM | op), dst, 0, ofs, imm }
#define EBPF_JMP_REG(op, dst, src, ofs) \
	{ (EBPF_CLS_JMP | EBPF_SRC_REG | op), dst, src, ofs, 0 }
#define EBPF_JMP_CALL(id) \
	{ (EBPF_CLS_JMP | EBPF_CALL), 0, 0, 0, id }
#define EBPF_JMP_EXIT \
	{ (EBPF_CLS_JMP | EBPF_EXIT), 0, 0, 0, 0 }

/* ---- the 90 opcodes the reference interpreter dispatches (ebpf_interpreter.c:41-366) ---- */
/* ALU (32-bit) */
#define EBPF_OP_ADD_IMM   0x04
#define EBPF_OP_ADD_REG   0x0c
#define EBPF_OP_SUB_IMM   0x14
#define EBPF_OP_SUB_REG   0x1c
#define EBPF_OP_MUL_IMM   0x24
#define EBPF_OP_MUL_REG   0x2c
#define EBPF_OP_DIV_IMM   0x34
#define EBPF_OP_DIV_REG   0x3c
#define EBPF_OP_OR_IMM    0x44
#define EBPF_OP_OR_REG    0x4c
#define EBPF_OP_AND_IMM   0x54
#define EBPF_OP_AND_REG   0x5c
#define EBPF_OP_LSH_IMM   0x64
#define EBPF_OP_LSH_REG   0x6c
#define EBPF_OP_RSH_IMM   0x74
#define EBPF_OP_RSH_REG   0x7c
#define EBPF_OP_NEG       0x84
#define EBPF_OP_MOD_IMM   0x94
#define EBPF_OP_MOD_REG   0x9c
#define EBPF_OP_XOR_IMM   0xa4
#define EBPF_OP_XOR_REG   0xac
#define EBPF_OP_MOV_IMM   0xb4
#define EBPF_OP_MOV_REG   0xbc
#define EBPF_OP_ARSH_IMM  0xc4
#define EBPF_OP_ARSH_REG  0xcc
#define EBPF_OP_LE        0xd4
#define EBPF_OP_BE        0xdc
/* ALU64 */
#define EBPF_OP_ADD64_IMM  0x07
#define EBPF_OP_ADD64_REG  0x0f
#define EBPF_OP_SUB64_IMM  0x17
#define EBPF_OP_SUB64_REG  0x1f
#define EBPF_OP_MUL64_IMM  0x27
#define EBPF_OP_MUL64_REG  0x2f
#define EBPF_OP_DIV64_IMM  0x37
#define EBPF_OP_DIV64_REG  0x3f
#define EBPF_OP_OR64_IMM   0x47
#define EBPF_OP_OR64_REG   0x4f
#define EBPF_OP_AND64_IMM  0x57
#define EBPF_OP_AND64_REG  0x5f
#define EBPF_OP_LSH64_IMM  0x67
#define EBPF_OP_LSH64_REG  0x6f
#define EBPF_OP_RSH64_IMM  0x77
#define EBPF_OP_RSH64_REG  0x7f
#define EBPF_OP_NEG64      0x87
#define EBPF_OP_MOD64_IMM  0x97
#define EBPF_OP_MOD64_REG  0x9f
#define EBPF_OP_XOR64_IMM  0xa7
#define EBPF_OP_XOR64_REG  0xaf
#define EBPF_OP_MOV64_IMM  0xb7
#define EBPF_OP_MOV64_REG  0xbf
#define EBPF_OP_ARSH64_IMM 0xc7
#define EBPF_OP_ARSH64_REG 0xcf
/* memory */
#define EBPF_OP_LDXW   0x61
#define EBPF_OP_LDXH   0x69
#define EBPF_OP_LDXB   0x71
#define EBPF_OP_LDXDW  0x79
#define EBPF_OP_STW    0x62
#define EBPF_OP_STH    0x6a
#define EBPF_OP_STB    0x72
#define EBPF_OP_STDW   0x7a
#define EBPF_OP_STXW   0x63
#define EBPF_OP_STXH   0x6b
#define EBPF_OP_STXB   0x73
#define EBPF_OP_STXDW  0x7b
#define EBPF_OP_LDDW   0x18
/* jumps */
#define EBPF_OP_JA       0x05
#define EBPF_OP_JEQ_IMM  0x15
#define EBPF_OP_JEQ_REG  0x1d
#define EBPF_OP_JGT_IMM  0x25
#define EBPF_OP_JGT_REG  0x2d
#define EBPF_OP_JGE_IMM  0x35
#define EBPF_OP_JGE_REG  0x3d
#define EBPF_OP_JSET_IMM 0x45
#define EBPF_OP_JSET_REG 0x4d
#define EBPF_OP_JNE_IMM  0x55
#define EBPF_OP_JNE_REG  0x5d
#define EBPF_OP_JSGT_IMM 0x65
#define EBPF_OP_JSGT_REG 0x6d
#define EBPF_OP_JSGE_IMM 0x75
#define EBPF_OP_JSGE_REG 0x7d
#define EBPF_OP_CALL     0x85
#define EBPF_OP_EXIT     0x95
#define EBPF_OP_JLT_IMM  0xa5
#define EBPF_OP_JLT_REG  0xad
#define EBPF_OP_JLE_IMM  0xb5
#define EBPF_OP_JLE_REG  0xbd
#define EBPF_OP_JSLT_IMM 0xc5
#define EBPF_OP_JSLT_REG 0xcd
#define EBPF_OP_JSLE_IMM 0xd5
#define EBPF_OP_JSLE_REG 0xdd

#endif /* EBPF_AMD_VM_ISA_H */
