/* Dumps the bytes of every reference ISA construction macro that compiles
 * (sys/sys/ebpf_vm_isa.h:107-143), for comparing the drop-in header with the reference's.
 * Built twice by tests/test_isa_macros.py: against include/ebpf_vm_isa.h and against the
 * reference header itself (EBPF_ISA_HEADER). */
#include <stdint.h>
#include <stdio.h>
#include EBPF_ISA_HEADER

static struct ebpf_inst insns[] = {
	EBPF_ALU_IMM(EBPF_ADD, 1, -5), EBPF_ALU_IMM(EBPF_MOV, 9, 0x7fffffff),
	EBPF_ALU_REG(EBPF_SUB, 2, 3), EBPF_ALU_REG(EBPF_XOR, 10, 1),
	EBPF_ALU64_IMM(EBPF_MUL, 4, 12345), EBPF_ALU64_IMM(EBPF_ARSH, 0, 63),
	EBPF_ALU64_REG(EBPF_MOV, 5, 6), EBPF_ALU64_REG(EBPF_DIV, 7, 8),
	EBPF_LE(3, 16), EBPF_LE(4, 64), EBPF_BE(5, 32), EBPF_BE(6, 64),
	EBPF_JMP_IMM(EBPF_JEQ, 1, -3, 99), EBPF_JMP_IMM(EBPF_JSLE, 2, 7, -1),
	EBPF_JMP_REG(EBPF_JGT, 3, 4, 12), EBPF_JMP_REG(EBPF_JSET, 9, 10, -32768),
	EBPF_JMP_CALL(0), EBPF_JMP_CALL(63), EBPF_JMP_EXIT,
};

int
main(void)
{
	fwrite(insns, 1, sizeof(insns), stdout);
	return 0;
}
