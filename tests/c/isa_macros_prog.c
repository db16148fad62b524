/*
 * A consumer of the drop-in headers (include/ebpf.h, include/ebpf_vm_isa.h, include/ebpf_gpu.h):
 * builds a program with the reference's ISA construction macros (sys/sys/ebpf_vm_isa.h:107-143,
 * the ones that compile, with their encodings as they are: EBPF_ALU_REG / EBPF_ALU64_REG carry
 * the immediate source bit), laid out on the reference's cumulative stepping path
 * (slots 0,1,3,6,10,15,21,28 straight on; a taken jump adds its offset to
 * the stride: ebpf_interpreter.c:39,209-211), links lib/libebpf.so and runs it.
 *
 *   isa_macros_prog cpu   N out.bin   ebpf_prog_run once per packet (the reference API)
 *   isa_macros_prog batch N out.bin   ebpf_prog_run_batch on the GPU (include/ebpf_gpu.h)
 *
 * out.bin = the program bytes (NSLOTS x 8) followed by N u64 results.  Packet i is 64 bytes,
 * byte j = (i * 7 + j * 13) & 0xff.  Expected r0 for byte0 = b: b <= 0x70 -> 0x71;
 * b > 0xc0 -> 0x170; otherwise 0x70 (tests/test_isa_macros.py checks this and the oracle).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdbool.h>
#include <stdint.h>

#include "ebpf.h"
#include "ebpf_vm_isa.h"
#include "ebpf_gpu.h"

#define NSLOTS 60

static struct ebpf_inst prog[NSLOTS] = {
	[0] = EBPF_ALU_IMM(EBPF_MOV, EBPF_R0, 7),              /* r0 = 7 */
	[1] = {EBPF_OP_LDXB, EBPF_R2, EBPF_R1, 0, 0},          /* r2 = pkt[0] (EBPF_LDX does not compile) */
	[3] = EBPF_ALU_REG(EBPF_ADD, EBPF_R0, EBPF_R2),        /* encodes ADD_IMM 0: r0 stays 7 */
	[6] = EBPF_ALU64_REG(EBPF_XOR, EBPF_R0, EBPF_R2),      /* encodes XOR64_IMM 0: r0 stays 7 */
	[10] = EBPF_ALU64_IMM(EBPF_LSH, EBPF_R0, 4),           /* r0 = 0x70 */
	[15] = EBPF_JMP_REG(EBPF_JGT, EBPF_R2, EBPF_R0, 2),    /* pkt[0] > 0x70: pc 6 -> 8, next slot 23 */
	[21] = EBPF_ALU_IMM(EBPF_ADD, EBPF_R0, 1),             /* not taken: r0 = 0x71 */
	[28] = EBPF_JMP_EXIT,
	[23] = EBPF_BE(EBPF_R2, 16),                           /* taken: r2 = pkt[0] << 8 */
	[32] = EBPF_JMP_IMM(EBPF_JGT, EBPF_R2, 1, 0xc000),     /* pkt[0] > 0xc0 */
	[42] = EBPF_LE(EBPF_R0, 16),                           /* r0 = 0x70 */
	[53] = EBPF_JMP_EXIT,
	[43] = EBPF_ALU_IMM(EBPF_OR, EBPF_R0, 0x100),          /* r0 = 0x170 */
	[55] = EBPF_JMP_EXIT,
};

static bool map_ok(struct ebpf_map_type *t) { (void)t; return true; }
static bool helper_ok(struct ebpf_helper_type *t) { (void)t; return true; }

int
main(int argc, char **argv)
{
	if (argc != 4)
		return 2;
	const int batch = strcmp(argv[1], "batch") == 0;
	const uint64_t n = strtoull(argv[2], NULL, 0);
	static struct ebpf_prog_type ptype;
	static struct ebpf_config cfg;
	strcpy(ptype.name, "test");
	ptype.ops.is_map_usable = map_ok;
	ptype.ops.is_helper_usable = helper_ok;
	cfg.prog_types[0] = &ptype;
	cfg.map_types[0] = &emt_array;
	cfg.helper_types[0] = &eht_map_lookup_elem;

	struct ebpf_env *ee;
	struct ebpf_prog *ep;
	if (ebpf_init() || ebpf_env_create(&ee, &cfg))
		return 3;
	struct ebpf_prog_attr attr = {.type = 0, .prog = prog, .prog_len = sizeof(prog)};
	if (ebpf_prog_create(ee, &ep, &attr))
		return 4;
	uint8_t *pk = malloc(n * 64 + 1);
	uint64_t *ret = calloc(n + 1, 8);
	for (uint64_t i = 0; i < n; i++)
		for (int j = 0; j < 64; j++)
			pk[i * 64 + j] = (uint8_t)(i * 7 + j * 13);
	if (batch) {
		struct ebpf_pkt_batch b = {.data = pk, .offsets = NULL, .count = n, .stride = 64, .flags = 0};
		struct ebpf_batch_stats st;
		int err = ebpf_prog_run_batch(ep, &b, ret, NULL, &st);
		if (err) {
			fprintf(stderr, "ebpf_prog_run_batch: %d %s\n", err, ebpf_gpu_last_error());
			return 5;
		}
		if (st.packets != n || st.faulted != 0)
			return 6;
	} else {
		for (uint64_t i = 0; i < n; i++)
			ret[i] = ebpf_prog_run(pk + i * 64, ep);
	}
	FILE *f = fopen(argv[3], "wb");
	if (!f || fwrite(prog, 8, NSLOTS, f) != NSLOTS || fwrite(ret, 8, n, f) != n)
		return 7;
	fclose(f);
	ebpf_prog_destroy(ep);
	if (ebpf_env_destroy(ee))
		return 8;
	ebpf_deinit();
	return 0;
}
