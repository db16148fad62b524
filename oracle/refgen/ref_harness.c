/*
 * ref_harness.c — CONTAINER-ONLY golden-vector generator.  Links the GENUINE reference
 * libebpf.so (generic-ebpf @ v0, built from /root/reference per SURVEY.md Appendix B) and runs
 * ebpf_prog_run over every packet of a case file written by tools/gen_golden.py.  Never built
 * or run on the GPU box; nothing from the reference is copied into the repository — this file
 * only calls the reference's public API (sys/sys/ebpf.h:107-136).
 *
 * Each packet is run twice, with the interpreter's stack frame pre-poisoned by 0xAA and by
 * 0x55 (registers r0, r2-r9 and the 512-B eBPF stack live there, ebpf_interpreter.c:26-28);
 * a differing r0 flags an undefined read, which makes the case unusable as a golden vector.
 *
 * Usage: ref_harness <case.bin> <out.bin>
 * case: u32 magic 'EBPC', u32 version(1), u32 prog_len, u32 nmaps,
 *       nmaps × { u32 value_size, u32 max_entries, bytes[value_size*max_entries] },
 *       u32 nrelocs, nrelocs × { u32 slot, u32 map }, bytes[prog_len],
 *       u64 count, u32 stride, u32 mode (0 = fixed stride, 1 = offsets),
 *       mode 1: u64 offsets[count+1], u64 data_len, bytes[data_len]
 * out:  u64 r0[count], u8 undefined_read[count], bytes data_after[data_len]  (0xAA pass)
 */
#include <errno.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <sys/ebpf.h>
#include <sys/ebpf_vm_isa.h>

extern int ebpf_init(void);
extern int ebpf_deinit(void);

static bool is_map_usable(struct ebpf_map_type *emt) { (void)emt; return true; }
static bool is_helper_usable(struct ebpf_helper_type *eht) { (void)eht; return true; }

static const struct ebpf_prog_type ept_harness = {"harness", {is_map_usable, is_helper_usable}};

static struct ebpf_config cfg; /* filled at runtime: tests/test_common.hpp:59-75 layout */

static void
die(const char *m)
{
	fprintf(stderr, "ref_harness: %s\n", m);
	exit(2);
}

static void
rd(FILE *f, void *p, size_t n)
{
	if (n && fread(p, 1, n, f) != n)
		die("short read");
}

static __attribute__((noinline)) void
poison_stack(uint8_t v)
{
	volatile uint8_t buf[32768];
	memset((void *)buf, v, sizeof(buf));
	__asm__ volatile("" ::"r"(buf) : "memory");
}

static __attribute__((noinline)) uint64_t
run_poisoned(void *ctx, struct ebpf_prog *ep, uint8_t v)
{
	poison_stack(v);
	return ebpf_prog_run(ctx, ep);
}

int
main(int argc, char **argv)
{
	if (argc != 3)
		die("usage: ref_harness case.bin out.bin");
	FILE *f = fopen(argv[1], "rb");
	if (!f)
		die("cannot open case");
	uint32_t magic, ver, prog_len, nmaps;
	rd(f, &magic, 4);
	rd(f, &ver, 4);
	if (magic != 0x43504245u || ver != 1)
		die("bad magic");
	rd(f, &prog_len, 4);
	rd(f, &nmaps, 4);

	if (ebpf_init() != 0)
		die("ebpf_init");
	cfg.prog_types[0] = &ept_harness;
	cfg.map_types[0] = &emt_array;
	cfg.helper_types[0] = &eht_map_lookup_elem;
	cfg.helper_types[1] = &eht_map_update_elem;
	cfg.helper_types[2] = &eht_map_delete_elem;
	struct ebpf_env *ee;
	if (ebpf_env_create(&ee, &cfg) != 0)
		die("env");

	struct ebpf_map **maps = calloc(nmaps + 1, sizeof(*maps));
	for (uint32_t m = 0; m < nmaps; m++) {
		uint32_t vs, me;
		rd(f, &vs, 4);
		rd(f, &me, 4);
		struct ebpf_map_attr ma = {.type = 0, .key_size = 4, .value_size = vs,
					   .max_entries = me, .flags = 0};
		if (ebpf_map_create(ee, &maps[m], &ma) != 0)
			die("map create");
		uint8_t *val = malloc(vs);
		for (uint32_t k = 0; k < me; k++) {
			rd(f, val, vs);
			if (ebpf_map_update_elem_from_user(maps[m], &k, val, EBPF_ANY) != 0)
				die("map update");
		}
		free(val);
	}
	uint32_t nrel;
	rd(f, &nrel, 4);
	uint32_t *rel = calloc(2 * nrel + 2, 4);
	rd(f, rel, 8 * (size_t)nrel);
	uint8_t *code = malloc(prog_len + 16);
	rd(f, code, prog_len);
	for (uint32_t r = 0; r < nrel; r++) {
		uint64_t h = (uint64_t)(uintptr_t)maps[rel[2 * r + 1]];
		uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
		memcpy(code + 8 * (size_t)rel[2 * r] + 4, &lo, 4);
		memcpy(code + 8 * (size_t)rel[2 * r] + 12, &hi, 4);
	}
	uint64_t count;
	uint32_t stride, mode;
	rd(f, &count, 8);
	rd(f, &stride, 4);
	rd(f, &mode, 4);
	uint64_t *offs = NULL;
	if (mode == 1) {
		offs = malloc(8 * (count + 1));
		rd(f, offs, 8 * (count + 1));
	}
	uint64_t dlen;
	rd(f, &dlen, 8);
	uint8_t *data = malloc(dlen + 1), *work_a = malloc(dlen + 1), *work_b = malloc(dlen + 1);
	rd(f, data, dlen);
	fclose(f);
	memcpy(work_a, data, dlen);
	memcpy(work_b, data, dlen);

	struct ebpf_prog *ep;
	struct ebpf_prog_attr pa = {.type = 0, .prog = (struct ebpf_inst *)code,
				    .prog_len = prog_len};
	if (ebpf_prog_create(ee, &ep, &pa) != 0)
		die("prog create");

	if (getenv("REF_HARNESS_TIME")) {
		/* calibration mode: time the genuine reference over the batch, no poisoning */
		struct timespec t0, t1;
		double best = 1e30;
		uint64_t sink = 0;
		for (int pass = 0; pass < 5; pass++) {
			clock_gettime(CLOCK_MONOTONIC, &t0);
			for (uint64_t i = 0; i < count; i++) {
				uint64_t o = mode == 1 ? offs[i] : i * (uint64_t)stride;
				sink += ebpf_prog_run(work_a + o, ep);
			}
			clock_gettime(CLOCK_MONOTONIC, &t1);
			double s = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
			if (s < best)
				best = s;
		}
		fprintf(stderr, "reference ebpf_prog_run: %.2f Mpkt/s (best of 5, %llu packets, sink %llu)\n",
			count / best / 1e6, (unsigned long long)count, (unsigned long long)sink);
		return 0;
	}
	uint64_t *r0 = malloc(8 * count + 8);
	uint8_t *undef = calloc(count + 1, 1);
	for (uint64_t i = 0; i < count; i++) {
		uint64_t o = mode == 1 ? offs[i] : i * (uint64_t)stride;
		uint64_t a = run_poisoned(work_a + o, ep, 0xAA);
		uint64_t b = run_poisoned(work_b + o, ep, 0x55);
		r0[i] = a;
		undef[i] = a != b;
	}
	if (memcmp(work_a, work_b, dlen) != 0)
		for (uint64_t i = 0; i < count; i++)
			undef[i] |= 2; /* stores depended on undefined state */

	FILE *o = fopen(argv[2], "wb");
	if (!o)
		die("cannot open out");
	fwrite(r0, 8, count, o);
	fwrite(undef, 1, count, o);
	fwrite(work_a, 1, dlen, o);
	fclose(o);

	ebpf_prog_destroy(ep);
	for (uint32_t m = 0; m < nmaps; m++)
		ebpf_map_destroy(maps[m]);
	if (ebpf_env_destroy(ee) != 0)
		die("env busy");
	ebpf_deinit();
	return 0;
}
