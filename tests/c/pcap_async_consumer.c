/* A C consumer of the host-input entry points (include/ebpf_gpu.h): builds a small classic pcap
 * capture in memory, turns it into a batch with ebpf_pcap_batch, checks the batch, and with
 * argv[1] == "gpu" runs a program over it through ebpf_prog_run_batch_async / ebpf_batch_wait
 * and checks every verdict against ebpf_prog_run on the same record bytes.  Prints "ok". */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ebpf.h"
#include "ebpf_gpu.h"
#include "ebpf_vm_isa.h"

static size_t
put32(uint8_t *p, uint32_t v)
{
	memcpy(p, &v, 4);
	return 4;
}

int
main(int argc, char **argv)
{
	enum { N = 1000 };
	static uint8_t cap[24 + N * (16 + 80)];
	size_t at = 0;
	at += put32(cap + at, 0xa1b2c3d4u);
	at += put32(cap + at, 0x00040002u);
	at += put32(cap + at, 0);
	at += put32(cap + at, 0);
	at += put32(cap + at, 65535);
	at += put32(cap + at, 1);
	uint64_t want_len[N];
	for (int i = 0; i < N; i++) {
		const uint32_t len = (uint32_t)(i * 37 % 81); /* 0..80 bytes */
		at += put32(cap + at, 1700000000u + i);
		at += put32(cap + at, (uint32_t)i);
		at += put32(cap + at, len);
		at += put32(cap + at, len);
		for (uint32_t k = 0; k < len; k++)
			cap[at + k] = (uint8_t)(i * 7 + k * 13);
		at += len;
		want_len[i] = len;
	}
	struct ebpf_pkt_batch b;
	struct ebpf_pcap_info pi;
	if (ebpf_pcap_batch(cap, at, 0, &b, &pi) != 0 || b.count != N || pi.linktype != 1) {
		printf("pcap_batch failed: %s\n", ebpf_gpu_last_error());
		return 1;
	}
	for (int i = 0; i < N; i++) {
		const uint8_t *p = (const uint8_t *)b.data + b.offsets[i];
		if (b.offsets[i + 1] - b.offsets[i] != want_len[i] ||
		    (want_len[i] && p[want_len[i] - 1] != (uint8_t)(i * 7 + (want_len[i] - 1) * 13))) {
			printf("record %d differs\n", i);
			return 1;
		}
	}
	if (argc > 1 && strcmp(argv[1], "gpu") == 0) {
		/* r0 = the packet's byte 20 (records shorter than 21 bytes fault MEM) */
		struct ebpf_inst prog[] = {
			{.opcode = EBPF_OP_LDXB, .dst = EBPF_R0, .src = EBPF_R1, .offset = 20},
			{.opcode = EBPF_OP_EXIT},
		};
		struct ebpf_env *ee;
		struct ebpf_prog *ep;
		struct ebpf_config cfg;
		memset(&cfg, 0, sizeof(cfg));
		static struct ebpf_prog_type pt = {"test"};
		cfg.prog_types[0] = &pt;
		if (ebpf_init() || ebpf_env_create(&ee, &cfg) ||
		    ebpf_prog_create(ee, &ep, &(struct ebpf_prog_attr){.type = 0, .prog = prog,
								       .prog_len = sizeof(prog)})) {
			printf("setup failed\n");
			return 1;
		}
		uint64_t *v = calloc(N, 8);
		uint8_t *f = calloc(N, 1);
		struct ebpf_batch_job *job;
		struct ebpf_batch_stats st;
		if (ebpf_prog_run_batch_async(ep, &b, v, f, &job) || ebpf_batch_wait(job, &st)) {
			printf("async batch failed: %s\n", ebpf_gpu_last_error());
			return 1;
		}
		for (int i = 0; i < N; i++) {
			const int faults = want_len[i] < 21;
			if ((f[i] != 0) != faults ||
			    (!faults && v[i] != (uint64_t)(uint8_t)(i * 7 + 20 * 13))) {
				printf("verdict %d differs: %llu fault %u\n", i, (unsigned long long)v[i], f[i]);
				return 1;
			}
		}
		free(v);
		free(f);
		ebpf_prog_destroy(ep);
		ebpf_env_destroy(ee);
	}
	ebpf_pcap_batch_free(&b);
	printf("ok\n");
	return 0;
}
