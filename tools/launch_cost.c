/* Host cost of one device-resident launch: a C caller of
 * ebpf_prog_run_batch_dev, no Python, C2's shape (1M x 64-B packets, a short ALU program, the
 * verdict histogram in overwrite mode), on the default stream.
 *
 *   enqueue  : host us per call while the GPU falls behind (K calls, no wait)
 *   step     : wall us per call including the GPU (K calls, then synchronize)
 *   timed    : the same with ebpf_gpu_time_next_launch events on every 2nd call
 *   raw      : hipLaunchKernel-free floor: hipEventRecord pairs (two runtime calls) per call
 *
 * Build: tools/launch_cost.sh.  Usage: launch_cost [K] [packets] */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ebpf.h"
#include "ebpf_gpu.h"
#include "ebpf_vm_isa.h"

static double
now_us(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec * 1e6 + t.tv_nsec / 1e3;
}

int
main(int argc, char **argv)
{
	const int K = argc > 1 ? atoi(argv[1]) : 2000;
	const uint64_t n = argc > 2 ? strtoull(argv[2], NULL, 0) : (1u << 20);
	/* reference stepping visits slots 0, 1, 3, 6: LDXW r0 [r1+4]; ADD r0 7; (pad); RSH r0 3;
	 * (pad x2); EXIT at slot 10 */
	struct ebpf_inst prog[11];
	memset(prog, 0, sizeof(prog));
	prog[0] = (struct ebpf_inst){.opcode = EBPF_OP_LDXW, .dst = EBPF_R0, .src = EBPF_R1, .offset = 4};
	prog[1] = (struct ebpf_inst){.opcode = EBPF_OP_ADD_IMM, .dst = EBPF_R0, .imm = 7};
	prog[3] = (struct ebpf_inst){.opcode = EBPF_OP_AND_IMM, .dst = EBPF_R0, .imm = 0xff};
	prog[6] = (struct ebpf_inst){.opcode = EBPF_OP_RSH_IMM, .dst = EBPF_R0, .imm = 3};
	prog[10] = (struct ebpf_inst){.opcode = EBPF_OP_EXIT};
	struct ebpf_env *ee;
	struct ebpf_prog *ep;
	struct ebpf_config cfg;
	memset(&cfg, 0, sizeof(cfg));
	static struct ebpf_prog_type pt = {"bench"};
	cfg.prog_types[0] = &pt;
	if (ebpf_init() || ebpf_env_create(&ee, &cfg) ||
	    ebpf_prog_create(ee, &ep, &(struct ebpf_prog_attr){.type = 0, .prog = prog,
							       .prog_len = sizeof(prog)})) {
		printf("setup failed\n");
		return 1;
	}
	void *d_pk, *d_ret, *d_hist;
	if (hipMalloc(&d_pk, n * 64) || hipMalloc(&d_ret, n * 8) || hipMalloc(&d_hist, 257 * 8) ||
	    hipMemset(d_pk, 0x5a, n * 64)) {
		printf("hipMalloc failed\n");
		return 1;
	}
	struct ebpf_pkt_batch b = {d_pk, NULL, n, 64, EBPF_BATCH_HIST_OVERWRITE};
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	for (int i = 0; i < 50; i++)
		if (ebpf_prog_run_batch_dev(ep, 0, &b, d_ret, NULL, d_hist, NULL)) {
			printf("launch failed: %s\n", ebpf_gpu_last_error());
			return 1;
		}
	hipDeviceSynchronize();
	for (int rep = 0; rep < 3; rep++) {
		double t0 = now_us();
		for (int i = 0; i < K; i++)
			ebpf_prog_run_batch_dev(ep, 0, &b, d_ret, NULL, d_hist, NULL);
		double t1 = now_us();
		hipDeviceSynchronize();
		double t2 = now_us();
		for (int i = 0; i < K; i++) {
			if ((i & 1) == 0)
				ebpf_gpu_time_next_launch(e0, e1);
			ebpf_prog_run_batch_dev(ep, 0, &b, d_ret, NULL, d_hist, NULL);
		}
		hipDeviceSynchronize();
		double t3 = now_us();
		float kms = 0;
		hipEventElapsedTime(&kms, e0, e1);
		for (int i = 0; i < K; i++) {
			hipEventRecord(e0, NULL);
			hipEventRecord(e1, NULL);
		}
		double t4 = now_us();
		hipDeviceSynchronize();
		printf("{\"packets\": %llu, \"calls\": %d, \"enqueue_us\": %.2f, \"step_us\": %.2f, "
		       "\"timed_step_us\": %.2f, \"kernel_us\": %.2f, \"event_pair_us\": %.2f}\n",
		       (unsigned long long)n, K, (t1 - t0) / K, (t2 - t0) / K, (t3 - t2) / K, kms * 1e3,
		       (t4 - t3) / K);
	}
	hipFree(d_pk);
	hipFree(d_ret);
	hipFree(d_hist);
	ebpf_prog_destroy(ep);
	ebpf_env_destroy(ee);
	return 0;
}
