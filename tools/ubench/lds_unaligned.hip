// Correctness probe: do ds_read_u16 / ds_read_b32 / ds_read_b64 at addresses off their natural
// alignment return the bytes at that address on gfx950 (the LDS-staged general kernel reads
// packets staged from unaligned CSR offsets at any byte address)?  And what do they cost?
// Prints, per (instruction, address mod 8), OK or the first mismatch, then cycles per
// wave-instruction for aligned vs unaligned b32 / b64 (s_memtime around 256 reads).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__global__ void probe(uint64_t *out, uint64_t *cyc)
{
	__shared__ __attribute__((aligned(16))) uint8_t buf[4096];
	const int t = threadIdx.x;
	for (int i = t; i < 4096; i += 64)
		buf[i] = (uint8_t)(i * 7 + 3);
	__syncthreads();
	const uint32_t base = (uint32_t)(uintptr_t)buf;
	// lane t reads at byte 64*t + m for m = 0..7, three widths
	for (int m = 0; m < 8; m++) {
		uint32_t a = base + 64 * t + 16 + m;
		uint32_t r16, r32;
		uint64_t r64;
		asm volatile("ds_read_u16 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r16) : "v"(a) : "memory");
		asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r32) : "v"(a) : "memory");
		asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r64) : "v"(a) : "memory");
		out[(t * 8 + m) * 3 + 0] = r16;
		out[(t * 8 + m) * 3 + 1] = r32;
		out[(t * 8 + m) * 3 + 2] = r64;
	}
	// timing: 256 dependent-free reads, aligned (m = 0) and unaligned (m = 1), b32 and b64
	for (int w = 0; w < 2; w++)
		for (int m = 0; m < 2; m++) {
			uint32_t a = base + 68 * t + m;
			uint64_t acc = 0, t0, t1;
			asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
			for (int k = 0; k < 256; k++) {
				if (w == 0) {
					uint32_t x;
					asm volatile("ds_read_b32 %0, %1 offset:0\n" : "=v"(x) : "v"(a) : "memory");
					acc += x;
				} else {
					uint64_t x;
					asm volatile("ds_read_b64 %0, %1 offset:0\n" : "=v"(x) : "v"(a) : "memory");
					acc += x;
				}
			}
			asm volatile("s_waitcnt lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
			if (t == 0)
				cyc[w * 2 + m] = t1 - t0;
			if (acc == 0x1234567)
				out[0] = acc;
		}
}

int
main()
{
	uint64_t *d_out, *d_cyc;
	hipMalloc(&d_out, 64 * 8 * 3 * 8);
	hipMalloc(&d_cyc, 4 * 8);
	hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_out, d_cyc);
	if (hipDeviceSynchronize() != hipSuccess) {
		printf("kernel failed\n");
		return 1;
	}
	uint64_t out[64 * 8 * 3], cyc[4];
	hipMemcpy(out, d_out, sizeof(out), hipMemcpyDeviceToHost);
	hipMemcpy(cyc, d_cyc, sizeof(cyc), hipMemcpyDeviceToHost);
	const char *nm[3] = {"ds_read_u16", "ds_read_b32", "ds_read_b64"};
	const int w[3] = {2, 4, 8};
	for (int k = 0; k < 3; k++)
		for (int m = 0; m < 8; m++) {
			int bad = -1;
			for (int t = 0; t < 64 && bad < 0; t++) {
				uint64_t want = 0;
				for (int b = 0; b < w[k]; b++)
					want |= (uint64_t)(uint8_t)((64 * t + 16 + m + b) * 7 + 3) << (8 * b);
				if (out[(t * 8 + m) * 3 + k] != want)
					bad = t;
			}
			printf("%s addr%%8=%d: %s\n", nm[k], m, bad < 0 ? "OK" : "MISMATCH");
		}
	printf("cycles/256 reads: b32 aligned %llu unaligned %llu; b64 aligned %llu unaligned %llu\n",
	       (unsigned long long)cyc[0], (unsigned long long)cyc[1], (unsigned long long)cyc[2],
	       (unsigned long long)cyc[3]);
	return 0;
}
