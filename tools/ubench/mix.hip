// HBM ceilings for C4's traffic mix, with plain HIP kernels (no LDS DMA, no eBPF work): is the
// staged kernel's 8-B-result cost (0.22 ms on 64M packets) the skeleton's or HBM's?
//   rd      read 64M x 64 B, 16 B per lane coalesced (the read ceiling)
//   wr8     write 64M x 8 B only
//   wr64    write 64M x 64 B only
//   copy    read 64M x 64 B and write them back elsewhere (1:1 mix)
//   mix8    read 64M x 64 B, write 8 B per packet in 4-KB bursts per wave (C4's 8:1 mix)
//   lane8   the same mix, each lane loading its own packet's 64 B (4 x 16 B, 64-B lane stride:
//           direct per-lane staging without LDS)
//   memcpy  hipMemcpyDeviceToDevice of 4 GB
// Each at 16 and 32 waves per CU (grid-stride), stores nt and plain.  hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int OP, int NT>
__global__ void __launch_bounds__(256) k_mix(const v4u *__restrict__ in, v4u *__restrict__ out16,
					     uint64_t *__restrict__ out8, uint64_t ngroups) {
	const int lane = threadIdx.x & 63;
	const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
	const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
	uint32_t acc = 0;
	// superblocks of 8 groups (64 packets each) per wave, like the staged kernel
	for (uint64_t sg = wave; sg * 8 < ngroups; sg += nwaves) {
		uint64_t r[8];
#pragma unroll
		for (int k = 0; k < 8; k++) {
			const uint64_t g = sg * 8 + k;
			const v4u *p = in + g * 256;
			v4u a, b, c, d;
			if (OP == 5) { // lane's own packet
				a = p[lane * 4]; b = p[lane * 4 + 1]; c = p[lane * 4 + 2]; d = p[lane * 4 + 3];
			} else if (OP != 1 && OP != 2) {
				a = p[lane]; b = p[64 + lane]; c = p[128 + lane]; d = p[192 + lane];
			} else {
				a = b = c = d = (v4u){(unsigned)g, (unsigned)lane, 1u, 2u};
			}
			if (OP == 2 || OP == 3) { // 64 B per packet out
				v4u *q = out16 + g * 256;
				if (NT) {
					__builtin_nontemporal_store(a, q + lane); __builtin_nontemporal_store(b, q + 64 + lane);
					__builtin_nontemporal_store(c, q + 128 + lane); __builtin_nontemporal_store(d, q + 192 + lane);
				} else {
					q[lane] = a; q[64 + lane] = b; q[128 + lane] = c; q[192 + lane] = d;
				}
			}
			r[k] = (uint64_t)(a.x ^ b.y ^ c.z ^ d.w) | ((uint64_t)(a.w + d.x) << 32);
		}
		if (OP == 0) {
#pragma unroll
			for (int k = 0; k < 8; k++) acc ^= (uint32_t)r[k];
		} else if (OP == 1 || OP == 4 || OP == 5) {
#pragma unroll
			for (int k = 0; k < 8; k++) {
				uint64_t *q = out8 + (sg * 8 + k) * 64 + lane;
				if (NT) __builtin_nontemporal_store(r[k], q);
				else *q = r[k];
			}
		}
	}
	if (acc == 0x9e3779b9u) out8[0] = acc;
}

template <int OP, int NT>
float run(const v4u *in, v4u *out16, uint64_t *out8, uint64_t ngroups, int grid) {
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	for (int it = 0; it < 3; it++) k_mix<OP, NT><<<grid, 256>>>(in, out16, out8, ngroups);
	(void)hipEventRecord(a);
	for (int it = 0; it < 10; it++) k_mix<OP, NT><<<grid, 256>>>(in, out16, out8, ngroups);
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms;
	(void)hipEventElapsedTime(&ms, a, b);
	return ms / 10;
}

int main() {
	const uint64_t npk = 1ull << 26, ngroups = npk / 64;
	v4u *in, *out16;
	uint64_t *out8;
	if (hipMalloc(&in, npk * 64) || hipMalloc(&out16, npk * 64) || hipMalloc(&out8, npk * 8)) {
		printf("hipMalloc failed\n");
		return 1;
	}
	(void)hipMemset(in, 1, npk * 64);
	(void)hipDeviceSynchronize();
	const char *names[] = {"rd    ", "wr8   ", "wr64  ", "copy  ", "mix8  ", "lane8 "};
	const double rdb[] = {64, 0, 0, 64, 64, 64}, wrb[] = {0, 8, 64, 64, 8, 8};
	for (int rep = 0; rep < 2; rep++) {
		for (int op = 0; op < 6; op++)
			for (int nt = 0; nt < 2; nt++) {
				if (op == 0 && nt) continue;
				for (int wpc : {16, 32}) {
					const int grid = 256 * wpc / 4;
					float ms;
#define R(O) ms = nt ? run<O, 1>(in, out16, out8, ngroups, grid) : run<O, 0>(in, out16, out8, ngroups, grid)
					switch (op) {
					case 0: R(0); break;
					case 1: R(1); break;
					case 2: R(2); break;
					case 3: R(3); break;
					case 4: R(4); break;
					default: R(5); break;
					}
					const double rgb = npk * rdb[op] / 1e9, wgb = npk * wrb[op] / 1e9;
					printf("%s nt=%d waves/CU=%2d: %.4f ms  read %.2f GB  write %.2f GB  total %.0f GB/s  %.1f Gpkt/s\n",
					       names[op], nt, wpc, ms, rgb, wgb, (rgb + wgb) / ms * 1e3, npk / ms / 1e6);
				}
			}
		hipEvent_t a, b;
		(void)hipEventCreate(&a);
		(void)hipEventCreate(&b);
		for (int it = 0; it < 2; it++) (void)hipMemcpy(out16, in, npk * 64, hipMemcpyDeviceToDevice);
		(void)hipEventRecord(a);
		for (int it = 0; it < 5; it++) (void)hipMemcpyAsync(out16, in, npk * 64, hipMemcpyDeviceToDevice, 0);
		(void)hipEventRecord(b);
		(void)hipEventSynchronize(b);
		float ms;
		(void)hipEventElapsedTime(&ms, a, b);
		ms /= 5;
		printf("memcpy 4.29 GB d2d: %.4f ms  total %.0f GB/s\n", ms, 2 * npk * 64 / ms / 1e6);
	}
	return 0;
}
