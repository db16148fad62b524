// Design-point microbenchmark for the staged interpreter's memory pipeline (no eBPF work):
// each wave walks its 64-packet groups, LDS-DMAs each group's 4 KB (4 x global_load_lds_dwordx4,
// 1 KB each, coalesced) into one of NB per-wave LDS buffers PF groups ahead, reads its packets
// into registers, and writes one u64 result per packet, buffered over K groups (one K x 512-B
// burst, nt) — K = 1 is the interpreter's current pattern.  Groups are assigned in superblocks
// of K consecutive groups per wave.  Reports Gpkt/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))

template <int NB, int K>
__global__ void __launch_bounds__(256) k_pipe(const uint8_t *__restrict__ in, uint64_t *__restrict__ out,
					       uint32_t ngroups, uint32_t nwaves_total) {
	extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
	const int lane = threadIdx.x & 63;
	const int wave = threadIdx.x >> 6;
	uint8_t *buf = lds + wave * NB * 4096;
	const uint32_t gw = blockIdx.x * 4 + wave;
	// this wave's group sequence: superblocks of K groups
	auto group_at = [&](uint32_t i) -> uint32_t { return (gw + (i / K) * nwaves_total) * K + (i % K); };
	auto issue = [&](uint32_t i) {
		uint32_t g = group_at(i);
		if (g >= ngroups)
			return;
		const uint8_t *src = in + (uint64_t)g * 4096 + lane * 16;
		uint8_t *dst = buf + (i % NB) * 4096;
#pragma unroll
		for (int q = 0; q < 4; q++)
			__builtin_amdgcn_global_load_lds((const void *)(src + q * 1024), LDS_PTR(dst + q * 1024), 16, 0, 0);
	};
	uint64_t r[K];
	for (int p = 0; p < NB; p++)
		issue(p);
	for (uint32_t i = 0;; i++) {
		uint32_t g = group_at(i);
		if (g >= ngroups)
			break;
		// wait for the oldest buffer only: NB-1 younger groups of 4 DMA ops may be in flight
		// (a store burst issued in the previous iteration is younger than every DMA)
		const bool burst = i > 0 && ((i - 1) % K == K - 1);
		if (NB == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		else if (NB == 2) { if (burst) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(4 + K) : "memory");
				    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }
		else { if (burst) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(8 + K) : "memory");
		       else asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
		// LDS reads in inline asm: the compiler would otherwise drain every LDS-DMA (vmcnt(0))
		typedef unsigned v4u __attribute__((ext_vector_type(4)));
		v4u a, b, c, d;
		const uint32_t la = (uint32_t)(uintptr_t)(buf + (i % NB) * 4096 + lane * 64);
		asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\t"
			     "ds_read_b128 %2, %4 offset:32\n\tds_read_b128 %3, %4 offset:48\n\t"
			     "s_waitcnt lgkmcnt(0)"
			     : "=v"(a), "=v"(b), "=v"(c), "=v"(d) : "v"(la) : "memory");
		issue(i + NB);
		r[i % K] = (uint64_t)(a.x ^ b.y ^ c.z ^ d.w) | ((uint64_t)(a.w + d.x) << 32);
		if (i % K == K - 1) {
			uint32_t g0 = g - (K - 1);
#pragma unroll
			for (int k = 0; k < K; k++)
				__builtin_nontemporal_store(r[k], out + (uint64_t)(g0 + k) * 64 + lane);
		}
	}
}

template <int NB, int K>
void run(const uint8_t *in, uint64_t *out, uint32_t ngroups, uint64_t npk, int cus) {
	const int lds = 4 * NB * 4096;
	int wg_per_cu = 160 * 1024 / (lds + 4096); // + ~4 KB for the other interpreter regions
	if (wg_per_cu > 8) wg_per_cu = 8;
	uint32_t wgs = cus * wg_per_cu;
	if ((uint64_t)wgs * 4 * K > ngroups) wgs = ngroups / (4 * K);
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	for (int it = 0; it < 3; it++) k_pipe<NB, K><<<wgs, 256, lds>>>(in, out, ngroups, wgs * 4);
	(void)hipEventRecord(a);
	for (int it = 0; it < 10; it++) k_pipe<NB, K><<<wgs, 256, lds>>>(in, out, ngroups, wgs * 4);
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms;
	(void)hipEventElapsedTime(&ms, a, b);
	ms /= 10;
	printf("NB=%d K=%d waves/CU=%d: %.3f ms  %.1f Gpkt/s\n", NB, K, wg_per_cu * 4, ms, npk / ms / 1e6);
}

int main() {
	const uint64_t npk = 1ull << 26;
	const uint32_t ngroups = npk / 64;
	uint8_t *in;
	uint64_t *out;
	(void)hipMalloc(&in, npk * 64);
	(void)hipMalloc(&out, npk * 8);
	(void)hipMemset(in, 1, npk * 64);
	int cus = 256;
	run<1, 1>(in, out, ngroups, npk, cus);
	run<1, 8>(in, out, ngroups, npk, cus);
	run<2, 1>(in, out, ngroups, npk, cus);
	run<2, 4>(in, out, ngroups, npk, cus);
	run<2, 8>(in, out, ngroups, npk, cus);
	run<3, 8>(in, out, ngroups, npk, cus);
	run<1, 1>(in, out, ngroups, npk, cus);
	return 0;
}
