// Does phasing the result writes in time cut the read/write mixing cost?  On 64M x 64-B packets
// (tools/ubench/mix.hip): reads alone 0.626 ms, 8-B result writes alone 0.100 ms, both mixed
// (the staged kernel's skeleton) 0.855 ms.  Here the floor kernel's packet DMA (4 KB per group,
// one LDS buffer per wave) keeps each group's results in a per-wave LDS ring of R groups, and
// flushes the ring when the GPU's constant clock (s_memrealtime, 100 MHz, one counter for the
// chip) is inside a write window — (t & pmask) < win — or when the ring is full.  win = 0:
// flush only when full (no phasing, the baseline).  hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))

template <int R>
__global__ void __launch_bounds__(256) k_phase(const uint8_t *__restrict__ in, uint64_t *__restrict__ out, uint32_t ngroups,
					       uint32_t nwaves_total, uint32_t pmask, uint32_t win, uint32_t *stats, int hold) {
	extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
	const int lane = threadIdx.x & 63;
	const int wave = threadIdx.x >> 6;
	uint8_t *buf = lds + wave * (4096 + R * 512);
	uint64_t *ring = (uint64_t *)(buf + 4096);
	const uint32_t gw = blockIdx.x * 4 + wave;
	const int K = 8; // superblocks of 8 contiguous groups per wave, as in the staged kernel
	auto group_at = [&](uint32_t i) -> uint32_t { return (gw + (i / K) * nwaves_total) * K + (i % K); };
	auto issue = [&](uint32_t i) {
		uint32_t g = group_at(i);
		if (g >= ngroups) return;
		const uint8_t *src = in + (uint64_t)g * 4096 + lane * 16;
#pragma unroll
		for (int q = 0; q < 4; q++)
			__builtin_amdgcn_global_load_lds((const void *)(src + q * 1024), LDS_PTR(buf + q * 1024), 16, 0, 2);
	};
	uint32_t pend_g[R];
	int p = 0;
	uint32_t forced = 0, windows = 0;
	auto flush = [&]() {
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
		for (int k = 0; k < R; k++) {
			if (k >= p) break;
			__builtin_nontemporal_store(ring[k * 64 + lane], out + (uint64_t)pend_g[k] * 64 + lane);
		}
		p = 0;
	};
	issue(0);
	for (uint32_t i = 0;; i++) {
		uint32_t g = group_at(i);
		if (g >= ngroups) break;
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		typedef unsigned v4u __attribute__((ext_vector_type(4)));
		v4u a, b, c, d;
		const uint32_t la = (uint32_t)(uintptr_t)(buf + lane * 64);
		asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\t"
			     "ds_read_b128 %2, %4 offset:32\n\tds_read_b128 %3, %4 offset:48\n\t"
			     "s_waitcnt lgkmcnt(0)"
			     : "=v"(a), "=v"(b), "=v"(c), "=v"(d) : "v"(la) : "memory");
		uint64_t res = (uint64_t)(a.x ^ b.y ^ c.z ^ d.w) | ((uint64_t)(a.w + d.x) << 32);
		if (win == 0) {
			// baseline: results in the ring, flushed when it is full (R-group bursts)
			ring[p * 64 + lane] = res;
			pend_g[p] = g;
			p++;
			if (p == R) flush();
			issue(i + 1);
			continue;
		}
		ring[p * 64 + lane] = res;
		pend_g[p] = g;
		p++;
		const uint32_t t = (uint32_t)__builtin_amdgcn_s_memrealtime();
		if ((t & pmask) < win) {
			windows++;
			flush();
			// HOLD: no packet reads inside the window (write-only phases)
			if (hold)
				while (((uint32_t)__builtin_amdgcn_s_memrealtime() & pmask) < win)
					__builtin_amdgcn_s_sleep(2);
		} else if (p == R) {
			forced++;
			flush();
		}
		issue(i + 1);
	}
	if (p) flush();
	if (lane == 0 && stats) {
		atomicAdd(stats, forced);
		atomicAdd(stats + 1, windows);
	}
}

static uint32_t *stats;

template <int R>
void run(const uint8_t *in, uint64_t *out, uint32_t ngroups, uint64_t npk, int wpc, uint32_t pmask, uint32_t win, int hold = 0) {
	const int lds = 4 * (4096 + R * 512);
	const int wg_per_cu = wpc / 4;
	if (lds * wg_per_cu > 160 * 1024) {
		printf("R=%d waves/CU=%d: LDS does not fit\n", R, wpc);
		return;
	}
	const uint32_t wgs = 256 * wg_per_cu;
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	for (int it = 0; it < 3; it++) k_phase<R><<<wgs, 256, lds>>>(in, out, ngroups, wgs * 4, pmask, win, nullptr, hold);
	(void)hipEventRecord(a);
	for (int it = 0; it < 10; it++) k_phase<R><<<wgs, 256, lds>>>(in, out, ngroups, wgs * 4, pmask, win, nullptr, hold);
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms;
	(void)hipEventElapsedTime(&ms, a, b);
	ms /= 10;
	(void)hipMemset(stats, 0, 8);
	k_phase<R><<<wgs, 256, lds>>>(in, out, ngroups, wgs * 4, pmask, win, stats, hold);
	uint32_t h[2];
	(void)hipMemcpy(h, stats, 8, hipMemcpyDeviceToHost);
	printf("hold=%d R=%2d waves/CU=%d period=%5u ticks window=%4u: %.4f ms  %.1f Gpkt/s  (forced flushes %u, window flushes %u)\n", hold, R,
	       wpc, pmask + 1, win, ms, npk / ms / 1e6, h[0], h[1]);
}

int main(int argc, char **argv) {
	const uint64_t npk = 1ull << 26;
	const uint32_t ngroups = npk / 64;
	uint8_t *in;
	uint64_t *out;
	if (hipMalloc(&in, npk * 64) || hipMalloc(&out, npk * 8) || hipMalloc(&stats, 8)) {
		printf("hipMalloc failed\n");
		return 1;
	}
	(void)hipMemset(in, 1, npk * 64);
	if (argc > 1 && argv[1][0] == 'h') {
		// hold: waves issue no packet reads inside the window, against the kernel's way (reads go on)
		for (int rep = 0; rep < 2; rep++) {
			run<8>(in, out, ngroups, npk, 16, 0, 0);
			for (uint32_t w : {640u, 512u})
				run<8>(in, out, ngroups, npk, 16, 2047, w);
			for (uint32_t w : {256u, 341u, 512u})
				run<8>(in, out, ngroups, npk, 16, 2047, w, 1);
			for (uint32_t w : {128u, 192u, 256u})
				run<8>(in, out, ngroups, npk, 16, 1023, w, 1);
		}
		return 0;
	}
	for (int rep = 0; rep < 2; rep++) {
		run<8>(in, out, ngroups, npk, 16, 0, 0);
		run<12>(in, out, ngroups, npk, 16, 0, 0);
		// period 2^10..2^12 ticks (10-41 us), write window 1/8 .. 1/4 of it
		for (uint32_t pb : {10u, 11u, 12u})
			for (uint32_t wf : {8u, 6u, 4u}) {
				const uint32_t pm = (1u << pb) - 1, w = (1u << pb) / wf;
				run<12>(in, out, ngroups, npk, 16, pm, w);
			}
		run<8>(in, out, ngroups, npk, 16, 2047, 512);
	}
	return 0;
}
