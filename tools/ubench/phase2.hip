// Write phasing with the result slots in VGPRs, as the staged kernel keeps them: how much do
// more slots per wave buy?  The floor kernel's packet DMA (one 4-KB LDS buffer per wave,
// superblocks of K groups per wave, default 8), results of the last R groups in registers (slot = the
// group's sequence number mod R, static after unrolling by R), written when the constant clock
// is inside the window or when the next group's slot is taken.  16 waves per CU throughout.
// hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))

template <int R, int K = 8, int PW = 0, int SP = 0, int XS = 0>
__global__ void __launch_bounds__(256) k_phase2(const uint8_t *__restrict__ in, uint64_t *__restrict__ out, uint32_t ngroups,
						uint32_t nwaves_total, uint32_t pmask, uint32_t win) {
	extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
	const int lane = threadIdx.x & 63;
	const int wave = threadIdx.x >> 6;
	uint8_t *buf = lds + wave * 4096;
	const uint32_t gw = blockIdx.x * 4 + wave;
	auto group_at = [&](uint32_t i) -> uint32_t { return (gw + (i / K) * nwaves_total) * K + (i % K); };
	auto issue = [&](uint32_t i) {
		uint32_t g = group_at(i);
		if (g >= ngroups) return;
		const uint8_t *src = in + (uint64_t)g * 4096 + lane * 16;
#pragma unroll
		for (int q = 0; q < 4; q++)
			__builtin_amdgcn_global_load_lds((const void *)(src + q * 1024), LDS_PTR(buf + q * 1024), 16, 0, 2);
	};
	uint64_t r[R];
	uint32_t pend = 0;
	int nst = 0; // PW: result stores issued after the newest DMA (waited for only as far as needed)
	// write every pending slot; slot j holds sequence number base + j (j <= k) or base - R + j
	auto flush = [&](uint32_t base, int k) {
#pragma unroll
		for (int j = 0; j < R; j++)
			if (pend & (1u << j)) {
				const uint32_t seq = j <= k ? base + j : base - R + j;
				if (SP) out[(uint64_t)group_at(seq) * 64 + lane] = r[j];   // SP: plain stores
				else __builtin_nontemporal_store(r[j], out + (uint64_t)group_at(seq) * 64 + lane);
				nst++;
			}
		pend = 0;
	};
	// XS: each XCD's windows start XS ticks after the previous XCD's
	uint32_t xcc = 0;
	if (XS) asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
	const uint32_t tshift = XS * xcc;
	issue(0);
	for (uint32_t base = 0;; base += R) {
		bool done = false;
#pragma unroll
		for (int k = 0; k < R; k++) {
			const uint32_t i = base + k;
			const uint32_t g = group_at(i);
			if (g >= ngroups) {
				done = true;
				if (pend) flush(base, k - 1);
				break;
			}
			// the slot about to be written still pending: write everything first
			if (pend & (1u << k)) flush(base, k - 1);
			if (PW) {
				// vmcnt retires in order: the DMA is done once at most nst younger stores remain
#define W(n) case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
				switch (nst < 16 ? nst : 16) {
				W(0) W(1) W(2) W(3) W(4) W(5) W(6) W(7) W(8) W(9) W(10) W(11) W(12) W(13) W(14) W(15) W(16)
				}
#undef W
			} else {
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			}
			typedef unsigned v4u __attribute__((ext_vector_type(4)));
			v4u a, b, c, d;
			const uint32_t la = (uint32_t)(uintptr_t)(buf + lane * 64);
			asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\t"
				     "ds_read_b128 %2, %4 offset:32\n\tds_read_b128 %3, %4 offset:48\n\t"
				     "s_waitcnt lgkmcnt(0)"
				     : "=v"(a), "=v"(b), "=v"(c), "=v"(d) : "v"(la) : "memory");
			issue(i + 1);
			nst = 0;
			r[k] = (uint64_t)(a.x ^ b.y ^ c.z ^ d.w) | ((uint64_t)(a.w + d.x) << 32);
			pend |= 1u << k;
			const uint32_t t = (uint32_t)__builtin_amdgcn_s_memrealtime() + tshift;
			if (win && (t & pmask) < win) flush(base, k);
			else if (!win && k == R - 1) flush(base, k);   // no phasing: R-group bursts
		}
		if (done) break;
	}
}

template <int R, int K = 8, int PW = 0, int SP = 0, int XS = 0>
void run(const uint8_t *in, uint64_t *out, uint32_t ngroups, uint64_t npk, uint32_t pmask, uint32_t win) {
	const int lds = 4 * 4096, wgs = 256 * 4;
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	for (int it = 0; it < 3; it++) k_phase2<R, K, PW, SP, XS><<<wgs, 256, lds>>>(in, out, ngroups, wgs * 4, pmask, win);
	(void)hipEventRecord(a);
	for (int it = 0; it < 10; it++) k_phase2<R, K, PW, SP, XS><<<wgs, 256, lds>>>(in, out, ngroups, wgs * 4, pmask, win);
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms;
	(void)hipEventElapsedTime(&ms, a, b);
	ms /= 10;
	printf("SP=%d XS=%4d PW=%d K=%2d R=%2d period=%5u window=%5u: %.4f ms  %.1f Gpkt/s\n", SP, XS, PW, K, R, pmask + 1, win, ms, npk / ms / 1e6);
}

int main() {
	const uint64_t npk = 1ull << 26;
	const uint32_t ngroups = npk / 64;
	uint8_t *in;
	uint64_t *out;
	if (hipMalloc(&in, npk * 64) || hipMalloc(&out, npk * 8)) {
		printf("hipMalloc failed\n");
		return 1;
	}
	(void)hipMemset(in, 1, npk * 64);
	for (int rep = 0; rep < 3; rep++) {
		run<8>(in, out, ngroups, npk, 0, 0);
		run<16>(in, out, ngroups, npk, 4095, 1024);
		run<16, 8, 0, 1>(in, out, ngroups, npk, 4095, 1024);
		run<16, 8, 0, 0, 128>(in, out, ngroups, npk, 4095, 1024);
		run<16, 8, 0, 0, 512>(in, out, ngroups, npk, 4095, 1024);
	}
	return 0;
}
