// Memory-pipeline floor of the staged interpreter (no eBPF work), swept over the knobs that a
// rewrite of the kernel skeleton could change:
//   NB     per-wave LDS packet buffers (NB-1 groups of 4 KB DMA'd ahead of the running one)
//   K      groups whose u64 results are written together (K x 512 B contiguous per wave)
//   ST     0 = u64 per lane nt, 1 = u64 plain, 2 = no result write (read ceiling),
//          3 = results staged in LDS, written as dwordx4 nt (1 KB per wave instruction)
//   LDNT   packet DMA cache policy nt
//   MAP    0 = superblocks of K groups interleaved over waves, 1 = one contiguous range per wave
//   TR     0 = the DMA's contiguous layout (lane l's packet at 64 l: the staging ds_read_b128 of
//          64 lanes at a 64-B stride conflict), 1 = chunk-transposed by the DMA itself (lane l
//          of DMA q loads its packet's 16-B chunk q to 1024 q + 16 l: conflict-free reads),
//          2 = permuted inside each DMA's own 1 KB (lane l of DMA q loads chunk l >> 4 of packet
//          16 q + (l & 15): LDS chunk 64 q + 16 c + m holds packet 16 q + m's chunk c, so the
//          reads of one chunk by 16 lanes are 256 contiguous bytes)
// plus waves per CU (workgroups per CU x 4).  Reports Gpkt/s of 64-B packets.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))

template <int NB, int K, int ST, int LDNT, int MAP, int COMP = 0, int TR = 0>
__global__ void __launch_bounds__(256) k_floor(const uint8_t *__restrict__ in, uint64_t *__restrict__ out,
					       uint32_t ngroups, uint32_t nwaves_total) {
	extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
	const int lane = threadIdx.x & 63;
	const int wave = threadIdx.x >> 6;
	uint8_t *buf = lds + wave * (NB * 4096 + (ST == 3 ? K * 512 : 0));
	uint64_t *rbuf = (uint64_t *)(buf + NB * 4096);
	const uint32_t gw = blockIdx.x * 4 + wave;
	const uint32_t per = (ngroups + nwaves_total - 1) / nwaves_total;
	auto group_at = [&](uint32_t i) -> uint32_t {
		if (MAP == 1) {
			uint32_t g = gw * per + i;
			return (i < per) ? g : 0xffffffffu;
		}
		return (gw + (i / K) * nwaves_total) * K + (i % K);
	};
	auto issue = [&](uint32_t i) {
		uint32_t g = group_at(i);
		if (g >= ngroups)
			return;
		const uint8_t *src = in + (uint64_t)g * 4096 +
				     (TR == 2 ? 64 * (lane & 15) + 16 * (lane >> 4) : lane * (TR ? 64 : 16));
		uint8_t *dst = buf + (i % NB) * 4096;
#pragma unroll
		for (int q = 0; q < 4; q++)
			__builtin_amdgcn_global_load_lds((const void *)(src + q * (TR == 1 ? 16 : 1024)), LDS_PTR(dst + q * 1024),
							 16, 0, LDNT ? 2 : 0);
	};
	uint64_t r[K];
	for (int p = 0; p < NB; p++)
		issue(p);
	uint32_t acc = 0;
	for (uint32_t i = 0;; i++) {
		uint32_t g = group_at(i);
		if (g >= ngroups)
			break;
		// group i's DMA is the oldest outstanding operation but for stores issued before it;
		// the NB-1 younger groups (4 DMA ops each) and the stores issued after them may stay
		// in flight only if they are younger: waiting for vmcnt <= 4*(NB-1) is exact for the
		// DMA and merely stricter for stores (the interpreter's NB = 1 waits for everything)
		if (NB == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		else if (NB == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
		else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
		typedef unsigned v4u __attribute__((ext_vector_type(4)));
		v4u a, b, c, d;
		const uint32_t la = (uint32_t)(uintptr_t)(buf + (i % NB) * 4096 +
							  (TR == 2 ? 1024 * (lane >> 4) + 16 * (lane & 15) : lane * (TR ? 16 : 64)));
		if (TR == 2)
			asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:256\n\t"
				     "ds_read_b128 %2, %4 offset:512\n\tds_read_b128 %3, %4 offset:768\n\t"
				     "s_waitcnt lgkmcnt(0)"
				     : "=v"(a), "=v"(b), "=v"(c), "=v"(d) : "v"(la) : "memory");
		else if (TR)
			asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\t"
				     "ds_read_b128 %2, %4 offset:2048\n\tds_read_b128 %3, %4 offset:3072\n\t"
				     "s_waitcnt lgkmcnt(0)"
				     : "=v"(a), "=v"(b), "=v"(c), "=v"(d) : "v"(la) : "memory");
		else
			asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\t"
				     "ds_read_b128 %2, %4 offset:32\n\tds_read_b128 %3, %4 offset:48\n\t"
				     "s_waitcnt lgkmcnt(0)"
				     : "=v"(a), "=v"(b), "=v"(c), "=v"(d) : "v"(la) : "memory");
		issue(i + NB);
		uint64_t res = (uint64_t)(a.x ^ b.y ^ c.z ^ d.w) | ((uint64_t)(a.w + d.x) << 32);
		// synthetic per-group work like a classifier's hash: COMP dependent rounds of
		// 64-bit multiply + shift-xor (3 quarter-rate multiplies each)
#pragma unroll
		for (int q = 0; q < COMP; q++)
			res = (res ^ (res >> 29)) * 0x27d4eb2d165667c5ull + (uint64_t)q;
		if (ST == 2) {
			acc ^= (uint32_t)res;
			continue;
		}
		if (ST == 3) {
			rbuf[(i % K) * 64 + lane] = res;
		} else {
			r[i % K] = res;
		}
		if (i % K == K - 1 || (MAP == 1 && group_at(i + 1) >= ngroups)) {
			uint32_t g0 = g - (i % K);
			if (ST == 3) {
				asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // wave-local: LDS ops retire in order
				typedef unsigned v4u_t __attribute__((ext_vector_type(4)));
				const v4u_t *src = (const v4u_t *)rbuf;
				v4u_t *dst = (v4u_t *)(out + (uint64_t)g0 * 64);
#pragma unroll
				for (int q = 0; q < K / 2; q++)
					__builtin_nontemporal_store(src[q * 64 + lane], dst + q * 64 + lane);
			} else {
#pragma unroll
				for (int k = 0; k < K; k++) {
					if (k > (int)(i % K)) break;
					if (ST == 0) __builtin_nontemporal_store(r[k], out + (uint64_t)(g0 + k) * 64 + lane);
					else out[(uint64_t)(g0 + k) * 64 + lane] = r[k];
				}
			}
		}
	}
	if (ST == 2 && acc == 0x9e3779b9u)
		out[0] = acc;
}

template <int NB, int K, int ST, int LDNT, int MAP, int COMP = 0, int TR = 0>
void run(const uint8_t *in, uint64_t *out, uint32_t ngroups, uint64_t npk, int cus, int wpc) {
	const int lds = 4 * (NB * 4096 + (ST == 3 ? K * 512 : 0));
	int wg_per_cu = wpc / 4;
	if ((lds + 4096) * wg_per_cu > 160 * 1024 || wg_per_cu < 1) {
		printf("NB=%d K=%d ST=%d LDNT=%d MAP=%d waves/CU=%d: LDS does not fit\n", NB, K, ST, LDNT, MAP, wpc);
		return;
	}
	uint32_t wgs = cus * wg_per_cu;
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	for (int it = 0; it < 3; it++) k_floor<NB, K, ST, LDNT, MAP, COMP, TR><<<wgs, 256, lds>>>(in, out, ngroups, wgs * 4);
	(void)hipEventRecord(a);
	for (int it = 0; it < 10; it++) k_floor<NB, K, ST, LDNT, MAP, COMP, TR><<<wgs, 256, lds>>>(in, out, ngroups, wgs * 4);
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms;
	(void)hipEventElapsedTime(&ms, a, b);
	ms /= 10;
	printf("TR=%d COMP=%d NB=%d K=%2d ST=%d LDNT=%d MAP=%d waves/CU=%2d: %.3f ms  %.1f Gpkt/s  %.0f GB/s total\n", TR, COMP,
	       NB, K, ST, LDNT, MAP, wpc, ms, npk / ms / 1e6, npk * (ST == 2 ? 64.0 : 72.0) / ms / 1e6);
}

int main(int argc, char **argv) {
	const uint64_t npk = 1ull << 26;
	const uint32_t ngroups = npk / 64;
	uint8_t *in;
	uint64_t *out;
	(void)hipMalloc(&in, npk * 64);
	(void)hipMalloc(&out, npk * 8);
	(void)hipMemset(in, 1, npk * 64);
	const int cus = 256;
	if (argc > 1 && argv[1][0] == 't') {
		// round 5: the DMA's own layout against chunk-transposed DMA (conflict-free staging
		// reads), with u64 results (ST 0), the read ceiling (ST 2), a little work (COMP 16)
		for (int rep = 0; rep < 3; rep++) {
			run<1, 8, 0, 1, 0, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 0, 1, 0, 0, 1>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 0, 1, 0, 0, 0>(in, out, ngroups, npk, cus, 24);
			run<1, 8, 0, 1, 0, 0, 1>(in, out, ngroups, npk, cus, 24);
			run<1, 8, 2, 1, 0, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 2, 1, 0, 0, 1>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 0, 1, 0, 16, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 0, 1, 0, 16, 1>(in, out, ngroups, npk, cus, 16);
		}
		return 0;
	}
	if (argc > 1 && argv[1][0] == 'p') {
		// round 5: lanes permuted inside each DMA's 1 KB (TR 2) against the DMA's own layout
		for (int rep = 0; rep < 3; rep++) {
			run<1, 8, 0, 1, 0, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 0, 1, 0, 0, 2>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 2, 1, 0, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 2, 1, 0, 0, 2>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 0, 1, 0, 16, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 0, 1, 0, 16, 2>(in, out, ngroups, npk, cus, 16);
		}
		return 0;
	}
	if (argc > 1 && argv[1][0] == 'k') {
		// result-burst length K beyond the kernel's 8 (round 3): 8, 16, 32 groups per burst,
		// u64 per lane (ST 0) or staged in LDS and written as 16-B lanes (ST 3), 16 / 24 waves
		for (int rep = 0; rep < 2; rep++) {
			run<1, 8, 0, 1, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 16, 0, 1, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 32, 0, 1, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 3, 1, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 16, 3, 1, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<2, 16, 0, 1, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 0, 1, 0, 0>(in, out, ngroups, npk, cus, 24);
			run<1, 16, 0, 1, 0, 0>(in, out, ngroups, npk, cus, 24);
			run<1, 8, 2, 1, 0, 0>(in, out, ngroups, npk, cus, 16);
		}
		return 0;
	}
	if (argc > 1 && argv[1][0] == 'm') {
		// round 4: one contiguous range per wave (MAP 1) against interleaved superblocks, plain
		// (ST 1) against nt result stores, the read ceiling (ST 2) beside them
		for (int rep = 0; rep < 2; rep++) {
			run<1, 8, 0, 1, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 0, 1, 1, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 1, 1, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 1, 1, 1, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 0, 0, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 0, 1, 1, 0>(in, out, ngroups, npk, cus, 24);
			run<2, 8, 0, 1, 1, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 2, 1, 0, 0>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 2, 1, 1, 0>(in, out, ngroups, npk, cus, 16);
		}
		return 0;
	}
	if (argc > 1 && argv[1][0] == 'o') {
		// occupancy x prefetch depth, with a little per-group work (the staged kernel at 4
		// workgroups per CU, round 1)
		for (int rep = 0; rep < 2; rep++) {
			run<1, 8, 0, 1, 0, 16>(in, out, ngroups, npk, cus, 16);
			run<2, 8, 0, 1, 0, 16>(in, out, ngroups, npk, cus, 16);
			run<3, 8, 0, 1, 0, 16>(in, out, ngroups, npk, cus, 16);
			run<1, 8, 0, 1, 0, 16>(in, out, ngroups, npk, cus, 12);
			run<2, 8, 0, 1, 0, 16>(in, out, ngroups, npk, cus, 12);
			run<1, 8, 0, 1, 0, 16>(in, out, ngroups, npk, cus, 20);
			run<2, 8, 0, 1, 0, 16>(in, out, ngroups, npk, cus, 20);
			run<1, 8, 0, 1, 0, 16>(in, out, ngroups, npk, cus, 24);
			run<1, 8, 2, 1, 0, 16>(in, out, ngroups, npk, cus, 16);
			run<2, 8, 2, 1, 0, 16>(in, out, ngroups, npk, cus, 16);
		}
		return 0;
	}
	run<1, 8, 0, 1, 0, 0>(in, out, ngroups, npk, cus, 24);
	run<1, 8, 0, 1, 0, 16>(in, out, ngroups, npk, cus, 24);
	run<1, 8, 0, 1, 0, 32>(in, out, ngroups, npk, cus, 24);
	run<1, 8, 0, 1, 0, 64>(in, out, ngroups, npk, cus, 24);
	run<2, 8, 0, 1, 0, 0>(in, out, ngroups, npk, cus, 16);
	run<2, 8, 0, 1, 0, 16>(in, out, ngroups, npk, cus, 16);
	run<2, 8, 0, 1, 0, 32>(in, out, ngroups, npk, cus, 16);
	run<2, 8, 0, 1, 0, 64>(in, out, ngroups, npk, cus, 16);
	run<2, 8, 0, 1, 0, 32>(in, out, ngroups, npk, cus, 12);
	run<3, 8, 0, 1, 0, 32>(in, out, ngroups, npk, cus, 12);
	run<3, 8, 0, 1, 0, 64>(in, out, ngroups, npk, cus, 12);
	run<1, 8, 0, 1, 0, 32>(in, out, ngroups, npk, cus, 32);
	run<1, 8, 0, 1, 0, 64>(in, out, ngroups, npk, cus, 32);
	return 0;
}
