// Per-lane gather cost model for C5-like programs: every lane owns one packet of P bytes
// (packets contiguous, lane l of group g = packet 64g + l) and performs NL loads of 1/2/4/8
// bytes at fixed pseudo-random offsets inside it, XOR-folded into one u64 result per packet.
//   MODE 0: global loads, 64-bit per-lane address (what compiled C5 issues), all lanes
//   MODE 1: as 0, one lane in four active (does the address path cost per lane or per wave
//           instruction?)
//   MODE 2: the group's span (64 x P bytes) DMA'd into LDS with coalesced 16-B lane loads,
//           then the same loads as ds_read from LDS
//   MODE 3: as 0, SGPR base + 32-bit per-lane offset address form
//   MODE 4: NL distinct 16-B aligned windows per lane as dwordx4 loads (the same bytes fetched
//           with fewer, wider lane loads)
//   MODE 5: NL distinct 8-B aligned windows per lane as dwordx2 loads
//   MODE 6: as 2, but the loads are FLAT loads whose addresses fall in the LDS aperture (does
//           a flat load routed to LDS cost what ds_read does, or what the TA gather path does?)
//   MODE 7: as 6 with half the lanes' packets left in global memory (per-lane routing mix)
// Grid: waves per CU x 256 CUs workgroups of one wave.  Prints ms and lane-loads per ns.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))

constexpr uint32_t mix(uint32_t x) {
	x ^= x >> 16;
	x *= 0x7feb352dU;
	x ^= x >> 15;
	x *= 0x846ca68bU;
	x ^= x >> 16;
	return x;
}

template <int P, int I>
__device__ __forceinline__ uint64_t ld_global(const uint8_t *p) {
	constexpr uint32_t h = mix(I * 2654435761U + P);
	constexpr int z = 1 << (h & 3);
	constexpr uint32_t off = 18 + (h >> 8) % (uint32_t)(P - 26);
	if constexpr (z == 1)
		return *(const uint8_t *)(p + off);
	else if constexpr (z == 2)
		return *(const uint16_t *)(p + (off & ~1u));
	else if constexpr (z == 4)
		return *(const uint32_t *)(p + (off & ~3u));
	else
		return *(const uint64_t *)(p + (off & ~7u));
}

template <int P, int W, int I>
__device__ __forceinline__ uint64_t ld_window(const uint8_t *p) {
	constexpr uint32_t h = mix(I * 2246822519U + P * 7 + W);
	constexpr uint32_t off = (h >> 8) % (uint32_t)(P / W) * W;
	if constexpr (W == 16) {
		typedef unsigned v4u __attribute__((ext_vector_type(4)));
		const v4u v = *(const v4u *)(p + off);
		return ((uint64_t)(v.x ^ v.z) << 32) | (v.y ^ v.w);
	} else {
		return *(const uint64_t *)(p + off);
	}
}

template <int P, int NL, int W, int I = 0>
__device__ __forceinline__ void foldw(const uint8_t *p, uint64_t &acc) {
	if constexpr (I < NL) {
		acc = (acc ^ ld_window<P, W, I>(p)) * 0x9E3779B1ull;
		foldw<P, NL, W, I + 1>(p, acc);
	}
}

template <int P, int NL, int I = 0>
__device__ __forceinline__ void fold(const uint8_t *p, uint64_t &acc) {
	if constexpr (I < NL) {
		acc = (acc ^ ld_global<P, I>(p)) * 0x9E3779B1ull;
		fold<P, NL, I + 1>(p, acc);
	}
}

template <int P, int NL, int MODE>
__global__ void __launch_bounds__(64) k_gather(const uint8_t *__restrict__ in, uint64_t *__restrict__ out,
						uint32_t ngroups) {
	extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
	const uint32_t lane = threadIdx.x;
	for (uint32_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
		const uint64_t pkt = (uint64_t)g * 64 + lane;
		uint64_t acc = 0;
		if constexpr (MODE == 6 || MODE == 7) {
			const uint8_t *src = in + (uint64_t)g * 64 * P;
			constexpr uint32_t span = 64u * P;
			for (uint32_t q = 0; q < span; q += 1024)
				__builtin_amdgcn_global_load_lds((const void *)(src + q + lane * 16), LDS_PTR(lds + q), 16, 0, 2);
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			const uint8_t *gp = (const uint8_t *)lds + lane * P;
			if (MODE == 7 && (lane & 1))
				gp = in + pkt * P;
			asm volatile("" : "+v"(gp));   // generic pointer: flat loads
			fold<P, NL>(gp, acc);
			asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_barrier" ::: "memory");
		} else if constexpr (MODE == 2) {
			const uint8_t *src = in + (uint64_t)g * 64 * P;
			constexpr uint32_t span = 64u * P;
			for (uint32_t q = 0; q < span; q += 1024)
				__builtin_amdgcn_global_load_lds((const void *)(src + q + lane * 16), LDS_PTR(lds + q), 16, 0, 2);
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			fold<P, NL>(lds + lane * P, acc);
			asm volatile("s_waitcnt lgkmcnt(0)\n s_barrier" ::: "memory");
		} else if constexpr (MODE == 4) {
			foldw<P, NL, 16>(in + pkt * P, acc);
		} else if constexpr (MODE == 5) {
			foldw<P, NL, 8>(in + pkt * P, acc);
		} else if constexpr (MODE == 3) {
			const uint32_t off32 = (uint32_t)(pkt * P);
			fold<P, NL>(in + off32, acc);
		} else {
			if (MODE == 1 && (lane & 3))
				continue;
			fold<P, NL>(in + pkt * P, acc);
		}
		out[pkt] = acc;
	}
}

template <int P, int NL, int MODE>
static void run(int wpc, uint32_t npkt) {
	const uint32_t ngroups = npkt / 64;
	uint8_t *in;
	uint64_t *out;
	hipMalloc(&in, (size_t)npkt * P);
	hipMalloc(&out, (size_t)npkt * 8);
	hipMemset(in, 0x5b, (size_t)npkt * P);
	const size_t lds = (MODE == 2 || MODE >= 6) ? 64u * P : 0;
	if (lds > 65536)
		hipFuncSetAttribute((const void *)k_gather<P, NL, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
				    (int)lds);
	const int grid = 256 * wpc;
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	for (int w = 0; w < 2; w++)
		k_gather<P, NL, MODE><<<grid, 64, lds>>>(in, out, ngroups);
	hipEventRecord(a);
	const int reps = 5;
	for (int r = 0; r < reps; r++)
		k_gather<P, NL, MODE><<<grid, 64, lds>>>(in, out, ngroups);
	hipEventRecord(b);
	hipEventSynchronize(b);
	float ms = 0;
	hipEventElapsedTime(&ms, a, b);
	ms /= reps;
	const double lanes = MODE == 1 ? npkt / 4.0 : npkt;
	printf("P=%4d NL=%d mode=%d waves/CU=%2d  %.4f ms  %.2f lane-loads/ns  %.1f GB/s of packets\n", P, NL,
	       MODE, wpc, ms, lanes * NL / (ms * 1e6), (double)npkt * P / (ms * 1e6));
	fflush(stdout);
	hipFree(in);
	hipFree(out);
}

// C5's address shape without its divergence (round 6, the gather roofline's calibration): IMIX
// packets (64 / 576 / 1500 B in 7:4:1, each on a 64-B boundary, CSR offsets), every lane loading
// NL values of 1/2/4/8 bytes at offsets drawn, per size class, uniformly in [18, limit - 8) the
// way C5's leaves draw theirs (workloads._c5_nodes), all 64 lanes active and no other work.
constexpr int kImixNL = 26;   // C5: 109.4M TCP tag accesses / 4M packets (profiles/r06/gather/)
__constant__ uint16_t c_imix_off[3][kImixNL];

__global__ void __launch_bounds__(64) k_imix(const uint8_t *__restrict__ in, const uint64_t *__restrict__ offs,
					     const uint8_t *__restrict__ cls, uint64_t *__restrict__ out, uint32_t ngroups) {
	const uint32_t lane = threadIdx.x;
	for (uint32_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
		const uint64_t pkt = (uint64_t)g * 64 + lane;
		const uint8_t *p = in + offs[pkt];
		const uint32_t c = cls[pkt];
		uint64_t acc = 0;
#pragma unroll
		for (int i = 0; i < kImixNL; i++) {
			const uint32_t o = c_imix_off[c][i];
			uint64_t v;
			switch (i & 3) {
			case 0: v = *(const uint8_t *)(p + o); break;
			case 1: v = *(const uint16_t *)(p + (o & ~1u)); break;
			case 2: v = *(const uint32_t *)(p + (o & ~3u)); break;
			default: v = *(const uint64_t *)(p + (o & ~7u)); break;
			}
			acc = (acc ^ v) * 0x9E3779B1ull;
		}
		out[pkt] = acc;
	}
}

static void run_imix(int wpc, uint32_t npkt) {
	std::vector<uint64_t> offs(npkt);
	std::vector<uint8_t> cls(npkt);
	uint64_t at = 0, x = 0x9E3779B97F4A7C15ull;
	const uint32_t limit[3] = {64, 576, 1500};
	for (uint32_t i = 0; i < npkt; i++) {
		x ^= x << 13, x ^= x >> 7, x ^= x << 17;
		const uint32_t r = (uint32_t)(x % 12);   // IMIX 7:4:1
		cls[i] = r < 7 ? 0 : r < 11 ? 1 : 2;
		offs[i] = at;
		at += (limit[cls[i]] + 63) / 64 * 64;
	}
	uint16_t tab[3][kImixNL];
	for (int c = 0; c < 3; c++)
		for (int i = 0; i < kImixNL; i++) {
			x ^= x << 13, x ^= x >> 7, x ^= x << 17;
			tab[c][i] = (uint16_t)(18 + x % (limit[c] - 26));
		}
	hipMemcpyToSymbol(HIP_SYMBOL(c_imix_off), tab, sizeof(tab));
	uint8_t *in, *d_cls;
	uint64_t *d_offs, *out;
	hipMalloc(&in, at + 64);
	hipMemset(in, 0x5b, at + 64);
	hipMalloc(&d_offs, npkt * 8ull);
	hipMalloc(&d_cls, npkt);
	hipMalloc(&out, npkt * 8ull);
	hipMemcpy(d_offs, offs.data(), npkt * 8ull, hipMemcpyHostToDevice);
	hipMemcpy(d_cls, cls.data(), npkt, hipMemcpyHostToDevice);
	const int grid = 256 * wpc;
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	for (int w = 0; w < 2; w++)
		k_imix<<<grid, 64>>>(in, d_offs, d_cls, out, npkt / 64);
	hipEventRecord(a);
	const int reps = 5;
	for (int r = 0; r < reps; r++)
		k_imix<<<grid, 64>>>(in, d_offs, d_cls, out, npkt / 64);
	hipEventRecord(b);
	hipEventSynchronize(b);
	float ms = 0;
	hipEventElapsedTime(&ms, a, b);
	ms /= reps;
	printf("IMIX NL=%d waves/CU=%2d  %.4f ms  %.2f lane-loads/ns  %.1f GB/s of packets\n", kImixNL, wpc, ms,
	       (double)npkt * kImixNL / (ms * 1e6), (double)at / (ms * 1e6));
	fflush(stdout);
	hipFree(in);
	hipFree(d_offs);
	hipFree(d_cls);
	hipFree(out);
}

int main(int argc, char **argv) {
	const uint32_t n = 1u << 22;
	if (argc > 1 && argv[1][0] == 'f') {   // flat-to-LDS study
		for (int w : {1, 2, 4}) {
			run<576, 56, 2>(w, n);
			run<576, 56, 6>(w, n);
			run<576, 56, 7>(w, n);
		}
		run<576, 56, 0>(8, n);
		return 0;
	}
	if (argc > 1 && argv[1][0] == 'i') {   // C5's shape: the gather roofline's calibration
		for (int w : {4, 8, 16, 24})
			run_imix(w, n);
		return 0;
	}
	if (argc > 1 && argv[1][0] == 'c') {   // the counters of the per-class gathers (round 6)
		run<576, 56, 0>(8, n);
		run<576, 56, 1>(8, n);
		run<1536, 56, 0>(8, n);
		run<64, 56, 0>(8, n);
		return 0;
	}
	for (int w : {8, 24}) {
		run<576, 56, 0>(w, n);
		run<576, 29, 4>(w, n);
		run<576, 42, 5>(w, n);
		run<576, 29, 0>(w, n);
		run<1536, 56, 0>(w, n);
		run<1536, 46, 4>(w, n);
		run<1536, 52, 5>(w, n);
	}
	return 0;
}
