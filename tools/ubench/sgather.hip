// Sparse divergent gathers (C5's shape: a leaf runs with ~3 of 64 lanes, each lane loading ~40
// values at constant offsets from its own 1500-B packet): vector loads under a sparse exec mask
// (the texture data path, ~17 cycles per wave-instruction whatever the active lanes) against the
// scalar path (per active lane: v_readlane of the packet address, s_load of each value).
// Reports ms per launch for the same loads and a checksum (both must agree).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int NL = 40;      // loads per lane
constexpr int PKT = 1536;   // packet stride

__device__ __constant__ uint32_t c_off[NL];

template <int ACTIVE_EVERY>
__global__ void __launch_bounds__(256) k_vec(const uint8_t *__restrict__ buf, uint64_t npk, uint32_t *out)
{
	const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	if (tid >= npk || (threadIdx.x % ACTIVE_EVERY) != 0)
		return;
	const uint8_t *p = buf + tid * PKT;
	uint32_t acc = 0;
#pragma unroll
	for (int i = 0; i < NL; i++)
		acc ^= *(const uint32_t *)(p + c_off[i]) + i;
	out[tid] = acc;
}

template <int ACTIVE_EVERY>
__global__ void __launch_bounds__(256) k_scalar(const uint8_t *__restrict__ buf, uint64_t npk, uint32_t *out)
{
	const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	const bool act = tid < npk && (threadIdx.x % ACTIVE_EVERY) == 0;
	const uint64_t addr = (uint64_t)(buf + tid * PKT);
	uint64_t mask = __ballot(act);
	uint32_t mine = 0;
	while (mask) {
		const int lane = __builtin_ctzll(mask);
		mask &= mask - 1;
		const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)addr, lane);
		const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(addr >> 32), lane);
		const uint64_t a = ((uint64_t)hi << 32) | lo;
		uint32_t acc = 0;
#pragma unroll
		for (int i = 0; i < NL; i += 8) {
			uint32_t v[8];
#pragma unroll
			for (int k = 0; k < 8; k++) {
				const uint64_t ak = a + c_off[i + k];
				asm volatile("s_load_dword %0, %1, 0x0" : "=s"(v[k]) : "s"(ak));
			}
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
			for (int k = 0; k < 8; k++)
				acc ^= v[k] + (uint32_t)(i + k);
		}
		if ((int)(threadIdx.x & 63) == lane)
			mine = acc;
	}
	if (act)
		out[tid] = mine;
}

template <typename K>
float timeit(K kern, const uint8_t *buf, uint64_t npk, uint32_t *out)
{
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	const uint32_t grid = (uint32_t)((npk + 255) / 256);
	for (int w = 0; w < 3; w++)
		kern<<<grid, 256>>>(buf, npk, out);
	(void)hipEventRecord(a);
	for (int it = 0; it < 10; it++)
		kern<<<grid, 256>>>(buf, npk, out);
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms = 0;
	(void)hipEventElapsedTime(&ms, a, b);
	hipError_t e = hipGetLastError();
	if (e != hipSuccess)
		printf("launch error: %s\n", hipGetErrorString(e));
	return ms / 10;
}

int main()
{
	const uint64_t npk = 1ull << 20; // 1M packets of 1536 B: 1.5 GB
	uint8_t *buf;
	uint32_t *out;
	if (hipMalloc(&buf, npk * PKT + 64) != hipSuccess || hipMalloc(&out, npk * 4) != hipSuccess) {
		printf("hipMalloc failed\n");
		return 1;
	}
	(void)hipMemset(buf, 7, npk * PKT);
	uint32_t off[NL];
	uint32_t x = 12345;
	for (int i = 0; i < NL; i++) {
		x = x * 1103515245u + 12345u;
		off[i] = (x >> 8) % (1496 - 20) + 18;
		off[i] &= ~3u; // (scalar loads are dword-aligned)
	}
	hipError_t ce = hipMemcpyToSymbol(HIP_SYMBOL(c_off), off, sizeof(off));
	if (ce != hipSuccess)
		printf("hipMemcpyToSymbol: %s\n", hipGetErrorString(ce));
	uint32_t h1[8], h2[8];
	for (int rep = 0; rep < 2; rep++) {
		float v3 = timeit(k_vec<20>, buf, npk, out);
		(void)hipMemcpy(h1, out, 32, hipMemcpyDeviceToHost);
		float s3 = timeit(k_scalar<20>, buf, npk, out);
		(void)hipMemcpy(h2, out, 32, hipMemcpyDeviceToHost);
		float v8 = timeit(k_vec<8>, buf, npk, out);
		float s8 = timeit(k_scalar<8>, buf, npk, out);
		float v1 = timeit(k_vec<64>, buf, npk, out);
		float s1 = timeit(k_scalar<64>, buf, npk, out);
		printf("active lanes ~3/64: vector %.3f ms  scalar %.3f ms | ~8/64: vector %.3f  scalar %.3f | "
		       "1/64: vector %.3f  scalar %.3f | checksum %s\n",
		       v3, s3, v8, s8, v1, s1, h1[0] == h2[0] ? "equal" : "DIFFERENT");
	}
	return 0;
}
