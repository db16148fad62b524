// Streaming ceilings for the batch-interpreter access pattern: read N x 64 B packets (16 B per
// lane, coalesced) and write one u64 result per packet.  Variants differ only in how the
// results are stored.  Reports GB/s of (reads + writes) and packets/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

// one wave = one 64-packet group per iteration (4 KB read = 4 x 1 KB wave loads), like the
// interpreter's groups
template <int WMODE>
__global__ void __launch_bounds__(256) k_group(const uint4 *__restrict__ in, uint64_t *__restrict__ out, uint64_t ngroups) {
	const int lane = threadIdx.x & 63;
	uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
	uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
	for (uint64_t g = wave; g < ngroups; g += nwaves) {
		const uint4 *p = in + g * 256;
		uint4 v0 = p[lane], v1 = p[64 + lane], v2 = p[128 + lane], v3 = p[192 + lane];
		uint32_t x = v0.x ^ v1.y ^ v2.z ^ v3.w;
		if (WMODE == 0) {           // u64 per lane, 512 B per wave store
			out[g * 64 + lane] = x;
		} else if (WMODE == 1) {    // same, nontemporal
			__builtin_nontemporal_store((uint64_t)x, out + g * 64 + lane);
		} else if (WMODE == 2) {    // no write
			if (x == 0x12345678u) out[0] = x;
		} else if (WMODE == 3) {    // 16 B per lane: pairs of lanes combined, 32 lanes store 1 KB? (512 B)
			uint64_t y = __shfl_down((uint64_t)x, 1);
			if ((lane & 1) == 0) {
				ulonglong2 w; w.x = x; w.y = y;
				*(ulonglong2 *)(out + g * 64 + lane) = w;
			}
		}
	}
}

// results buffered for 8 consecutive groups, then written as one 4-KB burst
__global__ void __launch_bounds__(256) k_burst(const uint4 *__restrict__ in, uint64_t *__restrict__ out, uint64_t ngroups) {
	const int lane = threadIdx.x & 63;
	uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
	uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
	for (uint64_t sg = wave; sg * 8 < ngroups; sg += nwaves) {
		uint64_t r[8];
#pragma unroll
		for (int k = 0; k < 8; k++) {
			const uint4 *p = in + (sg * 8 + k) * 256;
			uint4 v0 = p[lane], v1 = p[64 + lane], v2 = p[128 + lane], v3 = p[192 + lane];
			r[k] = v0.x ^ v1.y ^ v2.z ^ v3.w;
		}
#pragma unroll
		for (int k = 0; k < 8; k++)
			__builtin_nontemporal_store(r[k], out + (sg * 8 + k) * 64 + lane);
	}
}

template <int W>
float run(const uint4 *in, uint64_t *out, uint64_t ngroups, int grid) {
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	for (int it = 0; it < 3; it++) {
		if (W == 4) k_burst<<<grid, 256>>>(in, out, ngroups);
		else k_group<W><<<grid, 256>>>(in, out, ngroups);
	}
	hipEventRecord(a);
	const int reps = 10;
	for (int it = 0; it < reps; it++) {
		if (W == 4) k_burst<<<grid, 256>>>(in, out, ngroups);
		else k_group<W><<<grid, 256>>>(in, out, ngroups);
	}
	hipEventRecord(b);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	return ms / reps;
}

int main() {
	const uint64_t npk = 1ull << 26, ngroups = npk / 64;
	uint4 *in;
	uint64_t *out;
	(void)hipMalloc(&in, npk * 64);
	(void)hipMalloc(&out, npk * 8);
	(void)hipMemset(in, 1, npk * 64);
	const char *names[] = {"u64/lane 512B", "u64/lane nt  ", "no write     ", "16B/lane     ", "burst 4KB nt "};
	for (int w = 0; w < 5; w++)
		for (int wpc : {16, 32}) {
			int grid = 256 * wpc / 4;
			float ms = w == 0 ? run<0>(in, out, ngroups, grid) : w == 1 ? run<1>(in, out, ngroups, grid)
				 : w == 2 ? run<2>(in, out, ngroups, grid) : w == 3 ? run<3>(in, out, ngroups, grid) : run<4>(in, out, ngroups, grid);
			double bytes = npk * 64.0 + (w == 2 ? 0 : npk * 8.0);
			printf("%s waves/CU=%d: %.3f ms  %.0f GB/s  %.1f Gpkt/s\n", names[w], wpc, ms, bytes / ms / 1e6, npk / ms / 1e6);
		}
	return 0;
}
