// Result-write burst size vs throughput, with ONE 4-KB group of packet loads in flight per wave
// (the interpreter's shape): each wave walks K consecutive 64-packet groups, keeps their u64
// results, then writes K x 512 B contiguously.  K = 1 is the interpreter's current pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int K, bool NT>
__global__ void __launch_bounds__(256) k_burst(const uint4 *__restrict__ in, uint64_t *__restrict__ out, uint64_t ngroups) {
	const int lane = threadIdx.x & 63;
	uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
	uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
	for (uint64_t sg = wave; sg * K < ngroups; sg += nwaves) {
		uint64_t r[K];
		for (int k = 0; k < K; k++) {
			const uint4 *p = in + (sg * K + k) * 256;
			uint4 v0 = p[lane], v1 = p[64 + lane], v2 = p[128 + lane], v3 = p[192 + lane];
			r[k] = v0.x ^ v1.y ^ v2.z ^ v3.w;
			asm volatile("" ::: "memory"); // keep the groups' loads sequential
		}
#pragma unroll
		for (int k = 0; k < K; k++) {
			if (NT) __builtin_nontemporal_store(r[k], out + (sg * K + k) * 64 + lane);
			else out[(sg * K + k) * 64 + lane] = r[k];
		}
	}
}

template <int K, bool NT>
void run(const uint4 *in, uint64_t *out, uint64_t ngroups, uint64_t npk) {
	for (int wpc : {16, 24, 32}) {
		int grid = 256 * wpc / 4;
		hipEvent_t a, b;
		(void)hipEventCreate(&a);
		(void)hipEventCreate(&b);
		for (int it = 0; it < 3; it++) k_burst<K, NT><<<grid, 256>>>(in, out, ngroups);
		(void)hipEventRecord(a);
		for (int it = 0; it < 10; it++) k_burst<K, NT><<<grid, 256>>>(in, out, ngroups);
		(void)hipEventRecord(b);
		(void)hipEventSynchronize(b);
		float ms;
		(void)hipEventElapsedTime(&ms, a, b);
		ms /= 10;
		printf("K=%d nt=%d waves/CU=%d: %.3f ms  %.1f Gpkt/s\n", K, NT, wpc, ms, npk / ms / 1e6);
	}
}

int main() {
	const uint64_t npk = 1ull << 26, ngroups = npk / 64;
	uint4 *in;
	uint64_t *out;
	(void)hipMalloc(&in, npk * 64);
	(void)hipMalloc(&out, npk * 8);
	(void)hipMemset(in, 1, npk * 64);
	run<1, false>(in, out, ngroups, npk);
	run<1, true>(in, out, ngroups, npk);
	run<2, true>(in, out, ngroups, npk);
	run<4, false>(in, out, ngroups, npk);
	run<4, true>(in, out, ngroups, npk);
	run<8, true>(in, out, ngroups, npk);
	run<1, false>(in, out, ngroups, npk);
	return 0;
}
