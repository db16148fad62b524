// VALU throughput of the integer instructions the code generator chooses between (gfx950):
// each kernel issues ITER x 16 independent copies of one instruction per wave, 8 waves per SIMD,
// every CU busy; reports SIMD cycles per wave-instruction (clock from s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP16(x) x x x x x x x x x x x x x x x x

#define KERNEL(name, body)                                                                          \
	__global__ void __launch_bounds__(256) name(uint64_t *out, int iters, uint64_t *clk) {      \
		uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 1;     \
		uint64_t b0 = a0 * 11ull, b1 = a0 * 13ull, b2 = a0 * 17ull, b3 = a0 * 19ull, bc = 99;   \
		uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();   \
		for (int i = 0; i < iters; i++) {                                                  \
			asm volatile(REP16(body)                                                   \
				     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(b0), "+v"(b1), \
				       "+v"(b2), "+v"(b3)                                            \
				     : "s"(0x27d4eb2du), "v"(bc) : "vcc", "scc", "s60", "s61", "s62", "s63");     \
		}                                                                                   \
		uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();   \
		if (threadIdx.x == 0 && blockIdx.x == 0) {                                         \
			clk[0] = t1 - t0;                                                           \
			clk[1] = r1 - r0;                                                           \
		}                                                                                   \
		out[blockIdx.x * 256 + threadIdx.x] = (uint64_t)a0 + a1 + a2 + a3 + a4 + b0 + b1 + b2 + b3; \
	}

// 4 independent instructions per REP (on the 8 registers as 4 pairs or 4 singles)
KERNEL(k_xor, "v_xor_b32 %0, %9, %0\n v_xor_b32 %1, %9, %1\n v_xor_b32 %2, %9, %2\n v_xor_b32 %3, %9, %3\n")
KERNEL(k_mul_lo, "v_mul_lo_u32 %0, %0, %9\n v_mul_lo_u32 %1, %1, %9\n v_mul_lo_u32 %2, %2, %9\n v_mul_lo_u32 %3, %3, %9\n")
KERNEL(k_mul_hi, "v_mul_hi_u32 %0, %0, %9\n v_mul_hi_u32 %1, %1, %9\n v_mul_hi_u32 %2, %2, %9\n v_mul_hi_u32 %3, %3, %9\n")
KERNEL(k_mad64, "v_mad_u64_u32 %5, s[60:61], %0, %9, %5\n v_mad_u64_u32 %6, s[60:61], %1, %9, %6\n v_mad_u64_u32 %7, s[60:61], %2, %9, %7\n v_mad_u64_u32 %8, s[60:61], %3, %9, %8\n")
KERNEL(k_u24, "v_mul_u32_u24 %0, %9, %0\n v_mul_u32_u24 %1, %9, %1\n v_mul_u32_u24 %2, %9, %2\n v_mul_u32_u24 %3, %9, %3\n")
KERNEL(k_lsh64, "v_lshlrev_b64 %5, 5, %5\n v_lshlrev_b64 %6, 5, %6\n v_lshlrev_b64 %7, 5, %7\n v_lshlrev_b64 %8, 5, %8\n")
KERNEL(k_add64, "v_lshl_add_u64 %5, %5, 0, %10\n v_lshl_add_u64 %6, %6, 0, %10\n v_lshl_add_u64 %7, %7, 0, %10\n v_lshl_add_u64 %8, %8, 0, %10\n")
KERNEL(k_mov64, "v_mov_b64 %5, %6\n v_mov_b64 %6, %7\n v_mov_b64 %7, %8\n v_mov_b64 %8, %5\n")
KERNEL(k_cmp64, "v_cmp_eq_u64 vcc, %5, %10\n v_cmp_eq_u64 s[62:63], %6, %10\n v_cmp_eq_u64 vcc, %7, %10\n v_cmp_eq_u64 s[62:63], %8, %10\n")
KERNEL(k_cmp32, "v_cmp_eq_u32 vcc, %9, %0\n v_cmp_eq_u32 s[62:63], %9, %1\n v_cmp_eq_u32 vcc, %9, %2\n v_cmp_eq_u32 s[62:63], %9, %3\n")
KERNEL(k_perm, "v_perm_b32 %0, %1, %0, %9\n v_perm_b32 %1, %2, %1, %9\n v_perm_b32 %2, %3, %2, %9\n v_perm_b32 %3, %4, %3, %9\n")
KERNEL(k_mix, "v_xor_b32 %0, %9, %0\n s_xor_b32 s60, s60, %9\n v_xor_b32 %1, %9, %1\n s_xor_b32 s61, s61, %9\n")
KERNEL(k_mix3, "v_xor_b32 %0, %9, %0\n v_xor_b32 %1, %9, %1\n v_xor_b32 %2, %9, %2\n s_xor_b32 s61, s61, %9\n")
KERNEL(k_salu, "s_xor_b32 s60, s60, %9\n s_xor_b32 s61, s61, %9\n s_xor_b32 s62, s62, %9\n s_xor_b32 s63, s63, %9\n")

typedef void (*kfn)(uint64_t *, int, uint64_t *);

int main() {
	uint64_t *out, *clk;
	int cus = 256;
	(void)hipMalloc(&out, sizeof(uint64_t) * cus * 8 * 256);
	(void)hipMalloc(&clk, 16);
	struct { const char *n; kfn f; } ks[] = {
		{"v_xor_b32", k_xor}, {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32", k_mul_hi},
		{"v_mad_u64_u32", k_mad64}, {"v_mul_u32_u24", k_u24}, {"v_lshlrev_b64", k_lsh64},
		{"v_lshl_add_u64", k_add64}, {"v_mov_b64", k_mov64}, {"v_cmp_eq_u64", k_cmp64},
		{"v_cmp_eq_u32", k_cmp32}, {"v_perm_b32", k_perm}, {"mix v/s 1:1", k_mix}, {"mix v/s 3:1", k_mix3}, {"s_xor_b32", k_salu}};
	const int iters = 2000;
	setvbuf(stdout, NULL, _IONBF, 0);
	for (auto &k : ks) {
		for (int wps : {1, 8}) {
			int grid = cus * wps; // 256-lane blocks: 4 waves, one per SIMD; wps blocks per CU
			hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, out, 10, clk);
			hipEvent_t a, b;
			(void)hipEventCreate(&a);
			(void)hipEventCreate(&b);
			(void)hipEventRecord(a);
			hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, out, iters, clk);
			(void)hipEventRecord(b);
			(void)hipEventSynchronize(b);
			float ms;
			(void)hipEventElapsedTime(&ms, a, b);
			uint64_t c[2];
			(void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
			double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
			// wave-instructions per SIMD: wps waves per SIMD x iters x 64
			double per_simd = (double)wps * iters * 64;
			double cyc = ms * 1e-3 * ghz * 1e9 / per_simd;
			fprintf(stdout, "%-16s waves/SIMD=%d: %.3f ms, clock %.2f GHz, %.2f SIMD cycles per wave-instruction\n",
			       k.n, wps, ms, ghz, cyc);
		}
	}
	return 0;
}
