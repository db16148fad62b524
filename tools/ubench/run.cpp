// Runner for tools/ubench kernels: per-iteration latency at 1 wave/CU and at W waves/CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
int main(int argc, char **argv) {
  hipModule_t m; CK(hipModuleLoad(&m, argv[1]));
  hipFunction_t f[4]; const char *names[4] = {"k_smem", "k_jump", "k_disp", "k_init"};
  for (int i = 0; i < 4; i++) CK(hipModuleGetFunction(&f[i], m, names[i]));
  uint64_t *out, *tab; CK(hipMalloc(&out, 8 * 65536)); CK(hipMalloc(&tab, 64 * 32 + 4096));
  std::vector<uint32_t> chase(1024); for (int i = 0; i < 1024; i++) chase[i] = ((i * 7 + 3) % 64) * 4; // small, cached
  struct { uint64_t o, t; uint32_t it, pad; } a;
  size_t sz = sizeof(a); void *ex[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  a.o = (uint64_t)out; a.t = (uint64_t)tab; a.it = 1;
  CK(hipModuleLaunchKernel(f[3], 1, 1, 1, 64, 1, 1, 0, 0, 0, ex)); CK(hipDeviceSynchronize());
  uint64_t *chasebuf; CK(hipMalloc(&chasebuf, 4096)); CK(hipMemcpy(chasebuf, chase.data(), 4096, hipMemcpyHostToDevice));
  for (int k = 0; k < 3; k++) {
    for (int waves : {256, 256 * 8, 256 * 32}) {
      a.it = k == 0 ? 4096 : 64; a.t = k == 0 ? (uint64_t)chasebuf : (uint64_t)tab;
      for (int rep = 0; rep < 2; rep++) {
        CK(hipModuleLaunchKernel(f[k], waves, 1, 1, 64, 1, 1, 0, 0, 0, ex)); CK(hipDeviceSynchronize());
      }
      std::vector<uint64_t> h(waves); CK(hipMemcpy(h.data(), out, 8 * waves, hipMemcpyDeviceToHost));
      double avg = 0; for (auto x : h) avg += x; avg /= waves;
      double per = avg / (k == 0 ? a.it : a.it * 64.0);
      printf("%s waves=%d (%.0f/CU): %.1f cycles per op per wave (s_memtime)\n", names[k], waves, waves / 256.0, per);
    }
  }
  return 0;
}
