// Probe: are raw buffer stores with an out-of-range offset dropped on gfx950?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k(float* p, int n, uint32_t drop) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, 0, n * 4, 0x00020000);
  const int t = threadIdx.x;
  const uint32_t off = (t & 1) ? (uint32_t)t * 4u : drop;
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(t + 1)), r, off, 0, 0);
}
int main() {
  const int n = 64, guard = 1 << 20;
  float* big;
  hipMalloc(&big, sizeof(float) * (2 * guard + n));
  hipMemset(big, 0, sizeof(float) * (2 * guard + n));
  uint32_t drops[] = {0x80000000u, 4096u};
  for (uint32_t d : drops) {
    hipMemset(big, 0, sizeof(float) * (2 * guard + n));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, big + guard, n, d);
    hipDeviceSynchronize();
    std::vector<float> h(2 * guard + n);
    hipMemcpy(h.data(), big, sizeof(float) * h.size(), hipMemcpyDeviceToHost);
    int bad_in = 0, bad_out = 0;
    for (int i = 0; i < n; ++i) {
      float want = (i & 1) ? (float)(i + 1) : 0.0f;
      if (h[guard + i] != want) ++bad_in;
    }
    for (size_t i = 0; i < h.size(); ++i)
      if ((i < (size_t)guard || i >= (size_t)guard + n) && h[i] != 0.0f) ++bad_out;
    printf("drop=0x%08x in-range mismatches=%d writes outside=%d :", d, bad_in, bad_out);
    for (int i = 0; i < 8; ++i) printf(" %g", h[guard + i]);
    int nz = 0; size_t first = 0;
    for (size_t i = 0; i < h.size(); ++i) if (h[i] != 0.0f) { if (!nz) first = i; ++nz; }
    printf(" | nonzero=%d first=%ld\n", nz, (long)first - guard);
  }
  return 0;
}
