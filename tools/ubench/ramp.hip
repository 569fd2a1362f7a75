// tools/ubench/ramp.hip -- wave launch ramp: every wave records s_memrealtime
// (100 MHz) at entry; prints the spread of start times for 4096 / 16384 waves
// by workgroup size, with and without a 16 KiB-per-wave global load at entry.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/ramp.hip -o build/ramp
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

__global__ void ramp(uint64_t* t, const uint4* src, uint4* dst, int load) {
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint4 acc = {0, 0, 0, 0};
  if (load) {
    const uint4* p = src + (size_t)wave * 1024 + (threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < 16; i++) {
      uint4 v = p[i * 64];
      acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) { t[2 * wave] = t0; t[2 * wave + 1] = t1; }
  if (acc.x == 0x12345678u) dst[wave] = acc;
}

int main() {
  const int maxw = 16384;
  uint64_t* t;
  uint4 *src, *dst;
  hipMalloc(&t, maxw * 16);
  hipMalloc(&src, (size_t)maxw * 16384);
  hipMalloc(&dst, maxw * 16);
  hipMemset(src, 1, (size_t)maxw * 16384);
  std::vector<uint64_t> h(2 * maxw);
  for (int load : {0, 1})
    for (int total : {4096, 16384})
      for (int wpg : {1, 4, 16}) {
        for (int rep = 0; rep < 3; rep++) {
          hipLaunchKernelGGL(ramp, dim3(total / wpg), dim3(64 * wpg), 0, 0, t, src, dst, load);
          hipDeviceSynchronize();
        }
        hipMemcpy(h.data(), t, total * 16, hipMemcpyDeviceToHost);
        std::vector<double> s(total), e(total);
        uint64_t mn = ~0ull;
        for (int i = 0; i < total; i++) mn = std::min(mn, h[2 * i]);
        for (int i = 0; i < total; i++) { s[i] = (h[2 * i] - mn) * 10.0; e[i] = (h[2 * i + 1] - mn) * 10.0; }
        std::sort(s.begin(), s.end());
        std::sort(e.begin(), e.end());
        printf("load %d waves %5d wpg %2d: start ns p10 %6.0f p50 %6.0f p90 %6.0f max %6.0f | loaded ns p50 %6.0f max %6.0f\n",
               load, total, wpg, s[total / 10], s[total / 2], s[total * 9 / 10], s[total - 1], e[total / 2], e[total - 1]);
      }
  return 0;
}
