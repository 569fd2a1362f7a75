// tools/ubench/xcd.hip -- launch timeline per XCD (design measurement).
//
// Every wave records s_memrealtime (100 MHz) at entry and exit and its XCC id.
// Kernels: 4096 waves in workgroups of 4 waves, with the codec's 33 KiB of
// dynamic LDS per workgroup, spinning `spin_ns` in each wave.  Prints, per XCD,
// the first/median/last entry and the last exit relative to the earliest entry,
// and the host-event duration of the launch -- so launch overhead and any
// stagger between XCDs can be told apart from counter offsets (each XCD's
// counter is only comparable with itself).
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/xcd.hip -o build/xcd
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

__global__ __launch_bounds__(256, 4) void timeline(uint64_t* t, uint32_t spin_ticks) {
  extern __shared__ uint32_t lds[];
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  lds[threadIdx.x] = (uint32_t)t0;
  uint64_t t1 = t0;
  while (t1 - t0 < spin_ticks) t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    t[3 * wave] = t0;
    t[3 * wave + 1] = t1 + lds[(threadIdx.x + 64) & 255] * 0;
    t[3 * wave + 2] = xcc;
  }
}

struct BigArgs {  // the codec's kernarg size (Geometry: 344 bytes)
  uint64_t w[43];
};

__global__ __launch_bounds__(256, 4) void timeline_bigargs(uint64_t* t, uint32_t spin_ticks, BigArgs a) {
  extern __shared__ uint32_t lds[];
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (wave >= a.w[40]) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  lds[threadIdx.x] = (uint32_t)t0;
  uint64_t t1 = t0;
  while (t1 - t0 < spin_ticks) t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    t[3 * wave] = t0;
    t[3 * wave + 1] = t1 + lds[(threadIdx.x + 64) & 255] * 0 + a.w[threadIdx.x & 31] * 0;
    t[3 * wave + 2] = xcc;
  }
}

int main() {
  const int waves = 4096;
  uint64_t* t;
  hipMalloc(&t, waves * 24);
  std::vector<uint64_t> h(3 * waves);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  BigArgs big{};
  big.w[40] = waves;
  // back-to-back launches (as in the bench): per-launch time minus the spin is
  // the launch + drain overhead a kernel pays in a stream of kernels
  for (uint32_t spin_us : {0u, 20u}) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      for (int k = 0; k < 50; k++)
        hipLaunchKernelGGL(timeline, dim3(waves / 4), dim3(256), 33 * 1024, 0, t, spin_us * 100);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep) printf("back-to-back, spin %2u us: %.2f us per launch\n", spin_us, ms * 1000 / 50);
    }
  }
  for (int variant = 0; variant < 2; variant++)
  for (uint32_t spin_us : {0u, 5u, 20u}) {
    const uint32_t ticks = spin_us * 100;
    float ms = 0;
    for (int rep = 0; rep < 5; rep++) {
      hipEventRecord(e0);
      if (variant == 0)
        hipLaunchKernelGGL(timeline, dim3(waves / 4), dim3(256), 33 * 1024, 0, t, ticks);
      else
        hipLaunchKernelGGL(timeline_bigargs, dim3(waves / 4), dim3(256), 33 * 1024, 0, t, ticks, big);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
    }
    hipMemcpy(h.data(), t, waves * 24, hipMemcpyDeviceToHost);
    uint64_t mn = ~0ull;
    for (int i = 0; i < waves; i++) mn = std::min(mn, h[3 * i]);
    printf("%s spin %2u us: event %.2f us\n", variant ? "344-byte kernargs" : "small kernargs", spin_us, ms * 1000);
    for (uint32_t x = 0; x < 8; x++) {
      std::vector<double> s, e;
      for (int i = 0; i < waves; i++)
        if (h[3 * i + 2] == x) { s.push_back((h[3 * i] - mn) * 10.0); e.push_back((h[3 * i + 1] - mn) * 10.0); }
      if (s.empty()) continue;
      std::sort(s.begin(), s.end());
      std::sort(e.begin(), e.end());
      printf("  xcc %u: %4zu waves  entry ns first %6.0f p50 %6.0f last %6.0f | exit last %6.0f  (span %6.0f)\n", x,
             s.size(), s[0], s[s.size() / 2], s.back(), e.back(), e.back() - s[0]);
    }
  }
  return 0;
}
