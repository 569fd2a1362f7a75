// tools/ubench/throughput.hip -- design measurements for the codec kernels:
//  (1) SIMD cycles per wave64 VALU instruction vs waves per SIMD (1..8), for
//      32-bit ops, 64-bit shifts and a VALU/SALU mix;
//  (2) dispatch ramp: time of a near-empty kernel of 4096 waves by workgroup size.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/throughput.hip -o build/throughput
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 1024

template <int KIND>
__global__ __launch_bounds__(64) void work(uint32_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = seed ^ threadIdx.x, c = 3 + threadIdx.x, d = 5 ^ threadIdx.x;
  uint64_t x = a, y = b;
  uint32_t s = seed;
  for (int it = 0; it < ITERS; it++) {
    if constexpr (KIND == 0) {  // 8 independent-ish 32-bit VALU per iteration
      asm volatile(
          "v_add_u32 %0, %0, %4\n v_xor_b32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_xor_b32 %3, %3, %4\n"
          "v_add_u32 %0, %0, %4\n v_xor_b32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_xor_b32 %3, %3, %4"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(seed));
    } else if constexpr (KIND == 1) {  // 64-bit shifts
      asm volatile(
          "v_lshlrev_b64 %0, 3, %0\n v_lshrrev_b64 %1, 5, %1\n v_lshlrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 1, %1\n"
          "v_lshlrev_b64 %0, 3, %0\n v_lshrrev_b64 %1, 5, %1\n v_lshlrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 1, %1"
          : "+v"(x), "+v"(y));
    } else if constexpr (KIND == 2) {  // 4 VALU + 4 SALU
      asm volatile(
          "v_add_u32 %0, %0, %4\n s_add_u32 %5, %5, 3\n v_xor_b32 %1, %1, %4\n s_xor_b32 %5, %5, 7\n"
          "v_add_u32 %2, %2, %4\n s_add_u32 %5, %5, 3\n v_xor_b32 %3, %3, %4\n s_xor_b32 %5, %5, 7"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(seed), "+s"(s) :: "scc");
    } else if constexpr (KIND == 3) {  // dependent chain of 8 32-bit VALU
      asm volatile(
          "v_add_u32 %0, %0, %1\n v_xor_b32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_xor_b32 %0, %0, %1\n"
          "v_add_u32 %0, %0, %1\n v_xor_b32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_xor_b32 %0, %0, %1"
          : "+v"(a) : "v"(seed));
    } else if constexpr (KIND == 4) {  // 64-bit adds (v_lshl_add_u64)
      asm volatile(
          "v_lshl_add_u64 %0, %0, 0, %1\n v_lshl_add_u64 %1, %1, 0, %0\n v_lshl_add_u64 %0, %0, 1, %1\n v_lshl_add_u64 %1, %1, 0, %0\n"
          "v_lshl_add_u64 %0, %0, 0, %1\n v_lshl_add_u64 %1, %1, 0, %0\n v_lshl_add_u64 %0, %0, 1, %1\n v_lshl_add_u64 %1, %1, 0, %0"
          : "+v"(x), "+v"(y));
    } else if constexpr (KIND == 5) {  // ds_read_b32 independent (LDS issue)
      // handled below
    }
  }
  out[blockIdx.x * 64 + threadIdx.x] = a ^ b ^ c ^ d ^ (uint32_t)x ^ (uint32_t)(y >> 7) ^ s;
}

__global__ void empty_kernel(uint32_t* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) out[0] = 1;
}

template <int KIND>
static void run_kind(const char* name, uint32_t* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int wps : {1, 2, 3, 4, 6, 8}) {
    const int waves = 1024 * wps;
    float best = 1e9;
    for (int rep = 0; rep < 5; rep++) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(work<KIND>, dim3(waves), dim3(64), 0, 0, d, 1u);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const double instr = (double)ITERS * 8 * wps;  // per SIMD
    printf("%-14s waves/SIMD %d: %.4f ms  %.2f SIMD-cycles per wave-instr (2.4 GHz)\n", name, wps, best,
           best * 1e-3 * 2.4e9 / instr);
  }
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 64 * 8192 * 4 * 8);
  run_kind<0>("valu32", d);
  run_kind<1>("shift64", d);
  run_kind<2>("valu+salu", d);
  run_kind<3>("valu32-dep", d);
  run_kind<4>("lshl_add_u64", d);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int wpg : {1, 2, 4, 8, 16}) {
    for (int total : {4096, 16384}) {
      float best = 1e9;
      for (int rep = 0; rep < 5; rep++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(empty_kernel, dim3(total / wpg), dim3(64 * wpg), 0, 0, d);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      printf("empty kernel %5d waves, %2d waves/WG: %.2f us\n", total, wpg, best * 1e3);
    }
  }
  return 0;
}
