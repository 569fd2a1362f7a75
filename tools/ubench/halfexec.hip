// tools/ubench/halfexec.hip -- does a wave64 VALU op with only 32 active lanes
// (one half of EXEC zero) cost fewer SIMD cycles on gfx950?  Design
// measurement: runs a VALU-bound loop with 8 waves per SIMD, EXEC = all 64
// lanes vs lanes 0-31 only vs lanes 0-15, and reports kernel time.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ __launch_bounds__(64) void work(uint32_t* out, uint32_t seed, int active) {
  uint32_t a = seed + threadIdx.x, b = seed ^ threadIdx.x, c = 3, d = 5;
  if ((int)threadIdx.x < active) {
    for (int it = 0; it < 2048; it++) {
      asm volatile("v_add_u32 %0, %0, %4\n v_xor_b32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_xor_b32 %3, %3, %4"
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(seed));
    }
  }
  out[blockIdx.x * 64 + threadIdx.x] = a ^ b ^ c ^ d;
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 64 * 8192 * 4 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int waves : {1024, 4096, 8192}) {
    for (int active : {64, 32, 16}) {
      float best = 1e9;
      for (int rep = 0; rep < 5; rep++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(work, dim3(waves), dim3(64), 0, 0, d, 1u, active);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      // 8192 VALU per wave
      double cyc_per_instr_simd = best * 1e-3 * 2.4e9 / ((double)waves / 1024 * 8192);
      printf("waves %5d active lanes %2d: %.3f ms  (%.2f SIMD cycles per wave-instruction at 2.4 GHz)\n",
             waves, active, best, cyc_per_instr_simd);
    }
  }
  return 0;
}
