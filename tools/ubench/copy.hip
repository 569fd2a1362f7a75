// tools/ubench/copy.hip -- achievable HBM copy bandwidth on MI355X by copy-kernel
// shape (design measurement for cuzfp_hip_copy, the bench's calibrator):
// non-temporal vs plain 16-byte accesses, loads in flight per lane, grid size.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/copy.hip -o build/copy_ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT, int U>
__global__ __launch_bounds__(256) void copy_k(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (NT) __builtin_nontemporal_store(v[u], dst + i + u * stride);
      else dst[i + u * stride] = v[u];
    }
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

template <bool NT, int U>
static void run(const char* name, const u32x4* s, u32x4* d, size_t bytes, int grid) {
  const size_t n16 = bytes / 16;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; w++) hipLaunchKernelGGL((copy_k<NT, U>), dim3(grid), dim3(256), 0, 0, s, d, n16);
  hipEventRecord(e0);
  const int reps = 20;
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL((copy_k<NT, U>), dim3(grid), dim3(256), 0, 0, s, d, n16);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("%-8s U=%d grid=%6d bytes=%zu: %.1f GB/s (read+write)\n", name, U, grid, bytes,
         2.0 * bytes * reps / (ms * 1e-3) / 1e9);
}

int main() {
  const size_t bytes = 1ull << 30;
  u32x4 *s, *d;
  hipMalloc(&s, bytes);
  hipMalloc(&d, bytes);
  hipMemset(s, 1, bytes);
  hipMemset(d, 0, bytes);
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int g : {cus * 4, cus * 8, cus * 16, cus * 32, (int)(bytes / 16 / 256)}) {
    run<true, 1>("nt", s, d, bytes, g);
    run<true, 4>("nt", s, d, bytes, g);
    run<false, 1>("plain", s, d, bytes, g);
    run<false, 4>("plain", s, d, bytes, g);
  }
  run<true, 8>("nt", s, d, bytes, cus * 8);
  run<false, 8>("plain", s, d, bytes, cus * 8);
  return 0;
}
