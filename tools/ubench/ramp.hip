// tools/ubench/ramp.hip -- wave launch ramp: every wave records s_memrealtime
// (100 MHz) at entry; prints the spread of start times for 4096 / 16384 waves
// by workgroup size, with and without a 16 KiB-per-wave global load at entry.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/ramp.hip -o build/ramp
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

// the same with the codec kernels' footprint: ~110 VGPRs and 29 KiB of LDS per workgroup
__global__ __launch_bounds__(256, 4) void ramp_heavy(uint64_t* t, const uint4* src, uint4* dst, int load) {
  extern __shared__ uint32_t lds[];
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  asm volatile("" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109");
  lds[threadIdx.x] = (uint32_t)t0;
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) { t[2 * wave] = t0; t[2 * wave + 1] = t1 + lds[(threadIdx.x + 64) & 255] * 0; }
  (void)src; (void)dst; (void)load;
}

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
  for (int heavy : {0, 1})
  for (int load : {0, 1})
    for (int total : {4096, 16384})
      for (int wpg : {1, 4, 16}) {
        for (int rep = 0; rep < 3; rep++) {
          if (heavy) {
            if (wpg != 4 || load) continue;
            hipLaunchKernelGGL(ramp_heavy, dim3(total / wpg), dim3(64 * wpg), 29 * 1024, 0, t, src, dst, load);
          } else {
            hipLaunchKernelGGL(ramp, dim3(total / wpg), dim3(64 * wpg), 0, 0, t, src, dst, load);
          }
          hipDeviceSynchronize();
        }
        hipMemcpy(h.data(), t, total * 16, hipMemcpyDeviceToHost);
        std::vector<double> s(total), e(total);
        uint64_t mn = ~0ull;
        for (int i = 0; i < total; i++) mn = std::min(mn, h[2 * i]);
        for (int i = 0; i < total; i++) { s[i] = (h[2 * i] - mn) * 10.0; e[i] = (h[2 * i + 1] - mn) * 10.0; }
        std::sort(s.begin(), s.end());
        std::sort(e.begin(), e.end());
        if (heavy && (wpg != 4 || load)) continue;
        printf("heavy %d load %d waves %5d wpg %2d: start ns p10 %6.0f p50 %6.0f p90 %6.0f max %6.0f | loaded ns p50 %6.0f max %6.0f\n",
               heavy, load, total, wpg, s[total / 10], s[total / 2], s[total * 9 / 10], s[total - 1], e[total / 2], e[total - 1]);
      }
  return 0;
}
