// cuzfp_amd/csrc/inst_f64.hip -- double instantiations of the codec kernels.
#include "kernels.hpp"

namespace cuzfp {
template int launch_encode_type<double>(const Problem&, const void*, bool, uint64_t*, uint32_t,
                                       uint32_t, hipStream_t);
template int launch_decode_type<double>(const Problem&, const uint64_t*, bool, void*, uint32_t,
                                       uint32_t, hipStream_t);
}  // namespace cuzfp

#if defined(CUZFP_PROBE) && CUZFP_PROBE == 9
// diagnostic export of this unit's phase stamps (tools/probe.py --dtype float64)
extern "C" int cuzfp_hip_probe_stamps_f64(void* dst, size_t bytes) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int cuzfp_hip_probe_clear_f64() {
  static uint64_t zero[CUZFP_STAMP_WAVES * 10];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
#endif
