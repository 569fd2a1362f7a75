// cuzfp_amd/csrc/inst_f32.hip -- float instantiations of the codec kernels.
#include "kernels.hpp"

namespace cuzfp {
template int launch_encode_type<float>(const Problem&, const void*, bool, uint64_t*, uint32_t,
                                       uint32_t, hipStream_t);
template int launch_decode_type<float>(const Problem&, const uint64_t*, bool, void*, uint32_t,
                                       uint32_t, hipStream_t);
}  // namespace cuzfp

#if defined(CUZFP_PROBE) && CUZFP_PROBE == 9
// diagnostic export of the phase stamps (tools/probe.py)
extern "C" int cuzfp_hip_probe_stamps(void* dst, size_t bytes) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int cuzfp_hip_probe_clear() {
  static uint64_t zero[CUZFP_STAMP_WAVES * 10];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
#endif
