// cuzfp_amd/csrc/inst_f64.hip -- double instantiations of the codec kernels.
#include "kernels.hpp"

namespace cuzfp {
template int launch_encode_type<double>(const Problem&, const void*, bool, uint64_t*, uint32_t,
                                       uint32_t, hipStream_t);
template int launch_decode_type<double>(const Problem&, const uint64_t*, bool, void*, uint32_t,
                                       uint32_t, hipStream_t);
}  // namespace cuzfp
