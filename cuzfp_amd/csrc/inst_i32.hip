// cuzfp_amd/csrc/inst_i32.hip -- int32_t instantiations of the codec kernels.
#include "kernels.hpp"

namespace cuzfp {
template int launch_encode_type<int32_t>(const Problem&, const void*, bool, uint64_t*, uint32_t,
                                       uint32_t, hipStream_t);
template int launch_decode_type<int32_t>(const Problem&, const uint64_t*, bool, void*, uint32_t,
                                       uint32_t, hipStream_t);
}  // namespace cuzfp
