// cuzfp_amd/csrc/launch.hpp -- host-side launch interface shared by the
// per-type kernel translation units and the C-ABI (capi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cuzfp_hip.h"

namespace cuzfp {

constexpr int kLanes = 64;  // blocks per wave64 (one per lane)

struct Geometry {
  uint32_t nx, ny, nz;   // array extent (1 for unused dimensions)
  uint32_t bx, by;       // blocks along x and y
  uint32_t nblocks;      // total blocks
  uint32_t maxbits;      // bits per block
  uint32_t wave0;        // first wave of this launch
  uint32_t wave_end;     // one past its last wave
  uint32_t vec_io;       // stream base 16-byte aligned and maxbits even
  uint32_t lds_words;    // LDS words per wave
  int64_t sx, sy, sz;    // element strides
};

struct Problem {
  int type;
  unsigned dims;
  Geometry g;
  bool fast_ok;  // contiguous, extents multiple of 4 (aligned base checked per call)
};

extern thread_local int t_last_hip;

template <typename Scalar>
int launch_encode_type(const Problem& p, const void* data, bool fast, uint64_t* stream,
                       uint32_t wave0, uint32_t nwaves, hipStream_t st);
template <typename Scalar>
int launch_decode_type(const Problem& p, const uint64_t* stream, bool fast, void* data,
                       uint32_t wave0, uint32_t nwaves, hipStream_t st);

}  // namespace cuzfp
