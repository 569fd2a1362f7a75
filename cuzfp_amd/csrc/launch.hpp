// cuzfp_amd/csrc/launch.hpp -- host-side launch interface shared by the
// per-type kernel translation units and the C-ABI (capi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cuzfp_hip.h"

namespace cuzfp {

constexpr int kLanes = 64;  // blocks per wave64 (one per lane)
constexpr int kMaxDevices = 64;  // per-device caches (launch policy, host pipeline)

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
  // block index -> position without an integer divide: q = (n * m) >> s for
  // n < 2^31 (set_divisor), by bx and by bx * by; divmagic = 0 when nblocks
  // is too large for it (plain division then)
  uint32_t dbx_m, dbx_s, dpl_m, dpl_s, divmagic;
  // 3D double decoder: rows a pass when its row stores are staged through the
  // wave's LDS image (0: stored straight from the lanes), see kernels.hpp
  uint32_t row_stage;
};

// q = floor(n / d) = (n * m) >> s for every n < 2^31, with s = 31 + ceil(log2 d)
// and m = ceil(2^s / d) < 2^32: m = (2^s + e) / d with 0 <= e < d, so
// n * m / 2^s = n / d + n e / (d 2^s) and n e < 2^31 * 2^ceil(log2 d) = 2^s
// keeps the error below 1 / d, inside the gap floor(n / d) leaves.
inline void set_divisor(uint32_t d, uint32_t& m, uint32_t& s) {
  uint32_t l = 0;
  while ((1ull << l) < d) l++;
  s = 31 + l;
  m = (uint32_t)(((1ull << s) + d - 1) / d);
}

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
