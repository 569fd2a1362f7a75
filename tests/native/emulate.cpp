// tests/native/emulate.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Runs the per-lane block codec of cuzfp_amd/csrc/zfp_block.hpp -- the exact
// functions the HIP kernels execute on every lane -- serially on the host, so
// tests/test_emulation.py can check the lane algorithm bit-for-bit against the
// CPU oracle on a machine without a GPU.  It is never part of the product: the
// shipped codec path is the HIP kernels in cuzfp_amd/csrc/kernels.hpp.
//
// Raster / padding / stream layout are restated here in the simplest form (the
// kernels' coalesced gathers and LDS staging are tested on the GPU itself).
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../cuzfp_amd/csrc/zfp_block.hpp"

namespace {

// Writes each block at its absolute offset into the zeroed stream, dropping
// bits past the block's maxbits (the device writers drop them by never
// flushing a word beyond the block).
struct HostWriter {
  uint64_t* s;
  size_t pos, end;
  bool full() const { return pos >= end; }
  void put(uint64_t v, unsigned n) {
    if (pos >= end) return;
    if (pos + n > end) {
      n = (unsigned)(end - pos);
      v &= cuzfp::lowmask(n);
    }
    if (!n) return;
    const unsigned sh = pos & 63;
    s[pos >> 6] |= v << sh;
    if (sh + n > 64) s[(pos >> 6) + 1] |= v >> (64 - sh);
    pos += n;
  }
  void zero_bit() {
    if (pos < end) pos++;
  }
  void finish() {}
  uint32_t spread(uint32_t b) const {
    static const cuzfp::SpreadLut t = cuzfp::make_spread_lut();
    return t.e[b];
  }
};

struct HostReader {
  const uint64_t* s;
  size_t words;
  size_t pos;
  uint64_t word(size_t i) const { return i < words ? s[i] : 0; }
  uint64_t peek() const {
    const unsigned sh = pos & 63;
    const size_t w = pos >> 6;
    return sh ? (word(w) >> sh) | (word(w + 1) << (64 - sh)) : word(w);
  }
  void peek2(uint64_t& a, uint64_t& b) {
    a = peek();
    pos += 64;
    b = peek();
    pos -= 64;
  }
  void skip(unsigned n) { pos += n; }
  void init(size_t p) { pos = p; }
  // table decoder interface (see LdsReader in kernels.hpp)
  void windows(unsigned m, uint64_t& w, uint32_t& g) {
    w = peek();
    pos += m;
    g = (uint32_t)peek();
    pos -= m;
  }
  static const cuzfp::ChunkLut& table() {
    static const cuzfp::ChunkLut t = cuzfp::make_chunk_lut();
    return t;
  }
  uint32_t lut(uint32_t i) const { return table().e[i]; }
  void lut2(uint32_t i, uint32_t& a, uint32_t& b) const {
    a = table().e[i];
    b = table().e[i + (1u << cuzfp::kChunkBits)];
  }
};

template <typename Scalar, int DIMS>
size_t run(bool enc, unsigned nx, unsigned ny, unsigned nz, long long sx, long long sy,
           long long sz, unsigned maxbits, Scalar* data, uint64_t* stream, size_t words) {
  constexpr int N = 1 << (2 * DIMS);
  const unsigned NY = DIMS > 1 ? ny : 1, NZ = DIMS > 2 ? nz : 1;
  if (!sx) sx = 1;
  if (!sy) sy = nx;
  if (!sz) sz = (long long)nx * NY;
  const size_t bx = (nx + 3) / 4, by = (NY + 3) / 4, bz = (NZ + 3) / 4, nb = bx * by * bz;
  const size_t need = (nb * maxbits + 63) / 64;
  if (words < need) return 0;
  if (enc) memset(stream, 0, need * 8);
  for (size_t b = 0; b < nb; b++) {
    const size_t ix = b % bx, iy = (b / bx) % by, iz = b / (bx * by);
    const int wx = (int)(nx - 4 * ix < 4 ? nx - 4 * ix : 4);
    const int wy = DIMS > 1 ? (int)(NY - 4 * iy < 4 ? NY - 4 * iy : 4) : 1;
    const int wz = DIMS > 2 ? (int)(NZ - 4 * iz < 4 ? NZ - 4 * iz : 4) : 1;
    long long off[N];
    bool valid[N];
    for (int i = 0; i < N; i++) {
      const int x = i & 3, y = (i >> 2) & 3, z = i >> 4;
      const int px = cuzfp::pad_src(x, wx), py = DIMS > 1 ? cuzfp::pad_src(y, wy) : 0,
                pz = DIMS > 2 ? cuzfp::pad_src(z, wz) : 0;
      off[i] = (long long)(4 * ix + px) * sx + (long long)(4 * iy + py) * sy +
               (long long)(4 * iz + pz) * sz;
      valid[i] = x < wx && (DIMS < 2 || y < wy) && (DIMS < 3 || z < wz);
    }
    Scalar f[N];
    if (enc) {
      for (int i = 0; i < N; i++) f[i] = data[off[i]];
      HostWriter wr{stream, b * (size_t)maxbits, (b + 1) * (size_t)maxbits};
      cuzfp::encode_block<Scalar, DIMS>(f, maxbits, wr);
    } else {
      HostReader rd{stream, words, b * (size_t)maxbits};
      cuzfp::decode_block<Scalar, DIMS>(f, maxbits, rd);
      for (int i = 0; i < N; i++)
        if (valid[i]) data[off[i]] = f[i];
    }
  }
  return need * 8;
}

template <typename Scalar>
size_t dispatch_dims(bool enc, unsigned nx, unsigned ny, unsigned nz, long long sx, long long sy,
                     long long sz, unsigned maxbits, void* data, void* stream, size_t bytes) {
  Scalar* d = (Scalar*)data;
  uint64_t* s = (uint64_t*)stream;
  if (nz) return run<Scalar, 3>(enc, nx, ny, nz, sx, sy, sz, maxbits, d, s, bytes / 8);
  if (ny) return run<Scalar, 2>(enc, nx, ny, nz, sx, sy, sz, maxbits, d, s, bytes / 8);
  return run<Scalar, 1>(enc, nx, ny, nz, sx, sy, sz, maxbits, d, s, bytes / 8);
}

size_t dispatch(bool enc, int type, unsigned nx, unsigned ny, unsigned nz, long long sx,
                long long sy, long long sz, unsigned maxbits, void* data, void* stream,
                size_t bytes) {
  switch (type) {
    case 1: return dispatch_dims<int32_t>(enc, nx, ny, nz, sx, sy, sz, maxbits, data, stream, bytes);
    case 2: return dispatch_dims<int64_t>(enc, nx, ny, nz, sx, sy, sz, maxbits, data, stream, bytes);
    case 3: return dispatch_dims<float>(enc, nx, ny, nz, sx, sy, sz, maxbits, data, stream, bytes);
    case 4: return dispatch_dims<double>(enc, nx, ny, nz, sx, sy, sz, maxbits, data, stream, bytes);
  }
  return 0;
}

}  // namespace

extern "C" {

size_t emu_compress(int type, unsigned nx, unsigned ny, unsigned nz, long long sx, long long sy,
                    long long sz, unsigned maxbits, const void* data, void* stream, size_t bytes) {
  return dispatch(true, type, nx, ny, nz, sx, sy, sz, maxbits, (void*)data, stream, bytes);
}

int emu_decompress(int type, unsigned nx, unsigned ny, unsigned nz, long long sx, long long sy,
                   long long sz, unsigned maxbits, const void* stream, size_t bytes, void* data) {
  return dispatch(false, type, nx, ny, nz, sx, sy, sz, maxbits, data, (void*)stream, bytes) != 0;
}

}  // extern "C"
