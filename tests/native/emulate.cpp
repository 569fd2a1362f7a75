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

}  // namespace
#include "host_io.hpp"
namespace {

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
      HostReader rd{stream, words, b * (size_t)maxbits, (b + 1) * (size_t)maxbits};
      if (!cuzfp::decode_block<Scalar, DIMS>(f, maxbits, rd))
        for (int i = 0; i < N; i++) f[i] = (Scalar)0;
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



// Differential fuzz of one plane step: the table decoder (decode_plane_any, the
// kernels' path) against the general decoder (decode_plane, itself checked
// against the oracle) from random states -- n, budget, stream bits of varied
// density -- over a window that reads as zeros past the budget, as the
// kernels' does.  Returns the number of mismatching (x, n, bits, pos) results.
extern "C" long long emu_fuzz_plane(unsigned long long seed, long long trials, int dims) {
  uint64_t st = seed;
  auto rnd = [&]() {
    st += 0x9e3779b97f4a7c15ull;
    uint64_t z = st;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  };
  const unsigned N = 1u << (2 * dims);
  long long bad = 0;
  for (long long t = 0; t < trials; t++) {
    uint64_t buf[6] = {0, 0, 0, 0, 0, 0};
    const unsigned dens = (unsigned)(rnd() % 9);  // 0..8 -> one-bit probability dens/8 (0: structured)
    for (int i = 0; i < 4; i++) {
      uint64_t v = 0;
      if (dens == 0) {
        v = rnd() & rnd() & rnd();
      } else {
        for (int b = 0; b < 64; b++) v |= (uint64_t)((rnd() & 7u) < dens) << b;
      }
      buf[i] = v;
    }
    const unsigned n0 = (unsigned)(rnd() % (N + 1));
    const unsigned bits0 = (unsigned)(rnd() % 161);  // 0: a lane whose block is done (it keeps stepping with its wave)
    const size_t end = bits0;  // the budget ends where the block does
    HostReader ra{buf, 6, 0, end}, rb{buf, 6, 0, end};
    // n = N-1 and n = N are the same state (the table steps keep n <= N-1)
    auto cap = [&](unsigned v) { return v < N - 1 ? v : N - 1; };
    unsigned na = cap(n0), nb = n0, bb = bits0;
    uint64_t xa, xb;
    if (dims == 3) {
      xa = cuzfp::decode_plane_any<3, uint64_t>(na, ra);
      xb = cuzfp::decode_plane<3, uint64_t>(bb, nb, rb);
    } else if (dims == 2) {
      xa = cuzfp::decode_plane_any<2, uint32_t>(na, ra);
      xb = cuzfp::decode_plane<2, uint32_t>(bb, nb, rb);
    } else {
      xa = cuzfp::decode_plane_any<1, uint32_t>(na, ra);
      xb = cuzfp::decode_plane<1, uint32_t>(bb, nb, rb);
    }
    // the table steps keep the budget as the reader's end position: the bits
    // left are end - pos
    if (xa != xb || na != cap(nb) || ra.pos != rb.pos || end - rb.pos != bb) bad++;
    {  // the fast step with the budget (decode_half's every step)
      HostReader rc{buf, 6, 0, end};
      unsigned nc = cap(n0);
      const uint64_t xc = dims == 3 ? cuzfp::decode_plane_fast_any<3, uint64_t>(nc, rc)
                          : dims == 2 ? (uint64_t)cuzfp::decode_plane_fast_any<2, uint32_t>(nc, rc)
                                      : (uint64_t)cuzfp::decode_plane_fast_any<1, uint32_t>(nc, rc);
      if (xc != xb || nc != cap(nb) || rc.pos != rb.pos) bad++;
    }
  }
  return bad;
}
