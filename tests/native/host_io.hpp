// tests/native/host_io.hpp -- TEST INFRASTRUCTURE ONLY: host-side bit writer
// and reader with the interfaces the per-lane codec of zfp_block.hpp expects
// (the kernels' LDS writers / readers, restated serially).  Used by
// tests/native/emulate.cpp and the design tools.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../cuzfp_amd/csrc/zfp_block.hpp"

// Writes each block at its absolute offset into the zeroed stream, dropping
// bits past the block's maxbits (the device writers drop them by never
// flushing a word beyond the block).
struct HostWriter {
  uint64_t* s;
  size_t pos, end;
  uint64_t fit_lim = 0x7fff;  // (see LdsOrWriter)
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
  void settle() {}
  void zero_bit() {
    if (pos < end) pos++;
  }
  void finish() {}
  void lds_wait() const {}
  uint32_t spread(uint32_t b) const {
    static const cuzfp::SpreadLut t = cuzfp::make_spread_lut();
    return t.e[b];
  }
  uint32_t sp0(uint32_t o) const { return tab().e[o >> 2]; }  // o: byte offset
  uint32_t sp1(uint32_t o) const { return tab().e[256 + (o >> 2)]; }
  static const cuzfp::SpreadTab& tab() {
    static const cuzfp::SpreadTab t = cuzfp::make_spread_tab();
    return t;
  }
  // the 1D pair table (o: byte offset)
  uint32_t pair1d(uint32_t o) const {
    static const cuzfp::Pair1dLut t = cuzfp::make_pair1d_lut();
    return t.e[o >> 2];
  }
};

struct HostReader {
  const uint64_t* s;
  size_t words;
  size_t pos;
  size_t end;  // the block's last bit + 1: the stream reads as zeros from there (as on the GPU)
  uint64_t word(size_t i) const { return i < words ? s[i] : 0; }
  uint64_t peek() const {
    if (pos >= end) return 0;
    const unsigned sh = pos & 63;
    const size_t w = pos >> 6;
    const uint64_t v = sh ? (word(w) >> sh) | (word(w + 1) << (64 - sh)) : word(w);
    return end - pos < 64 ? v & cuzfp::lowmask((unsigned)(end - pos)) : v;
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
  uint32_t window_g(unsigned m, cuzfp::WRaw& wr) {
    wr = cuzfp::WRaw{0u, 0u, 0u};
    pos += m;
    const uint32_t g = (uint32_t)peek();
    pos -= m;
    return g;
  }
  uint64_t window_w_make(const cuzfp::WRaw&) const { return peek(); }
  void lds_wait() const {}
  // the 1D plane table (o: byte offset) and the next 8 stream bits
  uint32_t dec1d(uint32_t o) const {
    static const cuzfp::Plane1dDecLut t = cuzfp::make_plane1d_dec_lut();
    return t.e[o >> 1];
  }
  uint32_t bits8() const { return (uint32_t)peek() & 0xffu; }
  static const cuzfp::ChunkLut& table() {
    static const cuzfp::ChunkLut t = cuzfp::make_chunk_lut();
    return t;
  }
  void chunks_fast(uint32_t g, uint32_t& e1, uint32_t& sel, uint32_t& e2a, uint32_t& e2b) const {
    const uint32_t* t = table().e;
    const uint32_t gm = (g & 1u) ? g : 0u;
    const uint32_t c2 = gm >> cuzfp::kChunkBits;
    e1 = t[cuzfp::lut_s2_index(gm)];
    sel = t[cuzfp::lut_s2_index(gm) + 1];
    e2a = t[cuzfp::lut_pair_index(c2, 0)];
    e2b = t[cuzfp::lut_pair_index(c2, 1)];
  }
  uint32_t chunk1_fast(uint32_t g) const { return table().e[cuzfp::lut_s2_index(g)]; }
  // continuation pairs: 32 stream bits at q, chunk A in state st, chunk B in states 0 and 1
  uint32_t window32(size_t q) {
    const size_t p = pos;
    pos = q;
    const uint32_t v = (uint32_t)peek();
    pos = p;
    return v;
  }
  void chunks_st(uint32_t g, uint32_t st, uint32_t& eA, uint32_t& eBa, uint32_t& eBb) const {
    const uint32_t* t = table().e;
    const uint32_t c2 = g >> cuzfp::kChunkBits;
    eA = t[cuzfp::lut_pair_index(g, st)];
    eBa = t[cuzfp::lut_pair_index(c2, 0)];
    eBb = t[cuzfp::lut_pair_index(c2, 1)];
  }
};

