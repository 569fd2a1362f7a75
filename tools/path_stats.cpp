// tools/path_stats.cpp -- how often the decoder's plane paths are taken, per
// lane and per wave (a wave pays for a path if any of its 64 lanes takes it).
// Design tool: /opt/rocm/llvm/bin/clang++ -O2 -std=c++17 tools/path_stats.cpp -o build/path_stats
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
static int g_path[64];  // per-plane-call path of the current lane: 0 no group, 1 g0=0, 2 complete, 3 limited, 4 fallback
static int g_calls;
#define ZFP_COUNT_PLANE(g0, fast, complete) \
  do { g_path[g_calls++ & 63] = !(g0) ? 1 : (fast) ? 2 : 4; } while (0)
#include "../cuzfp_amd/csrc/zfp_block.hpp"
#include <math.h>

struct Rd {
  const uint64_t* s; size_t pos;
  uint64_t w(size_t i) const { return s[i]; }
  uint64_t peek() const { unsigned sh = pos & 63; size_t i = pos >> 6; return sh ? (w(i) >> sh) | (w(i + 1) << (64 - sh)) : w(i); }
  void peek2(uint64_t& a, uint64_t& b) { a = peek(); pos += 64; b = peek(); pos -= 64; }
  void skip(unsigned n) { pos += n; }
  void init(size_t p) { pos = p; }
  void windows(unsigned m, uint64_t& w, uint32_t& g) { w = peek(); pos += m; g = (uint32_t)peek(); pos -= m; }
  static const cuzfp::ChunkLut& table() { static const cuzfp::ChunkLut t = cuzfp::make_chunk_lut(); return t; }
  void chunks(uint32_t g, bool group, uint32_t& e1, uint32_t& e2a, uint32_t& e2b) const {
    const uint32_t* t = table().e;
    const uint32_t c2 = (g >> cuzfp::kChunkBits) & cuzfp::kChunkMask;
    e1 = t[group ? (2u << cuzfp::kChunkBits) | (g & cuzfp::kChunkMask) : cuzfp::kNoGroupEntry];
    e2a = t[c2];
    e2b = t[c2 + (1u << cuzfp::kChunkBits)];
  }
  void chunks_fast(uint32_t g, bool last, uint32_t& e1, uint32_t& e2a, uint32_t& e2b) const {
    const uint32_t* t = table().e;
    const uint32_t gm = (g & 1u) ? g : 0u;
    const uint32_t c2 = (gm >> cuzfp::kChunkBits) & cuzfp::kChunkMask;
    e1 = t[last ? cuzfp::kLastPosEntry + (g & 1u) : (2u << cuzfp::kChunkBits) | (gm & cuzfp::kChunkMask)];
    e2a = t[c2];
    e2b = t[c2 + (1u << cuzfp::kChunkBits)];
  }
  uint32_t chunk1_fast(uint32_t g, bool last) const {
    const uint32_t gm = (g & 1u) ? g : 0u;
    return table().e[last ? cuzfp::kLastPosEntry + (g & 1u) : (2u << cuzfp::kChunkBits) | (gm & cuzfp::kChunkMask)];
  }
  uint32_t chunk1(uint32_t g, bool group) const {
    return table().e[group ? (2u << cuzfp::kChunkBits) | (g & cuzfp::kChunkMask) : cuzfp::kNoGroupEntry];
  }
  uint32_t window32(size_t q) { const size_t p = pos; pos = q; const uint32_t v = (uint32_t)peek(); pos = p; return v; }
  void chunks_st(uint32_t g, uint32_t st, uint32_t& eA, uint32_t& eBa, uint32_t& eBb) const {
    const uint32_t* t = table().e;
    const uint32_t c2 = (g >> cuzfp::kChunkBits) & cuzfp::kChunkMask;
    eA = t[(st << cuzfp::kChunkBits) | (g & cuzfp::kChunkMask)];
    eBa = t[c2];
    eBb = t[c2 + (1u << cuzfp::kChunkBits)];
  }
};
struct Wr {
  uint64_t* s; size_t pos, end;
  bool full() const { return pos >= end; }
  void put(uint64_t v, unsigned n) {
    if (pos >= end) return;
    if (pos + n > end) { n = end - pos; v &= cuzfp::lowmask(n); }
    if (!n) return;
    unsigned sh = pos & 63; s[pos >> 6] |= v << sh; if (sh + n > 64) s[(pos >> 6) + 1] |= v >> (64 - sh); pos += n;
  }
  void settle() {}
  void zero_bit() { if (pos < end) pos++; }
  void finish() {}
  uint32_t spread(uint32_t b) const { static const cuzfp::SpreadLut t = cuzfp::make_spread_lut(); return t.e[b]; }
};

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 128;
  const int rough = argc > 2 ? atoi(argv[2]) : 0;
  const unsigned maxbits = 512;
  std::vector<float> a((size_t)n * n * n);
  uint64_t st = 42;
  for (int z = 0; z < n; z++) for (int y = 0; y < n; y++) for (int x = 0; x < n; x++) {
    auto f = [&](int i) { double t = (2.0 * i - n + 1) / n; return (float)(t - 3 * t * t + 4 * t * t * t * t); };
    float v;
    if (rough) { st += 0x9e3779b97f4a7c15ull; uint64_t zz = st; zz = (zz ^ (zz >> 30)) * 0xbf58476d1ce4e5b9ull; zz = (zz ^ (zz >> 27)) * 0x94d049bb133111ebull; zz ^= zz >> 31; v = (float)((double)(zz >> 11) / 9007199254740992.0 * 2 - 1); }
    else v = f(x) * f(y) * f(z);
    a[((size_t)z * n + y) * n + x] = v;
  }
  const int nb = n / 4;
  const size_t blocks = (size_t)nb * nb * nb;
  std::vector<uint64_t> s(blocks * maxbits / 64 + 4, 0);
  for (size_t b = 0; b < blocks; b++) {
    int bx = b % nb, by = (b / nb) % nb, bz = b / (nb * nb);
    float f[64];
    for (int i = 0; i < 64; i++) f[i] = a[((size_t)(4 * bz + i / 16) * n + 4 * by + (i / 4) % 4) * n + 4 * bx + i % 4];
    Wr w{s.data(), b * maxbits, (b + 1) * maxbits};
    cuzfp::encode_block<float, 3>(f, maxbits, w);
  }
  // per wave: for each plane call index, which paths occur among the lanes
  long lane_cnt[5] = {0}, wave_cnt[5] = {0}, wave_planes = 0;
  for (size_t w0 = 0; w0 < blocks; w0 += 64) {
    int seen[64][5];
    memset(seen, 0, sizeof seen);
    int maxcalls = 0;
    for (size_t b = w0; b < w0 + 64 && b < blocks; b++) {
      g_calls = 0;
      Rd r{s.data(), b * maxbits};
      float f[64];
      if (!cuzfp::decode_block<float, 3>(f, maxbits, r))
        for (int i = 0; i < 64; i++) f[i] = 0.0f;
      for (int c = 0; c < g_calls && c < 64; c++) { seen[c][g_path[c]] = 1; lane_cnt[g_path[c]]++; }
      if (g_calls > maxcalls) maxcalls = g_calls;
    }
    wave_planes += maxcalls;
    for (int c = 0; c < maxcalls; c++) for (int p = 0; p < 5; p++) wave_cnt[p] += seen[c][p];
  }
  const double nw = (double)blocks / 64;
  const char* nm[5] = {"no group part", "g0 = 0", "complete (fast)", "budget-limited (fast)", "fallback loop"};
  printf("%s %d^3: wave plane steps %.2f\n", rough ? "splitmix" : "polynomial", n, wave_planes / nw);
  for (int p = 0; p < 5; p++) printf("  %-22s lane avg %6.2f   wave executes %6.2f\n", nm[p], lane_cnt[p] / (double)blocks, wave_cnt[p] / nw);
}
