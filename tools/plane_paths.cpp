// tools/plane_paths.cpp -- how each plane's group code ends in the 3D rate-8
// stream (design tool for the decoder): per lane and per wave (a wave pays for
// a case if any of its 64 lanes has it at that plane step).
//   clang++ -O2 -std=c++17 tools/plane_paths.cpp -o build/plane_paths && build/plane_paths 128 [rough]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "../cuzfp_amd/csrc/zfp_block.hpp"

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

enum { NOGRP, G0, END, IMPLIED, BUDGET, NCASE };
static const char* names[NCASE] = {"no group part", "g0 = 0", "odd pair end", "implied N-1", "budget cut"};

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
  auto bit = [&](size_t p) { return (unsigned)(s[p >> 6] >> (p & 63)) & 1u; };
  long lane[NCASE] = {0}, wave[NCASE] = {0}, dense_l = 0, dense_w = 0, wave_planes = 0, full64 = 0;
  long hist_body[8] = {0}, wb[8] = {0}, wc[8] = {0};
  long heads_max_sum = 0, heads_sum = 0;
  for (size_t w0 = 0; w0 < blocks; w0 += 64) {
    int seen[40][NCASE + 1];
    memset(seen, 0, sizeof seen);
    int maxk = 0, hmax = 0;
    int bmax[40], cmax[40];
    for (int i = 0; i < 40; i++) bmax[i] = cmax[i] = 0;
    for (size_t b = w0; b < w0 + 64 && b < blocks; b++) {
      size_t p = b * maxbits;
      unsigned bits = maxbits;
      if (!bit(p)) continue;
      p += 9; bits -= 9;
      int emax = 0;
      (void)emax;
      unsigned nn = 0, k = 0, heads = 0;
      for (int pl = 31; bits && pl >= 0; pl--, k++) {
        unsigned m = nn < bits ? nn : bits;
        p += m; bits -= m;
        int cs;
        unsigned body = 0;
        const unsigned n0 = nn;
        if (nn >= 64 || !bits) cs = NOGRP;
        else {
          bits--;
          if (!bit(p++)) cs = G0;
          else {
            cs = -1;
            for (;;) {
              while (nn < 63 && bits) { bits--; body++; if (bit(p++)) break; nn++; }
              heads++;
              nn++;
              if (nn >= 64) { cs = IMPLIED; break; }
              if (!bits) { cs = BUDGET; break; }
              bits--; body++;
              if (!bit(p++)) { cs = END; break; }
            }
          }
        }
        if (k < 40) { seen[k][cs] = 1; if (body > 63) seen[k][NCASE] = 1;
          if ((int)body > bmax[k]) bmax[k] = body;
          const int cov = (int)(nn - n0); if (cov > cmax[k]) cmax[k] = cov; }
        lane[cs]++;
        if (body > 63) dense_l++;
        hist_body[body > 127 ? 7 : body / 16 > 6 ? 6 : body / 16]++;
      }
      if (nn >= 64) full64++;
      heads_sum += heads;
      if ((int)heads > hmax) hmax = heads;
      if ((int)k > maxk) maxk = k;
    }
    heads_max_sum += hmax;
    wave_planes += maxk;
    for (int k = 0; k < maxk && k < 40; k++) {
      for (int t = 0; t < 8; t++) { if (bmax[k] > 8 * t + 7) wb[t]++; if (cmax[k] > 8 * t + 8) wc[t]++; }
      for (int c = 0; c < NCASE; c++) wave[c] += seen[k][c];
      dense_w += seen[k][NCASE];
    }
  }
  const double nw = (double)blocks / 64;
  printf("%s %d^3: wave plane steps %.2f, blocks reaching n=64: %.1f%%\n", rough ? "splitmix" : "polynomial", n,
         wave_planes / nw, 100.0 * full64 / blocks);
  printf("  heads per block: lane avg %.2f, wave max avg %.2f\n", heads_sum / (double)blocks, heads_max_sum / nw);
  for (int c = 0; c < NCASE; c++)
    printf("  %-16s lane avg %6.2f   wave plane-steps with any lane %6.2f\n", names[c], lane[c] / (double)blocks, wave[c] / nw);
  printf("  %-16s lane avg %6.2f   wave plane-steps with any lane %6.2f\n", "body > 63 bits", dense_l / (double)blocks, dense_w / nw);
  printf("  wave steps whose max body > 7,15,..: ");
  for (int t = 0; t < 8; t++) printf("%.2f ", wb[t] / nw);
  printf("\n  wave steps whose max covered positions > 8,16,..: ");
  for (int t = 0; t < 8; t++) printf("%.2f ", wc[t] / nw);
  printf("\n");
  printf("  body length hist (16-bit bins): ");
  for (int i = 0; i < 8; i++) printf("%.2f ", hist_body[i] / (double)blocks);
  printf("\n");
}
