// tools/wave_work.cpp -- per-wave work of the 3D f32 bench field (design tool):
// for each wave (64 consecutive blocks) the plane steps it walks, the encoder
// steps on the wide path and the decoder steps on a slow path, written as
// int32[nwaves][4] for tools/stamps_simd.py --work.
//   clang++ -O2 -std=c++17 tools/wave_work.cpp -o build/wave_work && build/wave_work 256 out.bin
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../cuzfp_amd/csrc/zfp_block.hpp"
using namespace cuzfp;

static float poly(float x) { const float xx = x * x; const float yy = xx * 4.0f - 3.0f; return x + xx * yy; }

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 256;
  const char* out = argc > 2 ? argv[2] : "wave_work.bin";
  const unsigned maxbits = 512, budget = maxbits - 9;
  std::vector<float> ax(n);
  for (int i = 0; i < n; i++) ax[i] = poly((float)(2 * i - n + 1) / (float)n);
  const int nb = n / 4;
  const size_t blocks = (size_t)nb * nb * nb, nwaves = blocks / 64;
  std::vector<int> res(nwaves * 4);
  for (size_t w = 0; w < nwaves; w++) {
    int steps = 0;
    bool wide[32] = {}, slow[32] = {};
    for (int l = 0; l < 64; l++) {
      const size_t b = w * 64 + l;
      const int bx = b % nb, by = (b / nb) % nb, bz = b / ((size_t)nb * nb);
      float f[64];
      for (int i = 0; i < 64; i++) f[i] = ax[4 * bx + i % 4] * ax[4 * by + (i / 4) % 4] * ax[4 * bz + i / 16];
      const int emax = fp<float>::emax<64>(f);
      const float s = fp<float>::pow2(30 - emax);
      uint32_t q[64], u[64];
      for (int i = 0; i < 64; i++) q[i] = (uint32_t)fp<float>::to_int(s * f[i]);
      fwd_xform<3>(q);
      permute_fwd_add<3>(q, u, 0xaaaaaaaau, make_seq<64>());
      planes<uint32_t, 3> P;
      P.load<true>(u);
      unsigned nn = 0, bits = budget;
      int k = 0;
      for (; k < 32 && bits; k++) {
        const uint64_t x = P.get(31 - k);
        const uint64_t r = nn < 64 ? x >> nn : 0;
        const unsigned n0 = nn;
        unsigned len = nn;
        if (nn < 64) {
          if (!r) len += 1;
          else {
            const unsigned bl = 64 - __builtin_clzll(r), t = __builtin_popcountll(r);
            len += 1 + bl + t - (nn + bl == 64 ? 2 : 0);
            nn += bl;
          }
        }
        if (!(r >> 15 == 0 && len <= 64)) wide[k] = true;
        // decoder: the two-chunk table step covers a group code of <= 20 bits ending within the budget
        const unsigned m = n0 < bits ? n0 : bits;
        const unsigned g = len - n0, b1 = bits - m;
        if (n0 < 64 && (g > 20 || g > b1 + 1)) slow[k] = true;
        bits = len >= bits ? 0 : bits - len;
      }
      if (k > steps) steps = k;
    }
    int nw = 0, ns = 0;
    for (int k = 0; k < 32; k++) { nw += wide[k]; ns += slow[k]; }
    res[w * 4 + 0] = steps; res[w * 4 + 1] = nw; res[w * 4 + 2] = ns; res[w * 4 + 3] = 0;
  }
  FILE* f = fopen(out, "wb");
  fwrite(res.data(), 4, res.size(), f);
  fclose(f);
  printf("wrote %zu waves to %s\n", nwaves, out);
  return 0;
}
