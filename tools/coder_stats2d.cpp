// tools/coder_stats2d.cpp -- plane-step statistics of the 2D f32 bench field
// (design tool): per block the planes the decoder walks before the budget
// ends, per wave (64 consecutive x-blocks) the plane steps the wave walks
// (the max over its lanes, rounded up to the unrolled loop's pairs).
//   g++ -O2 -std=c++17 tools/coder_stats2d.cpp -o build/coder_stats2d && build/coder_stats2d 8192 32
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../cuzfp_amd/csrc/zfp_block.hpp"

using namespace cuzfp;

static float poly(float x) {
  const float xx = x * x;
  const float yy = xx * 4.0f - 3.0f;
  return x + xx * yy;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 8192;
  const unsigned maxbits = argc > 2 ? atoi(argv[2]) : 32;
  const int rows = argc > 3 ? atoi(argv[3]) : 64;  // block rows sampled (evenly spaced)
  std::vector<float> ax(n);
  for (int i = 0; i < n; i++) ax[i] = poly((float)(2 * i - n + 1) / (float)n);
  const int nb = n / 4;
  const unsigned budget = maxbits - 9;
  long planes_hist[33] = {0}, wave_hist[33] = {0}, pair_hist[17] = {0}, n_hist[17] = {0};
  long blocks = 0, waves = 0, sum_planes = 0, sum_wave = 0, sum_pairs = 0;
  for (int r = 0; r < rows; r++) {
    const int by = (int)((long)r * nb / rows);
    for (int w0 = 0; w0 < nb; w0 += 64) {
      int wmax = 0;
      for (int l = 0; l < 64 && w0 + l < nb; l++) {
        const int bx = w0 + l;
        float f[16];
        for (int i = 0; i < 16; i++) f[i] = ax[4 * bx + i % 4] * ax[4 * by + i / 4];
        const int emax = fp<float>::emax<16>(f);
        int k = 0;
        unsigned nn = 0;
        if (precision<2>(emax, 32) && emax + 127) {
          const float s = fp<float>::pow2(30 - emax);
          uint32_t q[16], u[16];
          for (int i = 0; i < 16; i++) q[i] = (uint32_t)fp<float>::to_int(s * f[i]);
          fwd_xform<2>(q);
          permute_fwd_add<2>(q, u, 0xaaaaaaaau, make_seq<16>());
          planes<uint32_t, 2> P;
          P.load<true>(u);
          unsigned bits = budget;
          for (; k < 32 && bits; k++) {
            const uint32_t x = (uint32_t)P.get(31 - k);
            const uint32_t rr = nn < 16 ? x >> nn : 0;
            unsigned len = nn;
            if (nn < 16) {
              if (!rr) len += 1;
              else {
                const unsigned bl = 32 - __builtin_clz(rr), t = __builtin_popcount(rr);
                len += 1 + bl + t - (nn + bl == 16 ? 2 : 0);
                nn += bl;
              }
            }
            bits = len >= bits ? 0 : bits - len;
          }
        }
        planes_hist[k]++;
        n_hist[nn > 16 ? 16 : nn]++;
        sum_planes += k;
        blocks++;
        if (k > wmax) wmax = k;
      }
      wave_hist[wmax]++;
      sum_wave += wmax;
      pair_hist[(wmax + 1) / 2]++;
      sum_pairs += (wmax + 1) / 2;
      waves++;
    }
  }
  printf("%ld blocks, %ld waves: planes a block %.2f, plane steps a wave %.2f, pairs a wave %.2f\n", blocks, waves,
         (double)sum_planes / blocks, (double)sum_wave / waves, (double)sum_pairs / waves);
  printf("planes a block:");
  for (int k = 0; k <= 32; k++) if (planes_hist[k]) printf(" %d:%.3f", k, (double)planes_hist[k] / blocks);
  printf("\nsteps a wave:");
  for (int k = 0; k <= 32; k++) if (wave_hist[k]) printf(" %d:%.3f", k, (double)wave_hist[k] / waves);
  printf("\nfinal n:");
  for (int k = 0; k <= 16; k++) if (n_hist[k]) printf(" %d:%.3f", k, (double)n_hist[k] / blocks);
  printf("\n");
  return 0;
}
