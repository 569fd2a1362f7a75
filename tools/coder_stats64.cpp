// tools/coder_stats64.cpp -- plane statistics of the 3D f64 bench field
// (design tool): per block the planes coded before the budget ends (of 64),
// per wave (64 consecutive blocks) the lowest plane any lane reaches -- the
// question being whether a wave ever needs the low 32-bit half of its planes.
//   g++ -O2 -std=c++17 tools/coder_stats64.cpp -o build/coder_stats64 && build/coder_stats64 256 1024 [rough]
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../cuzfp_amd/csrc/zfp_block.hpp"

using namespace cuzfp;

static double poly(double x) {
  const double xx = x * x;
  const double yy = xx * 4.0 - 3.0;
  return x + xx * yy;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 256;
  const unsigned maxbits = argc > 2 ? atoi(argv[2]) : 1024;
  const int rough = argc > 3 ? atoi(argv[3]) : 0;
  std::vector<double> ax(n);
  for (int i = 0; i < n; i++) ax[i] = poly((double)(2 * i - n + 1) / (double)n);
  const int nb = n / 4;
  const size_t blocks = (size_t)nb * nb * nb;
  const unsigned budget = maxbits - 12;
  long planes_hist[65] = {0}, low_hist[65] = {0};
  long waves_low = 0, sum_planes = 0, nwaves = 0;
  uint64_t st = 42;
  for (size_t w = 0; w < (blocks + 63) / 64; w++) {
    int wmax = 0;
    for (int l = 0; l < 64; l++) {
      const size_t b = w * 64 + l;
      if (b >= blocks) break;
      const int bx = b % nb, by = (b / nb) % nb, bz = b / ((size_t)nb * nb);
      double f[64];
      for (int i = 0; i < 64; i++) {
        const int x = 4 * bx + i % 4, y = 4 * by + (i / 4) % 4, z = 4 * bz + i / 16;
        if (rough) {
          st += 0x9e3779b97f4a7c15ull; uint64_t zz = st;
          zz = (zz ^ (zz >> 30)) * 0xbf58476d1ce4e5b9ull; zz = (zz ^ (zz >> 27)) * 0x94d049bb133111ebull; zz ^= zz >> 31;
          f[i] = (double)(zz >> 11) * (2.0 / 9007199254740992.0) - 1.0;
        } else {
          f[i] = ax[x] * ax[y] * ax[z];
        }
      }
      const int emax = fp<double>::emax<64>(f);
      const double s = fp<double>::pow2(62 - emax);
      uint64_t q[64], u[64];
      for (int i = 0; i < 64; i++) q[i] = (uint64_t)fp<double>::to_int(s * f[i]);
      fwd_xform<3>(q);
      permute_fwd_add<3>(q, u, (uint64_t)0xaaaaaaaaaaaaaaaaull, make_seq<64>());
      planes<uint64_t, 3> P;
      P.load<true>(u);
      unsigned nn = 0, bits = budget;
      int k = 0;
      for (; k < 64 && bits; k++) {
        const uint64_t x = P.get(63 - k);
        const uint64_t r = nn < 64 ? x >> nn : 0;
        unsigned len = nn;
        if (nn < 64) {
          if (!r) len += 1;
          else {
            const unsigned bl = 64 - __builtin_clzll(r), t = __builtin_popcountll(r);
            len += 1 + bl + t - (nn + bl == 64 ? 2 : 0);
            nn += bl;
          }
        }
        bits = len >= bits ? 0 : bits - len;
      }
      planes_hist[k]++;
      sum_planes += k;
      if (k > wmax) wmax = k;
    }
    low_hist[wmax]++;
    waves_low += wmax > 32;
    nwaves++;
  }
  printf("%zu blocks, %ld waves: planes a block %.2f; waves reaching the low half (> 32 planes) %.4f\n", blocks, nwaves,
         (double)sum_planes / blocks, (double)waves_low / nwaves);
  printf("planes a block:");
  for (int k = 0; k <= 64; k++) if (planes_hist[k]) printf(" %d:%.4f", k, (double)planes_hist[k] / blocks);
  printf("\nwave max planes:");
  for (int k = 0; k <= 64; k++) if (low_hist[k]) printf(" %d:%.4f", k, (double)low_hist[k] / nwaves);
  printf("\n");
  return 0;
}
