// tools/coder_stats.cpp -- plane-coder statistics of the 3D f32 bench field
// (design tool): per block the planes coded, per plane n and the new ones r,
// and per wave (64 consecutive blocks, as the kernels group them) how many
// plane steps the wave walks and how many of them every lane could take on
// a cheap path.
//   g++ -O2 -std=c++17 tools/coder_stats.cpp -o build/coder_stats && build/coder_stats 256 [rough]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "../cuzfp_amd/csrc/zfp_block.hpp"

using namespace cuzfp;

static float poly(float x) {
  const float xx = x * x;
  const float yy = xx * 4.0f - 3.0f;
  return x + xx * yy;
}

static long g_wide_r15 = 0, g_wide_len_only = 0, g_med24 = 0, g_med31 = 0;
int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 256;
  const int rough = argc > 2 ? atoi(argv[2]) : 0;
  const unsigned maxbits = argc > 3 ? atoi(argv[3]) : 512;
  std::vector<float> ax(n);
  for (int i = 0; i < n; i++) ax[i] = poly((float)(2 * i - n + 1) / (float)n);
  const int nb = n / 4;
  const size_t blocks = (size_t)nb * nb * nb;
  const unsigned budget = maxbits - 9;
  // per-plane-step histograms (step = plane index from the top, 0..31)
  long lanes_active[32] = {0}, r_zero[32] = {0}, n_full[32] = {0}, r_wide[32] = {0};
  long wave_all_r0[32] = {0}, wave_any_active[32] = {0}, wave_any_wide[32] = {0}, wave_all_full[32] = {0};
  long wave_fit64[32] = {0}, wave_g20[32] = {0}, wave_g40[32] = {0}, wave_g60[32] = {0};
  long planes_hist[33] = {0}, wave_steps_hist[33] = {0};
  long sum_planes = 0, sum_wave_steps = 0;
  long slow_rem[26] = {0}, slow_n[65] = {0}, slow_len[16] = {0}, slow_fits_budget = 0, slow_total = 0;
  uint64_t st = 42;
  const size_t nwaves = (blocks + 63) / 64;
  for (size_t w = 0; w < nwaves; w++) {
    int wsteps = 0;
    bool act[64][32] = {}, rz[64][32] = {}, wide[64][32] = {}, full[64][32] = {}, fit[64][32] = {}, r15[64][32] = {};
    bool r24[64][32] = {}, r31[64][32] = {};
    unsigned glen[64][32] = {};
    for (int l = 0; l < 64; l++) {
      const size_t b = w * 64 + l;
      if (b >= blocks) break;
      const int bx = b % nb, by = (b / nb) % nb, bz = b / ((size_t)nb * nb);
      float f[64];
      for (int i = 0; i < 64; i++) {
        const int x = 4 * bx + i % 4, y = 4 * by + (i / 4) % 4, z = 4 * bz + i / 16;
        if (rough) {
          st += 0x9e3779b97f4a7c15ull; uint64_t zz = st;
          zz = (zz ^ (zz >> 30)) * 0xbf58476d1ce4e5b9ull; zz = (zz ^ (zz >> 27)) * 0x94d049bb133111ebull; zz ^= zz >> 31;
          f[i] = (float)((double)(zz >> 40) * (1.0 / 8388608.0) - 1.0);
        } else {
          f[i] = ax[x] * ax[y] * ax[z];
        }
      }
      const int emax = fp<float>::emax<64>(f);
      const float s = fp<float>::pow2(30 - emax);
      uint32_t q[64], u[64];
      for (int i = 0; i < 64; i++) q[i] = (uint32_t)fp<float>::to_int(s * f[i]);
      fwd_xform<3>(q);
      const uint32_t NB = 0xaaaaaaaau;
      permute_fwd_add<3>(q, u, NB, make_seq<64>());
      planes<uint32_t, 3> P;
      P.load<true>(u);
      unsigned nn = 0, bits = budget;
      int k = 0;
      for (; k < 32 && bits; k++) {
        const uint64_t x = P.get(31 - k);
        const unsigned nn0 = nn;
        const uint64_t r = nn < 64 ? x >> nn : 0;
        act[l][k] = true;
        rz[l][k] = r == 0;
        wide[l][k] = (r >> 16) != 0;
        r15[l][k] = (r >> 15) != 0;
        r24[l][k] = (r >> 24) != 0;
        r31[l][k] = (r >> 31) != 0;
        full[l][k] = nn == 64;
        // plane code length (unbudgeted)
        unsigned len = nn;
        if (nn < 64) {
          if (!r) len += 1;
          else {
            const unsigned bl = 64 - __builtin_clzll(r), t = __builtin_popcountll(r);
            len += 1 + bl + t - (nn + bl == 64 ? 2 : 0);
            nn += bl;
          }
        }
        fit[l][k] = len <= 64;
        glen[l][k] = len - nn0;
        if (!(r >> 15 == 0 && len <= 64)) {
          const unsigned rem = bits;
          slow_rem[rem > 200 ? 200 / 8 : rem / 8]++;
          slow_n[nn0 > 64 ? 64 : nn0]++;
          slow_len[len > 127 ? 15 : len / 8]++;
          slow_fits_budget += rem <= 64;
          slow_total++;
        }
        bits = len >= bits ? 0 : bits - len;
      }
      sum_planes += k;
      planes_hist[k]++;
      if (k > wsteps) wsteps = k;
    }
    sum_wave_steps += wsteps;
    wave_steps_hist[wsteps]++;
    if (getenv("WAVE_DUMP")) {  // per-wave plane steps, one line per wave (load-balance studies)
      static FILE* wf = fopen(getenv("WAVE_DUMP"), "w");
      fprintf(wf, "%d\n", wsteps);
    }
    for (int k = 0; k < wsteps; k++) {
      bool any15 = false, anylong = false, any24 = false, any31 = false;
      for (int l = 0; l < 64; l++) if (act[l][k]) { any15 |= r15[l][k]; anylong |= !fit[l][k]; any24 |= r24[l][k]; any31 |= r31[l][k]; }
      g_med24 += any15 && !any24 && !anylong;
      g_med31 += any15 && !any31 && !anylong;
      g_wide_r15 += any15; g_wide_len_only += !any15 && anylong;
      bool all0 = true, anyw = false, allf = true, allfit = true;
      unsigned gmax = 0;
      for (int l = 0; l < 64; l++) {
        if (act[l][k]) {
          lanes_active[k]++;
          r_zero[k] += rz[l][k];
          n_full[k] += full[l][k];
          r_wide[k] += wide[l][k];
          all0 &= rz[l][k];
          anyw |= wide[l][k];
          allf &= full[l][k];
          allfit &= fit[l][k];
          if (glen[l][k] > gmax) gmax = glen[l][k];
        }
      }
      wave_any_active[k]++;
      wave_all_r0[k] += all0;
      wave_any_wide[k] += anyw;
      wave_all_full[k] += allf;
      wave_fit64[k] += allfit;
      wave_g20[k] += gmax > 20;
      wave_g40[k] += gmax > 40;
      wave_g60[k] += gmax > 60;
    }
  }
  printf("wide wave-steps per wave: some lane r >= 2^15 %.2f, only len > 64 %.2f\n", (double)g_wide_r15 / nwaves, (double)g_wide_len_only / nwaves);
  printf("  of the r >= 2^15 ones, every lane r < 2^24 and len <= 64: %.2f; r < 2^31 and len <= 64: %.2f\n", (double)g_med24 / nwaves, (double)g_med31 / nwaves);
  printf("blocks %zu waves %zu: planes per block mean %.2f, wave steps mean %.2f\n", blocks, nwaves,
         (double)sum_planes / blocks, (double)sum_wave_steps / nwaves);
  printf("step lanes_act%%  r==0%%  n==64%%  r>=2^16%% | waves: steps  all_r0%%  any_wide%%  all_full%%  all_fit64%%  grp>20%% grp>40%% grp>60%%\n");
  for (int k = 0; k < 32; k++) {
    if (!wave_any_active[k]) break;
    const double la = lanes_active[k];
    printf("%3d %8.1f %7.1f %7.1f %8.2f | %7ld %7.1f %8.2f %8.1f %8.1f %7.1f %7.1f %7.1f\n", k, 100.0 * la / (wave_any_active[k] * 64.0),
           100.0 * r_zero[k] / la, 100.0 * n_full[k] / la, 100.0 * r_wide[k] / la, wave_any_active[k],
           100.0 * wave_all_r0[k] / wave_any_active[k], 100.0 * wave_any_wide[k] / wave_any_active[k],
           100.0 * wave_all_full[k] / wave_any_active[k], 100.0 * wave_fit64[k] / wave_any_active[k], 100.0 * wave_g20[k] / wave_any_active[k],
           100.0 * wave_g40[k] / wave_any_active[k], 100.0 * wave_g60[k] / wave_any_active[k]);
  }
  printf("planes-per-block histogram:");
  for (int k = 0; k <= 32; k++) if (planes_hist[k]) printf(" %d:%ld", k, planes_hist[k]);
  printf("\nwave-steps histogram:");
  for (int k = 0; k <= 32; k++) if (wave_steps_hist[k]) printf(" %d:%ld", k, wave_steps_hist[k]);
  printf("\n");
  printf("slow lane-steps %ld, remaining budget <= 64: %.1f%%\n", slow_total, 100.0 * slow_fits_budget / (slow_total ? slow_total : 1));
  printf("slow: remaining budget hist (8-bit bins):");
  for (int i = 0; i < 26; i++) if (slow_rem[i]) printf(" %d:%ld", i * 8, slow_rem[i]);
  printf("\nslow: n hist:");
  for (int i = 0; i <= 64; i++) if (slow_n[i]) printf(" %d:%ld", i, slow_n[i]);
  printf("\nslow: code len hist (8-bit bins):");
  for (int i = 0; i < 16; i++) if (slow_len[i]) printf(" %d:%ld", i * 8, slow_len[i]);
  printf("\n");
  return 0;
}
