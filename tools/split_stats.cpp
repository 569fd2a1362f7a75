// tools/split_stats.cpp -- design tool: plane-step statistics of the 3D f32
// encoders on a field, per wave (host, no GPU).  Per block: its 32 plane words
// (zfp_block.hpp's own path) and every plane's code length and one-put
// fitness (r < 2^15 and len <= 64: encode_plane_step).  Per wave: the plane
// steps the wave executes (while any lane has budget) and how many of them take
// the wide step (some lane unfit), for
//   per-lane: 64 blocks a wave, planes 31..0 (zfp_encode)
//   split:    32 blocks a wave, lane A planes 31..16, lane B planes 15..0
//             (zfp_encode3_split), B's budget fixed (lim) or shrinking with A's
//             position (lim - posA, re-read every plane pair)
// Build: g++ -O2 -std=c++17 tools/split_stats.cpp -o build/split_stats
// Run:   build/split_stats 256 512 [splitmix]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../cuzfp_amd/csrc/zfp_block.hpp"

using namespace cuzfp;

static float axis(uint32_t i, uint32_t n) {  // cuzfp_amd/datagen.py polynomial_field
  const float x = (float)(int)(2 * i - n + 1) / (float)n;
  const float xx = x * x;
  return x + xx * (xx * 4.0f - 3.0f);
}
static uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct PlaneInfo {
  uint64_t x[32];
  unsigned e;  // 0: zero block
};

static unsigned bitlen64(uint64_t v) { return v ? 64 - __builtin_clzll(v) : 0; }

// code length and fitness of plane x at n; n updated
static bool g_med;  // the last step's plane fits r < 2^15 (its code may be longer than 64 bits)
static unsigned step(uint64_t x, unsigned& n, bool& ok) {
  const uint64_t r = x >> n;
  const unsigned bl = bitlen64(r), L = (unsigned)__builtin_popcountll(r) + bl;
  const unsigned nn = n + bl, imp = nn >> 6;
  const unsigned len = n + L + 1 - 2 * imp;
  const unsigned bl16 = bitlen64(r & 0xffffffffull), L16 = (unsigned)__builtin_popcount((uint32_t)r) + bl16;
  const unsigned len16 = n + L16 + 1 - 2 * ((n + bl16) >> 6);
  ok = (r >> 15) == 0 && len16 <= 64;
  g_med = (r >> 15) == 0;
  n = nn - imp;
  return len;
}

int main(int argc, char** argv) {
  const unsigned E = argc > 1 ? atoi(argv[1]) : 256, mb = argc > 2 ? atoi(argv[2]) : 512;
  const bool sm = argc > 3;
  const size_t nb = (size_t)(E / 4) * (E / 4) * (E / 4);
  std::vector<PlaneInfo> P(nb);
  uint64_t seed = 42;
  std::vector<float> field;
  if (sm) {
    field.resize((size_t)E * E * E);
    for (auto& v : field) v = (float)((double)(splitmix(seed) >> 11) * 0x1.0p-53 * 2.0 - 1.0);
  }
  for (size_t b = 0; b < nb; b++) {
    const size_t bx = b % (E / 4), by = (b / (E / 4)) % (E / 4), bz = b / ((E / 4) * (E / 4));
    float f[64];
    for (int i = 0; i < 64; i++) {
      const uint32_t x = 4 * bx + (i & 3), y = 4 * by + ((i >> 2) & 3), z = 4 * bz + (i >> 4);
      f[i] = sm ? field[((size_t)z * E + y) * E + x] : axis(x, E) * axis(y, E) * axis(z, E);
    }
    const int emax = fp<float>::emax<64>(f);
    P[b].e = (unsigned)(emax + 127);
    const float s = fp<float>::pow2(30 - emax);
    uint32_t q[64], u[64];
    for (int i = 0; i < 64; i++) q[i] = (uint32_t)fp<float>::to_int(s * f[i]);
    fwd_xform<3>(q);
    permute_fwd_add<3>(q, u, 0xaaaaaaaau, make_seq<64>());
    planes<uint32_t, 3> pl;
    pl.load<true>(u);
    for (int k = 0; k < 32; k++) P[b].x[k] = pl.get<0>(k);
  }
  const unsigned lim = mb - 9;  // bits after the exponent
  // per-lane waves
  {
    double steps = 0, wide = 0, need = 0, nlanes = 0, wider = 0;
    size_t waves = 0;
    for (size_t w0 = 0; w0 < nb; w0 += 64, waves++) {
      unsigned n[64] = {}, pos[64] = {};
      for (int l = 0; l < 64 && w0 + l < nb; l++) {  // planes each block needs on its own
        unsigned nn = 0, p = 0, k = 32;
        bool ok;
        while (k > 0 && p < lim && P[w0 + l].e) p += step(P[w0 + l].x[--k], nn, ok);
        need += 32 - k, nlanes++;
      }
      bool full[64];
      for (int l = 0; l < 64; l++) full[l] = w0 + l >= nb || !P[w0 + l].e;
      for (int k = 31; k >= 0; k--) {
        if (k % 2 == 1) {
          bool any = false;
          for (int l = 0; l < 64; l++) any |= !full[l];
          if (!any) break;
        }
        bool anyw = false, anyr = false;
        for (int l = 0; l < 64; l++) {
          if (w0 + l >= nb) continue;
          bool ok;
          pos[l] += step(P[w0 + l].x[k], n[l], ok);
          anyw |= !ok;
          anyr |= !g_med;
          if (pos[l] >= lim) full[l] = true;
        }
        steps++, wide += anyw, wider += anyr;
      }
    }
    printf("per-lane: %zu waves of 64 blocks: %.2f plane steps a wave, %.2f wide (%.2f with r >= 2^15); a block needs %.2f planes on average\n",
           waves, steps / waves, wide / waves, wider / waves, need / nlanes);
  }
  for (int dyn = 0; dyn < 2; dyn++) {
    double steps = 0, wide = 0, wideA = 0, wideB = 0;
    size_t waves = 0;
    for (size_t w0 = 0; w0 < nb; w0 += 32, waves++) {
      unsigned n[64] = {}, pos[64] = {};
      bool full[64];
      for (int l = 0; l < 32; l++) {
        const bool dead = w0 + l >= nb || !P[w0 + l].e;
        full[l] = full[l + 32] = dead;
        if (dead) continue;
        uint64_t o = 0;
        for (int k = 16; k < 32; k++) o |= P[w0 + l].x[k];
        const unsigned bl = bitlen64(o);
        n[l + 32] = bl < 63 ? bl : 63;
      }
      for (int j = 15; j >= 0; j--) {
        if (j % 2 == 1) {
          if (dyn)
            for (int l = 0; l < 32; l++)
              if (pos[l + 32] + pos[l] >= lim) full[l + 32] = true;
          bool any = false;
          for (int l = 0; l < 64; l++) any |= !full[l];
          if (!any) break;
        }
        bool anyw = false, aw = false, bw = false;
        for (int l = 0; l < 64; l++) {
          const size_t b = w0 + (l & 31);
          if (b >= nb) continue;
          bool ok;
          pos[l] += step(P[b].x[l < 32 ? 16 + j : j], n[l], ok);
          anyw |= !ok;
          (l < 32 ? aw : bw) |= !ok;
          if (pos[l] >= lim) full[l] = true;
        }
        steps++, wide += anyw, wideA += aw, wideB += bw;
      }
    }
    printf("split%s: %zu waves of 32 blocks: %.2f plane steps a wave, %.2f wide (A %.2f, B %.2f)\n",
           dyn ? " (B's budget lim - posA)" : "", waves, steps / waves, wide / waves, wideA / waves, wideB / waves);
  }
  return 0;
}
