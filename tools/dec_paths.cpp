// tools/dec_paths.cpp -- which decoder plane steps a wave executes on the 3D
// (or, with a third argument 2, the 2D) f32 bench field (design tool): per plane call of each lane the path taken
// (ZFP_COUNT_PATH ids in zfp_block.hpp), then per wave (64 consecutive blocks,
// as the kernels group them) how many plane-call indices had at least one
// lane on each path -- a wave pays for a path when any lane takes it.
//   clang++ -O2 -std=c++17 tools/dec_paths.cpp -o build/dec_paths && build/dec_paths 256
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
static int g_path[96], g_calls;
static long g_reason[16];
#define ZFP_COUNT_PATH(id) \
  do { if ((id) >= 10) g_reason[(id) - 10]++; else if (g_calls < 96) g_path[g_calls++] = (id); } while (0)
#include "../cuzfp_amd/csrc/zfp_block.hpp"
#include "../tests/native/host_io.hpp"

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 128;
  const unsigned maxbits = argc > 2 ? atoi(argv[2]) : 512;
  const int dims = argc > 3 ? atoi(argv[3]) : 3;
  const bool dbl = argc > 4 && argv[4][0] == 'd';  // 3D double
  std::vector<float> ax(n);
  for (int i = 0; i < n; i++) {
    const float x = (float)(2 * i - n + 1) / (float)n, xx = x * x;
    ax[i] = x + xx * (xx * 4.0f - 3.0f);
  }
  const int nb = n / 4;
  const size_t blocks = dims == 3 ? (size_t)nb * nb * nb : (size_t)nb * nb;
  std::vector<uint64_t> s(blocks * maxbits / 64 + 4, 0);
  for (size_t b = 0; b < blocks; b++) {
    const int bx = b % nb, by = (b / nb) % nb, bz = b / ((size_t)nb * nb);
    float f[64];
    HostWriter w{s.data(), b * maxbits, (b + 1) * maxbits};
    if (dims == 3 && dbl) {
      double d[64];
      for (int i = 0; i < 64; i++) d[i] = (double)(ax[4 * bx + i % 4] * ax[4 * by + (i / 4) % 4] * ax[4 * bz + i / 16]);
      cuzfp::encode_block<double, 3>(d, maxbits, w);
    } else if (dims == 3) {
      for (int i = 0; i < 64; i++) f[i] = ax[4 * bx + i % 4] * ax[4 * by + (i / 4) % 4] * ax[4 * bz + i / 16];
      cuzfp::encode_block<float, 3>(f, maxbits, w);
    } else {
      for (int i = 0; i < 16; i++) f[i] = ax[4 * bx + i % 4] * ax[4 * by + i / 4];
      cuzfp::encode_block<float, 2>(f, maxbits, w);
    }
  }
  const char* nm[9] = {"fast ok", "fast rare (table)", "fast -> general", "-", "-",
                       "table ok", "table -> general", "-", "-"};
  long lane[9] = {0}, wave[9] = {0};
  double wave_calls = 0;
  for (size_t w0 = 0; w0 < blocks; w0 += 64) {
    static int seen[96][9];
    memset(seen, 0, sizeof seen);
    int maxc = 0;
    for (size_t b = w0; b < w0 + 64 && b < blocks; b++) {
      g_calls = 0;
      HostReader r{s.data(), s.size(), b * maxbits, (b + 1) * maxbits};
      float f[64];
      double dd[64];
      if (dims == 3 && dbl) cuzfp::decode_block<double, 3>(dd, maxbits, r);
      else if (dims == 3) cuzfp::decode_block<float, 3>(f, maxbits, r);
      else cuzfp::decode_block<float, 2>(f, maxbits, r);
      // calls are logged in order; a fast/lut entry opens a plane call, cont entries belong to it
      int call = -1;
      for (int c = 0; c < g_calls; c++) {
        const int id = g_path[c];
        if (id <= 2 || id == 5 || id == 6) call++;
        if (call >= 0 && call < 96) seen[call][id] = 1;
        lane[id]++;
      }
      if (call + 1 > maxc) maxc = call + 1;
    }
    wave_calls += maxc;
    for (int c = 0; c < maxc; c++)
      for (int p = 0; p < 9; p++) wave[p] += seen[c][p];
  }
  const double nw = (double)blocks / 64;
  printf("polynomial %d^%d maxbits %u: plane calls per wave %.2f\n", n, dims, maxbits, wave_calls / nw);
  for (int p = 0; p < 9; p++)
    printf("  %d %-18s lane-steps per block %6.3f   wave-steps per wave %6.3f\n", p, nm[p], lane[p] / (double)blocks,
           wave[p] / nw);
  printf("rare lane-steps per block: code past two chunks %.4f, reaching position N-1 %.4f, neither %.4f\n",
         g_reason[6] / (double)blocks, g_reason[7] / (double)blocks, g_reason[8] / (double)blocks);
  printf("table step outcomes per block: ok %.3f  implied+cut %.4f  implied %.4f  cut P>q %.4f  open %.4f  other %.4f\n",
         g_reason[0] / (double)blocks, g_reason[1] / (double)blocks, g_reason[2] / (double)blocks,
         g_reason[3] / (double)blocks, g_reason[4] / (double)blocks, g_reason[5] / (double)blocks);
}
