// tests/native/divmagic.cpp -- host check of the launch's block-index division
// (cuzfp::set_divisor in cuzfp_amd/csrc/launch.hpp): (n * m) >> s == n / d for
// n < 2^31, every divisor 1..5000, powers of two and their neighbours, and
// random 32-bit divisors.  Prints the number of mismatches.
#include <cstdio>
#include <random>
#include "../../cuzfp_amd/csrc/launch.hpp"

int main() {
  std::mt19937_64 rng(7);
  long bad = 0;
  auto chk = [&](uint32_t d, uint32_t n) {
    uint32_t m, s;
    cuzfp::set_divisor(d, m, s);
    if ((uint32_t)(((uint64_t)n * m) >> s) != n / d) bad++;
  };
  for (uint32_t d = 1; d <= 5000; d++) {
    for (int k = 0; k < 500; k++) chk(d, (uint32_t)rng() & 0x7fffffffu);
    for (uint32_t n = 0x7fffffffu - 500; n < 0x80000000u; n++) chk(d, n);
    for (uint32_t n = 0; n < 500; n++) chk(d, n);
  }
  for (uint32_t e = 1; e < 32; e++) {
    const uint32_t p = 1u << e;
    for (uint32_t d : {p - 1, p, p + 1})
      for (int k = 0; k < 2000; k++) chk(d, (uint32_t)rng() & 0x7fffffffu), chk(d, 0x7fffffffu - (uint32_t)k);
  }
  for (int k = 0; k < 2000000; k++) chk(1u + (uint32_t)(rng() % 0xffffffffull), (uint32_t)rng() & 0x7fffffffu);
  printf("%ld\n", bad);
  return bad != 0;
}
