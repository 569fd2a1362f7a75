// cuzfp_amd/csrc/split3.hpp -- the 3D fixed-rate encoder with every block
// split over a lane pair.
//
// Why: at 256^3 the one-block-per-lane encoder (kernels.hpp zfp_encode) is one
// resident round of 4 waves a SIMD (108 VGPRs).  The input arrives over ~11 us
// in wave-age order, and a SIMD's last wave can only start its whole block
// codec (~2,700 VALU) when its data lands, largely alone at the end.  Here a
// block is coded by lanes l (half A) and l + 32 (half B) of a wave: each lane
// holds 32 of the 64 values, so a wave is 32 blocks, half the work and <= 64
// VGPRs -- 8 waves a SIMD, one resident round of twice as many half-size waves.
//
// Per block (reference: zfp 0.5.0 encode.c / encode3.c, as zfp_block.hpp):
//   gather       A: z = 0, 1 rows; B: z = 2, 3 (register zl*16 + y*4 + x)
//   exponent     half maxima, combined across the pair
//   quantise, x and y lifts (encode3.c:303-320) on each half
//   z exchange   16 v_permlane32_swap: A takes the columns K, B their partners
//                PI(K), every z of them; then the z lifts
//   movers       7 swaps: A ends with perm[0..31] (the low 32 bits of every
//                bit plane, codec3.c:3-88), B with perm[32..63]
//   transpose    each lane's 32 coefficients into 32 half plane words
//                (transposition input t pairs perm[t] on A with perm[32+t] on B;
//                one select where they sit in different registers)
//   plane split  16 swaps: A holds whole planes 31..16, B planes 15..0
//   coder        A codes its planes from bit 9 (after the exponent); B codes its
//                planes into a scratch column from bit 0, starting from n =
//                bitlen(OR of planes 31..16) -- the n the reference has after
//                plane 16 (encode.c:121-151: n only grows, to the top one of
//                each plane, capped at N-1 here) -- while the budget lasts
//   merge        B ORs its bits into A's column at A's end position; bits past
//                maxbits land in the slack row (the reference stops there)
// The layout tables are searched by tools/split3_plan.py (fewest selects).
#pragma once
#include "zfp_block.hpp"

namespace cuzfp {
namespace split3 {

// z exchange: register (zl, K[i]) <-> (zl, PI[i]) for zl = 0, 1
constexpr int K[8] = {0, 1, 2, 3, 4, 5, 8, 9};
constexpr int PI[8] = {10, 12, 14, 6, 15, 11, 13, 7};
// mover swaps: v_permlane32_swap(vdst = q[SWAP[s][0]], vsrc = q[SWAP[s][1]])
constexpr int kMovers = 7;
constexpr int SWAP[kMovers][2] = {{1, 6}, {19, 7}, {3, 22}, {9, 23}, {17, 27}, {0, 29}, {8, 30}};

// Coefficient index (x + 4y + 16z) each half holds in each register, after the
// z exchange and after the mover swaps; the transposition's sources.
struct Layout {
  int a[32], b[32];       // after the movers
  int srcA[32], srcB[32]; // register of perm[t] on A / of perm[32+t] on B
  bool ok;
};
constexpr Layout make_layout() {
  Layout L{};
  int inv[16] = {};
  for (int i = 0; i < 8; i++) inv[PI[i]] = K[i] + 1;
  for (int zl = 0; zl < 2; zl++)
    for (int cc = 0; cc < 16; cc++) {
      const int r = zl * 16 + cc;
      bool inK = false;
      int p = 0;
      for (int i = 0; i < 8; i++)
        if (K[i] == cc) inK = true, p = PI[i];
      if (inK) {
        L.a[r] = cc + 16 * zl;        // A's own column, its z
        L.b[r] = p + 16 * zl;         // from A: column PI(cc), A's z
      } else {
        L.a[r] = (inv[cc] - 1) + 16 * (2 + zl);  // from B: column K, B's z
        L.b[r] = cc + 16 * (2 + zl);            // B's own
      }
    }
  for (int s = 0; s < kMovers; s++) {  // vdst = (a0, a1), vsrc = (b0, b1)
    const int v0 = SWAP[s][0], v1 = SWAP[s][1];
    const int a0 = L.a[v0], b0 = L.b[v0], a1 = L.a[v1], b1 = L.b[v1];
    L.a[v0] = a0, L.b[v0] = a1, L.a[v1] = b0, L.b[v1] = b1;
  }
  L.ok = true;
  for (int t = 0; t < 32; t++) {
    const int pa = perm<3>::at(t), pb = perm<3>::at(32 + t);
    int ra = -1, rb = -1;
    for (int r = 0; r < 32; r++) {
      if (L.a[r] == pa) ra = r;
      if (L.b[r] == pb) rb = r;
    }
    L.ok = L.ok && ra >= 0 && rb >= 0;
    L.srcA[t] = ra, L.srcB[t] = rb;
  }
  return L;
}
constexpr Layout kLayout = make_layout();
static_assert(kLayout.ok, "split3: every coefficient of the perm halves must sit on its lane");

// x and y lifts of a half block, register zl*16 + y*4 + x (encode3.c:303-320:
// x for all rows, then y for all columns; z after the exchange)
template <typename UInt>
ZFP_HD void lift_xy(UInt* q) {
#pragma unroll
  for (int r = 0; r < 8; r++) fwd_lift(q[4 * r], q[4 * r + 1], q[4 * r + 2], q[4 * r + 3]);
#pragma unroll
  for (int zl = 0; zl < 2; zl++)
#pragma unroll
    for (int x = 0; x < 4; x++) {
      UInt* p = q + 16 * zl + x;
      fwd_lift(p[0], p[4], p[8], p[12]);
    }
}

// z lifts after the exchange: column K[i] (A) / PI[i] (B) is (z0, z1, z2, z3) =
// registers (K[i], 16 + K[i], PI[i], 16 + PI[i])
template <typename UInt>
ZFP_HD void lift_z(UInt* q) {
#pragma unroll
  for (int i = 0; i < 8; i++) fwd_lift(q[K[i]], q[16 + K[i]], q[PI[i]], q[16 + PI[i]]);
}

// ---------------------------------------------------------------------------
// Device side
#if defined(__HIPCC__)

// v_permlane32_swap: vdst's upper 32 lanes <-> vsrc's lower 32 lanes, i.e. with
// v0 = (a0 | b0) and v1 = (a1 | b1) by half: v0 = (a0 | a1), v1 = (b0 | b1)
__device__ __forceinline__ void xswap(uint32_t& v0, uint32_t& v1) {
  const auto r = __builtin_amdgcn_permlane32_swap(v0, v1, false, false);
  v0 = r[0];
  v1 = r[1];
}
// both halves' values of v on every lane: A's in .x, B's in .y
__device__ __forceinline__ uint2 xboth(uint32_t v) {
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return uint2{r[0], r[1]};
}

#endif  // __HIPCC__

}  // namespace split3
}  // namespace cuzfp
