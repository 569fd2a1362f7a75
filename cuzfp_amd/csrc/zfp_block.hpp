// cuzfp_amd/csrc/zfp_block.hpp -- per-block zfp fixed-rate codec, one block per lane.
//
// This header is the arithmetic of the MI355X codec: everything a single lane
// does to turn one 4^d block of scalars into `maxbits` stream bits and back.
// The HIP kernels (kernels.hpp) wrap it with coalesced HBM gathers and an
// LDS-staged bitstream; tests/emulate.cpp runs the very same functions on the
// host so the per-lane algorithm is checked against the CPU oracle without a GPU.
//
// Layout of one lane's work (reference: zfp 0.5.0, the ground truth of cuZFP's
// differential harness src/utils/test.py:68-93; paths below are relative to
// src/thirdparty_builtin/zfp-0.5.0/src):
//
//   emax  = exponent of max |x|              template/encode.c:9-33
//   q[i]  = (Int)(2^(p-2-emax) * x[i])       encode.c:35-52  (p = 32 / 64)
//   fwd_xform: lifting along x, y, z         encode.c:76-103, encode3.c:303-320
//   u[i]  = negabinary(q[perm[i]])           encode.c:105-119, codec3.c:3-88
//   planes = bit-matrix transpose of u        (replaces the per-plane gather
//                                              loop of encode.c:136-138)
//   embedded plane coder, budget-truncated   encode.c:121-151
//
// What is different from the reference GPU code (src/cuZFP/encode3.cuh): there a
// 64-thread CTA cooperates on one block and thread 0 serially concatenates the
// planes (encode3.cuh:336-362); here one lane owns the block end to end, so
// there are no barriers, no atomics on shared words and no idle threads, and
// the bit-plane transpose costs ~8 VALU ops per value instead of 64.
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define ZFP_HD __host__ __device__ __forceinline__
#else
#define ZFP_HD inline
#endif

// Diagnostic phase stamps (tools/probe.py, CUZFP_PROBE == 9 builds only).
#ifndef ZFP_STAMP
#define ZFP_STAMP(i)
#endif
#ifndef ZFP_COUNT_PLANE  // host-side path statistics (tools/path_stats.cpp)
#define ZFP_COUNT_PLANE(g0, fast, complete)
#endif
#ifndef ZFP_COUNT_PATH  // host-side decoder path statistics (tools/path_stats.cpp)
#define ZFP_COUNT_PATH(id)
#endif

namespace cuzfp {

// ---------------------------------------------------------------------------
// Scalar traits (zfp-0.5.0/src/traitsf.h, traitsd.h; cuZFP type_info.cuh:6-58)

template <typename T> struct traits;
template <> struct traits<float> {
  typedef int32_t Int; typedef uint32_t UInt;
  static constexpr bool is_int = false;
  static constexpr int prec = 32, ebits = 8, ebias = 127;
};
template <> struct traits<double> {
  typedef int64_t Int; typedef uint64_t UInt;
  static constexpr bool is_int = false;
  static constexpr int prec = 64, ebits = 11, ebias = 1023;
};
template <> struct traits<int32_t> {
  typedef int32_t Int; typedef uint32_t UInt;
  static constexpr bool is_int = true;
  static constexpr int prec = 32, ebits = 0, ebias = 0;
};
template <> struct traits<int64_t> {
  typedef int64_t Int; typedef uint64_t UInt;
  static constexpr bool is_int = true;
  static constexpr int prec = 64, ebits = 0, ebias = 0;
};

template <typename UInt> struct nbmask;
template <> struct nbmask<uint32_t> { static constexpr uint32_t value = 0xaaaaaaaau; };
template <> struct nbmask<uint64_t> { static constexpr uint64_t value = 0xaaaaaaaaaaaaaaaaull; };

ZFP_HD uint64_t lowmask(unsigned n) { return n >= 64 ? ~0ull : ((1ull << n) - 1); }

// the raw dwords of a reader's 64-bit window (LDS readers: issued, not yet
// combined; register readers: unused)
struct WRaw {
  uint32_t a0, a1, a2;
};

// The scheduler may not move instructions across this point (device builds):
// keeps the fast step's LDS reads issued in order and its uses of them after
// the one wait that covers them all.
ZFP_HD void sched_fence() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_sched_barrier(0);
#endif
}

// x, opaque to the optimizer (an empty asm: no instruction, no hazard
// padding).  Stops instruction selection from seeing through a mask -- e.g.
// turning a v_bfi_b32 with a sign-splat mask into a compare and a VCC
// v_cndmask_b32 (a ~17-cycle issue), or dropping a v_bfi_b32's mask it can
// prove redundant in favour of two instructions.
ZFP_HD uint32_t launder(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(x));
#endif
  return x;
}
// a wave-uniform constant the compiler keeps in one SGPR instead of
// re-materialising it (s_movk) wherever it is used
ZFP_HD uint32_t uniform_const(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+s"(x));
#endif
  return x;
}
ZFP_HD uint64_t uniform_const64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+s"(x));
#endif
  return x;
}
ZFP_HD uint64_t launder(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(x));
#endif
  return x;
}

ZFP_HD unsigned ctz64(uint64_t x) { return (unsigned)__builtin_ctzll(x); }  // x != 0

ZFP_HD unsigned umin(unsigned a, unsigned b) { return a < b ? a : b; }

// ---------------------------------------------------------------------------
// Coefficient order (zfp-0.5.0/src/template/codec{1,2,3}.c; the same tables
// cuZFP uploads to __constant__ memory, constants.h:8-131).  Indices are used
// only with compile-time positions, so after unrolling a permutation is pure
// register renaming.

template <int DIMS> struct perm;
template <> struct perm<1> {
  ZFP_HD static constexpr int at(int i) { return i; }
};
template <> struct perm<2> {
  ZFP_HD static constexpr int at(int i) {
    // (i,j) ordered by i+j, then i^2+j^2 (codec2.c:3-27)
    return i == 0 ? 0 : i == 1 ? 1 : i == 2 ? 4 : i == 3 ? 5 : i == 4 ? 2 : i == 5 ? 8 :
           i == 6 ? 6 : i == 7 ? 9 : i == 8 ? 3 : i == 9 ? 12 : i == 10 ? 10 : i == 11 ? 7 :
           i == 12 ? 13 : i == 13 ? 11 : i == 14 ? 14 : 15;
  }
};
#define ZFP_I3(i, j, k) ((i) + 4 * ((j) + 4 * (k)))
template <> struct perm<3> {
  ZFP_HD static constexpr int at(int i) {
    // (i,j,k) ordered by i+j+k, then i^2+j^2+k^2 (codec3.c:3-88)
    constexpr int t[64] = {
      ZFP_I3(0,0,0),
      ZFP_I3(1,0,0), ZFP_I3(0,1,0), ZFP_I3(0,0,1),
      ZFP_I3(0,1,1), ZFP_I3(1,0,1), ZFP_I3(1,1,0),
      ZFP_I3(2,0,0), ZFP_I3(0,2,0), ZFP_I3(0,0,2),
      ZFP_I3(1,1,1),
      ZFP_I3(2,1,0), ZFP_I3(2,0,1), ZFP_I3(0,2,1), ZFP_I3(1,2,0), ZFP_I3(1,0,2), ZFP_I3(0,1,2),
      ZFP_I3(3,0,0), ZFP_I3(0,3,0), ZFP_I3(0,0,3),
      ZFP_I3(2,1,1), ZFP_I3(1,2,1), ZFP_I3(1,1,2),
      ZFP_I3(0,2,2), ZFP_I3(2,0,2), ZFP_I3(2,2,0),
      ZFP_I3(3,1,0), ZFP_I3(3,0,1), ZFP_I3(0,3,1), ZFP_I3(1,3,0), ZFP_I3(1,0,3), ZFP_I3(0,1,3),
      ZFP_I3(1,2,2), ZFP_I3(2,1,2), ZFP_I3(2,2,1),
      ZFP_I3(3,1,1), ZFP_I3(1,3,1), ZFP_I3(1,1,3),
      ZFP_I3(3,2,0), ZFP_I3(3,0,2), ZFP_I3(0,3,2), ZFP_I3(2,3,0), ZFP_I3(2,0,3), ZFP_I3(0,2,3),
      ZFP_I3(2,2,2),
      ZFP_I3(3,2,1), ZFP_I3(3,1,2), ZFP_I3(1,3,2), ZFP_I3(2,3,1), ZFP_I3(2,1,3), ZFP_I3(1,2,3),
      ZFP_I3(0,3,3), ZFP_I3(3,0,3), ZFP_I3(3,3,0),
      ZFP_I3(3,2,2), ZFP_I3(2,3,2), ZFP_I3(2,2,3),
      ZFP_I3(1,3,3), ZFP_I3(3,1,3), ZFP_I3(3,3,1),
      ZFP_I3(2,3,3), ZFP_I3(3,2,3), ZFP_I3(3,3,2),
      ZFP_I3(3,3,3)};
    return t[i];
  }
};
#undef ZFP_I3

// Permutation with the table index as a template constant (no runtime-indexed
// register array, hence no scratch): u[i] = negabinary(q[perm[i]]) and back.
template <int... I> struct seq {};
template <int N, int... I> struct seq_gen : seq_gen<N - 1, N - 1, I...> {};
template <int... I> struct seq_gen<0, I...> { typedef seq<I...> type; };
template <int N> using make_seq = typename seq_gen<N>::type;
template <int DIMS, int I> struct pidx { static constexpr int value = perm<DIMS>::at(I); };

// (q + nb) ^ nb in coefficient order, without the final "^ nb": the encoder
// applies that after the bit-plane transpose, where it inverts the odd planes
// for free (planes::load<true>)
template <int DIMS, typename UInt, int... I>
ZFP_HD void permute_fwd_add(const UInt* q, UInt* u, UInt nb, seq<I...>) {
  ((u[I] = q[pidx<DIMS, I>::value] + nb), ...);
}
// (u ^ nb) - nb: one v_xad_u32 ((a ^ b) + c) for 32-bit words on the device
ZFP_HD uint32_t from_negabinary(uint32_t u, uint32_t nb) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(u), "s"(nb), "v"(0u - nb));  // one SGPR per VOP3
  return r;
#else
  return (u ^ nb) - nb;
#endif
}
ZFP_HD uint64_t from_negabinary(uint64_t u, uint64_t nb) { return (u ^ nb) - nb; }

template <int DIMS, typename UInt, int... I>
ZFP_HD void permute_inv(const UInt* u, UInt* q, UInt nb, seq<I...>) {
  ((q[pidx<DIMS, I>::value] = from_negabinary(u[I], nb)), ...);
}
// the coefficients already finished (planes::store_hi<true>)
template <int DIMS, typename UInt, int... I>
ZFP_HD void permute_inv_copy(const UInt* u, UInt* q, seq<I...>) {
  ((q[pidx<DIMS, I>::value] = u[I]), ...);
}
// the same for u already XOR-ed with nb (planes::store<true>): one subtraction
template <int DIMS, typename UInt, int... I>
ZFP_HD void permute_inv_sub(const UInt* u, UInt* q, UInt nb, seq<I...>) {
  ((q[pidx<DIMS, I>::value] = u[I] - nb), ...);
}

// precision() (codec1.c:8-11, codec2.c:131-136, codec3.c:92-97): planes coded
// for a block with exponent emax in fixed-rate mode (maxprec = type precision,
// minexp = ZFP_MIN_EXP = -1074).
template <int DIMS>
ZFP_HD unsigned precision(int emax, int prec) {
  int p = emax + 1074 + 2 * (DIMS + 1);
  p = p < 0 ? 0 : p;
  return (unsigned)(p < prec ? p : prec);
}

// ---------------------------------------------------------------------------
// Lifting transform (encode.c:76-103 / decode.c:243-270) on the unsigned type,
// so the reference's wrap-around (x86 int arithmetic) is well defined here.

ZFP_HD uint32_t asr1(uint32_t v) { return (uint32_t)((int32_t)v >> 1); }
ZFP_HD uint64_t asr1(uint64_t v) { return (uint64_t)((int64_t)v >> 1); }

template <typename UInt>
ZFP_HD void fwd_lift(UInt& x, UInt& y, UInt& z, UInt& w) {
  x += w; x = asr1(x); w -= x;
  z += y; z = asr1(z); y -= z;
  x += z; x = asr1(x); z -= x;
  w += y; w = asr1(w); y -= w;
  w += asr1(y); y -= asr1(w);
}

// decode.c:243-270.  Each "a += b; b <<= 1; b -= a" step is written in its
// two-operation form b' = b - a, a' = a + b (2b - (a + b) = b - a in modular
// arithmetic), which the compiler does not find by itself.
template <typename UInt>
ZFP_HD void inv_lift(UInt& x, UInt& y, UInt& z, UInt& w) {
  UInt t;
  y += asr1(w); w -= asr1(y);
  t = w - y; y += w; w = t;
  t = x - z; z += x; x = t;
  t = z - y; y += z; z = t;
  t = x - w; w += x; x = t;
}

template <int DIMS, typename UInt>
ZFP_HD void fwd_xform(UInt* p) {
  if constexpr (DIMS == 1) {
    fwd_lift(p[0], p[1], p[2], p[3]);
  } else if constexpr (DIMS == 2) {
#pragma unroll
    for (int y = 0; y < 4; y++) fwd_lift(p[4 * y], p[4 * y + 1], p[4 * y + 2], p[4 * y + 3]);
#pragma unroll
    for (int x = 0; x < 4; x++) fwd_lift(p[x], p[x + 4], p[x + 8], p[x + 12]);
  } else {
#pragma unroll
    for (int zy = 0; zy < 16; zy++) fwd_lift(p[4 * zy], p[4 * zy + 1], p[4 * zy + 2], p[4 * zy + 3]);
#pragma unroll
    for (int z = 0; z < 4; z++)
#pragma unroll
      for (int x = 0; x < 4; x++) {
        UInt* q = p + 16 * z + x;
        fwd_lift(q[0], q[4], q[8], q[12]);
      }
#pragma unroll
    for (int yx = 0; yx < 16; yx++) fwd_lift(p[yx], p[yx + 16], p[yx + 32], p[yx + 48]);
  }
}

template <int DIMS, typename UInt>
ZFP_HD void inv_xform(UInt* p) {
  if constexpr (DIMS == 1) {
    inv_lift(p[0], p[1], p[2], p[3]);
  } else if constexpr (DIMS == 2) {
#pragma unroll
    for (int x = 0; x < 4; x++) inv_lift(p[x], p[x + 4], p[x + 8], p[x + 12]);
#pragma unroll
    for (int y = 0; y < 4; y++) inv_lift(p[4 * y], p[4 * y + 1], p[4 * y + 2], p[4 * y + 3]);
  } else {
#pragma unroll
    for (int yx = 0; yx < 16; yx++) inv_lift(p[yx], p[yx + 16], p[yx + 32], p[yx + 48]);
#pragma unroll
    for (int z = 0; z < 4; z++)
#pragma unroll
      for (int x = 0; x < 4; x++) {
        UInt* q = p + 16 * z + x;
        inv_lift(q[0], q[4], q[8], q[12]);
      }
#pragma unroll
    for (int zy = 0; zy < 16; zy++) inv_lift(p[4 * zy], p[4 * zy + 1], p[4 * zy + 2], p[4 * zy + 3]);
  }
}

// ---------------------------------------------------------------------------
// Bit-plane transpose.  R rows of 32-bit words are cut into 32/R square R x R
// tiles side by side; each tile is transposed in place by log2(R) butterfly
// stages of bit-field inserts.  Afterwards word j holds, in bits [R*s, R*s+R),
// column R*s + j of the input, i.e. plane (R*s + j) of R coefficients.  The
// operation is an involution, so the decoder uses it unchanged.

// (a & m) | (b & ~m), m in a VGPR
ZFP_HD uint32_t bfi_v(uint32_t m, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
#else
  return (a & m) | (b & ~m);
#endif
}

// (a & m) | (b & ~m), m a wave-uniform constant (SGPR)
ZFP_HD uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(m), "v"(a), "v"(b));
  return r;
#else
  return (a & m) | (b & ~m);
#endif
}

// ~((a & m) | (b & ~m)) in one v_bitop3_b32 (truth table 0x35: not of v_bfi's 0xca)
ZFP_HD uint32_t nbfi(uint32_t m, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x35" : "=v"(r) : "s"(m), "v"(a), "v"(b));
  return r;
#else
  return ~((a & m) | (b & ~m));
#endif
}

// (a & m) | (~b & ~m) in one v_bitop3_b32 (truth table 0xc5: v_bfi's 0xca with b
// inverted)
ZFP_HD uint32_t bfi_notb(uint32_t m, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xc5" : "=v"(r) : "s"(m), "v"(a), "v"(b));
  return r;
#else
  return (a & m) | (~b & ~m);
#endif
}

// bytes of {a = bytes 0-3, b = bytes 4-7} picked by sel (v_perm_b32)
ZFP_HD uint32_t perm_bytes(uint32_t b, uint32_t a, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(b, a, sel);
#else
  const uint64_t v = (uint64_t)a | ((uint64_t)b << 32);
  uint32_t r = 0;
  for (int i = 0; i < 4; i++) r |= (uint32_t)((v >> (8 * ((sel >> (8 * i)) & 7))) & 0xff) << (8 * i);
  return r;
#endif
}

// Output inversion folded into the last stage (J = 1) of a transpose:
//   kOddWords: the odd output words come out inverted (encoder: the odd planes),
//   kOddBits:  the odd bit positions of every output word come out inverted
//              (decoder: the odd planes again, now as bits of coefficients).
// Either is the "^ 0xaaaa..." of the negabinary conversion, at no cost.
enum { kInvNone = 0, kOddWords = 1, kOddBits = 2 };

// Two words shifted by one 64-bit instruction (bit-granular stages): the bits
// one word's shift moves into the other lie where the stage's mask drops them
// -- ~m has its low J bits clear (the left shifts' spill), m its top J bits
// (the right shifts') -- so a pair of 32-bit shifts becomes one v_lshlrev_b64 /
// v_lshrrev_b64 on the two words as a register pair.
// (The shift count goes in as an SGPR the optimizer cannot see through: a
// 64-bit shift by a known constant is split by the compiler into 32-bit shifts
// and a funnel shift, and an inline-asm shift makes the hazard recognizer pad
// each consumer with an s_nop.)
template <int J>
ZFP_HD uint32_t opaque_shift() {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t s;
  asm("s_mov_b32 %0, %1" : "=s"(s) : "i"(J));
  return s;
#else
  return J;
#endif
}
template <int J>
ZFP_HD void shl2(uint32_t& x, uint32_t& y, uint32_t sj) {
  const uint64_t r = ((uint64_t)x | ((uint64_t)y << 32)) << sj;
  x = (uint32_t)r;
  y = (uint32_t)(r >> 32);
}
template <int J>
ZFP_HD void shr2(uint32_t& x, uint32_t& y, uint32_t sj) {
  const uint64_t r = ((uint64_t)x | ((uint64_t)y << 32)) >> sj;
  x = (uint32_t)r;
  y = (uint32_t)(r >> 32);
}

template <int J, int INV = kInvNone>
ZFP_HD void transpose_stage(uint32_t* a, int rows, int r0 = 0) {  // rows r0 .. rows-1 (J < 16: a closed set)
  // swap the J x J off-diagonal sub-blocks of every 2J x 2J tile:
  //   lo' = (lo & m) | ((hi << J) & ~m),  hi' = ((lo >> J) & m) | (hi & ~m)
  // one v_perm_b32 per word for the byte-granular stages; the bit-granular
  // ones take two pairs (i, i + J), (i2, i2 + J) at a time, their shifts as
  // one 64-bit shift of the two hi words and one of the two lo words, then a
  // v_bfi_b32 per output word: 3 instructions a pair instead of 4
  constexpr uint32_t m = J == 16 ? 0x0000ffffu : J == 8 ? 0x00ff00ffu : J == 4 ? 0x0f0f0f0fu
                       : J == 2 ? 0x33333333u : 0x55555555u;
  if constexpr (J <= 4) {
    // the partner pair: i + 1 for J >= 2 (adjacent words), i + 2 for J = 1
    constexpr int D = J == 1 ? 2 : 1;
    const uint32_t sj = opaque_shift<J>();
#pragma unroll
    for (int i = 0; i < 32; i++) {
      if (i < r0 || i >= rows || (i & J) || (i & D)) continue;
      const int i2 = i + D;
      uint32_t h1 = a[i + J], h2 = a[i2 + J], l1 = a[i], l2 = a[i2];
      const uint32_t H1 = h1, H2 = h2;  // hi words as they were
      shl2<J>(h1, h2, sj);              // hi << J
      shr2<J>(l1, l2, sj);              // lo >> J
      if constexpr (INV == kOddBits) {  // J = 1, m = 0x5555...: the odd bits come from hi
        a[i] = bfi_notb(m, a[i], h1);
        a[i2] = bfi_notb(m, a[i2], h2);
        a[i + J] = bfi_notb(m, l1, H1);
        a[i2 + J] = bfi_notb(m, l2, H2);
      } else {
        a[i] = bfi(m, a[i], h1);
        a[i2] = bfi(m, a[i2], h2);
        a[i + J] = INV == kOddWords ? nbfi(m, l1, H1) : bfi(m, l1, H1);
        a[i2 + J] = INV == kOddWords ? nbfi(m, l2, H2) : bfi(m, l2, H2);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 32; i++) {
    if (i < r0 || i >= rows || (i & J)) continue;
    const uint32_t lo = a[i], hi = a[i + J];
    if constexpr (J == 16) {
      a[i] = perm_bytes(hi, lo, 0x05040100u);
      a[i + J] = perm_bytes(hi, lo, 0x07060302u);
    } else if constexpr (J == 8) {
      a[i] = perm_bytes(hi, lo, 0x06020400u);
      a[i + J] = perm_bytes(hi, lo, 0x07030501u);
    } else {
      if constexpr (INV == kOddBits) {  // J = 1, m = 0x5555...: the odd bits come from hi
        a[i] = bfi_notb(m, lo, hi << J);
        a[i + J] = bfi_notb(m, lo >> J, hi);
      } else {
        a[i] = bfi(m, lo, hi << J);
        a[i + J] = INV == kOddWords ? nbfi(m, lo >> J, hi) : bfi(m, lo >> J, hi);
      }
    }
  }
}

// INV: kOddWords inverts the odd output words, i.e. (R even) the odd planes;
// kOddBits the odd bits of every output word -- the "^ 0xaaaa..." of the
// negabinary conversion, applied to planes (encoder) or coefficients (decoder)
template <int R, int INV = kInvNone>
ZFP_HD void transpose_tiles(uint32_t* a) {
  // stages J = R/2, ..., 1 spelled out so every index is a compile-time constant
  if constexpr (R >= 32) transpose_stage<16>(a, R);
  if constexpr (R >= 16) transpose_stage<8>(a, R);
  if constexpr (R >= 8) transpose_stage<4>(a, R);
  if constexpr (R >= 4) transpose_stage<2>(a, R);
  if constexpr (R >= 2) transpose_stage<1, INV>(a, R);
}

// Storage of the plane words.  64-bit coefficients keep them as clang
// ext_vector_type values (one R-register tuple per row group), which the
// rolled plane loops index with a runtime, wave-uniform plane number:
// VGPR-relative addressing (s_set_gpr_idx_on + v_mov), one copy of the loop
// body in the instruction cache.  (A runtime index into a plain array, or
// into a vector wider than 32 registers, would be lowered to scratch memory.
// Unrolled with plain registers, the f64 kernels still need ~190-200 VGPRs --
// two waves a SIMD, as rolled -- and the unit takes 14 minutes to compile.)
// 32-bit coefficients are always coded down to plane 0 (precision() is 32 for
// every f32 exponent and for int32), so their plane loops are unrolled with
// compile-time plane numbers and the words are plain registers: no tuple the
// register allocator must keep contiguous.
template <int H, int G, int R, bool VEC> struct plane_words;
template <int H, int G, int R> struct plane_words<H, G, R, false> {
  uint32_t a[H][G][R];
  ZFP_HD uint32_t get(int h, int g, int r) const { return a[h][g][r]; }
  ZFP_HD void set(int h, int g, int r, uint32_t x) { a[h][g][r] = x; }
  ZFP_HD void zero() {
#pragma unroll
    for (int h = 0; h < H; h++)
#pragma unroll
      for (int g = 0; g < G; g++)
#pragma unroll
        for (int r = 0; r < R; r++) a[h][g][r] = 0u;
  }
};
template <int H, int G, int R> struct plane_words<H, G, R, true> {
  typedef uint32_t vec __attribute__((ext_vector_type(R)));
  vec v[H][G];
  ZFP_HD uint32_t get(int h, int g, int r) const { return v[h][g][r]; }
  ZFP_HD void set(int h, int g, int r, uint32_t x) { v[h][g][r] = x; }
  ZFP_HD void zero() {
#pragma unroll
    for (int h = 0; h < H; h++)
#pragma unroll
      for (int g = 0; g < G; g++) v[h][g] = (vec)0u;
  }
};

// Planes of N = 4^DIMS coefficients held as 32-bit words.  For 32-bit
// coefficients W = N words; 64-bit coefficients are split into low and high
// halves (planes 0..31 from the low words, 32..63 from the high words).
// Word (h, g, row) = word g*R + row of half h.
template <typename UInt, int DIMS> struct planes {
  static constexpr int N = 1 << (2 * DIMS);
  static constexpr int H = sizeof(UInt) / 4;      // 32-bit halves per value
  static constexpr int R = N < 32 ? N : 32;       // tile height
  static constexpr int G = N / R;                 // row groups (2 for 3D)
  plane_words<H, G, R, (H == 2)> w;

  // NEG_ODD: u holds q + 0xaaaa... and the planes get the negabinary's
  // final "^ 0xaaaa..." (the odd planes inverted) from the transpose
  template <bool NEG_ODD = false>
  ZFP_HD void load(const UInt* u) {
    uint32_t t[H][N];
#pragma unroll
    for (int i = 0; i < N; i++) {
      t[0][i] = (uint32_t)u[i];
      if (H == 2) t[H - 1][i] = (uint32_t)((uint64_t)u[i] >> 32);
    }
#pragma unroll
    for (int h = 0; h < H; h++)
#pragma unroll
      for (int g = 0; g < G; g++) transpose_tiles<R, NEG_ODD ? kOddWords : kInvNone>(&t[h][g * R]);
#pragma unroll
    for (int h = 0; h < H; h++)
#pragma unroll
      for (int g = 0; g < G; g++)
#pragma unroll
        for (int r = 0; r < R; r++) w.set(h, g, r, t[h][g * R + r]);
  }

  // NEG_ODD: the coefficients come out as u ^ 0xaaaa... (the first half of
  // the inverse negabinary conversion)
  template <bool NEG_ODD = false>
  ZFP_HD void store(UInt* u) const {
    uint32_t t[H][N];
#pragma unroll
    for (int h = 0; h < H; h++)
#pragma unroll
      for (int g = 0; g < G; g++)
#pragma unroll
        for (int r = 0; r < R; r++) t[h][g * R + r] = w.get(h, g, r);
#pragma unroll
    for (int h = 0; h < H; h++)
#pragma unroll
      for (int g = 0; g < G; g++) transpose_tiles<R, NEG_ODD ? kOddBits : kInvNone>(&t[h][g * R]);
#pragma unroll
    for (int i = 0; i < N; i++) {
      uint64_t x = t[0][i];
      if (H == 2) x |= (uint64_t)t[H - 1][i] << 32;
      u[i] = (UInt)x;
    }
  }

  ZFP_HD void zero() { w.zero(); }

  // 3D 64-bit blocks in three steps (round 6): BASELINE's 3D f64 rate 16
  // codes planes 63..~21, so the low half's planes 15..0 are rarely reached.
  //   load_split: the high half's tiles transposed (planes 63..32), the low
  //   half's through the J = 16 stage (it moves bits between the row halves;
  //   the stages commute, so it may go first);
  //   lo_part<UPPER>: the low half's J = 8..1 stages on rows 16..31 (planes
  //   31..16; their pairs stay within a 16-row half), lo_part<!UPPER> on rows
  //   0..15 (planes 15..0).
  // Together the same words as load(): 88 slow instructions a tile are left
  // out when no lane of the wave reaches plane 15.
  template <bool NEG_ODD = false>
  ZFP_HD void load_split(const UInt* u) {
    static_assert(H == 2 && N == 64, "3D 64-bit blocks");
    uint32_t t[H][N];
#pragma unroll
    for (int i = 0; i < N; i++) {
      t[0][i] = (uint32_t)u[i];
      t[1][i] = (uint32_t)((uint64_t)u[i] >> 32);
    }
#pragma unroll
    for (int g = 0; g < G; g++) {
      transpose_tiles<R, NEG_ODD ? kOddWords : kInvNone>(&t[1][g * R]);
      transpose_stage<16>(&t[0][g * R], R);
    }
#pragma unroll
    for (int h = 0; h < H; h++)
#pragma unroll
      for (int g = 0; g < G; g++)
#pragma unroll
        for (int r = 0; r < R; r++) w.set(h, g, r, t[h][g * R + r]);
  }
  template <bool NEG_ODD = false, bool UPPER = true>
  ZFP_HD void lo_part() {
    constexpr int INV = NEG_ODD ? kOddWords : kInvNone;
    constexpr int r0 = UPPER ? 16 : 0, r1 = UPPER ? 32 : 16;
#pragma unroll
    for (int g = 0; g < G; g++) {
      uint32_t t[R];
#pragma unroll
      for (int r = r0; r < r1; r++) t[r] = w.get(0, g, r);
      transpose_stage<8>(t, r1, r0);
      transpose_stage<4>(t, r1, r0);
      transpose_stage<2>(t, r1, r0);
      transpose_stage<1, INV>(t, r1, r0);
#pragma unroll
      for (int r = r0; r < r1; r++) w.set(0, g, r, t[r]);
    }
  }

  // 2D (16 coefficients of 32 bits), planes 16..31 only (round 6).  A 2D
  // block's word r holds plane r in its low half and plane r + 16 in its high
  // half, so the full transpose moves two 16 x 16 tiles at once; when only the
  // high tile matters -- the encoder's first planes, the decoder of a wave
  // whose lanes all stopped above plane 16 (BASELINE's 2D rate 2 stops above
  // plane 20) -- the high tile alone is one 16 x 16 bit transpose in 8 dwords:
  // dword k = row k | row k + 8 << 16, whose off-diagonal 8 x 8 blocks swap by
  // the same byte permute that packs the rows, then three butterfly stages of
  // 8 x 8 tiles.  8 v_perm_b32 and 36 stage instructions instead of 88.
  //   load_hi: plane 16 + k (k < 8) in the high half of word k, plane 24 + k
  //   in the high half of word k + 8 (get() of planes 16..31 reads these; the
  //   low halves hold other bits until load() fills the block for planes
  //   0..15).
  template <bool NEG_ODD = false>
  ZFP_HD void load_hi(const UInt* u) {
    static_assert(DIMS == 2 && H == 1, "2D 32-bit blocks");
    uint32_t d[8];
#pragma unroll
    for (int k = 0; k < 8; k++) d[k] = perm_bytes(u[k + 8], u[k], 0x07030602u);
    transpose_tiles<8, NEG_ODD ? kOddWords : kInvNone>(d);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      w.set(0, 0, k, d[k] << 16);
      w.set(0, 0, k + 8, d[k]);
    }
  }
  //   store_hi: the planes' low halves are zero (planes 0..15 unset); the
  //   coefficients come out finished, q = (u ^ NB) - NB for NEG_ODD (the odd
  //   bits inverted by the last stage, then the rest of the conversion on the
  //   16-bit halves: two fast instructions a coefficient).
  template <bool NEG_ODD = false>
  ZFP_HD void store_hi(UInt* q) const {
    static_assert(DIMS == 2 && H == 1, "2D 32-bit blocks");
    uint32_t d[8];
#pragma unroll
    for (int k = 0; k < 8; k++) d[k] = perm_bytes(w.get(0, 0, k + 8), w.get(0, 0, k), 0x07030602u);
    transpose_tiles<8, NEG_ODD ? kOddBits : kInvNone>(d);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if constexpr (NEG_ODD) {
        // u ^ NB = (d << 16) | 0xaaaa, so (u ^ NB) - NB = (d - 0xaaaa) << 16; the
        // high coefficient: (d & 0xffff0000) | 0xaaaa, less NB
        q[k] = (d[k] - 0xaaaau) << 16;
        q[k + 8] = (d[k] & 0xffff0000u) - 0xaaaa0000u;
      } else {
        q[k] = d[k] << 16;
        q[k + 8] = d[k] & 0xffff0000u;
      }
    }
  }

  // plane c (0..31) of half h as an N-bit word (bit i = that bit of
  // coefficient i); h is a compile-time constant, c may be a runtime value
  // (wave-uniform in the kernels) for 64-bit coefficients only.
  template <int h> ZFP_HD uint64_t get(int c) const {
    if constexpr (N == 64) return (uint64_t)w.get(h, 0, c) | ((uint64_t)w.get(h, 1, c) << 32);
    else return (w.get(h, 0, c % R) >> (R * (c / R))) & (uint32_t)lowmask(R);
  }
  ZFP_HD uint64_t get(int k) const {  // k compile-time after unrolling
    return (k >> 5) ? get<H - 1>(k & 31) : get<0>(k & 31);
  }
  // the word holding plane c of half h (1D/2D: with R planes a word)
  template <int h> ZFP_HD uint32_t word(int c) const { return w.get(h, 0, c % R); }

  // deposit plane c of half h (bits beyond N are zero; the plane was zero)
  template <int h> ZFP_HD void set(int c, uint64_t x) {
    if constexpr (N == 64) {
      w.set(h, 0, c, (uint32_t)x);
      w.set(h, 1, c, (uint32_t)(x >> 32));
    } else {
      w.set(h, 0, c % R, w.get(h, 0, c % R) | ((uint32_t)x << (R * (c / R))));
    }
  }
  ZFP_HD void set(int k, uint64_t x) {
    if (k >> 5) set<H - 1>(k & 31, x);
    else set<0>(k & 31, x);
  }
};

// ---------------------------------------------------------------------------
// Embedded plane coder with a bit budget (encode.c:121-151).  Per plane k,
// most significant first: the first n bits verbatim (coefficients already
// significant), then group tests: "1" + the bits up to and including the next
// one bit (the one at position N-1 is implied), until a "0" test or the end of
// the plane.

// Plane word type: 64 coefficients need 64 bits, 16 or 4 fit in 32.
template <int DIMS> struct plane_word { typedef uint32_t type; };
template <> struct plane_word<3> { typedef uint64_t type; };

ZFP_HD unsigned ctz(uint32_t x) { return (unsigned)__builtin_ctz(x); }  // x != 0
ZFP_HD unsigned ctz(uint64_t x) { return (unsigned)__builtin_ctzll(x); }

// count of trailing zeros of x; any value >= 64 when x == 0
ZFP_HD unsigned ctz64_or_64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  // v_ffbl_b32 returns ~0 for a zero word: min(lo, hi | 32) is the 64-bit
  // count (or ~0) in four instructions, without the compiler's zero checks
  unsigned lo, hi;
  asm("v_ffbl_b32 %0, %1" : "=v"(lo) : "v"((uint32_t)x));
  asm("v_ffbl_b32 %0, %1" : "=v"(hi) : "v"((uint32_t)(x >> 32)));
  hi |= 32u;
  return lo < hi ? lo : hi;
#else
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const unsigned zl = lo ? (unsigned)__builtin_ctz(lo) : 64u;
  const unsigned zh = hi ? 32u + (unsigned)__builtin_ctz(hi) : 64u;
  return zl < zh ? zl : zh;
#endif
}

// Plane loop, most significant plane first (encode.c:133-150).  The plane
// number is a runtime value but the same on every lane of the wave (lanes whose
// block is full drop out; the wave walks on while any lane has bits left), so
// P.get() is VGPR-relative addressing, not scratch.
// The plane number of a plane loop: the same on every active lane, so say so
// (the loops' exits are per lane, which makes the compiler treat the counter as
// divergent and wrap each indexed access in a readfirstlane loop).
ZFP_HD int uniform(int c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_readfirstlane(c);
#else
  return c;
#endif
}

// Plane-loop exit: the loops run while any lane of the wave still has budget,
// and a finished lane's steps are no-ops (the decoder's consume nothing and
// deposit zeros; the encoder's write into the lane's slack, see
// Writer::settle).  Exiting per lane instead costs ~15 exec-mask instructions
// a loop trip.  On the host a "wave" is one lane.
ZFP_HD bool any_lane(bool p) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(CUZFP_LANE_EXIT)
  return __builtin_amdgcn_ballot_w64(p) != 0;
#else
  return p;
#endif
}

// Wave priority from progress through the plane loop (c: the wave-uniform
// plane number, counting down): a wave that is further along yields issue
// slots to the other waves of its SIMD, so the SIMD's waves move through the
// coder together instead of oldest-first (which leaves the last wave running
// alone at the end, at a fraction of the SIMD's issue rate).
//
// The encoder drops to 2, 1, 0 at planes 17, 9, 1; its copy-out runs at 3
// again.  (Rounds 1-4: 21, 13, 5.  Round 5, after the decoder change below,
// four interleaved A/B rounds: 256^3 r8 step 47.2-47.7 -> 46.6-46.8 us on
// the polynomial field, the headline's, and 44.5-44.9 -> 44.7-45.0 on
// splitmix; 19/11/3 in between, profiles/r05_xvar_encoder_prio.txt.)  The decoder drops to 2 and 1 at planes 21 and 11, and a wave out of
// its plane loop takes priority 2 again for the inverse transform and the
// stores (CUZFP_DPRIO_AFTER).  Rounds 2-4 dropped it to 0 there, so that the
// transform filled the plane-looping waves' gaps; but a SIMD's four decode
// waves then ended at 13.2 / 15.4 / 18.0 / 20.6 us (profiles/r05_stamps.txt)
// and the 64 MiB of output left only behind them.  Finishing a wave that is
// out of the loop first starts its stores sooner: 256^3 r8 step 48.2-48.6 ->
// 47.2-47.4 us on the polynomial field, 44.8-44.9 -> 44.6 on splitmix (2 at
// 21/11; 3 measured 47.2-47.5 / 44.7-44.9, 3 with drops at 13/5 47.0-47.2 /
// 44.9-45.0; 2D, 1D and f64 unchanged: profiles/r05_prio.txt).
#ifndef CUZFP_PRIO_T2  // plane numbers (odd: the loops step by two) where the priority drops
#define CUZFP_PRIO_T2 17
#define CUZFP_PRIO_T1 9
#define CUZFP_PRIO_T0 1
#endif
#ifndef CUZFP_DPRIO_T2
#define CUZFP_DPRIO_T2 21
#define CUZFP_DPRIO_T1 11
#define CUZFP_DPRIO_T0 (-1)
#define CUZFP_DPRIO_AFTER 2
#endif
// The schedule pays off when the launch is one resident round of waves (256^3
// f32: 4 waves per SIMD, all resident at once).  Over several rounds it costs
// 12 % (1024^3: step 3.63 -> 3.19 ms without it; tools/variants.py): a wave
// that has lowered its priority is starved by freshly started waves, so the
// slots it holds free up late.  The launcher picks per launch (kernels.hpp,
// use_priority), and the coder reads the choice from its writer / reader type
// (kPrio; types without it keep the schedule).
template <typename T, typename = void> struct prio_of {
  static constexpr bool value = true;
};
template <typename T> struct prio_of<T, decltype((void)T::kPrio)> {
  static constexpr bool value = T::kPrio;
};

// Writers whose put() keeps only the low 32 bits of its value (kPut32: the
// register writer of a 32-bit block), and the exponent field's put (head(),
// where a writer has one)
// Writers that code a zero block inline (kZeroInline): the block is marked
// full (mark_full) and the coder runs on zero coefficients with the wave, its
// writes all landing in the lane's discarded slack -- so the coder is not
// nested in a per-lane branch (LdsOrWriter)
template <typename T, typename = void> struct zero_inline_of {
  static constexpr bool value = false;
};
template <typename T> struct zero_inline_of<T, decltype((void)T::kZeroInline)> {
  static constexpr bool value = T::kZeroInline;
};

template <typename T, typename = void> struct put32_of {
  static constexpr bool value = false;
};
template <typename T> struct put32_of<T, decltype((void)T::kPut32)> {
  static constexpr bool value = T::kPut32;
};
template <typename W>
ZFP_HD auto wr_head(W& wr, uint64_t v, unsigned n) -> decltype(wr.head(v, n)) {
  wr.head(v, n);
}
template <typename W, typename... Ignored>
ZFP_HD void wr_head(W& wr, uint64_t v, unsigned n, Ignored...) {
  wr.put(v, n);
}

template <int T2, int T1, int T0>
ZFP_HD void progress_priority(int c) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(CUZFP_NO_PRIO)
  // one bit test on the common path (a compare cascade costs ~20 SALU a trip)
  constexpr uint32_t kAt = (1u << T2) | (1u << T1) | (T0 >= 0 ? 1u << (T0 & 31) : 0u);
  if (__builtin_expect((kAt >> (c & 31)) & 1u, 0)) {
    if (c == T2) __builtin_amdgcn_s_setprio(2);
    else if (c == T1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  }
#else
  (void)c;
#endif
}

// Table-driven plane step (the common case).  The group code of the plane's
// not-yet-significant part r is "1", then for every position up to r's top
// one its bit, each one followed by a "1" group test -- i.e. r with every one
// doubled -- with the top one's test flipped to the closing "0" (or, when the
// top one sits at position N-1, that one and its test omitted: it is implied).
// The doubling is read from a 256-entry table per byte of r (Writer::spread),
// so a plane costs two table reads and no loop over its ones.  Returns false,
// writing nothing, when r has bits beyond its low 16 (a dense plane; the caller
// codes it with encode_plane).
constexpr uint32_t spread_entry(uint32_t b) {
  uint32_t e = 0, p = 0;
  for (int i = 0; i < 8; i++) {
    if ((b >> i) & 1u) {
      e |= 3u << p;
      p += 2;
    } else {
      p += 1;
    }
  }
  return e;
}
struct SpreadLut {
  uint32_t e[256];
};
constexpr SpreadLut make_spread_lut() {
  SpreadLut t{};
  for (uint32_t b = 0; b < 256; b++) t.e[b] = spread_entry(b);
  return t;
}

// The one-put coder's tables, one dword an entry: table 0 (r's low byte)
// entry b = (spread(b) << 1 | 1) << 5 | (popcount(b) + 8) -- the group code's
// leading "1" in place, and in the low 5 bits the shift that places the high
// byte's part; table 1 (r's high byte) entry b = spread(b) << 1.  The group
// code of r < 2^16 is then e1 << e0[4:0] | e0 >> 5: one v_lshl_or_b32 (whose
// shift count is the low 5 bits of its operand) and one shift.
struct SpreadTab {
  uint32_t e[512];
};
constexpr SpreadTab make_spread_tab() {
  SpreadTab t{};
  for (uint32_t b = 0; b < 256; b++) {
    uint32_t pop = 0;
    for (int i = 0; i < 8; i++) pop += (b >> i) & 1u;
    t.e[b] = (((spread_entry(b) << 1) | 1u) << 5) | (pop + 8u);
    t.e[256 + b] = spread_entry(b) << 1;
  }
  return t;
}

// bit length of x (0 for 0): 32 - clz(x), where v_ffbh_u32 gives ~0 for 0 and
// the saturating (clamp) subtraction turns 32 - ~0 into 0 -- one half-rate and
// one full-rate instruction, no zero test
ZFP_HD uint32_t bitlen16(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t e;
  asm("v_ffbh_u32 %0, %1\n\tv_sub_u32_e64 %0, 32, %0 clamp" : "=&v"(e) : "v"(x));
  return e;
#else
  return x ? 32u - (uint32_t)__builtin_clz(x) : 0u;
#endif
}

// v << s as one v_lshlrev_b64: the compiler otherwise turns x ^ ((x >> n) << n)
// into a mask with a zero-count guard (seven instructions)
ZFP_HD uint64_t shl64(uint64_t v, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t r;
  asm("v_lshlrev_b64 %0, %1, %2" : "=v"(r) : "v"(s), "v"(v));
  return r;
#else
  return v << (s & 63);
#endif
}

// byte I of v times 4: the byte offset of its entry in a table of dwords.
// Two full-rate instructions (shift by an immediate, AND with a literal); the
// compiler's SDWA form takes the shift count from a VGPR, which issues at half
// rate (tools/ubench/opcost.hip).
template <int I>
ZFP_HD uint32_t byte_off4(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  if constexpr (I == 0)
    asm("v_lshlrev_b32 %0, 2, %1\n\tv_and_b32 %0, 0x3fc, %0" : "=&v"(r) : "v"(v));
  else
    asm("v_lshrrev_b32 %0, %2, %1\n\tv_and_b32 %0, 0x3fc, %0" : "=&v"(r) : "v"(v), "i"(8 * I - 2));
  return r;
#else
  return ((v >> (8 * I)) & 0xffu) << 2;
#endif
}

// v_bfe_u32(v, 0, w): the low w bits of v, w = 0 .. 31
ZFP_HD uint32_t low_bits(uint32_t v, uint32_t w) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_ubfe(v, 0u, w);
#else
  return w ? v & (0xffffffffu >> (32 - (w & 31))) : 0u;
#endif
}

// One-put plane step (the common case).  The whole plane code -- n verbatim
// bits, then the group code -- goes out with one writer call when it fits 64
// bits.  With r = x >> n the code is x ^ ((r ^ g) << n), g = the group code:
// "1", then r with every one doubled (Writer::spread), cut before the top
// one's partner (the closing "0", which the zeroed image already holds), i.e.
// the low L = bitlen(r) + popcount(r) bits of (spread(r) << 1 | 1) -- or, when
// r's top one lands on position N-1 (imp: it is implied), the low L - 1 bits
// and no closing test.  No new ones: L = 0, g = 0 and the single "0" test.
// n is kept at most N-1: with n = N-1 the last position's code is its bit
// alone either way (a "1" test with the one implied, or a "0" test), so the
// plane codes are those of n = N, verbatim.  Requires width <= 31, which
// holds for r < 2^15 (3D: checked by the caller) and always in 1D/2D.
struct PlaneLen {  // the one-put step's lengths (plane_len)
  uint32_t nn, imp, width, len;
};
// nn = n + bitlen(r) <= N, imp = r's top one at N-1 (it is implied), width =
// the group code's bits after the leading "1" (L = bitlen + popcount, less the
// implied one), len = the whole plane code: n verbatim bits, "1", width bits,
// the closing "0" unless imp.  Computed once and shared by the fit test, the
// put and the next plane's n (the compiler does not merge 2*imp with imp).
template <int DIMS>
ZFP_HD PlaneLen plane_len(uint32_t nf, uint32_t bl, uint32_t L) {
  PlaneLen p;
  p.nn = nf + bl;
  p.imp = p.nn >> (2 * DIMS);
  p.width = L - p.imp;
  p.len = nf + p.width + 1u - p.imp;
  return p;
}

template <int DIMS, typename PW, typename Writer>
ZFP_HD void encode_plane_one_put(PW x, unsigned nf, uint64_t r, const PlaneLen& pl, unsigned& n, Writer& wr) {
  const uint32_t rl = (uint32_t)r;
  constexpr unsigned N = 1u << (2 * DIMS);
  const uint32_t width = pl.width;
  // "1" + r with every one doubled: one table entry a byte of r (3D: r < 2^15,
  // 2D: r < 2^16; where r's top bits move past bit 31 they lie past width)
  // both table reads, then one wait for both (the compiler would wait for
  // each before its first use: two s_waitcnt a plane)
  const uint32_t e0 = wr.sp0(byte_off4<0>(rl));
  const uint32_t e1 = N > 4 ? wr.sp1(byte_off4<1>(rl)) : 0u;
  sched_fence();
  wr.lds_wait();
  sched_fence();
  uint32_t G = e0 >> 5;
  if constexpr (N > 4) G |= e1 << (e0 & 31u);
  const uint32_t g = low_bits(G, width);
  if constexpr (N <= 16 && put32_of<Writer>::value) {
    // the writer keeps 32 bits of the code (a 32-bit block: the rest lies past
    // its end), and r < 2^16: 32-bit shifts
    wr.put((uint32_t)x ^ ((rl ^ g) << nf), pl.len);
  } else {
    // r < 2^32 here, so r ^ g is (r's high word, rl ^ g): the shift takes r's
    // register pair as it is instead of a zero-extended copy of rl ^ g
    const uint64_t code = (uint64_t)x ^ ((r ^ (uint64_t)g) << nf);
    wr.put(code, pl.len);
  }
  n = pl.nn - pl.imp;  // min(nn, N-1)
}

// r with every one doubled, for a 32-bit r: four byte lookups placed at
// 8 i + (ones below byte i); at most 64 bits
template <typename Writer>
ZFP_HD uint64_t spread32(uint32_t v, const Writer& wr) {
  const uint32_t b0 = v & 0xffu, b1 = (v >> 8) & 0xffu, b2 = (v >> 16) & 0xffu, b3 = v >> 24;
  const uint32_t o1 = (uint32_t)__builtin_popcount(b0) + 8u;
  const uint32_t o2 = (uint32_t)__builtin_popcount(v & 0xffffu) + 16u;
  const uint32_t o3 = (uint32_t)__builtin_popcount(v & 0xffffffu) + 24u;
  const uint32_t s01 = wr.spread(b0) | (wr.spread(b1) << o1);  // < 2^32
  return (uint64_t)s01 | ((uint64_t)wr.spread(b2) << o2) | ((uint64_t)wr.spread(b3) << o3);
}

ZFP_HD uint32_t bitlen32(uint32_t x) { return x ? 32u - (uint32_t)__builtin_clz(x) : 0u; }

// General 3D plane step without a loop over the new ones (replaces the
// one-put step when some lane's code is longer than 64 bits or has new ones
// past r's 15th bit: dense planes, the last few of a block).  Three puts:
// the verbatim bits with the leading group test (n + 1 <= 64 bits), then r's
// doubled form in two halves (r's low and high 32 positions, each <= 64
// bits), the top one's partner dropped and the closing "0" counted (imp: the
// top one dropped too and no closing test).  The high half is skipped when no
// lane of the wave has new ones past position 31.  Bits past the block's
// budget land in the writer's slack; settle() first bounds them.
template <typename Writer>
ZFP_HD void encode_plane_wide(uint64_t x, unsigned& n, Writer& wr) {
  wr.settle();
  const unsigned nf = n;  // <= 63
  const uint64_t r = x >> nf;
  const uint32_t lo = (uint32_t)r, hi = (uint32_t)(r >> 32);
  const uint32_t blh = bitlen32(hi);
  const uint32_t bl = blh ? 32u + blh : bitlen32(lo);
  const uint32_t nn = nf + bl;  // <= 64
  const uint32_t imp = nn >> 6;
  const uint64_t nz = r != 0 ? 1u : 0u;
  wr.put((x ^ (r << nf)) | (nz << nf), nf + 1u);  // verbatim bits, then "1" (new ones) or "0"
  const uint64_t slo = spread32(lo, wr);
  const uint32_t tlo = (uint32_t)__builtin_popcount(lo);
  uint64_t top = slo;
  uint32_t ltop = bl + tlo;  // bits of the doubled form in the top part
  if (__builtin_expect(any_lane(hi != 0), 0)) {
    const uint64_t shi = spread32(hi, wr);
    // hi != 0: the low half is whole (32 positions, 32 + tlo bits) and the
    // top part is the high half
    wr.put(hi ? slo : 0ull, hi ? 32u + tlo : 0u);
    top = hi ? shi : slo;
    ltop = hi ? blh + (uint32_t)__builtin_popcount(hi) : ltop;
  }
  // drop the top one's partner (imp: the top one too); ltop >= 2 when r != 0
  const uint64_t cut = nz ? (uint64_t)(2u + imp) << ((ltop - 2u) & 63) : 0ull;
  wr.put(top & ~cut, ltop - 2u * imp);  // + the closing "0" (unless imp)
  n = nn - imp;  // min(nn, 63)
}

template <int DIMS, typename PW, typename Writer>
ZFP_HD void encode_plane_step(PW x, unsigned& n, Writer& wr) {
  constexpr unsigned N = 1u << (2 * DIMS);
  const unsigned nf = n;  // both steps keep n <= N-1
  // (16-coefficient planes: a 32-bit shift, nf <= 15)
  const uint64_t r = N <= 16 ? (uint64_t)((uint32_t)x >> nf) : (uint64_t)x >> nf;
  const uint32_t rl = (uint32_t)r;
  const uint32_t bl = bitlen16(rl);
  const uint32_t L = (uint32_t)__builtin_popcount(rl) + bl;  // v_bcnt_u32_b32(rl, bl)
  const PlaneLen pl = plane_len<DIMS>(nf, bl, L);
  if constexpr (N <= 16) {
    // r has at most 16 bits and the code at most 48: always one put
    encode_plane_one_put<DIMS>(x, nf, r, pl, n, wr);
  } else {
    // one put while every lane's code fits 64 bits with r < 2^15 (3D rate 8
    // on smooth data: ~26 of ~29 plane steps, tools/coder_stats.cpp);
    // otherwise the wide step for the whole wave
    // (r < 2^15 against the writer's fit_lim = 2^15 - 1, a 64-bit constant
    // kept in SGPRs rather than re-materialised every step)
    const bool ok = (uint64_t)r <= wr.fit_lim && pl.len <= 64u;
    if (__builtin_expect(!any_lane(!ok), 1))
      encode_plane_one_put<DIMS>(x, nf, r, pl, n, wr);
    else
      encode_plane_wide((uint64_t)x, n, wr);
  }
}

// Planes 31 .. cmin of 32-bit half H, two at a time (an odd one left at the
// bottom goes alone); false once the block is full.
template <int H, typename UInt, int DIMS, typename Writer>
ZFP_HD bool encode_half(const planes<UInt, DIMS>& P, unsigned& n, int cmin, Writer& wr) {
  typedef typename plane_word<DIMS>::type PW;
  int c = 31;
  for (; c - 1 >= cmin; c -= 2) {
    if (!any_lane(!wr.full())) return false;
    wr.settle();
    const int u = uniform(c);
    if constexpr (prio_of<Writer>::value) progress_priority<CUZFP_PRIO_T2, CUZFP_PRIO_T1, CUZFP_PRIO_T0>(u);
    encode_plane_step<DIMS>((PW)P.template get<H>(u), n, wr);
    encode_plane_step<DIMS>((PW)P.template get<H>(u - 1), n, wr);
  }
  if (c >= cmin && c >= 0) {
    if (!any_lane(!wr.full())) return false;
    wr.settle();
    encode_plane_step<DIMS>((PW)P.template get<H>(uniform(c)), n, wr);
  }
  return true;
}

// Planes 31 .. 0 of half H with compile-time plane numbers (every lane of the
// wave codes all 32 planes while it has budget): each plane word is a fixed
// register, so there is no VGPR-relative addressing (s_set_gpr_idx_on / off
// around each read), no readfirstlane of the plane number, and the priority
// drops sit at fixed trips.
// (STOP: the lowest plane coded, STOP even; planes STOP-1 .. 0 are left to a
// later call, as the 2D split of encode_block does)
template <int H, int C, bool PRI = true, int STOP = 0, typename UInt, int DIMS, typename Writer>
ZFP_HD bool encode_half_fixed(const planes<UInt, DIMS>& P, unsigned& n, Writer& wr) {
  typedef typename plane_word<DIMS>::type PW;
  if constexpr (C >= STOP + 1) {
    if (!any_lane(!wr.full())) return false;
    wr.settle();
#if defined(__HIP_DEVICE_COMPILE__) && !defined(CUZFP_NO_PRIO)
    if constexpr (prio_of<Writer>::value && PRI) {
      if constexpr (C == CUZFP_PRIO_T2) __builtin_amdgcn_s_setprio(2);
      else if constexpr (C == CUZFP_PRIO_T1) __builtin_amdgcn_s_setprio(1);
      else if constexpr (C == CUZFP_PRIO_T0) __builtin_amdgcn_s_setprio(0);
    }
#endif
    encode_plane_step<DIMS>((PW)P.template get<H>(C), n, wr);
    encode_plane_step<DIMS>((PW)P.template get<H>(C - 1), n, wr);
    return encode_half_fixed<H, C - 2, PRI, STOP>(P, n, wr);
  }
  return true;
}

// ---------------------------------------------------------------------------
// 1D blocks by table (4 coefficients: a plane is a nibble).
//
// Encoder: one lookup codes two planes.  Entry (n, a, b) -- n the count of
// significant coefficients before plane a (kept at most N-1 = 3, see
// encode_plane_one_put), a and b the two planes' nibbles -- holds the two plane
// codes concatenated (at most 2 x 7 bits), their length and the n after plane
// b.  The codes are those of encode.c:121-151 without a budget: the writer
// drops what passes the block's maxbits, and the reference writes exactly the
// budget's prefix of the same bits.
//
// Decoder: one lookup decodes one plane, budget included.  Entry (n, c, s) --
// c = min(bits left, 7) (a 1D plane code has at most 7 bits, so c = 7 means
// "not cut"), s the next 8 stream bits -- holds the plane's nibble, the bits
// read and the n after it, from decode.c:288-321 run on those bits with that
// budget (its quirk -- a one deposited where the budget ends a run of zeros --
// included).  So the 1D plane loop has no rare path and no branch on the data.

// encode.c:136-150 for one 1D plane x (4 bits) with n significant: the code's
// bits (LSB first), their count, and n afterwards
constexpr void plane_code_1d(uint32_t x, uint32_t& n, uint32_t& code, uint32_t& len) {
  constexpr uint32_t N = 4;
  code = 0;
  len = 0;
  for (uint32_t i = 0; i < n; i++) code |= ((x >> i) & 1u) << len++;
  x >>= n;
  while (n < N) {
    const uint32_t t = x ? 1u : 0u;  // group test
    code |= t << len++;
    if (!t) break;
    while (n < N - 1) {  // the run up to the next one (the one at N-1 is implied)
      const uint32_t b = x & 1u;
      code |= b << len++;
      if (b) break;
      x >>= 1;
      n++;
    }
    x >>= 1;
    n++;
  }
}
struct Pair1dLut {
  uint32_t e[4 * 256];  // [n][a << 4 | b]: code [0,14) | length << 14 | n' << 30
};
constexpr Pair1dLut make_pair1d_lut() {
  Pair1dLut t{};
  for (uint32_t n0 = 0; n0 < 4; n0++)
    for (uint32_t ab = 0; ab < 256; ab++) {
      uint32_t n = n0, ca = 0, la = 0, cb = 0, lb = 0;
      plane_code_1d(ab >> 4, n, ca, la);
      n = n < 3 ? n : 3;
      plane_code_1d(ab & 15u, n, cb, lb);
      n = n < 3 ? n : 3;
      t.e[n0 * 256 + ab] = (ca | (cb << la)) | ((la + lb) << 14) | (n << 30);
    }
  return t;
}
// byte offset of the (n, a, b) entry, n given as n << 10
ZFP_HD uint32_t pair1d_off(uint32_t n10, uint32_t a, uint32_t b) { return n10 | (a << 6) | (b << 2); }

// decode.c:288-321 for one 1D plane: the stream bits s (LSB first), budget c
constexpr void plane_decode_1d(uint32_t s, uint32_t c, uint32_t& n, uint32_t& x, uint32_t& used) {
  constexpr uint32_t N = 4;
  uint32_t bits = c, p = 0;
  const uint32_t m = n < bits ? n : bits;
  x = s & ((1u << m) - 1u);
  p = m;
  bits -= m;
  while (n < N && bits) {
    bits--;
    if (!((s >> p++) & 1u)) break;  // group test "0"
    while (n < N - 1 && bits) {
      bits--;
      if ((s >> p++) & 1u) break;  // the one
      n++;
    }
    x += 1u << n;
    n++;
  }
  used = c - bits;
}
struct Plane1dDecLut {
  uint16_t e[4 * 8 * 256];  // [n][c][s]: nibble | used << 4 | n' << 12 (n' in place for the next index)
};
constexpr Plane1dDecLut make_plane1d_dec_lut() {
  Plane1dDecLut t{};
  for (uint32_t n0 = 0; n0 < 4; n0++)
    for (uint32_t c = 0; c < 8; c++)
      for (uint32_t s = 0; s < 256; s++) {
        uint32_t n = n0, x = 0, used = 0;
        plane_decode_1d(s, c, n, x, used);
        n = n < 3 ? n : 3;
        t.e[(n0 * 8 + c) * 256 + s] = (uint16_t)(x | (used << 4) | (n << 12));
      }
  return t;
}

// Writers that hold the 1D pair table (pair1d(byte offset) reads an entry)
template <typename T, typename = void> struct has_pair1d {
  static constexpr bool value = false;
};
template <typename T> struct has_pair1d<T, decltype((void)&T::pair1d)> {
  static constexpr bool value = true;
};

// Planes C, C-1, ... 1, 0 of 32-bit half H of a 1D block, two per lookup,
// while any lane of the wave has budget; false once every lane is full.
template <int H, int C, typename UInt, typename Writer>
ZFP_HD bool encode_pairs_1d(const planes<UInt, 1>& P, uint32_t& n10, Writer& wr) {
  if constexpr (C >= 1) {
    if (!any_lane(!wr.full())) return false;
    constexpr int S = 4 * (C / 4);  // planes C and C-1 share a nibble position (C odd)
    const uint32_t a = (P.template word<H>(C) >> S) & 15u, b = (P.template word<H>(C - 1) >> S) & 15u;
    const uint32_t e = wr.pair1d(pair1d_off(n10, a, b));
    wr.put(e & 0x3fffu, (e >> 14) & 31u);
    n10 = e >> 20;  // bits 19-29 of an entry are zero
    return encode_pairs_1d<H, C - 2>(P, n10, wr);
  }
  return true;
}

template <typename UInt, int DIMS, typename Writer>
ZFP_HD void encode_planes(const planes<UInt, DIMS>& P, unsigned maxprec, Writer& wr) {
  constexpr int PREC = (int)sizeof(UInt) * 8;
  unsigned n = 0;
  if constexpr (PREC == 32) {
    // 32-bit coefficients are coded down to plane 0: precision() is 32 for
    // every f32 exponent (emax >= -149), and int32 has maxprec 32
    (void)maxprec;
    if constexpr (DIMS == 1 && has_pair1d<Writer>::value) {
      uint32_t n10 = 0;
      encode_pairs_1d<0, 31>(P, n10, wr);
      return;
    }
    encode_half_fixed<0, 31>(P, n, wr);
  } else {
    const int kmin = PREC > (int)maxprec ? PREC - (int)maxprec : 0;
    if (!any_lane(kmin != 0)) {  // every lane codes down to plane 0 (normal doubles)
      if constexpr (DIMS == 1 && has_pair1d<Writer>::value) {
        uint32_t n10 = 0;
        if (encode_pairs_1d<1, 31>(P, n10, wr)) encode_pairs_1d<0, 31>(P, n10, wr);
        return;
      }
      // the priority schedule over the high half only
      if (encode_half_fixed<1, 31>(P, n, wr)) encode_half_fixed<0, 31, false>(P, n, wr);
      return;
    }
    if (!encode_half<1>(P, n, kmin > 32 ? kmin - 32 : 0, wr)) return;
    encode_half<0>(P, n, kmin, wr);
  }
}

// Decoder plane step (decode.c:288-321).
//
// Fast path, bit-parallel.  After the verbatim bits and a "1" group test the
// plane's code is a sequence of segments  0^z 1 g  (zeros, the new one, the
// group test after it: g = 1 means more ones follow) ending at the first g = 0.
// So in the code c every run of ones starts at a segment's one and consists of
// (one, g = 1) pairs -- except the last run, whose final one is followed by the
// closing 0: the code ends at the first run of ODD length.  With
//   F = the ones at even offsets inside their run      (the segments' ones)
// the end is the lowest bit of F that is also the last bit of its run, and the
// new plane ones are F's bits moved down past the g bits below them (the j-th
// one of F by j).  Runs starting at even positions are found with one carrying
// add (c + their start bits clears exactly those runs).
//
// When the budget ends inside the code, the reference has read a prefix of
// it: every one in the prefix is deposited, and unless the prefix ends with a
// one, one more one is deposited at the next position (decode.c:305-311: the
// group loop's increment runs after the budget stops the run loop) -- so the
// prefix needs no sequential loop either.
//
// Codes longer than one 64-bit window (dense planes) are taken in chunks,
// each consumed up to its last whole (one, "1") pair.  The plane in which the
// last coefficient becomes significant ends with a run of zeros up to position
// N-1 and an implied one; that end is also found without a per-bit loop.
// Whatever is left (a code the chunking cannot split) runs the exact
// sequential group loop, whose trips follow the reference's control flow bit
// for bit.  tests/test_emulation.py and test_gpu_parity.py decode arbitrary
// bit streams against the oracle to exercise every path.
// One chunk of a plane's group code: c holds `valid` code bits starting at a
// segment (its first bit is a run of zeros or a one).  Returns false if the
// chunk neither ends the code nor can be split at a pair (the caller then
// takes the sequential loop).  Otherwise sets cb (code bits consumed), Fb (the
// ones read, at their code positions), nong (plane positions advanced), quirk
// (a one deposited after the budget ran out) and done (the code ended here).
struct chunk_parse {
  uint64_t Fb;
  unsigned cb, nong;
  bool quirk, done;
};

template <int N>
ZFP_HD bool parse_chunk(uint64_t c, unsigned valid, unsigned bits, unsigned n, chunk_parse& r) {
  constexpr uint64_t EVEN = 0x5555555555555555ull;
  const uint64_t starts = c & ~(c << 1);
  const uint64_t erun = c & ~(c + (starts & EVEN));
  const uint64_t Fall = (erun & EVEN) | (c & ~erun & ~EVEN);  // segment ones
  const uint64_t F = Fall & lowmask(valid - 1);                // ... with their partner inside
  const uint64_t oddend = F & ~(c >> 1);                       // a one with a 0 partner
  const unsigned qe = ctz64_or_64(oddend);                     // >= 64 if none
  const bool complete = qe < 64 && qe + 2 <= bits;             // code ends: c[0 .. qe+1]
  const bool limited = !complete && bits <= valid;             // budget ends: c[0 .. bits-1]
  const unsigned ql = F ? 63u - (unsigned)__builtin_clzll(F) : 0u;
  r.cb = complete ? qe + 2 : limited ? bits : ql + 2;
  const uint64_t cm = lowmask(r.cb);
  r.Fb = Fall & cm;
  r.nong = r.cb - (unsigned)__builtin_popcountll((r.Fb << 1) & cm);
  const bool lastone = r.cb && ((r.Fb >> ((r.cb - 1) & 63)) & 1);
  r.quirk = limited && !lastone;
  r.done = complete || limited;
  return complete ? n + r.nong <= N - 1 : (limited || F) && n + r.nong <= N - 2;
}

// the j-th one of Fb moved down by j (the g bits below it removed), plus the
// one deposited after the budget ran out
template <typename PW>
ZFP_HD PW place_ones(uint64_t f, bool quirk, unsigned nong) {
  PW y = quirk ? (PW)1 << (nong & (8 * sizeof(PW) - 1)) : (PW)0;
  unsigned j = 0;
  while (f) {
    const uint64_t low = f & (0 - f);
    y |= (PW)(low >> j);
    f ^= low;
    j++;
  }
  return y;
}

template <int DIMS, typename PW, typename Reader>
ZFP_HD PW decode_plane(unsigned& bits, unsigned& n, Reader& rd) {
  constexpr unsigned N = 1u << (2 * DIMS);
  constexpr unsigned PWB = 8 * sizeof(PW);
  uint64_t v0, v1;
  rd.peek2(v0, v1);  // stream bits [pos, pos + 128)
  const unsigned m = umin(n, bits);
  PW x = (PW)(v0 & lowmask(m));
  bits -= m;
  // The group part exists while positions and budget remain; then m <= n < N
  // <= 64 and m < 64, and `win` is the window at the leading group test.  The
  // first chunk is computed for every lane and selected, so the wave does not
  // branch on the data (a lane without group part, or with a "0" group test,
  // places nothing and consumes 0 or 1 bit).
  const bool grp = n < N && bits;
  const uint64_t win = (v0 >> (m & 63)) | ((v1 << 1) << (63 - (m & 63)));
  const bool g0 = grp && (win & 1);
  const unsigned lead = grp ? 1u : 0u;
  bits -= lead;
  chunk_parse r;
  const bool ok = parse_chunk<N>(win >> 1, 63, bits, n, r);
  ZFP_COUNT_PLANE(g0, ok && r.done, r.cb);
  if (__builtin_expect(!g0 || (ok && r.done), 1)) {
    // where the next plane starts is known now: move the reader first, so its
    // reads overlap placing this plane's ones
    const unsigned used = g0 ? r.cb : 0u;
    rd.skip(m + lead + used);
    bits -= used;
    x |= place_ones<PW>(g0 ? r.Fb : 0ull, g0 && r.quirk, r.nong) << (n & (PWB - 1));
    n += g0 ? r.nong + (r.quirk ? 1u : 0u) : 0u;
    return x;
  }
  // Rare: a dense code longer than the first chunk, or a code that reaches
  // position N-1.  Chunks are consumed up to their last whole (one, "1") pair
  // while that is possible.
  rd.skip(m + lead);
  uint64_t c = win >> 1;
  unsigned valid = 63;
  bool okc = ok;
  while (okc) {
    rd.skip(r.cb);
    bits -= r.cb;
    x |= place_ones<PW>(r.Fb, r.quirk, r.nong) << (n & (PWB - 1));
    n += r.nong + (r.quirk ? 1u : 0u);
    if (r.done) return x;
    c = rd.peek();
    valid = 64;
    okc = parse_chunk<N>(c, valid, bits, n, r);
  }
  {
    // The code reaches position N-1 before it ends: there the one is implied
    // and nothing more is read (the plane in which coefficient N-1 becomes
    // significant).  The real ones are the chunk's segment ones below plane
    // offset N'-1 (N' = N - n); the code is those pairs plus the zeros up to
    // offset N'-2: N'-1 + ones bits, and every one in it must belong to
    // those pairs (a one whose partner lies past the chunk is not in F).
    constexpr uint64_t EVEN = 0x5555555555555555ull;
    const uint64_t starts = c & ~(c << 1);
    const uint64_t erun = c & ~(c + (starts & EVEN));
    const uint64_t F = ((erun & EVEN) | (c & ~erun & ~EVEN)) & lowmask(valid - 1);
    const int np = (int)(N - n);
    uint64_t f = F, fr = 0;
    PW y = 0;
    unsigned j = 0;
    while (f) {
      const uint64_t low = f & (0 - f);
      if ((int)(ctz64(low) - j) > np - 2) break;
      y |= (PW)(low >> j);
      fr |= low;
      f ^= low;
      j++;
    }
    const unsigned e = (unsigned)np - 1 + j;
    if (e <= bits && e <= valid && !((c ^ fr ^ (fr << 1)) & lowmask(e))) {
      x |= (y | ((PW)1 << ((unsigned)(np - 1) & (PWB - 1)))) << (n & (PWB - 1));
      n = N;
      rd.skip(e);
      bits -= e;
      return x;
    }
  }
  // Exact sequential group loop from the start of a segment: one trip per new
  // one -- the run of zeros, the one (unless implied) and the following group
  // test, all from one window -- following the reference's control flow bit
  // for bit.
  bool more = true;
  while (more) {
    const uint64_t w = rd.peek();
    const unsigned lim = umin(N - 1 - n, bits);   // zeros we may still read
    const unsigned z = ctz64_or_64(w);            // zeros before the one
    const bool found = z < lim;                   // the one is read, not implied
    const unsigned adv = found ? z : lim;
    n += adv;
    x |= (PW)1 << n;
    n++;
    const unsigned used = adv + (found ? 1u : 0u);
    // the group test after a read one: "1" = more ones follow
    const bool gt = found && used < bits && n < N && ((w >> used) & 1);
    const unsigned take = used + ((found && used < bits && n < N) ? 1u : 0u);
    rd.skip(take);
    bits -= take;
    more = gt;  // with bits == 0 the next trip deposits at n (decode.c:311)
  }
  return x;
}

// ---------------------------------------------------------------------------
// Table-driven plane decoder (the common case).
//
// A group code after its leading "1" test is a token string: "0" (a position
// that stays zero) or "1g" (a new one, then the group test g; g = 0 ends the
// code).  kChunkBits bits of it are parsed by one table lookup: the entry of
// (state, chunk) -- state 1 meaning the chunk's first bit is the pending g of
// a one that closed the previous chunk -- gives the ones it places (as a bit
// pattern over the positions it covers), how many positions it covers, and,
// if the code ends inside it, how many bits it used.  Two chunks are looked
// up side by side (the second in both states), so one plane costs three table
// reads and no loop.  The tables are generated at compile time from the token
// grammar (decode.c:302-317 read the same grammar bit by bit).
constexpr int kChunkBits = 10;
constexpr uint32_t kChunkMask = (1u << kChunkBits) - 1;
// entry (one dword): ones [0,10) | 0 | positions covered [11,16) | exit state
// bit 16 | 0 | bits used U [18,32).  The fields have room for the sum of two
// entries (ones < 2^11 and the states' sum < 4 carry into zero bits,
// positions <= 20 < 2^5, U's carry leaves the dword), so one add combines
// chunk 1 and chunk 2.  U also says whether the code ended, by a marker M =
// 2^13 (U's top bit, the dword's sign bit): a chunk-1 entry that did not end
// carries M, a chunk-2 entry that did end carries M too, so the sum's U holds
// M (mod 2^14) exactly when the code has not ended -- the sum is negative.
// (Round 6: the fields the common step reads sit where fast-issue
// instructions reach them -- the ones by an AND with an inline constant, the
// positions as a shift count taken from the low 5 bits of e >> 11, U by one
// shift, the marker as the sign bit -- instead of behind v_bfe_u32.)
constexpr unsigned kOnesShift = 0, kPosShift = 11, kStateShift = 16, kUsedShift = 18;
constexpr uint32_t kNotEnded = 1u << 13;           // in U's units
constexpr uint32_t kEntryState = 1u << kStateShift;
constexpr uint32_t kMarkerBit = kNotEnded << kUsedShift;  // bit 31

constexpr uint32_t pack_entry(uint32_t ones, uint32_t pos, uint32_t used, uint32_t flags) {
  return (ones << kOnesShift) | (pos << kPosShift) | (used << kUsedShift) | flags;
}
// an entry's (or a sum's) fields
ZFP_HD constexpr uint32_t ent_ones(uint32_t e) { return (e >> kOnesShift) & ((1u << kChunkBits) - 1u); }
ZFP_HD constexpr uint32_t ent_pos(uint32_t e) { return (e >> kPosShift) & 31u; }
ZFP_HD constexpr uint32_t ent_state(uint32_t e) { return (e >> kStateShift) & 1u; }
ZFP_HD constexpr uint32_t ent_used(uint32_t e) { return e >> kUsedShift; }  // 14 bits, the marker included

// state 0: at a token boundary; 1: the first bit is the pending group test of
// a one that closed the previous chunk; 2: the first bit is the plane's
// leading group test (0 = no new ones in this plane)
constexpr uint32_t chunk_entry(unsigned state, uint32_t b) {
  // the marker: state 2 (chunk 1) entries that do not end, state 0/1 (chunk 2)
  // entries that do
  const uint32_t mark_end = state == 2 ? 0u : kNotEnded, mark_open = state == 2 ? kNotEnded : 0u;
  uint32_t ones = 0, pos = 0;
  unsigned i = 0;
  if (state == 2 || state == 1) {
    i = 1;
    if (!(b & 1u)) return pack_entry(0, 0, 1 + mark_end, 0);
  }
  while (i < (unsigned)kChunkBits) {
    if (!((b >> i) & 1u)) {  // a position that stays zero
      pos++;
      i++;
      continue;
    }
    ones |= 1u << pos;  // a new one
    pos++;
    i++;
    if (i == (unsigned)kChunkBits)  // its group test is in the next chunk
      return pack_entry(ones, pos, kChunkBits + mark_open, kEntryState);
    const bool more = (b >> i) & 1u;
    i++;
    if (!more) return pack_entry(ones, pos, i + mark_end, 0);
  }
  return pack_entry(ones, pos, kChunkBits + mark_open, 0);
}

// The chunk-2 entry a chunk-1 entry selects, as one v_perm_b32 of the pair
// (e2a: state 0, e2b: state 1) by the selector stored beside chunk 1's entry:
// bytes 0-3 (e2a) or 4-7 (e2b) by chunk 1's exit state, or 0x0c bytes (zero)
// when chunk 1 ended the code -- one slow-class instruction where the select
// by the exit state and the mask by the marker took four (round 6).
constexpr uint32_t kSelState0 = 0x03020100u, kSelState1 = 0x07060504u, kSelNone = 0x0c0c0c0cu;
constexpr uint32_t chunk_sel(uint32_t e1) {
  return !(e1 & kMarkerBit) ? kSelNone : (e1 & kEntryState) ? kSelState1 : kSelState0;
}
// v_perm_b32(b, a, sel): byte i of the result is selector byte i's pick of
// {a = bytes 0-3, b = bytes 4-7}, 0x00 for 12, 0xff for 13 and up (the
// sign-replicating selectors 8-11 are not used here)
ZFP_HD uint32_t perm_sel(uint32_t b, uint32_t a, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(b, a, sel);
#else
  const uint64_t v = (uint64_t)a | ((uint64_t)b << 32);
  uint32_t r = 0;
  for (int i = 0; i < 4; i++) {
    const uint32_t k = (sel >> (8 * i)) & 0xffu;
    const uint32_t byte = k < 8 ? (uint32_t)(v >> (8 * k)) & 0xffu : k == 12 ? 0u : 0xffu;
    r |= byte << (8 * i);
  }
  return r;
#endif
}

// Table layout (16 KiB): chunk 1 (state 2, the leading group test first) at
// dwords [0, 2^(B+1)), chunk b's entry at 2b and its chunk-2 selector at
// 2b + 1, so one ds_read_b64 reads both; states 0 and 1 side by side at
// [2^(B+1), 2^(B+2)), chunk b's pair at 2^(B+1) + 2b, one ds_read_b64 too (64
// banks, one LDS instruction, where two ds_read_b32 -- or one
// ds_read2st64_b32, served as two -- each take the 32-bank conflicts of the
// lanes' random entries).  1D reads the chunk-1 table alone.
constexpr uint32_t kLutS2 = 0, kLutPairs = 2u << kChunkBits;
ZFP_HD constexpr uint32_t lut_s2_index(uint32_t b) { return kLutS2 + 2u * (b & kChunkMask); }
ZFP_HD constexpr uint32_t lut_pair_index(uint32_t b, uint32_t state) { return kLutPairs + 2u * (b & kChunkMask) + state; }
struct ChunkLut {
  uint32_t e[4u << kChunkBits];
};
constexpr ChunkLut make_chunk_lut() {
  ChunkLut t{};
  for (uint32_t b = 0; b <= kChunkMask; b++) {
    const uint32_t e1 = chunk_entry(2, b);
    t.e[lut_s2_index(b)] = e1;
    t.e[lut_s2_index(b) + 1] = chunk_sel(e1);
    t.e[lut_pair_index(b, 0)] = chunk_entry(0, b);
    t.e[lut_pair_index(b, 1)] = chunk_entry(1, b);
  }
  return t;
}

// m = 0 .. 64 low bits set
ZFP_HD uint64_t lowmask64(unsigned m) { return m ? ~0ull >> ((64u - m) & 63u) : 0ull; }

// (ones << s) above bit s, w below it: the mask ~0 << s, the shift, and one
// v_bfi_b32 a dword (the compiler's form of the same expression ORs the
// shifted ones in after the insert: two more instructions)
template <typename PW>
ZFP_HD PW merge_at(uint32_t s, uint64_t ones, uint64_t w) {
  if constexpr (sizeof(PW) == 8) {
    // (s <= 63: the shifts' counts need no mask; o laundered, or the
    // compiler drops the mask o already satisfies and ORs it in separately)
    const uint64_t hi = ~0ull << (s & 63u), o = launder(ones << (s & 63u));
    return (o & hi) | (w & ~hi);
  } else {
    // 16-bit planes (2D: s <= 15, ones below bit 16 - s): the low s bits of w
    // (one v_bfe_u32) under the shifted ones (one v_lshl_or_b32)
    return (PW)(((uint32_t)ones << s) | low_bits((uint32_t)w, s));
  }
}

// (a & m) | c in one v_and_or_b32
ZFP_HD uint32_t and_or(uint32_t a, uint32_t m, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(m), "v"(c));
  return r;
#else
  return (a & m) | c;
#endif
}


// v unless e carries the marker (its sign bit): one arithmetic shift and an
// AND-NOT, both fast-issue
ZFP_HD uint32_t drop_if_marked(uint32_t v, uint32_t e) { return v & ~(uint32_t)((int32_t)e >> 31); }

// A two-chunk parse that covers position N-1 (npos > q = N-1-n): there the
// reference reads nothing -- its zero loop stops at N-1 and the one there is
// implied (decode.c:305-311) -- so the parse past N-1 is not the code.  The
// code's real end is the start of position N-1's token: in chunk 1 (state 2:
// its first bit is the leading test) at bit 1 + q + (ones before q), in chunk
// 2 (chunk 1 read whole, its exit state s1 = a pending group test first) at
// kChunkBits + s1 + (q - p1) + (ones before q - p1).  Returns that bit count
// and sets `ones` to the ones below N-1 plus the implied one.
ZFP_HD uint32_t implied_end(uint32_t e1, uint32_t e2, uint32_t q, uint64_t& ones) {
  const uint32_t p1 = ent_pos(e1);
  const uint32_t o1 = ent_ones(e1), o2 = ent_ones(e2);
  uint32_t o;
  if (p1 > q) {
    o = 1u + q + (uint32_t)__builtin_popcount(o1 & ((1u << q) - 1u));
  } else {
    const uint32_t q2 = q - p1;
    o = kChunkBits + ent_state(e1) + q2 + (uint32_t)__builtin_popcount(o2 & ((1u << q2) - 1u));
  }
  ones = (ones & ((1ull << q) - 1ull)) | (1ull << q);
  return o;
}

// One plane by table lookup, with the budget.  Reader: windows(m, w, g) gives
// the 64 stream bits at the read position (w) and the 32 bits m further on
// (g); chunks_fast(g, e1, e2a, e2b) reads the entry of g's first chunk in
// state 2 and of its second chunk in states 0 and 1, chunk1_fast(g) only the
// first; window32 / chunks_st read continuation pairs.  Sets `slow` for a
// plane the tables cannot finish (see below); the caller then discards this
// step's result and state and decodes the plane again with decode_plane.  So
// nothing here is gated on `slow`: a lane out of budget (b1 = 0) reads zeros
// past its block (its group test reads as a "0" it does not consume).
// The budget-aware step's resolution from the first pair's entries (e1, e2 as
// chunks_fast and the exit-state select give them) and the verbatim window w
// at the read position; nf = min(n, N-1), m = min(nf, bits).  Shared by
// decode_plane_lut and the fast step's rare branch , which
// reads the group window at nf rather than m: when m < nf both lie past the
// block's end and read zeros.
template <int DIMS, typename PW, typename Reader>
ZFP_HD PW lut_finish(unsigned& bits, unsigned& n, Reader& rd, bool& slow, unsigned nf, unsigned m,
                     uint64_t w, uint32_t e1, uint32_t e2) {
  constexpr unsigned N = 1u << (2 * DIMS);
  const unsigned b1 = bits - m;                // budget after the verbatim bits
  const uint32_t S = e1 + e2;                  // field-wise sums
  uint32_t npos = ent_pos(S);
  const uint32_t used = ent_used(S);           // >= kNotEnded: the code has not ended
  uint64_t ones = ent_ones(e1) | (ent_ones(e2) << ent_pos(e1));
  bool ended = used < kNotEnded;
  uint32_t parsed = used & (kNotEnded - 1u);  // code bits read (all of the chunks' if not ended)
  uint32_t st = ent_state(DIMS == 1 ? e1 : e2);       // exit state of the last chunk read
  const uint32_t q = N - 1 - nf;
  // the code bits up to position N-1's token when a continuation pair reaches
  // it (the first pair's case is implied_end below)
  uint32_t io = 0;
  if constexpr (DIMS >= 2) {
    // A code longer than the two chunks (a dense plane, the last few of a
    // block): further chunk pairs from the exit state, while the budget
    // reaches past what has been read.  In a continuation pair both chunks
    // are in state 0/1, whose entries carry the marker when they end.
    bool open = !ended && parsed < b1 && nf + npos < N;
    if (__builtin_expect(any_lane(open), 0)) {
      while (any_lane(open)) {
        if (open) {
          const uint32_t gg = rd.window32(rd.pos + m + parsed);
          uint32_t eA, eBa, eBb;
          rd.chunks_st(gg, st, eA, eBa, eBb);
          const uint32_t eB = drop_if_marked((eA & kEntryState) ? eBb : eBa, eA);
          const uint32_t T = eA + eB;
          const uint32_t pA = ent_pos(eA);
          const uint32_t oA = ent_ones(eA), oB = ent_ones(eB);
          const uint64_t o = oA | ((uint64_t)oB << pA);
          // this pair reaches position N-1 (offset q2 into it): the code ends
          // at the start of that position's token -- st + q2 + the ones'
          // "more" bits below it in chunk A, or chunk A whole and the same
          // count in chunk B (as implied_end for the first pair)
          const uint32_t q2 = q - npos;  // npos <= q while open
          io = pA > q2 ? parsed + st + q2 + (uint32_t)__builtin_popcount(oA & ((1u << q2) - 1u))
                       : parsed + kChunkBits + ent_state(eA) + (q2 - pA) +
                             (uint32_t)__builtin_popcount(oB & ((1u << ((q2 - pA) & 31u)) - 1u));
          ones |= o << (npos & 63u);
          npos += ent_pos(T);
          const uint32_t u = ent_used(T);
          ended = u >= kNotEnded;
          parsed += u & (kNotEnded - 1u);
          st = ent_state(eB);
          open = !ended && parsed < b1 && nf + npos < N;
        }
      }
    }
  }
  // The stream reads as zeros past the block's last bit (the kernels and the
  // host reader guarantee it) and the budget always ends there.  So:
  //  - a code that ended within the budget, or one bit past it (a one read
  //    with the budget's last bit, followed by the zero group test that is
  //    not in the stream), is taken as read (decode.c:302-317);
  //  - a code the budget cuts short inside the two chunks reads on as zero
  //    positions: the reference deposited one more one at the position it
  //    had reached when the budget ran out (decode.c:305-311), npos less the
  //    bits read past the budget.
  // A code whose parse reaches position N-1 (where the one is implied) is
  // resolved from the first two chunks' entries if that happens within the
  // budget; anything else left takes the general decoder.
  // (bitwise rather than short-circuit logic below: one mask each, no
  // divergent branches)
  const uint32_t d = parsed - b1;  // code bits parsed past the budget (wraps when within)
  // a one on the budget's last bit (its group test unread) also ends the code
  const bool done = ended | ((d == 0u) & (st != 0u));
  const bool cut = !done & ((int32_t)d >= 0);
  const uint32_t P = npos - (cut ? d : 0u);  // cut: the position of the deposited one
  slow = (cut & (P > q)) | (!cut & (!done | ((int32_t)d > 1) | (npos > q)));
  uint64_t ones64 = ones | ((uint64_t)(cut ? 1u : 0u) << (P & 63u));
  uint32_t np = P + (cut ? 1u : 0u), take = umin(parsed, b1);
  if (__builtin_expect(any_lane(npos > q), 0)) {  // the parse reaches position N-1 (implied one)
    if (npos > q) {
      uint64_t o64 = ones;
      uint32_t o = implied_end(e1, e2, q, o64);
      // reached in a continuation pair: its count from the loop
      if (ent_pos(e1) + ent_pos(e2) <= q) o = io;
      // position N-1 within the budget: the code ends there; the budget
      // running out first leaves the cut result above (slow unless its one
      // lies at or below N-1)
      if (o <= b1) {
        slow = false;
        ones64 = o64;
        np = q + 1u;
        take = o;
      } else if (!cut) {
        slow = true;
      }
    }
  }
  ZFP_COUNT_PATH(slow ? (npos > q ? (cut ? 11 : 12) : (cut ? 13 : (!ended ? 14 : 15))) : 10);
  // the verbatim bits below m, the new ones at n >= m: one v_bfi_b32 a dword
  // under the mask ~0 << m (m <= N-1)
  const PW hi = (PW)(~0ull << m);
  const PW x = (hi & ((PW)ones64 << nf)) | (~hi & (PW)w);
  n = nf + np;
  const unsigned adv = m + take;
  rd.pos += adv;
  bits -= adv;
  return x;
}

template <int DIMS, typename PW, typename Reader>
ZFP_HD PW decode_plane_lut(unsigned& bits, unsigned& n, Reader& rd, bool& slow) {
  constexpr unsigned N = 1u << (2 * DIMS);
  // n is taken as at most N-1: with n = N-1 the group part is the last
  // position's bit alone (a "0" test, or a "1" test with the one implied),
  // which reads the same bits as N verbatim ones; the implied-one rule
  // resolves it from the state-2 entry of that bit
  const unsigned nf = n < N - 1 ? n : N - 1;
  const unsigned m = umin(nf, bits);
  uint64_t w;
  uint32_t g;
  rd.windows(m, w, g);
  // chunk 1 starts at the leading group test (table state 2), chunk 2 is read
  // in both states and chosen by chunk 1's exit state; nothing follows a
  // chunk 1 that ended the code
  uint32_t e1, e2;
  if constexpr (DIMS == 1) {
    // a 1D code (4 positions, at most 7 bits with the leading test) fits chunk 1
    e1 = rd.chunk1_fast(g);
    e2 = 0;
  } else {
    uint32_t sel, e2a, e2b;
    rd.chunks_fast(g, e1, sel, e2a, e2b);
    e2 = perm_sel(e2b, e2a, sel);  // by chunk 1's exit state; nothing after a chunk 1 that ended
  }
  return lut_finish<DIMS, PW>(bits, n, rd, slow, nf, m, w, e1, e2);
}

// Plane loop: the table decoder for every lane, then, only when some lane of
// the wave needs it, the general decoder for those lanes.  (n <= N-1 in and
// out.)  Used for a rolled loop's trailing odd plane.
template <int DIMS, typename PW, typename Reader>
ZFP_HD PW decode_plane_any(unsigned& n, Reader& rd) {
  constexpr unsigned N = 1u << (2 * DIMS);
  const auto pos0 = rd.pos;
  const unsigned n0 = n;
  unsigned bits = rd.end - pos0;
  bool slow;
  PW x = decode_plane_lut<DIMS, PW>(bits, n, rd, slow);
  ZFP_COUNT_PATH(slow ? 6 : 5);
  if (__builtin_expect(any_lane(slow), 0)) {  // wave-uniform test first: the per-lane branch costs exec-mask work
    if (slow) {
      rd.init(pos0);
      n = n0;
      bits = rd.end - pos0;
      x = decode_plane<DIMS, PW>(bits, n, rd);
    }
  }
  n = umin(n, N - 1);
  return x;
}

// The decoder's plane step, every dimensionality (1D reads chunk 1 only).
// The reader holds the block's budget as an end position (rd.end: the read
// position never passes it), so the common path clips its advance with one
// min and keeps no separate bit count; the rare paths compute the budget left
// as rd.end - rd.pos.  n is kept at most N-1 (with n = N-1 the group part is
// the last position's bit alone, looked up in two dedicated entries, which
// reads the same bits as n = N), so the window offset and the verbatim mask
// take n as it is.  Common case: the code ends within the two chunks, below
// position N-1 (one wave-uniform test covers both).


template <int DIMS, typename PW, typename Reader>
ZFP_HD PW decode_plane_fast_any(unsigned& n, Reader& rd) {
  constexpr unsigned N = 1u << (2 * DIMS);
  const unsigned nf = n;  // <= N-1
  // the group window first (the lookups wait on it), the verbatim window's
  // reads after the lookups' (Reader::window_g / window_w)
  WRaw wr;
  const uint32_t g = rd.window_g(nf, wr);
  uint32_t e1, e2, sel = 0, e2a = 0, e2b = 0;
  if constexpr (DIMS == 1)
    e1 = rd.chunk1_fast(g);  // a 1D code fits chunk 1
  else
    rd.chunks_fast(g, e1, sel, e2a, e2b);
  sched_fence();
  rd.lds_wait();  // one wait for the lookups (and the window's dwords)
  sched_fence();
  const uint64_t w = rd.window_w_make(wr);
  if constexpr (DIMS == 1) {
    e2 = 0;
  } else {
    // the chunk-2 entry by chunk 1's exit state, or none after a chunk 1 that
    // ended: one v_perm_b32 by the selector stored beside chunk 1's entry
    e2 = perm_sel(e2b, e2a, sel);
  }
  const uint32_t S = e1 + e2;
  const uint32_t nfp = nf + ent_pos(S);
  // One wave-uniform test for both rare cases: a code longer than the two
  // chunks (the sum carries the marker: it is negative) and one reaching
  // position N-1 (nf + npos >= N).  As one sign test: (nfp + 64 - N) << 25
  // has its sign bit set exactly when nfp >= N (nfp + 64 - N < 128), and the
  // OR with S keeps S's (bits 25-30 of both are don't-cares).
  // (the biased count laundered: the compiler otherwise distributes the shift,
  // (nfp << 25) + (64 - N) << 25, and re-materialises that constant every step)
  const int32_t rare = (int32_t)(S | ((N == 64 ? nfp : launder(nfp + (64u - N))) << 25));
  if (__builtin_expect(any_lane(rare < 0), 0)) {
    const auto pos0 = rd.pos;
    // The budget-aware resolution from the entries already read
    // (lut_finish) for the whole wave, and for the lanes it cannot finish
    // (none on the bench fields: tools/dec_paths.cpp) the general decoder.
    // Everything rare stays in this one branch, so the common path carries
    // no flag from it.
    // (design statistics, tools/dec_paths.cpp: why a lane is rare)
    ZFP_COUNT_PATH((S & kMarkerBit) ? 16 : (nfp >= N) ? 17 : 18);
    unsigned bits = rd.end - rd.pos;
    bool slow;
    PW x = lut_finish<DIMS, PW>(bits, n, rd, slow, nf, umin(nf, bits), w, e1, e2);
    n = umin(n, N - 1);
    ZFP_COUNT_PATH(slow ? 2 : 1);
    if (any_lane(slow)) {
      if (slow) {
        rd.init(pos0);
        n = nf;
        bits = rd.end - pos0;
        x = decode_plane<DIMS, PW>(bits, n, rd);
        n = umin(n, N - 1);
      }
    }
    // leave no LDS read of the rare paths in flight: the common path's wait
    // bookkeeping after the join then needs no extra waits of its own
    rd.lds_wait();
    return x;
  }
  ZFP_COUNT_PATH(0);
  // The budget: past its budget a block reads as zeros (it ends there), so a
  // code that ended did so within the budget or with the zero group test that
  // follows a one read with the budget's last bit: taken as read, min(used,
  // bits - nf) bits.  A lane with fewer than nf bits reads zeros for the rest
  // of its verbatim part and a "0" leading test past its block: a
  // verbatim-only plane, all its bits.  So the common path only clips the
  // advance at the budget.
  // (the ones: two ANDs with an inline constant and a v_lshl_or_b32 whose
  // shift count is the low 5 bits of e1 >> 11, chunk 1's positions)
  const uint32_t ones = ent_ones(e1) | (ent_ones(e2) << ((e1 >> kPosShift) & 31u));
  PW x;
  if constexpr (sizeof(PW) == 8) {
    // bits >= nf of the plane from the group code, below it verbatim: w with
    // its bits from nf on replaced by the ones, as w ^ (((w >> nf) ^ ones) <<
    // nf) -- two 64-bit shifts and three XORs where the mask ~0 << nf, the
    // shifted ones and two v_bfi_b32 took four slow-issue instructions
    x = (PW)(w ^ (((w >> nf) ^ (uint64_t)ones) << nf));
  } else {
    x = merge_at<PW>(nf, ones, w);
  }
  n = nfp;
  rd.pos = umin(rd.pos + nf + ent_used(S), rd.end);
  return x;
}

// Planes 31 .. cmin of 32-bit half H, two per loop trip, while any lane of the
// wave has budget (a lane without deposits zeros).  Returns the highest plane
// left unset (-1: none); those below it are unset too.
template <int H, typename UInt, int DIMS, typename Reader>
ZFP_HD int decode_half(planes<UInt, DIMS>& P, unsigned& n, int cmin, Reader& rd) {
  typedef typename plane_word<DIMS>::type PW;
  int c = 31;
  for (; c - 1 >= cmin; c -= 2) {
    if (!any_lane(rd.pos < rd.end)) return c;
    if constexpr (prio_of<Reader>::value)
      progress_priority<CUZFP_DPRIO_T2, CUZFP_DPRIO_T1, CUZFP_DPRIO_T0>(uniform(c));
    PW xa, xb;
    xa = decode_plane_fast_any<DIMS, PW>(n, rd);
    xb = decode_plane_fast_any<DIMS, PW>(n, rd);
    ZFP_STAMP(4);  // diagnostic builds: the last fast pair's end
    const int u = uniform(c);
    P.template set<H>(u, xa);
    P.template set<H>(u - 1, xb);
  }
  if (c >= cmin && c >= 0 && any_lane(rd.pos < rd.end)) {
    P.template set<H>(uniform(c), decode_plane_any<DIMS, PW>(n, rd));
    c--;
  }
  return c;
}

// decode_half with compile-time plane numbers (32-bit halves whose every lane
// decodes down to plane 0, the common case): each plane is a fixed register
// (no VGPR-relative or compare-select writes of a runtime plane number) and
// the priority drops sit at fixed trips.  Returns the highest plane left
// unset (-1: none), as decode_half.
// Planes left unset by the loop must read as zero.  In 3D (set() assigns a
// whole plane) only those are zeroed, after the loop; zeroing the whole array
// before it costs ~90 moves a wave (the compiler then also shuffles the array
// into the layout its indexed moves use).  1D/2D planes share registers and
// set() ORs, so that array is zeroed up front.  (CUZFP_EAGER_ZERO: zero up
// front in 3D too.)
// 3D 64-bit encoder: the low half's planes transposed in two parts
// (planes::load_split; 0: the whole block up front).  (The decoder's mirror
// image -- the inverse transpose from rows 16..31 when planes 15..0 are unset
// on every lane -- measured no gain, r06_ab_f64split.txt, and is not built.)
#ifndef CUZFP_F64_SPLIT
#define CUZFP_F64_SPLIT 1
#endif
#ifndef CUZFP_EAGER_ZERO
constexpr bool kLazyZero = true;
#else
constexpr bool kLazyZero = false;
#endif
// planes C .. 0 of half H set to zero (compile-time plane numbers)
template <int H, int C, typename UInt, int DIMS>
ZFP_HD void zero_fixed(planes<UInt, DIMS>& P) {
  if constexpr (C >= 0) {
    P.template set<H>(C, 0);
    zero_fixed<H, C - 1>(P);
  }
}

template <int H, int C, bool PRI = true, typename UInt, int DIMS, typename Reader>
ZFP_HD int decode_half_fixed(planes<UInt, DIMS>& P, unsigned& n, Reader& rd) {
  typedef typename plane_word<DIMS>::type PW;
  if constexpr (C >= 1) {
    if (!any_lane(rd.pos < rd.end)) {
      // the planes left: zero in 3D (set() assigns whole words there; 1D/2D
      // words were zeroed up front)
      if constexpr (kLazyZero && DIMS == 3) zero_fixed<H, C>(P);
      return C;
    }
#if defined(__HIP_DEVICE_COMPILE__) && !defined(CUZFP_NO_PRIO)
    if constexpr (prio_of<Reader>::value && PRI) {
      if constexpr (C == CUZFP_DPRIO_T2) __builtin_amdgcn_s_setprio(2);
      else if constexpr (C == CUZFP_DPRIO_T1) __builtin_amdgcn_s_setprio(1);
      else if constexpr (C == CUZFP_DPRIO_T0) __builtin_amdgcn_s_setprio(0);
    }
#endif
    const PW xa = decode_plane_fast_any<DIMS, PW>(n, rd);
    const PW xb = decode_plane_fast_any<DIMS, PW>(n, rd);
    ZFP_STAMP(4);  // diagnostic builds: the last pair's end
    P.template set<H>(C, xa);
    P.template set<H>(C - 1, xb);
    return decode_half_fixed<H, C - 2, PRI>(P, n, rd);
  }
  return C;
}


template <int H, typename UInt, int DIMS>
ZFP_HD void zero_planes(planes<UInt, DIMS>& P, int c) {
  if constexpr (kLazyZero && DIMS == 3)
    for (; c >= 0; c--) P.template set<H>(uniform(c), 0);
}

// Readers that hold the 1D plane table (dec1d(byte offset) reads an entry,
// bits8() the next 8 stream bits, zeros past the block)
template <typename T, typename = void> struct has_dec1d {
  static constexpr bool value = false;
};
template <typename T> struct has_dec1d<T, decltype((void)&T::dec1d)> {
  static constexpr bool value = true;
};

// Planes C, C-1, ... 0 of 32-bit half H of a 1D block, one lookup each
// (Plane1dDecLut), while any lane of the wave has budget (tested every other
// plane; a lane without budget looks up c = 0: nothing read, nothing set).
// n12 = n << 12, the byte offset of n's part of the table.
template <int H, int C, typename UInt, typename Reader>
ZFP_HD void decode_planes_1d(planes<UInt, 1>& P, uint32_t& n12, Reader& rd) {
  if constexpr (C >= 0) {
    if constexpr (C & 1)
      if (!any_lane(rd.pos < rd.end)) return;
    // (c << 9 | n12: one v_lshl_or_b32, s << 1 | that: another)
    const uint32_t c = umin(rd.end - rd.pos, 7u);
    const uint32_t e = rd.dec1d((rd.bits8() << 1) | ((c << 9) | n12));
    P.template set<H>(C, e & 15u);
    rd.pos += (e >> 4) & 15u;
    n12 = e & 0x3000u;
    decode_planes_1d<H, C - 1>(P, n12, rd);
  }
}

// Returns the highest plane left unset by a 32-bit coefficients' loop (-1:
// none; every plane below it is unset too), 31 otherwise (nothing known).
template <typename UInt, int DIMS, typename Reader>
ZFP_HD int decode_planes(planes<UInt, DIMS>& P, unsigned budget, unsigned maxprec, Reader& rd) {
  constexpr int PREC = (int)sizeof(UInt) * 8;
  unsigned n = 0;
  rd.end = rd.pos + budget;  // the reader never passes it
  if constexpr (!(kLazyZero && DIMS == 3)) P.zero();
  if constexpr (PREC == 32) {
    // every plane down to 0 (see encode_planes); the early exits of the
    // unrolled loop zero what they leave
    (void)maxprec;
    if constexpr (DIMS == 1 && has_dec1d<Reader>::value) {
      uint32_t n12 = 0;
      decode_planes_1d<0, 31>(P, n12, rd);
      return 31;
    }
    return decode_half_fixed<0, 31>(P, n, rd);
  } else {
    const int kmin = PREC > (int)maxprec ? PREC - (int)maxprec : 0;
    if constexpr (DIMS == 1 && has_dec1d<Reader>::value) {
      if (!any_lane(kmin != 0)) {  // every lane decodes down to plane 0
        uint32_t n12 = 0;
        decode_planes_1d<1, 31>(P, n12, rd);
        decode_planes_1d<0, 31>(P, n12, rd);
        return 31;
      }
    }
    // (64-bit values keep the rolled loop: unrolled, the f64 decoder measured
    // 61.8 -> 71.2 us at 256^3 rate 16 and took minutes to compile)
    zero_planes<1>(P, decode_half<1>(P, n, kmin > 32 ? kmin - 32 : 0, rd));
    if (kmin >= 32) {
      zero_planes<0>(P, 31);
      return 31;
    }
    zero_planes<0>(P, decode_half<0>(P, n, kmin, rd));
  }
  return 31;
}

// ---------------------------------------------------------------------------
// Block exponent and the float <-> int casts.

template <typename Scalar> struct fp;

template <> struct fp<float> {
  // exponent of max |x| (encode.c:9-33): frexp exponent, clamped to -126 for
  // denormals, -127 for an all-zero block; frexp(inf) gives 0 (glibc).  fmaxf
  // ignores NaNs exactly as the reference's `if (max < f)` loop does.
  template <int N>
  ZFP_HD static int emax(const float* f) {
    float m = 0.0f;
#pragma unroll
    for (int i = 0; i < N; i++) m = fmaxf(m, fabsf(f[i]));
    uint32_t b = __float_as_uint_(m);
    int E = (int)(b >> 23);
    if (b == 0) return -127;
    return E == 255 ? 0 : E - 126;
  }
  // 2^e as a float, e in [-160, 160], with IEEE underflow / overflow
  ZFP_HD static float pow2(int e) {
    if (e > 127) return __uint_as_float_(0x7f800000u);
    if (e >= -126) return __uint_as_float_((uint32_t)(e + 127) << 23);
    if (e >= -149) return __uint_as_float_(1u << (e + 149));
    return 0.0f;  // 2^-150 rounds (to even) to zero, like ldexpf
  }
  // (Int)(s * x) with x86-64 cvttss2si semantics: NaN or |y| >= 2^31 -> INT_MIN
  ZFP_HD static int32_t to_int(float y) {
    return fabsf(y) < 2147483648.0f ? (int32_t)y : (int32_t)0x80000000u;
  }
  ZFP_HD static float from_int(int32_t q) { return (float)q; }
  ZFP_HD static uint32_t __float_as_uint_(float f) { union { float f; uint32_t u; } c; c.f = f; return c.u; }
  ZFP_HD static float __uint_as_float_(uint32_t u) { union { float f; uint32_t u; } c; c.u = u; return c.f; }
};

template <> struct fp<double> {
  template <int N>
  ZFP_HD static int emax(const double* f) {
    double m = 0.0;
#pragma unroll
    for (int i = 0; i < N; i++) m = fmax(m, fabs(f[i]));
    uint64_t b = as_u64(m);
    int E = (int)(b >> 52);
    if (b == 0) return -1023;
    return E == 2047 ? 0 : E - 1022;
  }
  ZFP_HD static double pow2(int e) {
    if (e > 1023) return as_f64(0x7ff0000000000000ull);
    if (e >= -1022) return as_f64((uint64_t)(e + 1023) << 52);
    if (e >= -1074) return as_f64(1ull << (e + 1074));
    return 0.0;
  }
  ZFP_HD static int64_t to_int(double y) {
    return fabs(y) < 9223372036854775808.0 ? (int64_t)y : (int64_t)0x8000000000000000ull;
  }
  ZFP_HD static double from_int(int64_t q) { return (double)q; }
  ZFP_HD static uint64_t as_u64(double f) { union { double f; uint64_t u; } c; c.f = f; return c.u; }
  ZFP_HD static double as_f64(uint64_t u) { union { double f; uint64_t u; } c; c.u = u; return c.f; }
};

// ---------------------------------------------------------------------------
// Whole-block encode / decode.
// Writer: full() is true once the block's maxbits bits are written; while it is
//   false, put(value, n) appends n <= 64 low bits (value has no bits at or
//   above n; bits past maxbits are dropped) and zero_bit() appends one 0;
//   finish() zero-pads the block to maxbits; settle() is called before each
//   plane step and lets a full writer take (and discard) further steps.
// Reader: peek() returns the next 64 stream bits, skip(n) consumes n <= 64.

#if defined(__HIP_DEVICE_COMPILE__)
// max |f[i]| over an even number of floats, NaN if any is NaN: v_maximum3_f32
// with |.| source modifiers, four independent chains
template <int N>
__device__ __forceinline__ float absmax_nan(const float* f) {
  constexpr int C = N >= 16 ? 4 : 1;
  float m[C];
#pragma unroll
  for (int c = 0; c < C; c++) m[c] = 0.0f;
#pragma unroll
  for (int i = 0; i < N; i += 2) {
    float& a = m[(i / 2) % C];
    asm("v_maximum3_f32 %0, |%1|, |%2|, %0" : "+v"(a) : "v"(f[i]), "v"(f[i + 1]));
  }
  if constexpr (C == 4) {
    asm("v_maximum3_f32 %0, %0, %1, %2" : "+v"(m[0]) : "v"(m[1]), "v"(m[2]));
    asm("v_maximum3_f32 %0, %0, %1, %1" : "+v"(m[0]) : "v"(m[3]));
  }
  return m[0];
}
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// q = (Int)(s * f) for an even number of floats, with the reference's x86 cast
// (cvttss2si: NaN or |y| >= 2^31 -> INT_MIN).  fast: a block of finite values
// with a finite scale, where |y| < 2^30 (max |x| < 2^emax), so v_cvt_i32_f32's
// truncation is the x86 cast and the product pairs go through v_pk_mul_f32;
// otherwise the exact path (encode.c:35-52, oracle/zfp_oracle.c).
template <int N>
__device__ __forceinline__ void quantize_f32(const float* f, float s, bool fast, uint32_t* q) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  // 1D/2D: one path for the whole wave (the exact one is right for every
  // block): a per-lane choice is if-converted for these small blocks, i.e.
  // both paths run.  (3D keeps the per-lane branch the compiler lays out.)
  if constexpr (N <= 16) fast = !any_lane(!fast);
  if (fast) {
    const f2 ss = {s, s};
#pragma unroll
    for (int i = 0; i < N; i += 2) {
      const f2 y = f2{f[i], f[i + 1]} * ss;
      q[i] = (uint32_t)(int32_t)y.x;  // v_cvt_i32_f32 (|y| < 2^30 here)
      q[i + 1] = (uint32_t)(int32_t)y.y;
    }
  }
  if (fast) {
  } else {
    // Two values per statement, in place (tied operands), so the quantised
    // block reuses the input registers instead of doubling the block's
    // register footprint.  Each compare result is read >= 2 instructions
    // after it is written (VALU SGPR/VCC write -> v_cndmask read).
    const float lim = 2147483648.0f;
    const uint32_t imin = 0x80000000u;
#pragma unroll
    for (int i = 0; i < N; i += 2) {
      float a = f[i], b = f[i + 1];
      uint64_t m;
      uint32_t t;
      asm("v_mul_f32 %0, %0, %4\n\t"
          "v_mul_f32 %1, %1, %4\n\t"
          "v_cmp_gt_f32_e64 vcc, %5, |%0|\n\t"
          "v_cmp_gt_f32_e64 %2, %5, |%1|\n\t"
          "v_cvt_i32_f32 %3, %0\n\t"
          "v_cndmask_b32 %0, %6, %3, vcc\n\t"
          "v_cvt_i32_f32 %3, %1\n\t"
          "v_cndmask_b32_e64 %1, %6, %3, %2"
          : "+v"(a), "+v"(b), "=&s"(m), "=&v"(t)
          : "v"(s), "v"(lim), "v"(imin)
          : "vcc");
      q[i] = __builtin_bit_cast(uint32_t, a);
      q[i + 1] = __builtin_bit_cast(uint32_t, b);
    }
  }
}
#endif

template <typename Scalar, int DIMS, typename Writer>
ZFP_HD void encode_block(const Scalar* f, unsigned maxbits, Writer& wr) {
  typedef traits<Scalar> T;
  typedef typename T::Int Int;
  typedef typename T::UInt UInt;
  constexpr int N = 1 << (2 * DIMS);
  UInt q[N];
  unsigned maxprec = T::prec;
  (void)maxbits;  // the writer owns the budget
  if constexpr (!T::is_int) {
    // encode.c:187-216
#if defined(__HIP_DEVICE_COMPILE__)
    // f32 blocks of an even size: max |x| with NaN-propagating v_maximum3_f32,
    // so that one class test says whether the block is finite (the fast path
    // below); only a block holding inf or NaN computes the reference's
    // NaN-ignoring maximum as well.
    bool finite = false;
    int emax;
    if constexpr (sizeof(Scalar) == 4 && N % 2 == 0) {
      const float mx = absmax_nan<N>((const float*)f);
      finite = __builtin_isfinite(mx);
      if (__builtin_expect(finite, 1)) {
        const uint32_t bm = __builtin_bit_cast(uint32_t, mx);
        emax = bm ? (int)(bm >> 23) - 126 : -127;
      } else {
        emax = fp<Scalar>::template emax<N>((const Scalar*)f);
      }
    } else {
      emax = fp<Scalar>::template emax<N>((const Scalar*)f);
    }
#else
    const int emax = fp<Scalar>::template emax<N>((const Scalar*)f);
#endif
    ZFP_STAMP(1);
    maxprec = precision<DIMS>(emax, T::prec);
    const unsigned e = maxprec ? (unsigned)(emax + T::ebias) : 0u;
    // all-zero block: a single 0 bit, then padding (encode.c:206-215)
    bool zero = !e;
    if constexpr (zero_inline_of<Writer>::value) {
      // ... coded inline: marked full (its bits all go to the discarded
      // slack, its column stays zero), quantised with a zero scale (q = 0);
      // a wave of zero blocks returns at once
      if (!any_lane(!zero)) {
        wr.finish();
        return;
      }
      wr.mark_full(zero);
    } else if (zero) {
      wr.finish();
      return;
    }
    wr_head(wr, 2ull * e + 1, T::ebits + 1);
    // q = (Int)(2^sh * x) with the reference's x86 cast: NaN or |y| >= 2^(p-1)
    // gives INT_MIN.  That happens when 2^sh overflows (max |x| < 2^-97 for
    // f32, 2^-961 for f64) and in blocks holding inf or NaN; see
    // oracle/zfp_oracle.c.
    Scalar s = (Scalar)fp<Scalar>::pow2(T::prec - 2 - emax);
    if constexpr (zero_inline_of<Writer>::value) s = zero ? (Scalar)0 : s;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (sizeof(Scalar) == 4 && N % 2 == 0) {
      quantize_f32<N>((const float*)f, (float)s, finite && (emax >= -97 || zero), (uint32_t*)q);
    } else
#endif
    {
#pragma unroll
      for (int i = 0; i < N; i++) q[i] = (UInt)fp<Scalar>::to_int(s * (Scalar)f[i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < N; i++) q[i] = (UInt)(Int)f[i];
  }
  fwd_xform<DIMS>(q);
  UInt u[N];
  constexpr UInt NB = nbmask<UInt>::value;
  permute_fwd_add<DIMS>(q, u, NB, make_seq<N>());  // "^ NB" in P.load<true>
  ZFP_STAMP(2);
#if defined(CUZFP_PROBE) && (CUZFP_PROBE == 1 || CUZFP_PROBE == 2)
  // timing probes (tools/probe.py; never built into the product library):
  // 1 = no plane coder, 2 = no transpose either
  uint64_t acc = 0;
#if CUZFP_PROBE == 1
  planes<UInt, DIMS> P;
  P.load(u);
#pragma unroll
  for (int k = 0; k < (int)sizeof(UInt) * 8; k++) acc ^= (uint64_t)P.get(k) << (k & 7);
#else
#pragma unroll
  for (int i = 0; i < N; i++) acc ^= (uint64_t)u[i] << (i & 31);
#endif
  wr.put(acc, 64);
  (void)maxprec;
#else
  planes<UInt, DIMS> P;
  if constexpr (DIMS == 2 && sizeof(UInt) == 4) {
    // 2D 32-bit blocks: planes 31..16 from the high tile alone (load_hi),
    // the low tile only if some lane of the wave still has budget after
    // plane 16 (never at BASELINE's 2D rate 2, whose blocks stop above plane
    // 20).  (precision() is 32 here: every plane down to 0, as encode_planes.)
    P.template load_hi<true>(u);
    ZFP_STAMP(3);
    (void)maxprec;
    unsigned n = 0;
    if (encode_half_fixed<0, 31, true, 16>(P, n, wr)) {
      P.template load<true>(u);
      encode_half_fixed<0, 15>(P, n, wr);
    }
  } else if constexpr (CUZFP_F64_SPLIT && DIMS == 3 && sizeof(UInt) == 8 && zero_inline_of<Writer>::value) {
    // 3D 64-bit blocks: the low half's tiles transposed a 16-plane part at a
    // time, each only if some lane of the wave still has budget
    // (planes::load_split), in the lane-interleaved image's kernels (with the
    // bit-packed image the kernel spills in its main path).  One consumer of u: a second layout of u for a
    // separate rolled path made the kernel spill in its main path.
    planes<UInt, DIMS> PS;
    PS.template load_split<true>(u);
    ZFP_STAMP(3);
    unsigned n = 0;
    if (__builtin_expect(!any_lane(maxprec != T::prec), 1)) {  // normal doubles, int64: down to plane 0
      if (encode_half_fixed<1, 31>(PS, n, wr)) {
        PS.template lo_part<true, true>();
        if (encode_half_fixed<0, 31, false, 16>(PS, n, wr)) {
          PS.template lo_part<true, false>();
          encode_half_fixed<0, 15, false>(PS, n, wr);
        }
      }
    } else {  // some lane stops above plane 0: encode_planes' rolled loops
      PS.template lo_part<true, true>();
      PS.template lo_part<true, false>();
      const int kmin = 64 - (int)maxprec;
      if (encode_half<1>(PS, n, kmin > 32 ? kmin - 32 : 0, wr)) encode_half<0>(PS, n, kmin, wr);
    }
  } else {
    P.template load<true>(u);
    ZFP_STAMP(3);
    encode_planes<UInt, DIMS>(P, maxprec, wr);
  }
  ZFP_STAMP(4);
#endif
  wr.finish();
}

// Returns false, leaving f untouched, when every lane of the wave holds a
// zero block (the caller stores zeros: zeroing f here costs the kernel 64
// register moves a wave, made on every path before the branch); a zero block
// beside coded ones decodes to +0 values (see below).  On the host a "wave"
// is one lane.
template <typename Scalar, int DIMS, typename Reader>
ZFP_HD bool decode_block(Scalar* f, unsigned maxbits, Reader& rd) {
  typedef traits<Scalar> T;
  typedef typename T::Int Int;
  typedef typename T::UInt UInt;
  constexpr int N = 1 << (2 * DIMS);
  unsigned budget = maxbits, maxprec = T::prec;
  int emax = 0;
  if constexpr (!T::is_int) {
    // decode.c:352-381
    const uint64_t head = rd.peek();
    const bool coded = head & 1;
    // A zero block (decode.c:354-355) takes the coded path with no budget
    // inside a wave that holds coded blocks: it reads no planes, so its q
    // are zero and its values 0 * 2^(emax-p+2) = +0 whatever its header bits
    // -- the reference's zero block -- and the plane loop is not nested in a
    // per-lane branch (whose exec-mask bookkeeping costs every plane step).
    // A wave of zero blocks returns at once.
    if (!any_lane(coded)) return false;
    emax = (int)((head >> 1) & lowmask(T::ebits)) - T::ebias;
    const auto start = rd.pos;
    rd.skip(T::ebits + 1);
    maxprec = precision<DIMS>(emax, T::prec);
    budget = coded ? maxbits - (T::ebits + 1) : 0u;
    // (the plane steps take the stream as zeros past the budget's end, which
    // a zero block's bits need not be: its reads start at the block's end,
    // where the readers hold zeros)
    if (!coded) rd.pos = start + maxbits;
  }
  UInt u[N];
#if defined(CUZFP_PROBE) && CUZFP_PROBE == 2
  {
    const uint64_t base = rd.peek();
    (void)budget;
#pragma unroll
    for (int i = 0; i < N; i++) u[i] = (UInt)(base >> (i & 31)) + (UInt)i;
  }
#elif defined(CUZFP_PROBE) && CUZFP_PROBE == 1
  planes<UInt, DIMS> P;
  {
    const uint64_t base = rd.peek();
    (void)budget;
#pragma unroll
    for (int k = 0; k < (int)sizeof(UInt) * 8; k++)
      P.set(k, (typename plane_word<DIMS>::type)((base >> (k & 15)) ^ (uint64_t)k));
  }
  P.store(u);
#else
  planes<UInt, DIMS> P;
  const int unset = decode_planes<UInt, DIMS>(P, budget, maxprec, rd);
  (void)unset;
#if defined(__HIP_DEVICE_COMPILE__) && !defined(CUZFP_NO_PRIO) && CUZFP_DPRIO_AFTER >= 0
  if constexpr (prio_of<Reader>::value) __builtin_amdgcn_s_setprio(CUZFP_DPRIO_AFTER);  // see progress_priority
#endif
  ZFP_STAMP(1);
  UInt q[N];
  constexpr UInt NB = nbmask<UInt>::value;
  if constexpr (DIMS == 2 && sizeof(UInt) == 4) {
    // planes 15..0 unset on every lane of the wave (a wave-uniform loop
    // exit): the high tile alone, coefficients finished by store_hi
    if (unset >= 15) {
      P.template store_hi<true>(u);  // (u ^ NB) - NB
      permute_inv_copy<DIMS>(u, q, make_seq<N>());
    } else {
      P.template store<true>(u);  // u ^ NB
      permute_inv_sub<DIMS>(u, q, NB, make_seq<N>());  // (u ^ NB) - NB
    }
    ZFP_STAMP(2);
  } else {
    P.template store<true>(u);  // u ^ NB
    ZFP_STAMP(2);
    permute_inv_sub<DIMS>(u, q, NB, make_seq<N>());  // (u ^ NB) - NB
  }
#endif
#if defined(CUZFP_PROBE) && (CUZFP_PROBE == 1 || CUZFP_PROBE == 2)
  UInt q[N];
  constexpr UInt NB = nbmask<UInt>::value;
  permute_inv<DIMS>(u, q, NB, make_seq<N>());
#endif
  inv_xform<DIMS>(q);
  ZFP_STAMP(3);
  if constexpr (!T::is_int) {
    const Scalar s = (Scalar)fp<Scalar>::pow2(emax - (T::prec - 2));
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (sizeof(Scalar) == 4 && N % 2 == 0) {
      // two values per v_pk_mul_f32 (the same IEEE product as v_mul_f32)
      typedef float f2 __attribute__((ext_vector_type(2)));
      const f2 ss = {(float)s, (float)s};
#pragma unroll
      for (int i = 0; i < N; i += 2) {
        const f2 v = f2{(float)(Int)q[i], (float)(Int)q[i + 1]} * ss;
        f[i] = (Scalar)v.x;
        f[i + 1] = (Scalar)v.y;
      }
    } else
#endif
    if constexpr (sizeof(Scalar) == 8) {
      // (double)q as fma(hi, 2^32, lo): hi * 2^32 and lo are exact, so the
      // one rounding of the fused sum is the conversion's (the compiler's form
      // is two conversions, an ldexp and an add): 256^3 rate 16 decode 54.5 ->
      // 54.2 us (tools/variants.py, r04_ahead.txt)
#pragma unroll
      for (int i = 0; i < N; i++) {
        const int64_t v = (int64_t)(Int)q[i];
        const double d = __builtin_fma((double)(int32_t)(v >> 32), 4294967296.0, (double)(uint32_t)v);
        f[i] = (Scalar)(s * d);
      }
    } else {
#pragma unroll
      for (int i = 0; i < N; i++) f[i] = (Scalar)(s * (Scalar)(Int)q[i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < N; i++) f[i] = (Scalar)(Int)q[i];
  }
  return true;
}

// ---------------------------------------------------------------------------
// Partial-block padding (encode.c:54-74 pad_block, applied along x, y, z by
// encode3.c:284-301).  It is separable: padded index i of an edge with n valid
// values reads source index pad_src(i, n).

ZFP_HD int pad_src(int i, int n) { return i < n ? i : (i == 3 ? 0 : n - 1); }

}  // namespace cuzfp
