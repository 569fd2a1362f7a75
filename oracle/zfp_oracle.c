/*
 * oracle/zfp_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the zfp 0.5.0 fixed-rate codec, the ground truth of
 * the reference's differential harness (mclarsen/cuZFP src/utils/test.py:68-93).
 * It is the checker for the HIP codec in cuzfp_amd/: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * Citations are relative to /root/reference/src/thirdparty_builtin/zfp-0.5.0/
 * unless they start with src/cuZFP.  Pinned bit-exact against the reference
 * itself (oracle/_ref/libzfp_ref.so) and against tests/golden/ fixtures.
 *
 * Restatement choices (behaviour identical to the reference):
 *   - fixed rate means minbits == maxbits, so block b occupies stream bits
 *     [b*maxbits, (b+1)*maxbits) and every bit it does not write is zero
 *     (encode.c:166-169 stream_pad, zfp.c:627 stream_flush).  The restatement
 *     therefore writes each block at its absolute bit offset into a zeroed
 *     buffer instead of streaming sequentially.
 *   - the float->int cast `(Int)(s * x)` (encode.c:50) is undefined in C when
 *     the product is out of range or NaN; the reference build (gcc, x86-64,
 *     SSE cvttss2si / cvttsd2si) yields the "integer indefinite" value INT_MIN.
 *     That happens for f32 blocks whose max |x| < 2^-97 (the scale factor
 *     ldexpf(1, 30 - emax) overflows to +inf) and for f64 blocks with
 *     max |x| < 2^-961.  We spell that result out.
 */
#include "zfp_oracle.h"

#include <limits.h>
#include <math.h>
#include <string.h>

#define TYPE_INT32 1
#define TYPE_INT64 2
#define TYPE_FLOAT 3
#define TYPE_DOUBLE 4
#define ZFP_MIN_EXP (-1074) /* inc/zfp.h:80 */

/* ------------------------------------------------------------------------ */
/* bit access on a zeroed stream of 64-bit words, LSB first                   */
/* (inline/bitstream.c:194-220: bits enter each word at its low end)          */

static void put_bit(uint64_t* s, size_t pos, unsigned bit)
{
  s[pos >> 6] |= (uint64_t)(bit & 1u) << (pos & 63);
}

static unsigned get_bit(const uint64_t* s, size_t pos)
{
  return (unsigned)(s[pos >> 6] >> (pos & 63)) & 1u;
}

/* ------------------------------------------------------------------------ */
/* coefficient orderings: template/codec1.c:2-5, codec2.c:3-27, codec3.c:3-88 */
/* (order by total degree i+j+k, then by i^2+j^2+k^2)                          */

#define I2(i, j) ((i) + 4 * (j))
#define I3(i, j, k) ((i) + 4 * ((j) + 4 * (k)))
static const unsigned char PERM1[4] = {0, 1, 2, 3};
static const unsigned char PERM2[16] = {
  I2(0,0), I2(1,0), I2(0,1), I2(1,1), I2(2,0), I2(0,2), I2(2,1), I2(1,2),
  I2(3,0), I2(0,3), I2(2,2), I2(3,1), I2(1,3), I2(3,2), I2(2,3), I2(3,3)};
static const unsigned char PERM3[64] = {
  I3(0,0,0),
  I3(1,0,0), I3(0,1,0), I3(0,0,1),
  I3(0,1,1), I3(1,0,1), I3(1,1,0), I3(2,0,0), I3(0,2,0), I3(0,0,2),
  I3(1,1,1), I3(2,1,0), I3(2,0,1), I3(0,2,1), I3(1,2,0), I3(1,0,2), I3(0,1,2),
  I3(3,0,0), I3(0,3,0), I3(0,0,3),
  I3(2,1,1), I3(1,2,1), I3(1,1,2), I3(0,2,2), I3(2,0,2), I3(2,2,0),
  I3(3,1,0), I3(3,0,1), I3(0,3,1), I3(1,3,0), I3(1,0,3), I3(0,1,3),
  I3(1,2,2), I3(2,1,2), I3(2,2,1), I3(3,1,1), I3(1,3,1), I3(1,1,3),
  I3(3,2,0), I3(3,0,2), I3(0,3,2), I3(2,3,0), I3(2,0,3), I3(0,2,3),
  I3(2,2,2),
  I3(3,2,1), I3(3,1,2), I3(1,3,2), I3(2,3,1), I3(2,1,3), I3(1,2,3),
  I3(0,3,3), I3(3,0,3), I3(3,3,0),
  I3(3,2,2), I3(2,3,2), I3(2,2,3), I3(1,3,3), I3(3,1,3), I3(3,3,1),
  I3(2,3,3), I3(3,2,3), I3(3,3,2),
  I3(3,3,3)};

static const unsigned char* perm_for(unsigned dims)
{
  return dims == 1 ? PERM1 : dims == 2 ? PERM2 : PERM3;
}

/* ------------------------------------------------------------------------ */
/* Integer block coder, instantiated for 32- and 64-bit integers.            */
/*  fwd_lift / inv_lift        template/encode.c:76-103, decode.c:243-270     */
/*  int2uint / uint2int        encode.c:105-110, decode.c:272-277              */
/*  fwd_xform / inv_xform      encode1.c:172-178, encode2.c:232-243,           */
/*                             encode3.c:303-320; decode{1,2,3}.c inv_xform    */
/*  encode_ints / decode_ints  encode.c:121-151, decode.c:288-321              */
/* Arithmetic is done on the unsigned type so wrap-around is defined; `>>`    */
/* on the signed type is arithmetic (as on every target the reference ran). */

#define DEFINE_INT_CODEC(SFX, Int, UInt, INTPREC, NBMASK)                          \
static void fwd_lift_##SFX(Int* p, unsigned s)                                     \
{                                                                                  \
  UInt x = (UInt)p[0], y = (UInt)p[s], z = (UInt)p[2 * s], w = (UInt)p[3 * s];     \
  x += w; x = (UInt)((Int)x >> 1); w -= x;                                         \
  z += y; z = (UInt)((Int)z >> 1); y -= z;                                         \
  x += z; x = (UInt)((Int)x >> 1); z -= x;                                         \
  w += y; w = (UInt)((Int)w >> 1); y -= w;                                         \
  w += (UInt)((Int)y >> 1); y -= (UInt)((Int)w >> 1);                              \
  p[0] = (Int)x; p[s] = (Int)y; p[2 * s] = (Int)z; p[3 * s] = (Int)w;             \
}                                                                                  \
static void inv_lift_##SFX(Int* p, unsigned s)                                     \
{                                                                                  \
  UInt x = (UInt)p[0], y = (UInt)p[s], z = (UInt)p[2 * s], w = (UInt)p[3 * s];     \
  y += (UInt)((Int)w >> 1); w -= (UInt)((Int)y >> 1);                              \
  y += w; w <<= 1; w -= y;                                                         \
  z += x; x <<= 1; x -= z;                                                         \
  y += z; z <<= 1; z -= y;                                                         \
  w += x; x <<= 1; x -= w;                                                         \
  p[0] = (Int)x; p[s] = (Int)y; p[2 * s] = (Int)z; p[3 * s] = (Int)w;             \
}                                                                                  \
static void fwd_xform_##SFX(Int* p, unsigned dims)                                 \
{                                                                                  \
  unsigned a, b;                                                                   \
  if (dims == 1) { fwd_lift_##SFX(p, 1); return; }                                 \
  if (dims == 2) {                                                                 \
    for (a = 0; a < 4; a++) fwd_lift_##SFX(p + 4 * a, 1); /* along x */            \
    for (a = 0; a < 4; a++) fwd_lift_##SFX(p + a, 4);     /* along y */            \
    return;                                                                        \
  }                                                                                \
  for (b = 0; b < 4; b++) for (a = 0; a < 4; a++) fwd_lift_##SFX(p + 4 * a + 16 * b, 1); \
  for (b = 0; b < 4; b++) for (a = 0; a < 4; a++) fwd_lift_##SFX(p + a + 16 * b, 4);     \
  for (b = 0; b < 4; b++) for (a = 0; a < 4; a++) fwd_lift_##SFX(p + a + 4 * b, 16);     \
}                                                                                  \
static void inv_xform_##SFX(Int* p, unsigned dims)                                 \
{                                                                                  \
  unsigned a, b;                                                                   \
  if (dims == 1) { inv_lift_##SFX(p, 1); return; }                                 \
  if (dims == 2) {                                                                 \
    for (a = 0; a < 4; a++) inv_lift_##SFX(p + a, 4);     /* along y */            \
    for (a = 0; a < 4; a++) inv_lift_##SFX(p + 4 * a, 1); /* along x */            \
    return;                                                                        \
  }                                                                                \
  for (b = 0; b < 4; b++) for (a = 0; a < 4; a++) inv_lift_##SFX(p + a + 4 * b, 16);     \
  for (b = 0; b < 4; b++) for (a = 0; a < 4; a++) inv_lift_##SFX(p + a + 16 * b, 4);     \
  for (b = 0; b < 4; b++) for (a = 0; a < 4; a++) inv_lift_##SFX(p + 4 * a + 16 * b, 1); \
}                                                                                  \
/* Embedded coding of `size` coefficients, most significant bit plane first,   \
 * at most `budget` bits written starting at stream bit `pos`.  Returns bits    \
 * written (encode.c:121-151).  Per plane k: the first n bits (coefficients     \
 * already known significant) verbatim, then a group test (is any remaining     \
 * bit set?) followed, when set, by the bits up to and including the next one  \
 * -- the last position's one being implied -- repeated until the test fails.  \
 * Every write is skipped once the budget is spent, so the output is a prefix. */ \
static unsigned encode_ints_##SFX(uint64_t* s, size_t pos, unsigned budget,      \
                                  unsigned maxprec, const UInt* u, unsigned size) \
{                                                                                  \
  unsigned kmin = INTPREC > maxprec ? INTPREC - maxprec : 0;                       \
  unsigned bits = budget, n = 0, i;                                                \
  int k;                                                                           \
  for (k = INTPREC - 1; bits && k >= (int)kmin; k--) {                             \
    uint64_t x = 0;                                                                \
    for (i = 0; i < size; i++) x |= (uint64_t)((u[i] >> k) & 1u) << i;             \
    for (i = 0; i < n && bits; i++, bits--) put_bit(s, pos++, (unsigned)(x >> i) & 1u); \
    while (n < size && bits) {                                                     \
      unsigned any = (x >> n) != 0;                                                \
      bits--; put_bit(s, pos++, any);                                              \
      if (!any) break;                                                             \
      while (n < size - 1 && bits) {                                               \
        unsigned b = (unsigned)(x >> n) & 1u;                                      \
        bits--; put_bit(s, pos++, b);                                              \
        if (b) break;                                                              \
        n++;                                                                       \
      }                                                                            \
      n++;                                                                         \
    }                                                                              \
  }                                                                                \
  return budget - bits;                                                            \
}                                                                                  \
/* decode.c:288-321.  Mirrors the encoder; note that when the budget runs out  \
 * inside a run of zeros the decoder still deposits a one at the current       \
 * position (the `x += 1 << n++` step of decode.c:311), which we keep.          */ \
static unsigned decode_ints_##SFX(const uint64_t* s, size_t pos, unsigned budget,\
                                  unsigned maxprec, UInt* u, unsigned size)        \
{                                                                                  \
  unsigned kmin = INTPREC > maxprec ? INTPREC - maxprec : 0;                       \
  unsigned bits = budget, n = 0, i;                                                \
  int k;                                                                           \
  for (i = 0; i < size; i++) u[i] = 0;                                             \
  for (k = INTPREC - 1; bits && k >= (int)kmin; k--) {                             \
    uint64_t x = 0;                                                                \
    for (i = 0; i < n && bits; i++, bits--) x |= (uint64_t)get_bit(s, pos++) << i; \
    while (n < size && bits) {                                                     \
      bits--;                                                                      \
      if (!get_bit(s, pos++)) break;                                               \
      while (n < size - 1 && bits) {                                               \
        bits--;                                                                    \
        if (get_bit(s, pos++)) break;                                              \
        n++;                                                                       \
      }                                                                            \
      x |= (uint64_t)1 << n;                                                       \
      n++;                                                                         \
    }                                                                              \
    for (i = 0; i < size; i++) u[i] |= (UInt)((x >> i) & 1u) << k;                \
  }                                                                                \
  return budget - bits;                                                            \
}                                                                                  \
/* encode_block (encode.c:153-171) minus the padding, which the zeroed fixed  \
 * layout provides: transform, reorder + negabinary, embedded coding.        */  \
static void encode_int_block_##SFX(uint64_t* s, size_t pos, unsigned budget,     \
                                   unsigned maxprec, Int* q, unsigned dims)        \
{                                                                                  \
  UInt u[64];                                                                      \
  const unsigned char* perm = perm_for(dims);                                      \
  unsigned size = 1u << (2 * dims), i;                                             \
  fwd_xform_##SFX(q, dims);                                                        \
  for (i = 0; i < size; i++) u[i] = ((UInt)q[perm[i]] + NBMASK) ^ NBMASK;          \
  encode_ints_##SFX(s, pos, budget, maxprec, u, size);                             \
}                                                                                  \
static void decode_int_block_##SFX(const uint64_t* s, size_t pos, unsigned budget,\
                                   unsigned maxprec, Int* q, unsigned dims)        \
{                                                                                  \
  UInt u[64];                                                                      \
  const unsigned char* perm = perm_for(dims);                                      \
  unsigned size = 1u << (2 * dims), i;                                             \
  decode_ints_##SFX(s, pos, budget, maxprec, u, size);                             \
  for (i = 0; i < size; i++) q[perm[i]] = (Int)((u[i] ^ NBMASK) - NBMASK);         \
  inv_xform_##SFX(q, dims);                                                        \
}

DEFINE_INT_CODEC(i32, int32_t, uint32_t, 32u, (uint32_t)0xaaaaaaaau)
DEFINE_INT_CODEC(i64, int64_t, uint64_t, 64u, (uint64_t)0xaaaaaaaaaaaaaaaaull)

/* ------------------------------------------------------------------------ */
/* Floating-point block coder: encode.c:187-216, decode.c:352-381            */

/* precision(): template/codec1.c:8-11 (+4), codec2.c:131-136 (+6),
 * codec3.c:92-97 (+8) */
static unsigned precision(int emax, unsigned maxprec, int minexp, unsigned dims)
{
  int p = emax - minexp + 2 * (int)(dims + 1);
  if (p < 0) p = 0;
  return (unsigned)p < maxprec ? (unsigned)p : maxprec;
}

/* x86-64 cvtt semantics of (Int)(s * x): NaN or out of range -> INT_MIN. */
static int32_t cast_i32(float y)
{
  if (!(y >= -2147483648.0f && y < 2147483648.0f)) return INT32_MIN;
  return (int32_t)y;
}

static int64_t cast_i64(double y)
{
  if (!(y >= -9223372036854775808.0 && y < 9223372036854775808.0)) return INT64_MIN;
  return (int64_t)y;
}

/* exponent() (encode.c:9-20): frexp exponent of x > 0, clamped at 1 - EBIAS
 * for denormals; -EBIAS for x == 0.  exponent_block (encode.c:22-33) takes it
 * of the block's max |x|, comparing with `<` so NaNs never become the max. */
static int emax_f32(const float* f, unsigned n)
{
  float m = 0;
  unsigned i;
  int e;
  for (i = 0; i < n; i++) {
    float a = fabsf(f[i]);
    if (m < a) m = a;
  }
  if (!(m > 0)) return -127;
  frexp((double)m, &e);
  return e > -126 ? e : -126;
}

static int emax_f64(const double* f, unsigned n)
{
  double m = 0;
  unsigned i;
  int e;
  for (i = 0; i < n; i++) {
    double a = fabs(f[i]);
    if (m < a) m = a;
  }
  if (!(m > 0)) return -1023;
  frexp(m, &e);
  return e > -1022 ? e : -1022;
}

static void encode_block_f32(uint64_t* s, size_t pos, unsigned maxbits, const float* f, unsigned dims)
{
  unsigned size = 1u << (2 * dims), i;
  int emax = emax_f32(f, size);
  unsigned maxprec = precision(emax, 32, ZFP_MIN_EXP, dims);
  unsigned e = maxprec ? (unsigned)(emax + 127) : 0;
  if (e) {
    int32_t q[64];
    float sc = ldexpf(1.0f, 30 - emax); /* quantize(1, emax), encode.c:35-40 */
    for (i = 0; i < 9; i++) put_bit(s, pos + i, ((2 * e + 1) >> i) & 1u);
    for (i = 0; i < size; i++) q[i] = cast_i32(sc * f[i]); /* fwd_cast, encode.c:42-52 */
    encode_int_block_i32(s, pos + 9, maxbits - 9, maxprec, q, dims);
  }
  /* else: a single 0 bit, then padding (encode.c:206-215): nothing to set */
}

static void encode_block_f64(uint64_t* s, size_t pos, unsigned maxbits, const double* f, unsigned dims)
{
  unsigned size = 1u << (2 * dims), i;
  int emax = emax_f64(f, size);
  unsigned maxprec = precision(emax, 64, ZFP_MIN_EXP, dims);
  unsigned e = maxprec ? (unsigned)(emax + 1023) : 0;
  if (e) {
    int64_t q[64];
    double sc = ldexp(1.0, 62 - emax);
    for (i = 0; i < 12; i++) put_bit(s, pos + i, ((2 * e + 1) >> i) & 1u);
    for (i = 0; i < size; i++) q[i] = cast_i64(sc * f[i]);
    encode_int_block_i64(s, pos + 12, maxbits - 12, maxprec, q, dims);
  }
}

static void decode_block_f32(const uint64_t* s, size_t pos, unsigned maxbits, float* f, unsigned dims)
{
  unsigned size = 1u << (2 * dims), i;
  if (get_bit(s, pos)) {
    int32_t q[64];
    int emax = 0;
    unsigned maxprec;
    float sc;
    for (i = 0; i < 8; i++) emax |= (int)get_bit(s, pos + 1 + i) << i;
    emax -= 127;
    maxprec = precision(emax, 32, ZFP_MIN_EXP, dims);
    decode_int_block_i32(s, pos + 9, maxbits - 9, maxprec, q, dims);
    sc = ldexpf(1.0f, emax - 30); /* dequantize(1, emax), decode.c:224-229 */
    for (i = 0; i < size; i++) f[i] = sc * (float)q[i]; /* inv_cast, decode.c:231-241 */
  }
  else
    for (i = 0; i < size; i++) f[i] = 0;
}

static void decode_block_f64(const uint64_t* s, size_t pos, unsigned maxbits, double* f, unsigned dims)
{
  unsigned size = 1u << (2 * dims), i;
  if (get_bit(s, pos)) {
    int64_t q[64];
    int emax = 0;
    unsigned maxprec;
    double sc;
    for (i = 0; i < 11; i++) emax |= (int)get_bit(s, pos + 1 + i) << i;
    emax -= 1023;
    maxprec = precision(emax, 64, ZFP_MIN_EXP, dims);
    decode_int_block_i64(s, pos + 12, maxbits - 12, maxprec, q, dims);
    sc = ldexp(1.0, emax - 62);
    for (i = 0; i < size; i++) f[i] = sc * (double)q[i];
  }
  else
    for (i = 0; i < size; i++) f[i] = 0;
}

/* ------------------------------------------------------------------------ */
/* Array raster: template/compress.c:219-291, decompress.c:59-104.           */
/* Blocks in z, then y, then x order; partial blocks are gathered with       */
/* pad_block (encode.c:54-74) along x, then y, then z (encode3.c:284-301).   */
/* pad_block is separable: padded index i of an n-wide edge reads source     */
/* PADSRC[n][i] (n=1: 0,0,0,0  n=2: 0,1,1,0  n=3: 0,1,2,0).                   */

static const unsigned char PADSRC[5][4] = {
  {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 1, 1, 0}, {0, 1, 2, 0}, {0, 1, 2, 3}};

typedef struct {
  unsigned dims, nx, ny, nz;
  ptrdiff_t sx, sy, sz;
  size_t bx, by, bz;
} raster;

static int make_raster(raster* r, unsigned nx, unsigned ny, unsigned nz, int sx, int sy, int sz)
{
  if (!nx) return 0;
  r->dims = nz ? 3 : ny ? 2 : 1;
  if (nz && !ny) return 0;
  r->nx = nx; r->ny = ny ? ny : 1; r->nz = nz ? nz : 1;
  /* default strides: compress.c:228-229,257-259 */
  r->sx = sx ? sx : 1;
  r->sy = sy ? sy : (ptrdiff_t)nx;
  r->sz = sz ? sz : (ptrdiff_t)nx * (ptrdiff_t)r->ny;
  r->bx = (nx + 3) / 4;
  r->by = (r->ny + 3) / 4;
  r->bz = (r->nz + 3) / 4;
  return 1;
}

static size_t raster_blocks(const raster* r) { return r->bx * r->by * r->bz; }

/* element offsets of block b's 4^d values (padded) */
static void block_offsets(const raster* r, size_t b, ptrdiff_t* off, unsigned* valid)
{
  size_t ix = b % r->bx, iy = (b / r->bx) % r->by, iz = b / (r->bx * r->by);
  unsigned wx = r->nx - 4 * ix, wy = r->ny - 4 * iy, wz = r->nz - 4 * iz;
  unsigned i, j, k, n = 0;
  if (wx > 4) wx = 4;
  if (wy > 4) wy = 4;
  if (wz > 4) wz = 4;
  for (k = 0; k < (r->dims > 2 ? 4u : 1u); k++)
    for (j = 0; j < (r->dims > 1 ? 4u : 1u); j++)
      for (i = 0; i < 4; i++, n++) {
        unsigned si = PADSRC[wx][i], sj = r->dims > 1 ? PADSRC[wy][j] : 0, sk = r->dims > 2 ? PADSRC[wz][k] : 0;
        off[n] = (ptrdiff_t)(4 * ix + si) * r->sx + (ptrdiff_t)(4 * iy + sj) * r->sy +
                 (ptrdiff_t)(4 * iz + sk) * r->sz;
        valid[n] = i < wx && (r->dims < 2 || j < wy) && (r->dims < 3 || k < wz);
      }
}

unsigned oracle_rate_to_maxbits(double rate, int type, unsigned dims, int wra)
{
  unsigned n = 1u << (2 * dims);
  unsigned bits = (unsigned)floor(n * rate + 0.5); /* zfp.c:407-408 */
  if (type == TYPE_FLOAT && bits < 9) bits = 9;    /* zfp.c:409-418 */
  if (type == TYPE_DOUBLE && bits < 12) bits = 12;
  if (wra) bits = (bits + 63) & ~63u;               /* zfp.c:419-423 */
  return bits;
}

size_t oracle_stream_bytes(size_t nblocks, unsigned maxbits)
{
  return ((nblocks * maxbits + 63) / 64) * 8;
}

static int check_args(int type, int want_float, unsigned maxbits)
{
  if (want_float && type != TYPE_FLOAT && type != TYPE_DOUBLE) return 0;
  if (!want_float && type != TYPE_INT32 && type != TYPE_INT64) return 0;
  if (type == TYPE_FLOAT && maxbits < 9) return 0;
  if (type == TYPE_DOUBLE && maxbits < 12) return 0;
  if (!maxbits) return 0;
  return 1;
}

size_t oracle_compress(int type, unsigned nx, unsigned ny, unsigned nz,
                       int sx, int sy, int sz, unsigned maxbits,
                       const void* data, void* stream, size_t stream_bytes)
{
  raster r;
  size_t nb, b, bytes;
  if (!check_args(type, 1, maxbits) || !make_raster(&r, nx, ny, nz, sx, sy, sz)) return 0;
  nb = raster_blocks(&r);
  bytes = oracle_stream_bytes(nb, maxbits);
  if (stream_bytes < bytes) return 0;
  memset(stream, 0, bytes);
  for (b = 0; b < nb; b++) {
    ptrdiff_t off[64];
    unsigned valid[64], i, size = 1u << (2 * r.dims);
    block_offsets(&r, b, off, valid);
    if (type == TYPE_FLOAT) {
      float f[64];
      for (i = 0; i < size; i++) f[i] = ((const float*)data)[off[i]];
      encode_block_f32((uint64_t*)stream, b * maxbits, maxbits, f, r.dims);
    } else {
      double f[64];
      for (i = 0; i < size; i++) f[i] = ((const double*)data)[off[i]];
      encode_block_f64((uint64_t*)stream, b * maxbits, maxbits, f, r.dims);
    }
  }
  return bytes;
}

int oracle_decompress(int type, unsigned nx, unsigned ny, unsigned nz,
                      int sx, int sy, int sz, unsigned maxbits,
                      const void* stream, size_t stream_bytes, void* data)
{
  raster r;
  size_t nb, b;
  if (!check_args(type, 1, maxbits) || !make_raster(&r, nx, ny, nz, sx, sy, sz)) return 0;
  nb = raster_blocks(&r);
  if (stream_bytes < oracle_stream_bytes(nb, maxbits)) return 0;
  for (b = 0; b < nb; b++) {
    ptrdiff_t off[64];
    unsigned valid[64], i, size = 1u << (2 * r.dims);
    block_offsets(&r, b, off, valid);
    if (type == TYPE_FLOAT) {
      float f[64];
      decode_block_f32((const uint64_t*)stream, b * maxbits, maxbits, f, r.dims);
      for (i = 0; i < size; i++) if (valid[i]) ((float*)data)[off[i]] = f[i];
    } else {
      double f[64];
      decode_block_f64((const uint64_t*)stream, b * maxbits, maxbits, f, r.dims);
      for (i = 0; i < size; i++) if (valid[i]) ((double*)data)[off[i]] = f[i];
    }
  }
  return 1;
}

size_t oracle_compress_int(int type, unsigned nx, unsigned ny, unsigned nz,
                           int sx, int sy, int sz, unsigned maxbits,
                           const void* data, void* stream, size_t stream_bytes)
{
  raster r;
  size_t nb, b, bytes;
  if (!check_args(type, 0, maxbits) || !make_raster(&r, nx, ny, nz, sx, sy, sz)) return 0;
  nb = raster_blocks(&r);
  bytes = oracle_stream_bytes(nb, maxbits);
  if (stream_bytes < bytes) return 0;
  memset(stream, 0, bytes);
  for (b = 0; b < nb; b++) {
    ptrdiff_t off[64];
    unsigned valid[64], i, size = 1u << (2 * r.dims);
    block_offsets(&r, b, off, valid);
    if (type == TYPE_INT32) {
      int32_t q[64];
      for (i = 0; i < size; i++) q[i] = ((const int32_t*)data)[off[i]];
      encode_int_block_i32((uint64_t*)stream, b * maxbits, maxbits, 32, q, r.dims);
    } else {
      int64_t q[64];
      for (i = 0; i < size; i++) q[i] = ((const int64_t*)data)[off[i]];
      encode_int_block_i64((uint64_t*)stream, b * maxbits, maxbits, 64, q, r.dims);
    }
  }
  return bytes;
}

int oracle_decompress_int(int type, unsigned nx, unsigned ny, unsigned nz,
                          int sx, int sy, int sz, unsigned maxbits,
                          const void* stream, size_t stream_bytes, void* data)
{
  raster r;
  size_t nb, b;
  if (!check_args(type, 0, maxbits) || !make_raster(&r, nx, ny, nz, sx, sy, sz)) return 0;
  nb = raster_blocks(&r);
  if (stream_bytes < oracle_stream_bytes(nb, maxbits)) return 0;
  for (b = 0; b < nb; b++) {
    ptrdiff_t off[64];
    unsigned valid[64], i, size = 1u << (2 * r.dims);
    block_offsets(&r, b, off, valid);
    if (type == TYPE_INT32) {
      int32_t q[64];
      decode_int_block_i32((const uint64_t*)stream, b * maxbits, maxbits, 32, q, r.dims);
      for (i = 0; i < size; i++) if (valid[i]) ((int32_t*)data)[off[i]] = q[i];
    } else {
      int64_t q[64];
      decode_int_block_i64((const uint64_t*)stream, b * maxbits, maxbits, 64, q, r.dims);
      for (i = 0; i < size; i++) if (valid[i]) ((int64_t*)data)[off[i]] = q[i];
    }
  }
  return 1;
}

/* Jenkins one-at-a-time hash, the array checksum of zfp-0.5.0/tests/testzfp.cpp:74-89 */
uint32_t oracle_jenkins_hash(const void* p, size_t n)
{
  const unsigned char* q = (const unsigned char*)p;
  uint32_t h = 0;
  for (; n; q++, n--) {
    h += *q;
    h += h << 10;
    h ^= h >> 6;
  }
  h += h << 3;
  h ^= h >> 11;
  h += h << 15;
  return h;
}
