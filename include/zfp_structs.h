// include/zfp_structs.h -- parameter and array descriptors of the cuZFP C++ API.
//
// Drop-in for the reference's src/cuZFP/zfp_structs.h (installed next to
// cuZFP.h by src/cuZFP/CMakeLists.txt:33): same type names, field order, enum
// values and header-only helpers, so callers written against cuZFP compile
// unchanged (e.g. the reference tests call these unqualified after
// `using namespace cuZFP`, t_sanity_check_3.cpp:9,39-49).
#ifndef CUZFP_ZFP_STRUCTS
#define CUZFP_ZFP_STRUCTS

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstddef>
#include <cstdlib>

#define ZFP_MAX_PREC 64          /* maximum precision supported */
#define ZFP_MIN_EXP -1074        /* minimum floating-point base-2 exponent */
#define ZFP_MAX_BITS 4171        /* maximum number of bits per block */
#define ZFP_MIN_BITS 0           /* minimum number of bits per block */
#define ZFP_HEADER_MAX_BITS 148  /* max number of header bits */

typedef unsigned int uint;
typedef unsigned long long Word;  // stream word (zfp_structs.h:16)
#ifndef wsize
#define wsize ((uint)(CHAR_BIT * sizeof(Word)))
#endif

namespace cuZFP {

// zfp_structs.h:22-29 -- only maxbits is used by the fixed-rate codec
typedef struct {
  uint minbits;
  uint maxbits;
  uint maxprec;
  int minexp;
  Word* stream;  // host or device pointer to the compressed words
} zfp_stream;

// zfp_structs.h:31-37
typedef enum {
  zfp_type_none = 0,
  zfp_type_int32 = 1,
  zfp_type_int64 = 2,
  zfp_type_float = 3,
  zfp_type_double = 4
} zfp_type;

// zfp_structs.h:39-44.  Unlike the reference, which ignores sx/sy/sz
// (SURVEY.md 8a row a1), non-zero strides are honoured as in CPU zfp.
typedef struct {
  zfp_type type;
  uint nx, ny, nz;  // sizes (zero for unused dimensions)
  int sx, sy, sz;   // strides (zero for contiguous a[nz][ny][nx])
  void* data;
} zfp_field;

// zfp_structs.h:46-76: bits/block = floor(4^d * rate + 0.5), at least
// 1 + exponent bits; 3D rounded up to a multiple of 64 (as the reference does).
static double stream_set_rate(zfp_stream* zfp, double rate, zfp_type type, uint dims) {
  const uint n = 1u << (2 * dims);
  uint bits = (uint)std::floor(n * rate + 0.5);
  if (type == zfp_type_float) bits = std::max(bits, 1u + 8u);
  if (type == zfp_type_double) bits = std::max(bits, 1u + 11u);
  if (dims == 3) bits = (bits + wsize - 1) & ~(wsize - 1);
  zfp->minbits = bits;
  zfp->maxbits = bits;
  zfp->maxprec = ZFP_MAX_PREC;
  zfp->minexp = ZFP_MIN_EXP;
  return (double)bits / n;
}

static zfp_field* zfp_field_alloc() {
  zfp_field* f = (zfp_field*)std::malloc(sizeof(zfp_field));
  if (f) {
    f->type = zfp_type_none;
    f->nx = f->ny = f->nz = 0;
    f->sx = f->sy = f->sz = 0;
    f->data = 0;
  }
  return f;
}

static zfp_field* zfp_field_1d(void* data, zfp_type type, uint nx) {
  zfp_field* f = zfp_field_alloc();
  if (f) { f->type = type; f->nx = nx; f->data = data; }
  return f;
}

static zfp_field* zfp_field_2d(void* data, zfp_type type, uint nx, uint ny) {
  zfp_field* f = zfp_field_alloc();
  if (f) { f->type = type; f->nx = nx; f->ny = ny; f->data = data; }
  return f;
}

static zfp_field* zfp_field_3d(void* data, zfp_type type, uint nx, uint ny, uint nz) {
  zfp_field* f = zfp_field_alloc();
  if (f) { f->type = type; f->nx = nx; f->ny = ny; f->nz = nz; f->data = data; }
  return f;
}

static void zfp_field_free(zfp_field* field) { std::free(field); }

static zfp_stream* zfp_stream_open(Word* stream) {
  zfp_stream* z = (zfp_stream*)std::malloc(sizeof(zfp_stream));
  if (z) {
    z->stream = stream;
    z->minbits = ZFP_MIN_BITS;
    z->maxbits = ZFP_MAX_BITS;
    z->maxprec = ZFP_MAX_PREC;
    z->minexp = ZFP_MIN_EXP;
  }
  return z;
}

static void zfp_stream_close(zfp_stream* zfp) { std::free(zfp); }

static uint zfp_field_dimensionality(const zfp_field* field) {
  return field->nx ? field->ny ? field->nz ? 3 : 2 : 1 : 0;
}

static uint type_precision(zfp_type type) {
  switch (type) {
    case zfp_type_int32: return CHAR_BIT * (uint)sizeof(int);
    case zfp_type_int64: return CHAR_BIT * (uint)sizeof(long long int);
    case zfp_type_float: return CHAR_BIT * (uint)sizeof(float);
    case zfp_type_double: return CHAR_BIT * (uint)sizeof(double);
    default: return 0;
  }
}

template <typename T> static zfp_type get_zfp_type() { return zfp_type_none; }
template <> zfp_type get_zfp_type<int>() { return zfp_type_int32; }
template <> zfp_type get_zfp_type<long long int>() { return zfp_type_int64; }
template <> zfp_type get_zfp_type<float>() { return zfp_type_float; }
template <> zfp_type get_zfp_type<double>() { return zfp_type_double; }

static size_t zfp_type_size(zfp_type type) {
  switch (type) {
    case zfp_type_int32: return sizeof(int);
    case zfp_type_int64: return sizeof(long long int);
    case zfp_type_float: return sizeof(float);
    case zfp_type_double: return sizeof(double);
    default: return 0;
  }
}

// zfp_structs.h:222-251: worst-case stream bytes for `field` under `zfp`.
static size_t zfp_stream_maximum_size(const zfp_stream* zfp, const zfp_field* field) {
  const uint dims = zfp_field_dimensionality(field);
  if (!dims || field->type == zfp_type_none) return 0;
  const size_t blocks = (size_t)((std::max(field->nx, 1u) + 3) / 4) *
                        (size_t)((std::max(field->ny, 1u) + 3) / 4) *
                        (size_t)((std::max(field->nz, 1u) + 3) / 4);
  const uint values = 1u << (2 * dims);
  uint maxbits = 1;
  if (field->type == zfp_type_float) maxbits += 8;
  if (field->type == zfp_type_double) maxbits += 11;
  maxbits += values - 1 + values * std::min(zfp->maxprec, type_precision(field->type));
  maxbits = std::min(maxbits, zfp->maxbits);
  maxbits = std::max(maxbits, zfp->minbits);
  return ((ZFP_HEADER_MAX_BITS + blocks * maxbits + wsize - 1) & ~(size_t)(wsize - 1)) / CHAR_BIT;
}

}  // namespace cuZFP
#endif
