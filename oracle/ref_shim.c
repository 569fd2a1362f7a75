/*
 * oracle/ref_shim.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A ctypes-friendly shim over the reference's vendored CPU zfp 0.5.0
 * (src/thirdparty_builtin/zfp-0.5.0).  It is linked with the reference objects
 * into oracle/_ref/libzfp_ref.so and used by tests/ as the ground truth, and by
 * bench.py's cpu_baseline leg ("kind": "reference").  It never ships.
 *
 * Every call goes through the reference's public API exactly the way its own
 * harness does (zfp-0.5.0/utils/zfp.c:330-400, tests/testzfp.cpp:92-140):
 * zfp_stream_open -> zfp_stream_set_params/set_rate -> stream_open ->
 * zfp_stream_rewind -> zfp_compress / zfp_decompress.
 */
#define _POSIX_C_SOURCE 199309L
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "zfp.h"

static zfp_field* make_field(int type, unsigned nx, unsigned ny, unsigned nz,
                             int sx, int sy, int sz, void* data)
{
  zfp_field* f;
  zfp_type t = (zfp_type)type;
  if (nz)      f = zfp_field_3d(data, t, nx, ny, nz);
  else if (ny) f = zfp_field_2d(data, t, nx, ny);
  else         f = zfp_field_1d(data, t, nx);
  if (sx || sy || sz) {
    if (nz)      zfp_field_set_stride_3d(f, sx, sy, sz);
    else if (ny) zfp_field_set_stride_2d(f, sx, sy);
    else         zfp_field_set_stride_1d(f, sx);
  }
  return f;
}

/* zfp_stream_set_rate(..., wra=0) as zfp-0.5.0/src/zfp.c:405-430; returns maxbits. */
unsigned ref_rate_to_maxbits(double rate, int type, unsigned dims, int wra)
{
  zfp_stream* z = zfp_stream_open(NULL);
  unsigned bits;
  zfp_stream_set_rate(z, rate, (zfp_type)type, dims, wra);
  bits = z->maxbits;
  zfp_stream_close(z);
  return bits;
}

static zfp_stream* open_fixed(int type, unsigned maxbits)
{
  zfp_stream* z = zfp_stream_open(NULL);
  unsigned prec = (type == zfp_type_float || type == zfp_type_int32) ? 32u : 64u;
  /* fixed-rate mode: minbits == maxbits, full precision (zfp.c:424-428) */
  zfp_stream_set_params(z, maxbits, maxbits, prec, ZFP_MIN_EXP);
  return z;
}

size_t ref_maximum_size(int type, unsigned nx, unsigned ny, unsigned nz, unsigned maxbits)
{
  zfp_field* f = make_field(type, nx, ny, nz, 0, 0, 0, NULL);
  zfp_stream* z = open_fixed(type, maxbits);
  size_t n = zfp_stream_maximum_size(z, f);
  zfp_stream_close(z);
  zfp_field_free(f);
  return n;
}

/* Compress with explicit maxbits; returns compressed bytes (0 on failure). */
size_t ref_compress(int type, unsigned nx, unsigned ny, unsigned nz,
                    int sx, int sy, int sz, unsigned maxbits,
                    const void* data, void* out, size_t outcap)
{
  zfp_field* f = make_field(type, nx, ny, nz, sx, sy, sz, (void*)data);
  zfp_stream* z = open_fixed(type, maxbits);
  bitstream* s = stream_open(out, outcap);
  size_t n;
  zfp_stream_set_bit_stream(z, s);
  zfp_stream_rewind(z);
  n = zfp_compress(z, f);
  stream_close(s);
  zfp_stream_close(z);
  zfp_field_free(f);
  return n;
}

int ref_decompress(int type, unsigned nx, unsigned ny, unsigned nz,
                   int sx, int sy, int sz, unsigned maxbits,
                   const void* in, size_t incap, void* data)
{
  zfp_field* f = make_field(type, nx, ny, nz, sx, sy, sz, data);
  zfp_stream* z = open_fixed(type, maxbits);
  bitstream* s = stream_open((void*)in, incap);
  int ok;
  zfp_stream_set_bit_stream(z, s);
  zfp_stream_rewind(z);
  ok = zfp_decompress(z, f);
  stream_close(s);
  zfp_stream_close(z);
  zfp_field_free(f);
  return ok;
}

/* Block-level integer codec (zfp-0.5.0/src/template/encode.c:176-185,
 * decode.c:346-350): the oracle for int32/int64 fields, which zfp_compress
 * rejects (zfp.c:618-624).  Encodes `nblocks` contiguous blocks of 4^dims ints. */
size_t ref_encode_int_blocks(int type, unsigned dims, unsigned maxbits, size_t nblocks,
                             const void* blocks, void* out, size_t outcap)
{
  zfp_stream* z = open_fixed(type, maxbits);
  bitstream* s = stream_open(out, outcap);
  size_t b, n = (size_t)1 << (2 * dims);
  zfp_stream_set_bit_stream(z, s);
  zfp_stream_rewind(z);
  for (b = 0; b < nblocks; b++) {
    if (type == zfp_type_int32) {
      const int32* p = (const int32*)blocks + b * n;
      if (dims == 1) zfp_encode_block_int32_1(z, p);
      else if (dims == 2) zfp_encode_block_int32_2(z, p);
      else zfp_encode_block_int32_3(z, p);
    } else {
      const int64* p = (const int64*)blocks + b * n;
      if (dims == 1) zfp_encode_block_int64_1(z, p);
      else if (dims == 2) zfp_encode_block_int64_2(z, p);
      else zfp_encode_block_int64_3(z, p);
    }
  }
  zfp_stream_flush(z);
  n = stream_size(s);
  stream_close(s);
  zfp_stream_close(z);
  return n;
}

int ref_decode_int_blocks(int type, unsigned dims, unsigned maxbits, size_t nblocks,
                          const void* in, size_t incap, void* blocks)
{
  zfp_stream* z = open_fixed(type, maxbits);
  bitstream* s = stream_open((void*)in, incap);
  size_t b, n = (size_t)1 << (2 * dims);
  zfp_stream_set_bit_stream(z, s);
  zfp_stream_rewind(z);
  for (b = 0; b < nblocks; b++) {
    if (type == zfp_type_int32) {
      int32* p = (int32*)blocks + b * n;
      if (dims == 1) zfp_decode_block_int32_1(z, p);
      else if (dims == 2) zfp_decode_block_int32_2(z, p);
      else zfp_decode_block_int32_3(z, p);
    } else {
      int64* p = (int64*)blocks + b * n;
      if (dims == 1) zfp_decode_block_int64_1(z, p);
      else if (dims == 2) zfp_decode_block_int64_2(z, p);
      else zfp_decode_block_int64_3(z, p);
    }
  }
  stream_close(s);
  zfp_stream_close(z);
  return 1;
}

/* ---- CPU baseline timing (bench.py cpu_baseline, SURVEY.md 8d "CPU side") ----
 * Times zfp_compress + zfp_decompress of a contiguous array with steady
 * (monotonic) clocks, `reps` repetitions, single thread or `threads` threads
 * on disjoint z-slabs (3D) / y-slabs (2D) / x-ranges (1D).  Slab boundaries are
 * block-aligned and each slab's stream starts on a 64-bit word, so the slab
 * streams concatenate to the whole-array stream whenever the slab block count
 * times maxbits is a multiple of 64.  Returns the median
 * round-trip seconds; enc/dec medians through the out-pointers. */
typedef struct {
  int type; unsigned nx, ny, nz, maxbits;
  const char* in; char* out; char* stream; size_t cap;
  double enc, dec;
  int valid;
} slab_job;

static double now_s(void)
{
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void* slab_run(void* arg)
{
  slab_job* j = (slab_job*)arg;
  double t0 = now_s(), t1;
  ref_compress(j->type, j->nx, j->ny, j->nz, 0, 0, 0, j->maxbits, j->in, j->stream, j->cap);
  t1 = now_s();
  ref_decompress(j->type, j->nx, j->ny, j->nz, 0, 0, 0, j->maxbits, j->stream, j->cap, j->out);
  j->enc = t1 - t0;
  j->dec = now_s() - t1;
  return NULL;
}

static int cmp_d(const void* a, const void* b)
{
  double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

double ref_time_roundtrip(int type, unsigned nx, unsigned ny, unsigned nz, unsigned maxbits,
                          const void* in, void* out, int threads, int reps,
                          double* enc_med, double* dec_med)
{
  size_t esz = (type == zfp_type_float) ? 4 : 8;
  unsigned dims = nz ? 3 : ny ? 2 : 1;
  unsigned slow = dims == 3 ? nz : dims == 2 ? ny : nx;
  size_t plane = dims == 3 ? (size_t)nx * ny : dims == 2 ? (size_t)nx : 1;
  size_t bplane = dims == 3 ? (size_t)((nx + 3) / 4) * ((ny + 3) / 4) : dims == 2 ? (nx + 3) / 4 : 1;
  unsigned nblk = (slow + 3) / 4, per, t, r;
  if (threads < 1) threads = 1;
  if (reps < 1) reps = 1;
  double *rt = (double*)malloc(sizeof(double) * reps), *et = (double*)malloc(sizeof(double) * reps),
         *dt = (double*)malloc(sizeof(double) * reps), med;
  slab_job* jobs = (slab_job*)calloc(threads, sizeof(slab_job));
  pthread_t* tid = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  per = (nblk + threads - 1) / threads;
  for (t = 0; t < (unsigned)threads; t++) {
    unsigned b0 = t * per, b1 = b0 + per > nblk ? nblk : b0 + per;
    unsigned s0 = 4 * b0, s1 = 4 * b1 > slow ? slow : 4 * b1;
    slab_job* j = &jobs[t];
    j->type = type; j->maxbits = maxbits; j->valid = s1 > s0;
    j->nx = dims == 1 ? (s1 > s0 ? s1 - s0 : 0) : nx;
    j->ny = dims == 1 ? 0 : dims == 2 ? (s1 > s0 ? s1 - s0 : 0) : ny;
    j->nz = dims == 3 ? (s1 > s0 ? s1 - s0 : 0) : 0;
    j->in = (const char*)in + (size_t)s0 * plane * esz;
    j->out = (char*)out + (size_t)s0 * plane * esz;
    j->cap = ((size_t)(b1 - b0) * bplane * maxbits + 64 + 148) / 8 + 64;
    j->stream = (char*)malloc(j->cap);
  }
  for (r = 0; r < (unsigned)reps; r++) {
    double t0 = now_s(), emax = 0, dmax = 0;
    for (t = 0; t < (unsigned)threads; t++)
      if (jobs[t].valid)
        pthread_create(&tid[t], NULL, slab_run, &jobs[t]);
    for (t = 0; t < (unsigned)threads; t++)
      if (jobs[t].valid) {
        pthread_join(tid[t], NULL);
        if (jobs[t].enc > emax) emax = jobs[t].enc;
        if (jobs[t].dec > dmax) dmax = jobs[t].dec;
      }
    rt[r] = now_s() - t0; et[r] = emax; dt[r] = dmax;
  }
  qsort(rt, reps, sizeof(double), cmp_d);
  qsort(et, reps, sizeof(double), cmp_d);
  qsort(dt, reps, sizeof(double), cmp_d);
  med = rt[reps / 2];
  if (enc_med) *enc_med = et[reps / 2];
  if (dec_med) *dec_med = dt[reps / 2];
  for (t = 0; t < (unsigned)threads; t++) free(jobs[t].stream);
  free(jobs); free(tid); free(rt); free(et); free(dt);
  return med;
}
