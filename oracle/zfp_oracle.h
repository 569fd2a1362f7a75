/*
 * oracle/zfp_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the zfp 0.5.0 fixed-rate codec that the reference
 * (mclarsen/cuZFP) is checked against (src/utils/test.py:68-93).  Used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker; the shipped HIP codec never links or calls it.
 *
 * Parity is pinned two ways (see tests/test_oracle.py):
 *   - bit-exact against oracle/_ref/libzfp_ref.so, the reference's own vendored
 *     zfp 0.5.0 compiled from /root/reference, and
 *   - against committed golden fixtures (tests/golden/) generated from that
 *     build, plus testzfp's checksums and max-error tables.
 *
 * Types follow the reference enum (src/cuZFP/zfp_structs.h:46-52):
 *   1 = int32, 2 = int64, 3 = float, 4 = double.
 */
#ifndef CUZFP_AMD_ZFP_ORACLE_H
#define CUZFP_AMD_ZFP_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* zfp_stream_set_rate (zfp-0.5.0/src/zfp.c:405-430); wra=1 rounds bits up to a
 * multiple of 64 as cuZFP's stream_set_rate does for 3D (zfp_structs.h:77-84). */
unsigned oracle_rate_to_maxbits(double rate, int type, unsigned dims, int wra);

/* Bytes of a fixed-rate stream of `nblocks` blocks: zfp_compress flushes to a
 * 64-bit word (zfp.c:627, inline/bitstream.c stream_flush). */
size_t oracle_stream_bytes(size_t nblocks, unsigned maxbits);

/* zfp_compress / zfp_decompress restricted to fixed-rate mode
 * (minbits == maxbits, maxprec = type precision, minexp = ZFP_MIN_EXP).
 * ny == 0 -> 1D, nz == 0 -> 2D; strides of 0 mean contiguous a[nz][ny][nx].
 * Returns compressed bytes (0 on a bad argument); decompress returns 1 / 0. */
size_t oracle_compress(int type, unsigned nx, unsigned ny, unsigned nz,
                       int sx, int sy, int sz, unsigned maxbits,
                       const void* data, void* stream, size_t stream_bytes);
int oracle_decompress(int type, unsigned nx, unsigned ny, unsigned nz,
                      int sx, int sy, int sz, unsigned maxbits,
                      const void* stream, size_t stream_bytes, void* data);

/* Integer fields (int32/int64), which zfp 0.5.0's zfp_compress rejects
 * (zfp.c:618-624).  Same block raster, partial-block padding and fixed-rate
 * stream layout as the float path; each block is coded by the reference's
 * block-level integer coder (template/encode.c:176-185, decode.c:346-350),
 * which carries no exponent header. */
size_t oracle_compress_int(int type, unsigned nx, unsigned ny, unsigned nz,
                           int sx, int sy, int sz, unsigned maxbits,
                           const void* data, void* stream, size_t stream_bytes);
int oracle_decompress_int(int type, unsigned nx, unsigned ny, unsigned nz,
                          int sx, int sy, int sz, unsigned maxbits,
                          const void* stream, size_t stream_bytes, void* data);

/* Jenkins one-at-a-time hash (zfp-0.5.0/tests/testzfp.cpp:74-89). */
uint32_t oracle_jenkins_hash(const void* p, size_t n);

#ifdef __cplusplus
}
#endif
#endif
