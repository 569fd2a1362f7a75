/*
 * include/cuzfp_hip.h -- C-ABI of the MI355X-native zfp fixed-rate codec.
 *
 * This is the drop-in boundary: plain pointers, sizes and a HIP stream, no C++
 * or torch types.  The C++ surface of the reference (`cuZFP::compress`,
 * `cuZFP::decompress`, include/cuZFP.h) is implemented on top of it
 * (cuzfp_amd/csrc/cuZFP.cpp); Python, ctypes, cgo or JNI callers bind it
 * directly.
 *
 * Each entry point names the reference interface it replaces (paths relative to
 * /root/reference/src/cuZFP):
 *
 *   cuzfp_hip_encode  <- internal::encode<T>(dims, maxbits, d_data, d_stream)
 *                        cuZFP.cu:26-64, i.e. encode1launch / encode2launch /
 *                        encode3launch (encode1.cuh:458-526, encode2.cuh:462-528,
 *                        encode3.cuh:428-508) and their kernels.
 *   cuzfp_hip_decode  <- internal::decode<T>(dims, maxbits, d_stream, d_data)
 *                        cuZFP.cu:66-105 -> decode{1,2,3}launch (decode1.cuh:102-145,
 *                        decode2.cuh:141-182, decode3.cuh:217-264).
 *   cuzfp_hip_stream_bytes <- the byte count those launchers return
 *                        (calc_device_mem{1,2,3}d, e.g. encode3.cuh:413-423).
 *   cuzfp_hip_maximum_size <- zfp_stream_maximum_size (zfp_structs.h:222-251).
 *   cuzfp_hip_rate_to_maxbits <- stream_set_rate (zfp_structs.h:46-76).
 *   cuzfp_hip_compress_host / cuzfp_hip_decompress_host <- the host-pointer
 *                        staging of cuZFP::compress / decompress
 *                        (cuZFP.cu:107-170, 174-269), as a pinned, chunked,
 *                        stream-overlapped pipeline.
 *
 * Stream format: bit-exact with zfp 0.5.0 fixed-rate mode (the ground truth of
 * the reference's src/utils/test.py:68-93): 64-bit little-endian words, bits
 * LSB first, block b (raster order z, y, x) at bits [b*maxbits, (b+1)*maxbits),
 * zero padded to a whole word; no header.
 *
 * Unlike the reference (cuZFP.cu:174-269: errors printed, execution continues),
 * every call returns a cuzfp_status.  Device calls are asynchronous on
 * `stream` (0 = the null stream) and never allocate or synchronise, so they
 * can be captured into a hipGraph.
 */
#ifndef CUZFP_HIP_H
#define CUZFP_HIP_H

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CUZFP_HIP_ABI_VERSION 1

/* scalar type codes: the reference's zfp_type enum (zfp_structs.h:31-37) */
#define CUZFP_TYPE_INT32 1
#define CUZFP_TYPE_INT64 2
#define CUZFP_TYPE_FLOAT 3
#define CUZFP_TYPE_DOUBLE 4

/* Largest accepted maxbits (bits per block).  Calls with more return
 * CUZFP_ERROR_INVALID_ARGUMENT.  It is far above ZFP_MAX_BITS = 4171
 * (zfp_structs.h:12), the most bits any block can use; beyond that a stream is
 * padding.  The bound keeps one wave's LDS stream image within a gfx950
 * workgroup's LDS (160 KiB, hipDeviceAttributeMaxSharedMemoryPerBlock): the
 * decoder's image at 16384 bits is 129 KiB plus 12 KiB of tables.  On a device
 * with less LDS per workgroup (e.g. 64 KiB) the launchers check one wave's image
 * plus the tables against the device's budget before launching and return
 * CUZFP_ERROR_INVALID_ARGUMENT for a call that does not fit (3D f32/f64 past
 * about 6,500 bits on a 64 KiB device); the environment variable
 * CUZFP_LDS_CAP_BYTES lowers the budget (tests). */
#define CUZFP_MAX_BITS 16384

/* Pinned staging slots of the host-memory pipeline for pageable buffers
 * (callers' default `nstreams` for cuzfp_hip_compress_host / decompress_host). */
#define CUZFP_HOST_STREAMS 4

typedef enum {
  CUZFP_SUCCESS = 0,
  CUZFP_ERROR_INVALID_ARGUMENT = 1, /* bad dims, maxbits or null pointer   */
  CUZFP_ERROR_UNSUPPORTED_TYPE = 2, /* type code not 1..4                   */
  CUZFP_ERROR_BUFFER_TOO_SMALL = 3, /* stream capacity < needed bytes       */
  CUZFP_ERROR_HIP = 4               /* a HIP runtime call failed            */
} cuzfp_status;

int cuzfp_hip_abi_version(void);
const char* cuzfp_hip_status_string(int status);
/* last HIP error seen by this thread (hipSuccess if none) */
int cuzfp_hip_last_hip_error(void);

/* maxbits for `rate` bits/value: floor(4^dims * rate + 0.5), at least 1 + the
 * exponent bits (9 float, 12 double); wra != 0 rounds up to a multiple of 64,
 * which is what the reference's stream_set_rate does for 3D arrays. */
unsigned cuzfp_hip_rate_to_maxbits(double rate, int type, unsigned dims, int wra);

/* Exact compressed size: ceil(blocks * maxbits / 64) * 8.  ny == 0 -> 1D,
 * nz == 0 -> 2D. Returns 0 for invalid arguments. */
size_t cuzfp_hip_stream_bytes(int type, unsigned nx, unsigned ny, unsigned nz, unsigned maxbits);

/* Worst-case buffer size, the reference's zfp_stream_maximum_size. */
size_t cuzfp_hip_maximum_size(int type, unsigned nx, unsigned ny, unsigned nz, unsigned maxbits);

/* Compress a device-resident array into a device-resident stream.
 * Strides are in elements (0 = contiguous a[nz][ny][nx]; negative allowed).
 * *out_bytes (optional) receives cuzfp_hip_stream_bytes(). */
int cuzfp_hip_encode(const void* d_data, int type, unsigned nx, unsigned ny, unsigned nz,
                     long long sx, long long sy, long long sz, unsigned maxbits,
                     uint64_t* d_stream, size_t stream_capacity, size_t* out_bytes,
                     hipStream_t stream);

/* Decompress a device-resident stream into a device-resident array. */
int cuzfp_hip_decode(const uint64_t* d_stream, size_t stream_bytes, int type, unsigned nx,
                     unsigned ny, unsigned nz, long long sx, long long sy, long long sz,
                     unsigned maxbits, void* d_data, hipStream_t stream);

/* Host-memory end to end: the array and the stream live in
 * host memory; the library moves them in z-slab (3D) / y-slab (2D) / x-range
 * (1D) chunks on three HIP streams -- input copies, kernels, output copies,
 * each in chunk order -- so the copies overlap the kernels and each other
 * (64 MiB chunks between pinned buffers, smaller ones at the pipeline's ends;
 * 8 MiB through `nstreams` pinned staging buffers for pageable ones).
 * Synchronous; contiguous arrays only.  Environment (read per call):
 * CUZFP_HOST_CHUNK_BYTES sets the chunk size, CUZFP_HOST_ORDERED=0 selects
 * round 4's schedule (chunk i's copies and kernel on stream i % nstreams),
 * CUZFP_HOST_ZEROCOPY: 1 (default) compresses a pinned array into a pinned
 * stream in one kernel that loads and stores them over PCIe itself, 2 also
 * lets the decode kernels store to a pinned array, 0 copies everything
 * (capi.hip host_zero_copy has the measurements).  The first call on a device
 * also times which of its streams carry which copies (~15 ms, once).
 *
 * Retention: the first call on a device allocates, and keeps for later calls,
 * device buffers for the array and the stream (grown to the largest call, up
 * to 1 GiB each; larger calls use buffers freed on return), its HIP streams
 * with their events, and (for pageable user buffers) pinned staging buffers of
 * one chunk each (at most 64 MiB apiece).  This memory is outside any
 * framework allocator (e.g. torch's caching allocator).  Calls on one device
 * are serialised; calls on different devices run concurrently. */
int cuzfp_hip_compress_host(const void* h_data, int type, unsigned nx, unsigned ny,
                            unsigned nz, unsigned maxbits, void* h_stream,
                            size_t stream_capacity, size_t* out_bytes, int nstreams);
int cuzfp_hip_decompress_host(const void* h_stream, size_t stream_bytes, int type,
                              unsigned nx, unsigned ny, unsigned nz, unsigned maxbits,
                              void* h_data, int nstreams);

/* Frees the host pipeline's retained buffers, streams and events for `device`
 * (-1: the current device) after its pending work; the next host-pipeline call
 * allocates them again.  Not a reference entry point. */
int cuzfp_hip_release_host_cache(int device);

/* Diagnostic, not a reference entry point: device-to-device copy of `bytes`
 * (a multiple of 16, both pointers 16-byte aligned) with 16-byte non-temporal
 * loads and stores -- the codec's access width and cache policy.  bench.py
 * times it as the achievable-HBM-bandwidth calibrator. */
int cuzfp_hip_copy(const void* d_src, void* d_dst, size_t bytes, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif
