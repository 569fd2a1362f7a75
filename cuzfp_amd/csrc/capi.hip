// cuzfp_amd/csrc/capi.hip -- the C-ABI of include/cuzfp_hip.h: argument
// checking, kernel dispatch and the pinned host-memory pipeline.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <chrono>
#include <vector>

#include "launch.hpp"

namespace cuzfp {

thread_local int t_last_hip = hipSuccess;

static int make_problem(int type, unsigned nx, unsigned ny, unsigned nz, long long sx,
                        long long sy, long long sz, unsigned maxbits, Problem* pr) {
  if (type < CUZFP_TYPE_INT32 || type > CUZFP_TYPE_DOUBLE) return CUZFP_ERROR_UNSUPPORTED_TYPE;
  if (!nx || (nz && !ny)) return CUZFP_ERROR_INVALID_ARGUMENT;
  const unsigned dims = nz ? 3 : ny ? 2 : 1;
  const unsigned ebits = type == CUZFP_TYPE_FLOAT ? 9 : type == CUZFP_TYPE_DOUBLE ? 12 : 1;
  // One wave's LDS image must fit a workgroup's LDS beside the tables: the
  // decoder's (maxbits / 32 + 5 rows of 256 B + 12 KiB of chunk tables) takes
  // 141 KiB at CUZFP_MAX_BITS (16,384) of gfx950's 160 KiB (the launchers
  // check the device's budget).  The cap is far above the most bits any block
  // can use (zfp's ZFP_MAX_BITS, 4,171: 3D double at full precision); past
  // that a stream is padding.
  if (maxbits < ebits || maxbits > CUZFP_MAX_BITS) return CUZFP_ERROR_INVALID_ARGUMENT;
  Geometry& g = pr->g;
  g.nx = nx;
  g.ny = dims > 1 ? ny : 1;
  g.nz = dims > 2 ? nz : 1;
  g.bx = (g.nx + 3) / 4;
  g.by = (g.ny + 3) / 4;
  const uint64_t nb = (uint64_t)g.bx * g.by * ((g.nz + 3) / 4);
  if (nb >= (1ull << 32) - kLanes) return CUZFP_ERROR_INVALID_ARGUMENT;
  g.nblocks = (uint32_t)nb;
  set_divisor(g.bx, g.dbx_m, g.dbx_s);
  set_divisor(g.bx * g.by, g.dpl_m, g.dpl_s);
  g.divmagic = nb < (1ull << 31) ? 1u : 0u;
  g.maxbits = maxbits;
  g.wave0 = 0;
  g.vec_io = 0;
  g.row_stage = 0;
  g.sx = sx ? sx : 1;
  g.sy = sy ? sy : (long long)g.nx;
  g.sz = sz ? sz : (long long)g.nx * g.ny;
  pr->type = type;
  pr->dims = dims;
  pr->fast_ok = (type == CUZFP_TYPE_FLOAT || type == CUZFP_TYPE_DOUBLE) && g.sx == 1 &&
                g.sy == (long long)g.nx && g.sz == (long long)g.nx * g.ny && g.nx % 4 == 0 &&
                (dims < 2 || g.ny % 4 == 0) && (dims < 3 || g.nz % 4 == 0);
  return CUZFP_SUCCESS;
}

static int launch_encode(const Problem& p, const void* data, uint64_t* stream, uint32_t wave0,
                         uint32_t nwaves, hipStream_t st) {
  if (!nwaves) return CUZFP_SUCCESS;
  const bool fast = p.fast_ok && ((uintptr_t)data & 15) == 0;
  switch (p.type) {
    case CUZFP_TYPE_INT32: return launch_encode_type<int32_t>(p, data, false, stream, wave0, nwaves, st);
    case CUZFP_TYPE_INT64: return launch_encode_type<int64_t>(p, data, false, stream, wave0, nwaves, st);
    case CUZFP_TYPE_FLOAT: return launch_encode_type<float>(p, data, fast, stream, wave0, nwaves, st);
    default: return launch_encode_type<double>(p, data, fast, stream, wave0, nwaves, st);
  }
}

static int launch_decode(const Problem& p, const uint64_t* stream, void* data, uint32_t wave0,
                         uint32_t nwaves, hipStream_t st) {
  if (!nwaves) return CUZFP_SUCCESS;
  const bool fast = p.fast_ok && ((uintptr_t)data & 15) == 0;
  switch (p.type) {
    case CUZFP_TYPE_INT32: return launch_decode_type<int32_t>(p, stream, false, data, wave0, nwaves, st);
    case CUZFP_TYPE_INT64: return launch_decode_type<int64_t>(p, stream, false, data, wave0, nwaves, st);
    case CUZFP_TYPE_FLOAT: return launch_decode_type<float>(p, stream, fast, data, wave0, nwaves, st);
    default: return launch_decode_type<double>(p, stream, fast, data, wave0, nwaves, st);
  }
}

static size_t stream_bytes_of(const Geometry& g) {
  return (((size_t)g.nblocks * g.maxbits + 63) / 64) * 8;
}

static uint32_t waves_of(const Geometry& g) { return (g.nblocks + kLanes - 1) / kLanes; }


// Bandwidth calibrator (cuzfp_hip_copy, below; also the stand-in kernel of
// pick_copy_queues): a device-to-device copy with 16-byte
// non-temporal loads and stores, one per lane, one grid over the whole buffer
// -- the codec's own access width, cache policy and one-touch-per-wave shape.
// bench.py times it at 1 GiB beside the codec as the achievable-HBM reference
// (roofline.frac_of_copy).  tools/ubench/copy.hip (profiles/r02_copy_ubench.txt):
// this shape 6.64 TB/s (read + write) at 1 GiB; grid-stride loops over
// 1-32 workgroups per CU with 1-8 accesses in flight a lane 4.6-6.4 TB/s;
// plain (temporal) accesses 0.3-0.5 TB/s below non-temporal.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void copy16_nt(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                 size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// ---------------------------------------------------------------------------
// Host-memory pipeline (cuzfp_hip_compress_host / cuzfp_hip_decompress_host).
//
// The array is cut into chunks of whole block slabs along its slowest axis
// (4 z-planes in 3D, 4 rows in 2D, 4 values in 1D), ~kChunkBytes of scalars
// each.  Chunk i runs on stream i % S:
//   encode: H2D slabs -> encode the waves whose blocks are now all resident
//           -> D2H their stream words
//   decode: H2D the stream words of a wave range -> decode -> D2H the slabs
//           whose blocks are now all decoded
// Waves straddle slab boundaries, so each kernel / D2H also waits on the
// previous S-1 chunks' events (chunks further back ran on the same streams).
// Pinned (hipHostMalloc / registered) user buffers are DMA'd in place;
// pageable ones go through a ring of pinned staging buffers.

// Chunk size: 64 MiB between pinned buffers (ordered schedule, 256^3 f32
// rate 8: compression 50.4 GB/s, decompression 48.9 against a 54.8 / 55.3 GB/s
// link; 32 MiB 49.7 / 48.1, 16 MiB 49.0 / 47.3; the round-4 schedule at 8 MiB
// 44.1 / 47.4: tools/host_sweep.py, profiles/r05_host_sweep.txt).  Pageable
// buffers go through pinned staging buffers a chunk each, bound by the host
// copies into them: 8 MiB keeps that staging small.
constexpr size_t kChunkBytes = 64u << 20, kStagedChunkBytes = 8u << 20;

// chunk size: the above, or CUZFP_HOST_CHUNK_BYTES from the environment
// (read per call; tests use small chunks to run the multi-chunk paths)
static size_t chunk_bytes(bool staged) {
  const char* e = getenv("CUZFP_HOST_CHUNK_BYTES");
  if (e && *e) {
    const long long v = atoll(e);
    if (v > 0) return (size_t)v;
  }
  return staged ? kStagedChunkBytes : kChunkBytes;
}

// schedule: ordered copy queues (host_pipeline); CUZFP_HOST_ORDERED=0 -> the
// round-4 schedule, chunk i's copies and kernel on stream i % S (tests run both)
static bool host_ordered() {
  const char* e = getenv("CUZFP_HOST_ORDERED");
  return !(e && *e == '0');
}

// Zero-copy level (CUZFP_HOST_ZEROCOPY): 0 none; 1 (default): compression of
// a pinned array into a pinned stream is one encode launch that loads the
// array and stores the stream over PCIe itself; 2: also decompression into a
// pinned array, the decode kernels storing to it (the stream still copied in
// chunks).  256^3 f32 rate 8 (tools/zero_copy.py,
// tools/host_sweep.py, tools/hostpath_probe.py, profiles/r05_host_*.txt):
// compression 50.2-50.6 GB/s whatever streams the process made before, where
// the copy pipeline measured 47-51 after its queue calibration
// (pick_copy_queues) and 41 without it; decompression at level 2 42-43
// (with the kernels also loading the stream: 41-42) against 49-50 for the copies -- the kernels' own PCIe stores
// reach 49.6 GB/s (53.1 for a plain copy kernel) where the copy engine
// reaches 55-57.  So compression uses level 1 and decompression the copies.
static int host_zero_copy() {
  const char* e = getenv("CUZFP_HOST_ZEROCOPY");
  return (e && *e) ? atoi(e) : 1;
}

// The device address of [p, p + bytes) when the whole range lies in one pinned
// host allocation mapped into the device's address space (hipHostMalloc, a
// pinned torch tensor), else null.  Registered memory reports no allocation
// base (hipMemGetAddressRange; tools/zero_copy.py --ranges) and is not used.
static char* mapped_view(const void* p, size_t bytes) {
  hipPointerAttribute_t a;
  void* d = nullptr;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  const bool ok = hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost &&
                  hipHostGetDevicePointer(&d, const_cast<void*>(p), 0) == hipSuccess && d &&
                  hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)d) == hipSuccess && base &&
                  (char*)d >= (char*)base && (size_t)((char*)d - (char*)base) + bytes <= size;
  (void)hipGetLastError();
  return ok ? (char*)d : nullptr;
}

// CUZFP_HOST_SPLIT=0: fill the ordered schedule's queues chunk by chunk
// between pinned buffers too (A/B of host_pipeline's three passes)
static bool host_split_passes() {
  const char* e = getenv("CUZFP_HOST_SPLIT");
  return !(e && *e == '0');
}

static bool is_pinned_host(const void* ptr) {
  hipPointerAttribute_t a;
  const hipError_t e = hipPointerGetAttributes(&a, ptr);
  (void)hipGetLastError();
  return e == hipSuccess && a.type == hipMemoryTypeHost;
}

namespace {
struct Chunk {
  size_t d0, d1;    // data byte range
  size_t s0, s1;    // stream byte range
  uint32_t w0, w1;  // wave range for the kernel
};

// The pipeline's device buffers, streams, events and pinned staging ring,
// kept between calls (per device; one call at a time per device, calls on
// different devices run concurrently): allocating and freeing them per call
// cost about as much as the transfers of a 64 MiB array.  Device buffers grow
// to the largest call seen up to kCacheLimit bytes (larger calls use buffers
// of their own, freed on return); the pinned staging buffers are chunk-sized
// (chunk_bytes(), capped at kPinCacheLimit each; larger chunks stage through
// buffers freed on return).  cuzfp_hip_release_host_cache() frees a device's
// cache (include/cuzfp_hip.h documents the retention).
constexpr size_t kCacheLimit = 1ull << 30;
constexpr size_t kPinCacheLimit = 64ull << 20;
constexpr int kMaxStreams = 8;

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t get(size_t bytes) {  // at least `bytes`, contents undefined
    if (bytes <= cap) return hipSuccess;
    release();
    const hipError_t e = hipMalloc(&p, std::max<size_t>(bytes, 16));
    if (e == hipSuccess) cap = bytes;
    else p = nullptr;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t get(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    release();
    const hipError_t e = hipHostMalloc(&p, std::max<size_t>(bytes, 16), hipHostMallocDefault);
    if (e == hipSuccess) cap = bytes;
    else p = nullptr;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// a pinned staging buffer for one call: the cache's up to kPinCacheLimit,
// else the call's own (freed on return)
struct CallHostBuf {
  void* p = nullptr;
  bool own = false;
  ~CallHostBuf() {
    if (own && p) (void)hipHostFree(p);
  }
  hipError_t get(HostBuf& cached, size_t bytes) {
    if (bytes <= kPinCacheLimit) {
      const hipError_t e = cached.get(bytes);
      p = cached.p;
      return e;
    }
    own = true;
    const hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e != hipSuccess) p = nullptr;
    return e;
  }
};

struct PipelineCache {
  std::mutex mu;  // one call at a time on this device
  DevBuf d_data, d_stream;
  hipStream_t st[kMaxStreams] = {};
  hipEvent_t ev_in[kMaxStreams] = {}, ev_kernel[kMaxStreams] = {}, ev_done[kMaxStreams] = {};
  HostBuf pin_in[kMaxStreams], pin_out[kMaxStreams];
  int nst = 0;
  // the ordered schedule's queues: indices into st (pick_copy_queues)
  int q_in = 0, q_k = 1, q_out = 2;
  bool queues_picked = false;
  // one input-copy and one kernel event per chunk (the ordered schedule
  // between pinned buffers enqueues every chunk's input copy first)
  std::vector<hipEvent_t> ev_chunk_in, ev_chunk_kernel;
  hipError_t chunk_events(size_t n) {
    while (ev_chunk_in.size() < n) {
      hipEvent_t a = nullptr, b = nullptr;
      hipError_t e = hipEventCreateWithFlags(&a, hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&b, hipEventDisableTiming);
      if (e != hipSuccess) {
        if (a) (void)hipEventDestroy(a);
        return e;
      }
      ev_chunk_in.push_back(a);
      ev_chunk_kernel.push_back(b);
    }
    return hipSuccess;
  }
};

// by device ordinal; kept for the process lifetime unless released
PipelineCache g_pipeline[kMaxDevices];

// device buffers for one call: the cache's, or the call's own past kCacheLimit
struct CallBuf {
  void* p = nullptr;
  bool own = false;
  ~CallBuf() {
    if (own && p) (void)hipFree(p);
  }
  hipError_t get(DevBuf& cached, size_t bytes) {
    if (bytes <= kCacheLimit) {
      const hipError_t e = cached.get(bytes);
      p = cached.p;
      return e;
    }
    own = true;
    return hipMalloc(&p, bytes);
  }
};
}  // namespace

#define CUZFP_HIP_TRY(x)            \
  do {                              \
    const hipError_t e_ = (x);      \
    if (e_ != hipSuccess) {         \
      t_last_hip = e_;              \
      return CUZFP_ERROR_HIP;       \
    }                               \
  } while (0)

// Which of the cache's first eight streams carry the input copies, the
// kernels and the output copies.  HIP spreads streams over GPU_MAX_HW_QUEUES
// (4 on these boxes) hardware queues in creation order, and the same pipeline
// ran at 50 GB/s each way or at 41 according to how many streams the process
// had created before it (tools/hostpath_probe.py --streams N,
// profiles/r05_hostpath_streams.txt: N = 0, 1, 4, 5 fast, 2, 3 slow).  Among
// four consecutive streams no assignment was fast for N = 2; among eight one
// was (profiles/r05_host_queues.txt).  So, once per device, a small model of
// the schedule -- three 4 MiB chunks, each an H2D copy, a copy kernel waiting
// on it and a D2H copy waiting on the kernel -- is timed for each choice of
// one role's stream with the other two held (output, then kernels, then
// input; 16 candidates, the better of two ~0.4 ms runs each) and the
// fastest assignment is kept.
#ifndef CUZFP_PICK_STREAMS
#define CUZFP_PICK_STREAMS 8
#endif
constexpr int kPickStreams = CUZFP_PICK_STREAMS;
static hipError_t pick_copy_queues(PipelineCache& r) {
  constexpr size_t kB = 4u << 20;
  constexpr int kChunks = 3;
  void *h = nullptr, *d = nullptr;
  hipError_t e = hipHostMalloc(&h, 2 * kChunks * kB, hipHostMallocDefault);
  if (e == hipSuccess) e = hipMalloc(&d, 2 * kChunks * kB);
  if (e != hipSuccess) {
    if (h) (void)hipHostFree(h);
    return e;
  }
  std::memset(h, 0, 2 * kChunks * kB);
  char* hc = (char*)h;
  char* dc = (char*)d;
  hipEvent_t ev[2 * kChunks] = {};
  for (int i = 0; i < 2 * kChunks && e == hipSuccess; i++) e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
  const unsigned grid = (unsigned)(kB / 16 / 256);
  // every stream copies both ways once before anything is timed
  for (int q = 0; q < kPickStreams && e == hipSuccess; q++) {
    e = hipMemcpyAsync(dc, hc, kB, hipMemcpyHostToDevice, r.st[q]);
    if (e == hipSuccess) e = hipMemcpyAsync(hc + kB, dc + kB, kB, hipMemcpyDeviceToHost, r.st[q]);
    if (e == hipSuccess) e = hipStreamSynchronize(r.st[q]);
  }
  auto trial1 = [&](int a, int k, int b, double& t) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int c = 0; c < kChunks && e == hipSuccess; c++) {
      e = hipMemcpyAsync(dc + c * kB, hc + c * kB, kB, hipMemcpyHostToDevice, r.st[a]);
      if (e == hipSuccess) e = hipEventRecord(ev[c], r.st[a]);
    }
    for (int c = 0; c < kChunks && e == hipSuccess; c++) {
      e = hipStreamWaitEvent(r.st[k], ev[c], 0);
      if (e == hipSuccess) {
        hipLaunchKernelGGL(copy16_nt, dim3(grid), dim3(256), 0, r.st[k], (const u32x4*)(dc + c * kB),
                           (u32x4*)(dc + (kChunks + c) * kB), kB / 16);
        e = hipGetLastError();
      }
      if (e == hipSuccess) e = hipEventRecord(ev[kChunks + c], r.st[k]);
    }
    for (int c = 0; c < kChunks && e == hipSuccess; c++) {
      e = hipStreamWaitEvent(r.st[b], ev[kChunks + c], 0);
      if (e == hipSuccess)
        e = hipMemcpyAsync(hc + (kChunks + c) * kB, dc + (kChunks + c) * kB, kB, hipMemcpyDeviceToHost, r.st[b]);
    }
    for (int q : {a, k, b})
      if (e == hipSuccess) e = hipStreamSynchronize(r.st[q]);
    t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (getenv("CUZFP_HOST_DEBUG")) fprintf(stderr, "cuzfp host queues: in %d kernels %d out %d: %.1f us\n", a, k, b, t * 1e6);
  };
  auto trial = [&](int a, int k, int b, double& t) {  // the better of two runs
    double t2 = 0;
    trial1(a, k, b, t);
    trial1(a, k, b, t2);
    t = std::min(t, t2);
  };
  int role[3] = {0, 1, 2};  // in, kernels, out
  double best = 1e30;
  trial(role[0], role[1], role[2], best);
  for (int which : {2, 1, 0}) {
    for (int q = 0; q < kPickStreams && e == hipSuccess; q++) {
      if (q == role[0] || q == role[1] || q == role[2]) continue;
      int cand[3] = {role[0], role[1], role[2]};
      cand[which] = q;
      double t = 0;
      trial(cand[0], cand[1], cand[2], t);
      if (t < best) {
        best = t;
        role[which] = q;
      }
    }
  }
  // nothing of a failed trial may still use the buffers when they are freed
  if (e != hipSuccess)
    for (int q = 0; q < kPickStreams; q++) (void)hipStreamSynchronize(r.st[q]);
  for (int i = 0; i < 2 * kChunks; i++)
    if (ev[i]) (void)hipEventDestroy(ev[i]);
  (void)hipFree(d);
  (void)hipHostFree(h);
  if (e != hipSuccess) return e;
  r.q_in = role[0];
  r.q_k = role[1];
  r.q_out = role[2];
  r.queues_picked = true;
  return hipSuccess;
}

static int host_pipeline(const Problem& p, bool encode, void* h_data, void* h_stream,
                         int nstreams) {
  const Geometry& g = p.g;
  const size_t es = (p.type == CUZFP_TYPE_FLOAT || p.type == CUZFP_TYPE_INT32) ? 4 : 8;
  // slabs along the slowest axis
  const size_t slab_vals = p.dims == 3 ? 4ull * g.nx * g.ny : p.dims == 2 ? 4ull * g.nx : 4ull;
  const size_t slab_blocks = p.dims == 3 ? (size_t)g.bx * g.by : p.dims == 2 ? g.bx : 1;
  const size_t total_vals = (size_t)g.nx * g.ny * g.nz;
  const size_t nslabs = ((size_t)(p.dims == 3 ? g.nz : p.dims == 2 ? g.ny : g.nx) + 3) / 4;
  const uint32_t nwaves = waves_of(g);
  const size_t data_bytes = total_vals * es;
  const size_t sbytes = stream_bytes_of(g);
  const size_t wave_bytes = (size_t)g.maxbits * 8;  // stream bytes per full wave
  const bool data_pinned = is_pinned_host(h_data);
  const bool stream_pinned = is_pinned_host(h_stream);
  const size_t per = std::max<size_t>(1, chunk_bytes(!data_pinned || !stream_pinned) / (slab_vals * es));

  const bool ordered = host_ordered();
  // chunk lengths in slabs: `per` each, except (ordered schedule) at the
  // pipeline's exposed end -- the last chunks of a compression, whose kernels
  // and stream copies trail the input copies, and the first of a
  // decompression, before whose kernel no output copy can start -- which grow
  // by 3x from about nslabs / 32 (256^3 f32, 1 MiB slabs, 64 MiB chunks:
  // compression 38, 18, 6, 2 slabs; decompression 2, 6, 18, 38).  The stream
  // is a quarter of the data or less, so chunk i + 1's stream copy and kernel
  // finish within chunk i's data copy at 3x growth, and the copy queue that
  // binds never waits; every copy also costs ~10-15 us of its own
  // (tools/copy_chunks.py), so the chunks stay few.
  std::vector<size_t> lens;
  {
    std::vector<size_t> edge;  // from the exposed end inward
    size_t sum = 0;
    if (ordered) {
      for (size_t l = std::max<size_t>(1, nslabs / 32); sum + l < nslabs && l < per; l *= 3) {
        edge.push_back(l);
        sum += l;
      }
    }
    // the rest in equal chunks of at most `per`
    const size_t body = nslabs - sum, nb = (body + per - 1) / per;
    if (!encode) lens = edge;
    for (size_t k = 0; k < nb; k++) lens.push_back(body / nb + (k < body % nb ? 1 : 0));
    if (encode) lens.insert(lens.end(), edge.rbegin(), edge.rend());
  }
  std::vector<Chunk> chunks;
  uint32_t w_prev = 0;
  size_t d_prev = 0;
  size_t sl = 0;  // first slab of the chunk
  for (size_t len : lens) {
    const size_t e = sl + len;
    const bool last = e == nslabs;
    Chunk c;
    if (encode) {
      c.d0 = std::min(data_bytes, sl * slab_vals * es);
      c.d1 = last ? data_bytes : e * slab_vals * es;
      c.w0 = w_prev;
      c.w1 = last ? nwaves : (uint32_t)(e * slab_blocks / kLanes);
      w_prev = c.w1;
    } else {
      c.w0 = w_prev;
      c.w1 = last ? nwaves : (uint32_t)(e * slab_blocks / kLanes);
      w_prev = c.w1;
      const size_t done_slabs = last ? nslabs : (size_t)c.w1 * kLanes / slab_blocks;
      c.d0 = d_prev;
      c.d1 = std::min(data_bytes, done_slabs * slab_vals * es);
      d_prev = c.d1;
    }
    c.s0 = std::min(sbytes, (size_t)c.w0 * wave_bytes);
    c.s1 = last ? sbytes : std::min(sbytes, (size_t)c.w1 * wave_bytes);
    chunks.push_back(c);
    sl = e;
  }

  const int S = std::max(1, std::min(nstreams, kMaxStreams));
  int dev = 0;
  CUZFP_HIP_TRY(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDevices) return CUZFP_ERROR_INVALID_ARGUMENT;
  PipelineCache& r = g_pipeline[dev];
  std::lock_guard<std::mutex> lock(r.mu);
  // zero-copy views (host_zero_copy): both buffers for a compression, the
  // array for a decompression (ordered schedule)
  const int zc = host_zero_copy();
  char* in_view = nullptr;
  char* out_view = nullptr;
  if (encode && zc >= 1) {
    in_view = mapped_view(h_data, data_bytes);
    out_view = in_view ? mapped_view(h_stream, sbytes) : nullptr;
    if (!out_view) in_view = nullptr;
  } else if (!encode && zc >= 2 && ordered) {
    out_view = mapped_view(h_data, data_bytes);
  }
  CallBuf bd, bs;
  if (!out_view) CUZFP_HIP_TRY(bd.get(r.d_data, data_bytes));
  if (!in_view) CUZFP_HIP_TRY(bs.get(r.d_stream, sbytes));
  size_t max_in = 0, max_out = 0;
  for (const Chunk& c : chunks) {
    max_in = std::max(max_in, encode ? c.d1 - c.d0 : c.s1 - c.s0);
    max_out = std::max(max_out, encode ? c.s1 - c.s0 : c.d1 - c.d0);
  }
  const bool in_pinned = encode ? data_pinned : stream_pinned;
  const bool out_pinned = encode ? stream_pinned : data_pinned;
  // the ordered schedule uses three of kPickStreams streams (pick_copy_queues)
  // whatever S is
  const int NS = ordered ? std::max(S, kPickStreams) : S;
  for (int i = r.nst; i < NS; i++) {
    CUZFP_HIP_TRY(hipStreamCreateWithFlags(&r.st[i], hipStreamNonBlocking));
    CUZFP_HIP_TRY(hipEventCreateWithFlags(&r.ev_in[i], hipEventDisableTiming));
    CUZFP_HIP_TRY(hipEventCreateWithFlags(&r.ev_kernel[i], hipEventDisableTiming));
    CUZFP_HIP_TRY(hipEventCreateWithFlags(&r.ev_done[i], hipEventDisableTiming));
    r.nst = i + 1;
  }
  if (ordered && !r.queues_picked && pick_copy_queues(r) != hipSuccess) {
    // The calibration only tunes which streams carry the copies: if it cannot
    // run (e.g. its 24 MiB of pinned and device memory are not available),
    // clear the error, keep the default roles and do not retry every call.
    (void)hipGetLastError();
    r.q_in = 0;
    r.q_k = 1;
    r.q_out = 2;
    r.queues_picked = true;
  }
  CallHostBuf pin_in[kMaxStreams], pin_out[kMaxStreams];
  for (int i = 0; i < S; i++) {
    if (!in_pinned) CUZFP_HIP_TRY(pin_in[i].get(r.pin_in[i], max_in));
    if (!out_pinned) CUZFP_HIP_TRY(pin_out[i].get(r.pin_out[i], max_out));
  }
  // on every return (an error included) nothing of this call is left running
  // on the cached streams when the next call reuses them (declared after the
  // call's own buffers, so it runs before they are freed)
  struct Drain {
    PipelineCache& r;
    int S;
    ~Drain() {
      for (int i = 0; i < S; i++) (void)hipStreamSynchronize(r.st[i]);
    }
  } drain{r, NS};
  char* hd = (char*)h_data;
  char* hs = (char*)h_stream;
  char* dd = (char*)bd.p;
  char* ds = (char*)bs.p;
  auto out_range = [&](const Chunk& c, size_t* o0, size_t* o1) {
    *o0 = encode ? c.s0 : c.d0;
    *o1 = encode ? c.s1 : c.d1;
  };
  const size_t n = chunks.size();
  if (in_view) {
    // one launch over the whole array: its loads of the pinned array and
    // stores of the pinned stream cross PCIe as the waves run
    return launch_encode(p, in_view, (uint64_t*)out_view, 0, nwaves, r.st[0]);  // Drain waits for it
  }
  if (ordered) {
    // three queues, each in chunk order: input copies, kernels, output copies
    // (on the streams pick_copy_queues chose).  Chunk i's input lands at (i + 1) input
    // copies' time, so its kernel and output copy start then, and only the
    // last chunk's kernel and output copy trail the input stream.  Slots
    // (i % S) only matter for the pinned staging buffers: a slot is reused
    // once its previous chunk's copies are done.
    hipStream_t sin = r.st[r.q_in], sk = r.st[r.q_k], sout = r.st[r.q_out];
    if (in_pinned && (out_pinned || out_view) && host_split_passes()) {
      // Between pinned buffers nothing waits on the host, so the queues are
      // filled in three passes -- every input copy, then every kernel, then
      // every output copy -- each chunk's input and kernel with an event of
      // its own.  (Filled chunk by chunk, an input copy was submitted after
      // the previous chunk's output copy, which waits on that chunk's kernel,
      // and the trace showed the input copies of a decompression starting
      // only after that kernel, 12-48 us late: tools/host_trace.py,
      // profiles/r05_host_trace_chunkwise.txt; in three passes
      // r05_host_trace.txt.  Decompression 48.7 -> 50.1 GB/s, compression
      // 49.2 -> 49.5: profiles/r05_host_sweep.txt.)
      CUZFP_HIP_TRY(r.chunk_events(n));
      for (size_t i = 0; i < n; i++) {
        const Chunk& c = chunks[i];
        const size_t i0 = encode ? c.d0 : c.s0, i1 = encode ? c.d1 : c.s1;
        if (i1 > i0)
          CUZFP_HIP_TRY(hipMemcpyAsync((encode ? dd : ds) + i0, (encode ? hd : hs) + i0, i1 - i0,
                                       hipMemcpyHostToDevice, sin));
        CUZFP_HIP_TRY(hipEventRecord(r.ev_chunk_in[i], sin));
      }
      for (size_t i = 0; i < n; i++) {
        const Chunk& c = chunks[i];
        CUZFP_HIP_TRY(hipStreamWaitEvent(sk, r.ev_chunk_in[i], 0));
        int rc = encode ? launch_encode(p, dd, (uint64_t*)ds, c.w0, c.w1 - c.w0, sk)
                        : launch_decode(p, (const uint64_t*)ds, out_view ? out_view : dd, c.w0, c.w1 - c.w0, sk);
        if (rc) return rc;
        CUZFP_HIP_TRY(hipEventRecord(r.ev_chunk_kernel[i], sk));
      }
      if (out_view) return CUZFP_SUCCESS;  // the kernels stored to the pinned array themselves
      for (size_t i = 0; i < n; i++) {
        size_t o0, o1;
        out_range(chunks[i], &o0, &o1);
        CUZFP_HIP_TRY(hipStreamWaitEvent(sout, r.ev_chunk_kernel[i], 0));
        if (o1 > o0)
          CUZFP_HIP_TRY(hipMemcpyAsync((encode ? hs : hd) + o0, (encode ? ds : dd) + o0, o1 - o0,
                                       hipMemcpyDeviceToHost, sout));
      }
      return CUZFP_SUCCESS;
    }
    for (size_t i = 0; i < n + S; i++) {
      if (i >= (size_t)S) {
        const size_t j = i - S;
        const int sj = (int)(j % S);
        if (!out_pinned) {
          CUZFP_HIP_TRY(hipEventSynchronize(r.ev_done[sj]));
          size_t o0, o1;
          out_range(chunks[j], &o0, &o1);
          if (o1 > o0) std::memcpy((encode ? hs : hd) + o0, pin_out[sj].p, o1 - o0);
        } else if (!in_pinned) {
          CUZFP_HIP_TRY(hipEventSynchronize(r.ev_in[sj]));
        }
      }
      if (i >= n) continue;
      const Chunk& c = chunks[i];
      const int s = (int)(i % S);
      const size_t i0 = encode ? c.d0 : c.s0, i1 = encode ? c.d1 : c.s1;
      char* src = (encode ? hd : hs) + i0;
      if (i1 > i0) {
        if (!in_pinned) {
          std::memcpy(pin_in[s].p, src, i1 - i0);
          src = (char*)pin_in[s].p;
        }
        CUZFP_HIP_TRY(hipMemcpyAsync((encode ? dd : ds) + i0, src, i1 - i0, hipMemcpyHostToDevice, sin));
      }
      CUZFP_HIP_TRY(hipEventRecord(r.ev_in[s], sin));
      // every earlier chunk's input (encode) / kernel (decode) is ahead of
      // this one in its queue, so one wait covers the straddling waves
      CUZFP_HIP_TRY(hipStreamWaitEvent(sk, r.ev_in[s], 0));
      int rc = encode ? launch_encode(p, dd, (uint64_t*)ds, c.w0, c.w1 - c.w0, sk)
                      : launch_decode(p, (const uint64_t*)ds, out_view ? out_view : dd, c.w0, c.w1 - c.w0, sk);
      if (rc) return rc;
      CUZFP_HIP_TRY(hipEventRecord(r.ev_kernel[s], sk));
      if (out_view) continue;  // the kernel stored its blocks to the pinned array itself
      CUZFP_HIP_TRY(hipStreamWaitEvent(sout, r.ev_kernel[s], 0));
      size_t o0, o1;
      out_range(c, &o0, &o1);
      if (o1 > o0)
        CUZFP_HIP_TRY(hipMemcpyAsync(out_pinned ? (encode ? hs : hd) + o0 : (char*)pin_out[s].p,
                                     (encode ? ds : dd) + o0, o1 - o0, hipMemcpyDeviceToHost, sout));
      CUZFP_HIP_TRY(hipEventRecord(r.ev_done[s], sout));
    }
    return CUZFP_SUCCESS;
  }
  for (size_t i = 0; i < n + S; i++) {
    // retire chunk i - S: its slot's buffers become free
    if (i >= (size_t)S) {
      const size_t j = i - S;
      const int sj = (int)(j % S);
      CUZFP_HIP_TRY(hipEventSynchronize(r.ev_done[sj]));
      if (!out_pinned) {
        size_t o0, o1;
        out_range(chunks[j], &o0, &o1);
        if (o1 > o0) std::memcpy((encode ? hs : hd) + o0, pin_out[sj].p, o1 - o0);
      }
    }
    if (i >= n) continue;
    const Chunk& c = chunks[i];
    const int s = (int)(i % S);
    hipStream_t st = r.st[s];
    // input copy
    const size_t i0 = encode ? c.d0 : c.s0, i1 = encode ? c.d1 : c.s1;
    char* src = (encode ? hd : hs) + i0;
    char* dst = (encode ? dd : ds) + i0;
    if (i1 > i0) {
      if (!in_pinned) {
        std::memcpy(pin_in[s].p, src, i1 - i0);
        src = (char*)pin_in[s].p;
      }
      CUZFP_HIP_TRY(hipMemcpyAsync(dst, src, i1 - i0, hipMemcpyHostToDevice, st));
    }
    CUZFP_HIP_TRY(hipEventRecord(r.ev_in[s], st));
    // encode kernel over waves [w0, w1): needs the neighbouring chunks' input
    if (encode)
      for (size_t k = (i >= (size_t)S - 1 ? i - S + 1 : 0); k < i; k++)
      CUZFP_HIP_TRY(hipStreamWaitEvent(st, r.ev_in[k % S], 0));
    int rc = encode ? launch_encode(p, dd, (uint64_t*)ds, c.w0, c.w1 - c.w0, st)
                    : launch_decode(p, (const uint64_t*)ds, dd, c.w0, c.w1 - c.w0, st);
    if (rc) return rc;
    CUZFP_HIP_TRY(hipEventRecord(r.ev_kernel[s], st));
    // output copy: decoded slabs may contain blocks of earlier chunks' kernels
    if (!encode)
      for (size_t k = (i >= (size_t)S - 1 ? i - S + 1 : 0); k < i; k++)
        CUZFP_HIP_TRY(hipStreamWaitEvent(st, r.ev_kernel[k % S], 0));
    size_t o0, o1;
    out_range(c, &o0, &o1);
    if (o1 > o0) {
      char* osrc = (encode ? ds : dd) + o0;
      char* odst = out_pinned ? (encode ? hs : hd) + o0 : (char*)pin_out[s].p;
      CUZFP_HIP_TRY(hipMemcpyAsync(odst, osrc, o1 - o0, hipMemcpyDeviceToHost, st));
    }
    CUZFP_HIP_TRY(hipEventRecord(r.ev_done[s], st));
  }
  return CUZFP_SUCCESS;
}

// ---------------------------------------------------------------------------
}  // namespace cuzfp


// ---------------------------------------------------------------------------
// C-ABI

using namespace cuzfp;

extern "C" {

int cuzfp_hip_abi_version(void) { return CUZFP_HIP_ABI_VERSION; }

const char* cuzfp_hip_status_string(int status) {
  switch (status) {
    case CUZFP_SUCCESS: return "success";
    case CUZFP_ERROR_INVALID_ARGUMENT: return "invalid argument";
    case CUZFP_ERROR_UNSUPPORTED_TYPE: return "unsupported scalar type";
    case CUZFP_ERROR_BUFFER_TOO_SMALL: return "stream buffer too small";
    case CUZFP_ERROR_HIP: return "HIP runtime error";
  }
  return "unknown status";
}

int cuzfp_hip_last_hip_error(void) { return t_last_hip; }

unsigned cuzfp_hip_rate_to_maxbits(double rate, int type, unsigned dims, int wra) {
  if (dims < 1 || dims > 3 || !(rate >= 0)) return 0;
  const unsigned n = 1u << (2 * dims);
  unsigned bits = (unsigned)floor(n * rate + 0.5);
  if (type == CUZFP_TYPE_FLOAT) bits = std::max(bits, 1u + 8u);
  if (type == CUZFP_TYPE_DOUBLE) bits = std::max(bits, 1u + 11u);
  if (wra) bits = (bits + 63) & ~63u;
  return bits;
}

size_t cuzfp_hip_stream_bytes(int type, unsigned nx, unsigned ny, unsigned nz, unsigned maxbits) {
  Problem p;
  if (make_problem(type, nx, ny, nz, 0, 0, 0, maxbits, &p) != CUZFP_SUCCESS) return 0;
  return stream_bytes_of(p.g);
}

size_t cuzfp_hip_maximum_size(int type, unsigned nx, unsigned ny, unsigned nz, unsigned maxbits) {
  // zfp_structs.h:222-251 in fixed-rate mode: minbits == maxbits, so every
  // block is exactly maxbits bits; plus the reference's 148-bit header allowance
  Problem p;
  if (make_problem(type, nx, ny, nz, 0, 0, 0, maxbits, &p) != CUZFP_SUCCESS) return 0;
  return ((148 + (size_t)p.g.nblocks * maxbits + 63) & ~(size_t)63) / 8;
}

int cuzfp_hip_encode(const void* d_data, int type, unsigned nx, unsigned ny, unsigned nz,
                     long long sx, long long sy, long long sz, unsigned maxbits,
                     uint64_t* d_stream, size_t stream_capacity, size_t* out_bytes,
                     hipStream_t stream) {
  Problem p;
  int rc = make_problem(type, nx, ny, nz, sx, sy, sz, maxbits, &p);
  if (rc) return rc;
  if (!d_data || !d_stream) return CUZFP_ERROR_INVALID_ARGUMENT;
  const size_t need = stream_bytes_of(p.g);
  if (stream_capacity < need) return CUZFP_ERROR_BUFFER_TOO_SMALL;
  rc = launch_encode(p, d_data, d_stream, 0, waves_of(p.g), stream);
  if (rc == CUZFP_SUCCESS && out_bytes) *out_bytes = need;
  return rc;
}

int cuzfp_hip_decode(const uint64_t* d_stream, size_t stream_bytes, int type, unsigned nx,
                     unsigned ny, unsigned nz, long long sx, long long sy, long long sz,
                     unsigned maxbits, void* d_data, hipStream_t stream) {
  Problem p;
  int rc = make_problem(type, nx, ny, nz, sx, sy, sz, maxbits, &p);
  if (rc) return rc;
  if (!d_data || !d_stream) return CUZFP_ERROR_INVALID_ARGUMENT;
  if (stream_bytes < stream_bytes_of(p.g)) return CUZFP_ERROR_BUFFER_TOO_SMALL;
  return launch_decode(p, d_stream, d_data, 0, waves_of(p.g), stream);
}

int cuzfp_hip_copy(const void* d_src, void* d_dst, size_t bytes, hipStream_t stream) {
  if (!d_src || !d_dst || (bytes & 15) || (((uintptr_t)d_src | (uintptr_t)d_dst) & 15))
    return CUZFP_ERROR_INVALID_ARGUMENT;
  if (!bytes) return CUZFP_SUCCESS;
  const size_t n16 = bytes / 16;
  // one grid over the buffer up to 16 Mi workgroups (the measured shape, 4 GiB
  // a launch); past that the kernel's grid-stride loop covers the rest, so a
  // launch never nears the 2^32 work-item limit
  const unsigned grid = (unsigned)std::min<size_t>((n16 + 255) / 256, 1u << 24);
  hipLaunchKernelGGL(copy16_nt, dim3(grid), dim3(256), 0, stream, (const u32x4*)d_src, (u32x4*)d_dst, n16);
  const hipError_t e = hipGetLastError();
  t_last_hip = e;
  return e == hipSuccess ? CUZFP_SUCCESS : CUZFP_ERROR_HIP;
}

int cuzfp_hip_compress_host(const void* h_data, int type, unsigned nx, unsigned ny,
                            unsigned nz, unsigned maxbits, void* h_stream,
                            size_t stream_capacity, size_t* out_bytes, int nstreams) {
  Problem p;
  int rc = make_problem(type, nx, ny, nz, 0, 0, 0, maxbits, &p);
  if (rc) return rc;
  if (!h_data || !h_stream) return CUZFP_ERROR_INVALID_ARGUMENT;
  const size_t need = stream_bytes_of(p.g);
  if (stream_capacity < need) return CUZFP_ERROR_BUFFER_TOO_SMALL;
  rc = host_pipeline(p, true, (void*)h_data, h_stream, nstreams);
  if (!rc && out_bytes) *out_bytes = need;
  return rc;
}

int cuzfp_hip_release_host_cache(int device) {
  if (device < -1 || device >= kMaxDevices) return CUZFP_ERROR_INVALID_ARGUMENT;
  if (device == -1) CUZFP_HIP_TRY(hipGetDevice(&device));
  if (device < 0 || device >= kMaxDevices) return CUZFP_ERROR_INVALID_ARGUMENT;
  PipelineCache& r = g_pipeline[device];
  std::lock_guard<std::mutex> lock(r.mu);
  if (!r.nst && !r.d_data.p && !r.d_stream.p) return CUZFP_SUCCESS;  // never used
  int prev = 0;
  CUZFP_HIP_TRY(hipGetDevice(&prev));
  CUZFP_HIP_TRY(hipSetDevice(device));
  for (int i = 0; i < r.nst; i++) (void)hipStreamSynchronize(r.st[i]);
  r.d_data.release();
  r.d_stream.release();
  for (int i = 0; i < kMaxStreams; i++) {
    r.pin_in[i].release();
    r.pin_out[i].release();
  }
  for (int i = 0; i < r.nst; i++) {
    (void)hipEventDestroy(r.ev_in[i]);
    (void)hipEventDestroy(r.ev_kernel[i]);
    (void)hipEventDestroy(r.ev_done[i]);
    (void)hipStreamDestroy(r.st[i]);
  }
  for (size_t i = 0; i < r.ev_chunk_in.size(); i++) {
    (void)hipEventDestroy(r.ev_chunk_in[i]);
    (void)hipEventDestroy(r.ev_chunk_kernel[i]);
  }
  r.ev_chunk_in.clear();
  r.ev_chunk_kernel.clear();
  r.nst = 0;
  r.queues_picked = false;
  CUZFP_HIP_TRY(hipSetDevice(prev));
  return CUZFP_SUCCESS;
}

int cuzfp_hip_decompress_host(const void* h_stream, size_t stream_bytes, int type,
                              unsigned nx, unsigned ny, unsigned nz, unsigned maxbits,
                              void* h_data, int nstreams) {
  Problem p;
  int rc = make_problem(type, nx, ny, nz, 0, 0, 0, maxbits, &p);
  if (rc) return rc;
  if (!h_data || !h_stream) return CUZFP_ERROR_INVALID_ARGUMENT;
  if (stream_bytes < stream_bytes_of(p.g)) return CUZFP_ERROR_BUFFER_TOO_SMALL;
  return host_pipeline(p, false, h_data, (void*)h_stream, nstreams);
}

}  // extern "C"
