// cuzfp_amd/csrc/kernels.hpp -- MI355X (gfx950) zfp fixed-rate kernels.
//
// One zfp block per lane, 64 blocks (one wave) per workgroup:
//
//   encode: coalesced 16-byte HBM gathers of the 4^d block  ->  per-lane block
//           coder (zfp_block.hpp: exponent, quantize, lifting, negabinary,
//           bit-plane transpose, embedded plane coder)  ->  the lane's bits land
//           in an LDS image of the wave's contiguous stream segment
//           (64 * maxbits bits = maxbits words)  ->  one coalesced copy-out.
//   decode: coalesced copy-in of the wave's stream segment to LDS  ->  per-lane
//           128-bit window reader + block decoder  ->  16-byte stores.
//
// Replaces the reference's six CUDA kernels (src/cuZFP/encode{1,2,3}.cuh,
// decode{1,2,3}.cuh), which use one 64-thread CTA per 3D block with serial
// tid-0 packing (encode3.cuh:336-362, decode3.cuh:111-144) and 64-bit global
// atomics to share stream words in 1D/2D (shared.h:394-424).  Here a wave's
// stream segment is word aligned (64 * maxbits is a multiple of 64), so
// workgroups never share a stream word and no global atomics are needed.
//
// Instantiated per scalar type in inst_{f32,f64,i32,i64}.hip (parallel build).
#pragma once
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <atomic>
#include <type_traits>

#if defined(CUZFP_PROBE) && CUZFP_PROBE == 9
// Diagnostic build (tools/probe.py stamps): lane 0 of every wave records
// s_memtime at the codec's phase boundaries, plus its HW_ID / XCC_ID.
#define CUZFP_STAMP_WAVES 65536
__device__ uint64_t g_stamps[CUZFP_STAMP_WAVES * 10];
__device__ __forceinline__ uint32_t stamp_wave() { return blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); }
#define ZFP_STAMP(i)                                                              \
  do {                                                                            \
    if ((threadIdx.x & 63) == 0 && stamp_wave() < CUZFP_STAMP_WAVES)              \
      g_stamps[stamp_wave() * 10 + 1 + (i)] = __builtin_amdgcn_s_memtime();      \
  } while (0)
__device__ __forceinline__ void stamp_hwid() {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if ((threadIdx.x & 63) == 0 && stamp_wave() < CUZFP_STAMP_WAVES)
    g_stamps[stamp_wave() * 10] = (uint64_t)hw | ((uint64_t)xcc << 32);
}
// global 100 MHz clock, comparable across CUs: slot 8 = start, 9 = end
__device__ __forceinline__ void stamp_real(int slot) {
  if ((threadIdx.x & 63) == 0 && stamp_wave() < CUZFP_STAMP_WAVES)
    g_stamps[stamp_wave() * 10 + slot] = __builtin_amdgcn_s_memrealtime();
}
#define ZFP_STAMP_REAL(slot) stamp_real(slot)
#define ZFP_STAMP_HWID() stamp_hwid()
#else
#define ZFP_STAMP_HWID()
#define ZFP_STAMP_REAL(slot)
#endif

#include "zfp_block.hpp"
#include "launch.hpp"

namespace cuzfp {

// The plane decoder's chunk tables (zfp_block.hpp), generated at compile time;
// each decode workgroup copies them to LDS.
__device__ const ChunkLut g_chunk_lut = make_chunk_lut();
constexpr size_t kChunkLutBytes = sizeof(ChunkLut);
// the part a DIMS-dimensional decoder holds in LDS: 1D reads chunk 1's table
// alone (a 1D group code fits one chunk), 8 of the 16 KiB
template <int DIMS>
constexpr size_t chunk_lut_bytes() { return DIMS == 1 ? kLutPairs * 4 : kChunkLutBytes; }
// ... and the plane coder's spread tables (2 KiB): a static LDS array at
// address 0, so a lookup is one ds_read_b32 at (byte << 2) with the table in
// the offset field.  Every wave of a workgroup writes the whole table itself
// (the same values to the same addresses) and waits only for its own writes,
// so the waves need no barrier.
__device__ const SpreadTab g_spread_tab = make_spread_tab();
// ... and the 1D tables (zfp_block.hpp): the encoder's pair table, the
// decoder's plane table
__device__ const Pair1dLut g_pair1d_lut = make_pair1d_lut();
__device__ const Plane1dDecLut g_plane1d_lut = make_plane1d_dec_lut();
constexpr size_t kSpreadTabBytes = sizeof(SpreadTab);
typedef __attribute__((address_space(3))) const uint32_t lds_spread;
typedef lds_spread* P1dPtr;

// n / d and n % d for a wave-uniform d: shifts when d is a power of two (the
// words or dwords a block takes at rates 4, 8, 16, ...), the compiler's
// reciprocal-based division (~15 VALU and a readfirstlane) otherwise
__device__ __forceinline__ void udivmod_uniform(uint32_t n, uint32_t d, uint32_t& q, uint32_t& r) {
  if (__builtin_expect((d & (d - 1)) == 0, 1)) {
    const uint32_t sh = (uint32_t)__builtin_ctz(d);
    q = n >> sh;
    r = n & (d - 1);
  } else {
    q = n / d;
    r = n % d;
  }
}

// ---------------------------------------------------------------------------
// LDS bit writers / reader (one lane, one block)

// maxbits % 64 == 0: the lane owns LDS words [lane*(W+4), lane*(W+4) + W) of a
// zeroed image, plus 4 slack words.  A put ORs its bits in at the running bit
// position (ds_or_b64 on the two words it can touch), so consecutive puts do
// not form a read-modify-write chain through an accumulator and need no
// flush branch; the coder's only serial state is `pos`.  Once W words are
// filled the block is full; what the coder still produces (it finishes the
// pair of planes it is in: at most 2 x 128 bits + one straddled word) lands in
// the slack, which the copy-out skips.
constexpr uint32_t kSlackWords = 6;
template <bool PRIO = true>
struct LdsOrWriter {
  static constexpr bool kPrio = PRIO;  // progress_priority schedule (zfp_block.hpp)
  static constexpr bool kZeroInline = true;  // zero blocks coded inline (encode_block)
  uint64_t* p;          // the lane's column: word j at p[64 j], W + kSlackWords words, zeroed
  lds_spread* lut;      // the workgroup's spread tables
  uint32_t pos, lim;    // bits produced; 64 * W
  P1dPtr p1d;           // 1D: the workgroup's pair table (Pair1dLut)
  uint64_t fit_lim;     // 2^15 - 1 in SGPRs (encode_plane_step's fit test)
  __device__ __forceinline__ uint32_t pair1d(uint32_t o) const { return *(P1dPtr)((uintptr_t)p1d + o); }
  __device__ __forceinline__ bool full() const { return pos >= lim; }
  __device__ __forceinline__ void put(uint64_t v, unsigned n) {  // v < 2^n
    const uint32_t w = pos >> 6;
    uint64_t* q = p + w * 64;
    // the 64-bit shifts use the low 6 bits of their counts: pos & 63 and
    // 63 - (pos & 63) = (pos ^ 63) & 63 (one full-rate XOR); plain shifts
    // (an inline-asm shift read by the next one costs an s_nop)
    const uint64_t lo = v << (pos & 63u);
    const uint64_t hi = (v >> 1) >> ((pos ^ 63u) & 63u);
    atomicOr((unsigned long long*)&q[0], (unsigned long long)lo);
    atomicOr((unsigned long long*)&q[64], (unsigned long long)hi);
    pos += n;
  }
  // o: byte offset of the entry (byte_off8)
  __device__ __forceinline__ uint32_t sp0(uint32_t o) const { return *(lds_spread*)((uintptr_t)lut + o); }
  __device__ __forceinline__ uint32_t sp1(uint32_t o) const { return *(lds_spread*)((uintptr_t)(lut + 256) + o); }
  __device__ __forceinline__ uint32_t spread(uint32_t b) const { return lut[256 + b] >> 1; }
  __device__ __forceinline__ void zero_bit() { pos++; }
  // every LDS access issued so far has completed (s_waitcnt lgkmcnt(0))
  __device__ __forceinline__ void lds_wait() const { __builtin_amdgcn_s_waitcnt(0xc07f); }
  __device__ __forceinline__ void finish() {}
  // a full lane keeps stepping with its wave: restart it at the first slack
  // row each plane, so its (discarded) pieces stay within rows W .. W + 3
  __device__ __forceinline__ void settle() { pos = pos < lim ? pos : lim; }
  // a zero block: full from the start, so every bit of it lands in the slack
  __device__ __forceinline__ void mark_full(bool z) { pos = z ? lim : pos; }
};

// general maxbits: the lane's bits are [pos0, end) of the wave's segment;
// 64-bit chunks are OR-ed into the (zeroed) LDS image with ds_or_b64, since
// the first and last words of a lane's range are shared with its neighbours.
template <bool PRIO = true>
struct LdsBitWriter {
  static constexpr bool kPrio = PRIO;
  uint64_t* lds;
  lds_spread* lut;         // the workgroup's spread tables
  uint32_t pos, end, cnt;  // pos: stream offset of acc's bit 0
  uint64_t acc;
  P1dPtr p1d;              // 1D: the workgroup's pair table (Pair1dLut)
  uint64_t fit_lim;        // 2^15 - 1 in SGPRs (encode_plane_step's fit test)
  __device__ __forceinline__ uint32_t pair1d(uint32_t o) const { return *(P1dPtr)((uintptr_t)p1d + o); }
  __device__ __forceinline__ uint32_t sp0(uint32_t o) const { return *(lds_spread*)((uintptr_t)lut + o); }
  __device__ __forceinline__ uint32_t sp1(uint32_t o) const { return *(lds_spread*)((uintptr_t)(lut + 256) + o); }
  __device__ __forceinline__ uint32_t spread(uint32_t b) const { return lut[256 + b] >> 1; }
  __device__ __forceinline__ bool full() const { return pos + cnt >= end; }
  __device__ __forceinline__ void emit(uint64_t v) {
    if (pos >= end) return;  // bits past maxbits are dropped
    const uint32_t room = end - pos;
    if (room < 64) v &= lowmask(room);
    const uint32_t w = pos >> 6, sh = pos & 63;
    atomicOr((unsigned long long*)&lds[w], (unsigned long long)(v << sh));
    if (sh) atomicOr((unsigned long long*)&lds[w + 1], (unsigned long long)(v >> (64 - sh)));
    pos += 64;
  }
  __device__ __forceinline__ void put(uint64_t v, unsigned n) {
    acc |= v << cnt;
    const unsigned c = cnt + n;
    if (c >= 64) {
      emit(acc);
      acc = (v >> 1) >> (63 - cnt);
      cnt = c - 64;
    } else {
      cnt = c;
    }
  }
  __device__ __forceinline__ void zero_bit() {
    if (++cnt == 64) {
      emit(acc);
      acc = 0;
      cnt = 0;
    }
  }
  __device__ __forceinline__ void finish() {
    if (cnt && pos < end) emit(acc);
  }
  __device__ __forceinline__ void settle() {}  // emit() drops bits past maxbits
  // every LDS access issued so far has completed (s_waitcnt lgkmcnt(0))
  __device__ __forceinline__ void lds_wait() const { __builtin_amdgcn_s_waitcnt(0xc07f); }
};

// maxbits <= 64 (1D rate <= 16, 2D rate <= 4: BASELINE's 2D 8192^2 rate 2 and
// 1D rate 8): the lane's whole block is one 64-bit register.  A put ORs its
// bits in at the count; the count stops at maxbits, so a full lane's further
// puts land at or past bit maxbits, which the kernel masks off.  With maxbits
// = 64 (FULL64) a full lane's puts are masked to zero instead (a shift by 64
// would wrap).  No LDS image, no flush.
template <bool PRIO = true, bool FULL64 = false>
struct RegWriter {
  static constexpr bool kPrio = PRIO;
  lds_spread* lut;  // the workgroup's spread tables
  P1dPtr p1d;       // 1D: the pair table
  uint64_t acc;
  uint32_t cnt, mb;  // bits produced (at most mb); maxbits
  __device__ __forceinline__ bool full() const { return cnt >= mb; }
  __device__ __forceinline__ void put(uint64_t v, unsigned n) {
    if constexpr (FULL64) v &= (uint64_t)(int64_t)((int32_t)(cnt - 64u) >> 31);  // all ones while cnt < 64
    acc |= shl64(v, cnt);
    cnt = umin(cnt + n, mb);
  }
  __device__ __forceinline__ void zero_bit() { cnt = umin(cnt + 1, mb); }
  __device__ __forceinline__ uint32_t sp0(uint32_t o) const { return *(lds_spread*)((uintptr_t)lut + o); }
  __device__ __forceinline__ uint32_t sp1(uint32_t o) const { return *(lds_spread*)((uintptr_t)(lut + 256) + o); }
  __device__ __forceinline__ uint32_t spread(uint32_t b) const { return lut[256 + b] >> 1; }
  __device__ __forceinline__ uint32_t pair1d(uint32_t o) const { return *(P1dPtr)((uintptr_t)p1d + o); }
  __device__ __forceinline__ void finish() {}
  __device__ __forceinline__ void settle() {}
  __device__ __forceinline__ uint64_t bits() const { return acc & lowmask(mb); }
  // every LDS access issued so far has completed (s_waitcnt lgkmcnt(0))
  __device__ __forceinline__ void lds_wait() const { __builtin_amdgcn_s_waitcnt(0xc07f); }
};

// maxbits 32 for floating-point blocks: a coded block's first stream bit is
// the low bit of its exponent field 2e + 1, always one, so the writer keeps
// stream bits 1 .. 32 in a 32-bit register at bit positions 0 .. 31 and the
// count one less than the bits produced.  Every put then shifts by at most 31
// (a 32-bit shift: the 64-bit one is a slow-issue VALU instruction), a full
// lane's further bits land at position 31 (stream bit 32, dropped by bits())
// or beyond (gone), and a zero block (no head()) stays all zeros.  Integer
// blocks, which have no exponent, keep RegWriter.
template <bool PRIO = true>
struct RegWriter32 {
  static constexpr bool kPrio = PRIO;
  static constexpr bool kPut32 = true;  // put() keeps the low 32 bits of its value
  lds_spread* lut;
  P1dPtr p1d;
  uint32_t acc, cnt;  // stream bits 1 .., at bit 0 ..; bits produced - 1 (0 before the exponent)
  __device__ __forceinline__ bool full() const { return cnt >= 31u; }
  __device__ __forceinline__ void head(uint64_t v, unsigned n) {  // the exponent field, v odd
    acc = (uint32_t)(v >> 1);
    cnt = n - 1u;
  }
  __device__ __forceinline__ void put(uint32_t v, unsigned n) {
    acc |= v << cnt;
    cnt = umin(cnt + n, 31u);
  }
  __device__ __forceinline__ void zero_bit() { cnt = umin(cnt + 1u, 31u); }
  __device__ __forceinline__ uint32_t sp0(uint32_t o) const { return *(lds_spread*)((uintptr_t)lut + o); }
  __device__ __forceinline__ uint32_t sp1(uint32_t o) const { return *(lds_spread*)((uintptr_t)(lut + 256) + o); }
  __device__ __forceinline__ uint32_t spread(uint32_t b) const { return lut[256 + b] >> 1; }
  __device__ __forceinline__ uint32_t pair1d(uint32_t o) const { return *(P1dPtr)((uintptr_t)p1d + o); }
  __device__ __forceinline__ void finish() {}
  __device__ __forceinline__ void settle() {}
  __device__ __forceinline__ uint64_t bits() const { return cnt ? (acc << 1) | 1u : 0u; }
  // every LDS access issued so far has completed (s_waitcnt lgkmcnt(0))
  __device__ __forceinline__ void lds_wait() const { __builtin_amdgcn_s_waitcnt(0xc07f); }
};

// the register writer of a maxbits-32 (REG 1) / 64 (REG 2) block
template <typename Scalar, bool PRIO, int REG>
using reg_writer = typename std::conditional<REG == 1 && !traits<Scalar>::is_int, RegWriter32<PRIO>,
                                             RegWriter<PRIO, REG == 2>>::type;

// Reader over the lane's block in the wave's lane-interleaved LDS image
// (dword j of the block at lds32[64 * j]; pos counts bits from the block's
// start).  The table decoder reads its windows fresh per plane; the general
// decoder (decode_plane) keeps the five dwords that
// cover bits [pos, pos + 128) in registers: peek()/peek2() funnel them into
// place with v_alignbit_b32, and skip() moves the bit offset and issues the
// LDS reads for the new position at once.  The plane decoder skips as soon as
// it knows where the next plane starts -- before it places the plane's ones --
// so those reads land while it still has work to do.
template <bool PRIO = true>
struct LdsReader {
  static constexpr bool kPrio = PRIO;
  const uint32_t* lds32;
  const uint32_t* lut32;  // the workgroup's copy of the chunk tables (static LDS)
  const uint16_t* d1d;    // 1D: the workgroup's plane table (Plane1dDecLut)
  uint32_t pos;
  uint32_t end;  // the block's budget end (decode_planes sets it; pos never passes it)
  uint32_t x0, x1, x2, x3, x4;
  // byte address of the row holding bit p: lds32 + 256 * (p >> 5), in two
  // instructions (the compiler's form of the same expression takes three)
  typedef __attribute__((address_space(3))) const uint32_t lds_u32;
  __device__ __forceinline__ lds_u32* row(uint32_t p) const {
    uint32_t a;
    asm("v_lshl_add_u32 %0, %1, 8, %2"
        : "=v"(a)
        : "v"(p >> 5), "v"((uint32_t)(uintptr_t)(lds_u32*)lds32));
    return (lds_u32*)(uintptr_t)a;
  }
  // table decoder: 64 bits at pos and 32 bits at pos + m, read fresh
  __device__ __forceinline__ void windows(uint32_t m, uint64_t& w, uint32_t& g) const {
    const uint32_t q = pos + m;
    lds_u32* r = row(pos);
    lds_u32* t = row(q);
    const uint32_t a0 = r[0], a1 = r[64], a2 = r[128];
    const uint32_t b0 = t[0], b1 = t[64];
    w = (uint64_t)__builtin_amdgcn_alignbit(a1, a0, pos) |
        ((uint64_t)__builtin_amdgcn_alignbit(a2, a1, pos) << 32);
    g = __builtin_amdgcn_alignbit(b1, b0, q);
  }
  // The fast plane step's windows: the group window m bits on (the step's
  // critical path: its chunk lookups need it) and the 64-bit window at the
  // position (needed only at the step's end).  Both are issued here, the
  // group window's read first, and only it is waited for (lgkmcnt(2): the
  // window's two reads may still be in flight); the window's dwords land in
  // the lookups' shadow and window_w_make combines them after the step's one
  // other wait.  (The compiler's own placement waits before each first use:
  // six waits a plane.)
  __device__ __forceinline__ uint32_t window_g(uint32_t m, WRaw& wr) const {
    const uint32_t q = pos + m;
    lds_u32* t = row(q);
    const uint32_t b0 = t[0], b1 = t[64];
    __builtin_amdgcn_sched_barrier(0);
    lds_u32* r = row(pos);
    wr = WRaw{r[0], r[64], r[128]};
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xc27f);  // lgkmcnt(2); vmcnt / expcnt not waited for
    __builtin_amdgcn_sched_barrier(0);
    return __builtin_amdgcn_alignbit(b1, b0, q);
  }
  __device__ __forceinline__ uint64_t window_w_make(const WRaw& a) const {
    return (uint64_t)__builtin_amdgcn_alignbit(a.a1, a.a0, pos) | ((uint64_t)__builtin_amdgcn_alignbit(a.a2, a.a1, pos) << 32);
  }
  // every LDS read issued so far has landed (s_waitcnt lgkmcnt(0))
  __device__ __forceinline__ void lds_wait() const { __builtin_amdgcn_s_waitcnt(0xc07f); }
  // The chunk tables are the kernel's static LDS (address 0), so an entry's
  // byte offset goes straight into ds_read's address with the state in the
  // offset field.  (The plane loops are bound by the count of VALU
  // instructions -- SQ_ACTIVE_INST_VALU is one quad-cycle per instruction,
  // with two issued together in about a tenth of them, SQ_ACTIVE_INST_VALU2 --
  // so the offsets are built with the fewest instructions, three-input ones
  // included.)
  __device__ __forceinline__ uint32_t tab(uint32_t byte_off) const {
    return *(lds_u32*)((uintptr_t)(lds_u32*)lut32 + byte_off);
  }
  // (The chunk lookups index the tables with the window as read.  Masking it
  // to zero for lanes whose leading test is "0" -- entry 0, a broadcast --
  // cut the LDS bank-conflict cycles, but its two VALU a plane cost more:
  // 256^3 r8 decode 23.5 -> 23.2 us without it, tools/xvar.py, r04_nolead.)
  // byte offsets of chunk 1's state-2 entry and selector (chunk bits 0-9;
  // 8-byte entries, the table at LDS address 0) and of chunk 2's pair of
  // state-0/1 entries (bits 10-19; from the pair table's start, kLutPairs)
  static __device__ __forceinline__ uint32_t off1(uint32_t gm) {
    uint32_t a;
    asm("v_lshlrev_b32 %0, 3, %1\n\tv_and_b32 %0, 0x1ff8, %0" : "=&v"(a) : "v"(gm));
    return a;
  }
  static __device__ __forceinline__ uint32_t off2(uint32_t gm) {
    uint32_t a;
    asm("v_lshrrev_b32 %0, 7, %1\n\tv_and_b32 %0, 0x1ff8, %0" : "=&v"(a) : "v"(gm));
    return a;
  }
  static constexpr uint32_t kPairBytes = 4u * kLutPairs;  // byte address of the pair table
  typedef __attribute__((address_space(3))) const uint64_t lds_u64;
  __device__ __forceinline__ uint2 tab64(uint32_t byte_off) const {
    const uint64_t v = *(lds_u64*)((uintptr_t)(lds_u32*)lut32 + byte_off);
    return uint2{(uint32_t)v, (uint32_t)(v >> 32)};
  }
  // the table steps' lookups: entry (2, g's chunk 1) with its chunk-2
  // selector, and the pair (0, chunk 2), (1, chunk 2), each one ds_read_b64.
  // (With n = N-1 the group part is the last position's bit alone; the parse
  // then runs past position N-1, which the steps' implied-one rule resolves.)
  __device__ __forceinline__ void chunks_fast(uint32_t g, uint32_t& e1, uint32_t& sel, uint32_t& e2a,
                                              uint32_t& e2b) const {
    // (sending the lookups of lanes whose leading test is "0" to entry 0, a
    // broadcast, measured neutral in round 6: profiles/r06_ab_dmask.txt)
    const uint2 c = tab64(off1(g));
    const uint2 p = tab64(kPairBytes + off2(g));
    e1 = c.x;
    sel = c.y;
    e2a = p.x;
    e2b = p.y;
  }
  // continuation pairs (dense planes): 32 stream bits at bit q of the block,
  // chunk A in state st (0/1), chunk B in states 0 and 1
  __device__ __forceinline__ uint32_t window32(uint32_t q) const {
    lds_u32* t = row(q);
    return __builtin_amdgcn_alignbit(t[64], t[0], q);
  }
  __device__ __forceinline__ void chunks_st(uint32_t g, uint32_t st, uint32_t& eA, uint32_t& eBa,
                                            uint32_t& eBb) const {
    eA = tab(kPairBytes + ((g << 3) & 0x1ff8u) + 4u * st);
    const uint2 p = tab64(kPairBytes + off2(g));
    eBa = p.x;
    eBb = p.y;
  }
  __device__ __forceinline__ uint32_t chunk1_fast(uint32_t g) const {
    return tab(off1(g));
  }
  // 1D: an entry of the plane table (o: byte offset) and the 8 stream bits at pos
  typedef __attribute__((address_space(3))) const uint16_t lds_u16;
  __device__ __forceinline__ uint32_t dec1d(uint32_t o) const { return *(lds_u16*)((uintptr_t)(lds_u16*)d1d + o); }
  __device__ __forceinline__ uint32_t bits8() const { return window32(pos) & 0xffu; }
  __device__ __forceinline__ void load() {
    const uint32_t* r = lds32 + (pos >> 5) * 64;
    x0 = r[0];
    x1 = r[64];
    x2 = r[128];
    x3 = r[192];
    x4 = r[256];
  }
  __device__ __forceinline__ void init(uint32_t bitpos) {
    pos = bitpos;
    load();
  }
  __device__ __forceinline__ void peek2(uint64_t& a, uint64_t& b) const {
    const uint32_t sh = pos & 31;
    a = (uint64_t)__builtin_amdgcn_alignbit(x1, x0, sh) |
        ((uint64_t)__builtin_amdgcn_alignbit(x2, x1, sh) << 32);
    b = (uint64_t)__builtin_amdgcn_alignbit(x3, x2, sh) |
        ((uint64_t)__builtin_amdgcn_alignbit(x4, x3, sh) << 32);
  }
  __device__ __forceinline__ uint64_t peek() const {
    const uint32_t sh = pos & 31;
    return (uint64_t)__builtin_amdgcn_alignbit(x1, x0, sh) |
           ((uint64_t)__builtin_amdgcn_alignbit(x2, x1, sh) << 32);
  }
  __device__ __forceinline__ void skip(unsigned n) {
    pos += n;
    load();
  }
};

// maxbits <= 64 (1D rate <= 16, 2D rate <= 4: BASELINE's 2D 8192^2 rate 2 and
// 1D rate 8): the lane's whole block is one 64-bit register, zero past
// maxbits, read straight from HBM.  The windows are shifts of it, so a plane
// step waits on one LDS round trip (the chunk tables) instead of two, and
// there is no LDS stream image to fill.
// B32: a block of at most 32 bits (maxbits <= 32: BASELINE's 1D rate 8 and 2D
// rate 2).  Its read positions stay below 64 (pos <= 32 plus a window offset
// < 16), so a window is one 64-bit shift of the zero-extended block, without
// the bounds test and selects a block of up to 64 bits needs (five of the
// plane step's slow-issue VALU instructions).
// B32 also keeps the block shifted up by 3 (blk8): the group window is taken
// from it, so a chunk's 10 bits sit at bits 3-12, already a byte offset of
// chunk 1's 8-byte entries (one AND instead of a shift and an AND).
template <bool PRIO = true, bool B32 = false>
struct RegReader : LdsReader<PRIO> {
  uint64_t blk, blk8;
  __device__ __forceinline__ void set_block(uint64_t b) {
    blk = b;
    if constexpr (B32) blk8 = b << 3;
  }
  __device__ __forceinline__ uint64_t at(uint32_t p) const {
    if constexpr (B32) return blk >> p;
    return p < 64 ? blk >> p : 0ull;
  }
  __device__ __forceinline__ void windows(uint32_t m, uint64_t& w, uint32_t& g) const {
    w = at(this->pos);
    if constexpr (B32)
      g = (uint32_t)(blk8 >> (this->pos + m));  // the group window << 3
    else
      g = (uint32_t)at(this->pos + m);
  }
  __device__ __forceinline__ uint32_t window_g(uint32_t m, WRaw& wr) const {
    wr = WRaw{0u, 0u, 0u};
    if constexpr (B32) return (uint32_t)(blk8 >> (this->pos + m));  // the group window << 3
    return (uint32_t)at(this->pos + m);
  }
  __device__ __forceinline__ uint64_t window_w_make(const WRaw&) const { return at(this->pos); }
  // (B32: g from windows() is the group window << 3; its bit 3 is the leading
  // test)
  __device__ __forceinline__ void chunks_fast(uint32_t g, uint32_t& e1, uint32_t& sel, uint32_t& e2a,
                                              uint32_t& e2b) const {
    if constexpr (B32) {
      // (no lead mask here: at 8 waves a SIMD the 2D decoder's LDS is not
      // what it waits on, and the mask's two VALU a plane are)
      const uint2 c = this->tab64(g & 0x1ff8u);
      e1 = c.x;
      sel = c.y;
      const uint2 p = this->tab64(LdsReader<PRIO>::kPairBytes + ((g >> 10) & 0x1ff8u));
      e2a = p.x;
      e2b = p.y;
    } else {
      LdsReader<PRIO>::chunks_fast(g, e1, sel, e2a, e2b);
    }
  }
  __device__ __forceinline__ uint32_t chunk1_fast(uint32_t g) const {
    if constexpr (B32) {
      uint32_t t;
      asm("v_bfe_i32 %0, %1, 3, 1" : "=v"(t) : "v"(g));
      return this->tab((g & t) & 0x1ff8u);
    } else {
      return LdsReader<PRIO>::chunk1_fast(g);
    }
  }
  __device__ __forceinline__ uint64_t peek() const { return at(this->pos); }
  __device__ __forceinline__ uint32_t window32(uint32_t q) const { return (uint32_t)at(q); }
  // (B32: pos <= 32.  v_bfe_u32 takes its offset mod 32, so at pos = 32 it
  // reads bits 0-7 of the block, not zeros; that is harmless because pos = 32
  // means the budget is spent, c = 0, and every c = 0 entry of Plane1dDecLut
  // is the same whatever the stream bits s)
  __device__ __forceinline__ uint32_t bits8() const {
    if constexpr (B32) return __builtin_amdgcn_ubfe((uint32_t)blk, this->pos, 8u);
    return (uint32_t)(blk >> (this->pos & 63)) & 0xffu;
  }
  __device__ __forceinline__ void peek2(uint64_t& a, uint64_t& b) const {
    a = at(this->pos);
    b = 0;  // bits past 64: past the block
  }
  __device__ __forceinline__ void load() {}
  __device__ __forceinline__ void init(uint32_t bitpos) { this->pos = bitpos; }
  __device__ __forceinline__ void skip(unsigned n) { this->pos += n; }
};

// ---------------------------------------------------------------------------
// Gather / scatter of one block.  FAST: contiguous layout, every extent a
// multiple of 4 and a 16-byte aligned base, so each row of 4 values is one
// 16-byte access and consecutive lanes (consecutive x-blocks) read consecutive
// 16-byte segments: 1 KiB per wave instruction.

// f32 values move with non-temporal hints (global_load/store ... nt): each
// array is read or written once per kernel, each instruction covering 1 KiB
// of a row.  At 256^3 the stores take the decode from 33.4 to 29.9 us and the
// encode+decode step by 1.3 %; the gathers another 1-2 % of the step
// (tools/variants.py).  f64 rows are two 16-byte accesses a lane, each
// instruction covering every other 16 bytes, and there the store hint cost
// 32 % (61.5 -> 81.1 us), so f64 stays plain, as does the compressed stream
// (a hint on it measured neutral or worse).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#ifndef CUZFP_TEMPORAL_VALUES
constexpr bool kNtValues = true;
#else
constexpr bool kNtValues = false;  // A/B builds
#endif
// A/B builds: the gathers (CUZFP_TEMPORAL_LOADS) or the value stores
// (CUZFP_TEMPORAL_STORES) alone without the hint
#ifndef CUZFP_TEMPORAL_LOADS
constexpr bool kNtLoads = kNtValues;
#else
constexpr bool kNtLoads = false;
#endif
#ifndef CUZFP_TEMPORAL_STORES
constexpr bool kNtStores = kNtValues;
#else
constexpr bool kNtStores = false;
#endif
#ifndef CUZFP_NT_STREAM
constexpr bool kNtStream = false;
#else
constexpr bool kNtStream = true;  // A/B builds: the compressed stream with the hint
#endif
template <bool NT>
__device__ __forceinline__ uint4 ld16(const void* p) {
  if constexpr (NT) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
    return uint4{v.x, v.y, v.z, v.w};
  } else {
    return *(const uint4*)p;
  }
}
template <bool NT>
__device__ __forceinline__ void st16(void* p, uint4 v) {
  if constexpr (NT)
    __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, (u32x4*)p);
  else
    *(uint4*)p = v;
}

template <typename Scalar>
__device__ __forceinline__ void load_row(const Scalar* p, Scalar* f) {
  if constexpr (sizeof(Scalar) == 4) {
    const uint4 v = ld16<kNtLoads>(p);
    __builtin_memcpy(f, &v, 16);
  } else {
    const uint4 a = ld16<false>(p);
    const uint4 b = ld16<false>(p + 2);
    __builtin_memcpy(f, &a, 16);
    __builtin_memcpy(f + 2, &b, 16);
  }
}

template <typename Scalar>
__device__ __forceinline__ void store_row(Scalar* p, const Scalar* f) {
  if constexpr (sizeof(Scalar) == 4) {
    uint4 v;
    __builtin_memcpy(&v, f, 16);
    st16<kNtStores>(p, v);
  } else {
    uint4 a, b;
    __builtin_memcpy(&a, f, 16);
    __builtin_memcpy(&b, f + 2, 16);
    st16<false>(p, a);
    st16<false>(p + 2, b);
  }
}

struct BlockPos {
  uint32_t ix, iy, iz;
};

__device__ __forceinline__ uint32_t div_magic(uint32_t n, uint32_t m, uint32_t s) {
  return (uint32_t)(((uint64_t)n * m) >> s);
}

// (the divisions by multiply-high with the launch's magic numbers: about a
// dozen VALU instructions fewer each than the compiler's division)
template <int DIMS>
__device__ __forceinline__ BlockPos block_pos(const Geometry& g, uint32_t b) {
  BlockPos p;
  if constexpr (DIMS == 1) {
    p.ix = b; p.iy = 0; p.iz = 0;
  } else if constexpr (DIMS == 2) {
    p.iy = g.divmagic ? div_magic(b, g.dbx_m, g.dbx_s) : b / g.bx;
    p.ix = b - p.iy * g.bx; p.iz = 0;
  } else {
    const uint32_t plane = g.bx * g.by;
    p.iz = g.divmagic ? div_magic(b, g.dpl_m, g.dpl_s) : b / plane;
    const uint32_t r = b - p.iz * plane;
    p.iy = g.divmagic ? div_magic(r, g.dbx_m, g.dbx_s) : r / g.bx;
    p.ix = r - p.iy * g.bx;
  }
  return p;
}

template <typename Scalar, int DIMS, bool FAST>
__device__ __forceinline__ void gather(const Scalar* __restrict__ data, const Geometry& g,
                                       BlockPos bp, Scalar* f) {
  constexpr int NY = DIMS > 1 ? 4 : 1, NZ = DIMS > 2 ? 4 : 1;
  if constexpr (FAST) {
    const Scalar* p = data + ((size_t)(4 * bp.iz) * g.ny + 4 * bp.iy) * g.nx + 4 * bp.ix;
#pragma unroll
    for (int z = 0; z < NZ; z++)
#pragma unroll
      for (int y = 0; y < NY; y++)
        load_row(p + ((size_t)z * g.ny + y) * g.nx, f + 16 * z + 4 * y);
  } else {
    const int wx = (int)min(4u, g.nx - 4 * bp.ix);
    const int wy = (int)min(4u, g.ny - 4 * bp.iy);
    const int wz = (int)min(4u, g.nz - 4 * bp.iz);
    const Scalar* p = data + (int64_t)(4 * bp.ix) * g.sx + (int64_t)(4 * bp.iy) * g.sy +
                      (int64_t)(4 * bp.iz) * g.sz;
#pragma unroll
    for (int z = 0; z < NZ; z++)
#pragma unroll
      for (int y = 0; y < NY; y++)
#pragma unroll
        for (int x = 0; x < 4; x++)
          f[16 * z + 4 * y + x] = p[(int64_t)pad_src(x, wx) * g.sx + (int64_t)pad_src(y, wy) * g.sy +
                                    (int64_t)pad_src(z, wz) * g.sz];
  }
}

template <typename Scalar, int DIMS, bool FAST>
__device__ __forceinline__ void scatter(Scalar* __restrict__ data, const Geometry& g, BlockPos bp,
                                        const Scalar* f) {
  constexpr int NY = DIMS > 1 ? 4 : 1, NZ = DIMS > 2 ? 4 : 1;
  if constexpr (FAST) {
    Scalar* p = data + ((size_t)(4 * bp.iz) * g.ny + 4 * bp.iy) * g.nx + 4 * bp.ix;
#pragma unroll
    for (int z = 0; z < NZ; z++)
#pragma unroll
      for (int y = 0; y < NY; y++)
        store_row(p + ((size_t)z * g.ny + y) * g.nx, f + 16 * z + 4 * y);
  } else {
    const int wx = (int)min(4u, g.nx - 4 * bp.ix);
    const int wy = (int)min(4u, g.ny - 4 * bp.iy);
    const int wz = (int)min(4u, g.nz - 4 * bp.iz);
    Scalar* p = data + (int64_t)(4 * bp.ix) * g.sx + (int64_t)(4 * bp.iy) * g.sy +
                (int64_t)(4 * bp.iz) * g.sz;
#pragma unroll
    for (int z = 0; z < NZ; z++)
#pragma unroll
      for (int y = 0; y < NY; y++)
#pragma unroll
        for (int x = 0; x < 4; x++)
          if (x < wx && y < wy && z < wz)
            p[(int64_t)x * g.sx + (int64_t)y * g.sy + (int64_t)z * g.sz] = f[16 * z + 4 * y + x];
  }
}

// ---------------------------------------------------------------------------
// Kernels

// Up to kWavesPerGroup independent waves share a workgroup (fewer workgroups
// for the dispatcher to launch); each has its own LDS image and they never
// synchronise with each other.  Within a wave, LDS traffic between lanes only
// needs the wave's own LDS operations to have completed.
constexpr int kWavesPerGroup = 4;
// The LDS-image kernels' workgroups (the 3D paths).  Alone, the encoder
// measured best at 1-2 waves a workgroup (256^3 r8 encode 27.8 -> 27.5 us)
// and the decoder, whose workgroup shares one table copy behind a barrier, at
// 8 (23.5 -> 23.0 us; 1-2 waves: 32-34 us) -- but the encode+decode step
// with different sizes took 55.6-56.7 us against 50.2 us with 4 and 4: a
// kernel whose workgroups need more wave slots per CU than the previous
// kernel's leave starts late (tools/xvar.py e1d8 / e2d8 / e2d16).
#ifndef CUZFP_ENC_WPG  // A/B builds
#define CUZFP_ENC_WPG 4
#endif
#ifndef CUZFP_DEC_WPG
#define CUZFP_DEC_WPG 4
#endif
constexpr int kEncWaves = CUZFP_ENC_WPG, kDecWaves = CUZFP_DEC_WPG;
// Workgroup size of the 1D register-reader decoder: 16 waves, so that the
// workgroup's 20 KiB of tables are shared by 16 waves that each decode 1 KiB
// of values (64M values: decode 151 -> 121 us).  The 2D decoder and the 1D/2D
// register-writer encoders measured best at 4 (16: 2D encode 66.6 -> 71.3
// us, 1D 97 -> 102 us; 2D decode unchanged).
#ifndef CUZFP_REG_WAVES_1D  // A/B builds
#define CUZFP_REG_WAVES_1D 16
#endif
constexpr int kRegWaves1d = CUZFP_REG_WAVES_1D;
#ifndef CUZFP_REG_WAVES_2D  // A/B builds
#define CUZFP_REG_WAVES_2D 4
#endif
constexpr int kRegWaves2d = CUZFP_REG_WAVES_2D;
// 1D batches: a wave of the register-path kernels codes K batches of 64
// blocks (zfp_encode_regk / zfp_decode_regk), so that it has K times the bytes
// in flight -- 1D waves are small (16-24 VGPRs) and 8 a SIMD is the hardware's
// cap -- and the decoder's workgroup copies its 20 KiB of tables once for
// W x K batches.  64M values, rate 8 (tools/xvar.py): encode 97.2 -> 79.6 us
// at K = 2 (4 equal, 8 spills), decode 120.3 -> 103.7 us at K = 4 with
// 8-wave workgroups (K = 4 in 16-wave or 4-wave groups 111.5, K = 8 110).
// 2D measured slower both ways (its waves are 34-62 VGPRs and move 4 KiB of
// values each: encode 67.5 -> 76-77 us, decode 73.6 -> 75.3 / 83.1 us), so 2D
// stays at one batch.  Used from kRegBatchMinWaves logical waves up: at 4M
// values (16,384 waves) the batches measured slower (step 18.9 -> 20.3 us), at
// 16M faster (62.8 -> 58.6 us), at 1M much slower (7.9 -> 12.4 us: idle CUs).
#ifndef CUZFP_REG_DEC_BATCH_1D  // A/B builds (1 = off)
#define CUZFP_REG_DEC_BATCH_1D 4
#endif
#ifndef CUZFP_REG_ENC_BATCH_1D
#define CUZFP_REG_ENC_BATCH_1D 2
#endif
#ifndef CUZFP_REG_BATCH_WAVES_1D  // workgroup size of the batched 1D decoder
#define CUZFP_REG_BATCH_WAVES_1D 8
#endif
#ifndef CUZFP_REG_BATCH_MIN_WAVES
#define CUZFP_REG_BATCH_MIN_WAVES 32768
#endif
constexpr int kRegDecBatch1d = CUZFP_REG_DEC_BATCH_1D, kRegEncBatch1d = CUZFP_REG_ENC_BATCH_1D;
constexpr int kRegBatchWaves1d = CUZFP_REG_BATCH_WAVES_1D;
constexpr uint32_t kRegBatchMinWaves = CUZFP_REG_BATCH_MIN_WAVES;
#ifndef CUZFP_REG_BATCH_PRIO
#define CUZFP_REG_BATCH_PRIO 0
#endif

// The wave's index in its workgroup, as a wave-uniform (SGPR) value: the
// compiler takes threadIdx.x >> 6 for a per-lane value, so every branch on
// the wave's number (a wave past the launch's end, a partial last wave) would
// otherwise be a divergent one, and everything after it an exec-masked region
// -- an s_cbranch_execz and exec-mask bookkeeping at every step of the coders.
__device__ __forceinline__ uint32_t wave_in_group() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// 3D double rows through the wave's LDS image.  A lane's row of 4 doubles is
// 32 bytes, so storing it straight from the lane takes two 16-byte stores that
// each cover every other 16 bytes of the wave's 2 KiB row span (64 blocks
// side by side along x).  Staged, each lane writes its rows into the wave's
// LDS and reads back the span's 16-byte pieces in lane order, so each store
// instruction covers 1 KiB contiguously and takes the non-temporal hint like
// the f32 rows: 256^3 rate 16 decode 59.7 -> 54.1 us in the timing experiment
// (the store pattern alone).  Needs the wave's 64 blocks on one x-row of
// blocks (bx a multiple of 64: every wave full and aligned) and ROWS x 2 KiB
// of the wave's LDS image, which the decoder no longer reads.  Every lane of
// the wave calls it; a lane with a zero block stages zeros.
template <int ROWS>
__device__ __forceinline__ void scatter_f64_staged(double* __restrict__ data, const Geometry& g, BlockPos bp,
                                                   const double* f, bool coded, uint64_t* wave_lds,
                                                   uint32_t lane) {
  static_assert(16 % ROWS == 0, "rows a pass");
  uint4* stage = (uint4*)wave_lds;  // row j of a pass: 128 pieces of 16 bytes
  // the row span's start: lane 0's block (ix - lane)
  double* base = data + ((size_t)(4 * bp.iz) * g.ny + 4 * bp.iy) * g.nx + 4 * (bp.ix - lane);
#pragma unroll
  for (int r0 = 0; r0 < 16; r0 += ROWS) {
    if (coded) {
#pragma unroll
      for (int j = 0; j < ROWS; j++) {
        uint4 a, b;
        __builtin_memcpy(&a, f + 4 * (r0 + j), 16);
        __builtin_memcpy(&b, f + 4 * (r0 + j) + 2, 16);
        stage[j * 128 + 2 * lane] = a;
        stage[j * 128 + 2 * lane + 1] = b;
      }
    } else {
#pragma unroll
      for (int j = 0; j < ROWS; j++) {
        stage[j * 128 + 2 * lane] = uint4{0, 0, 0, 0};
        stage[j * 128 + 2 * lane + 1] = uint4{0, 0, 0, 0};
      }
    }
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < ROWS; j++) {
      const int r = r0 + j, z = r >> 2, y = r & 3;
      double* row = base + ((size_t)z * g.ny + y) * g.nx;
      st16<true>(row + 2 * lane, stage[j * 128 + lane]);
      st16<true>(row + 128 + 2 * lane, stage[j * 128 + 64 + lane]);
    }
    // The next pass overwrites the pieces other lanes have just read: its
    // writes must not be moved above these reads (the compiler sees disjoint
    // per-lane addresses), so the wave waits for them (asm memory clobber;
    // at most 16 waits a block)
    if (r0 + ROWS < 16) wave_lds_sync();
  }
}

// Waves per SIMD the register budget is sized for: 4 (<= 128 VGPRs) in
// general.  3D double blocks hold 64 x 64-bit values (128 VGPRs) and then 64 x
// 64-bit planes, so 2 (<= 256 VGPRs) rather than spilling.  At 3 waves
// (<= 168) the encoder spills 40 B a lane and the decoder 268 B; the encoder at
// 3 measured 66.7 us against 56.7 us at 2 (256^3 rate 16, tools/variants.py
// f64w3 / f64w2), so CUZFP_F64_ENC_WAVES stays 2.
#ifndef CUZFP_F64_ENC_WAVES
#define CUZFP_F64_ENC_WAVES 2
#endif
#ifndef CUZFP_F64_DEC_WAVES  // A/B builds
#define CUZFP_F64_DEC_WAVES 2
#endif
#ifndef CUZFP_F32_DEC_WAVES  // A/B builds: 3D float decoder / encoder
#define CUZFP_F32_DEC_WAVES 4
#endif
#ifndef CUZFP_F32_ENC_WAVES
#define CUZFP_F32_ENC_WAVES 4
#endif
template <typename Scalar, int DIMS, bool ENC = false> struct occupancy {
  static constexpr int value = (sizeof(Scalar) == 8 && DIMS == 3) ? (ENC ? CUZFP_F64_ENC_WAVES : CUZFP_F64_DEC_WAVES)
                               : (sizeof(Scalar) == 4 && DIMS == 3) ? (ENC ? CUZFP_F32_ENC_WAVES : CUZFP_F32_DEC_WAVES)
                                                                    : 4;
};

// REG (1D/2D, maxbits 32 or 64): the block is coded into a register
// (RegWriter; 2 = maxbits 64) and stored straight from it: a lane's block is
// dword / word b of the stream.  No LDS image.
template <typename Scalar, int DIMS, bool FAST, bool ALIGNED, bool PRIO = true, int REG = 0, int WPG = kEncWaves>
__device__ __forceinline__ void zfp_encode_body(const Scalar* __restrict__ data, const Geometry& g,
                                                uint64_t* __restrict__ stream, uint32_t bid,
                                                uint32_t* stab, uint32_t* ptab) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds_all[];
  // (the tables: stab, the spread tables at LDS address 0; ptab, 1D: the pair
  // table, Pair1dLut, 4 KiB, one copy a workgroup -- the kernel's static LDS)
  constexpr int N = 1 << (2 * DIMS);
  const uint32_t wig = wave_in_group();
  const uint32_t wave = g.wave0 + bid * (blockDim.x >> 6) + wig;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t b = wave * kLanes + lane;
  const bool live_wave = wave < g.wave_end;
  uint64_t* lds = lds_all + (size_t)wig * g.lds_words;
  // the register-path kernels (1D/2D) copy the spread tables once a workgroup
  constexpr bool kGroupSpread = DIMS == 1 || REG != 0;
  if constexpr (DIMS == 2 && REG != 0) {
    for (uint32_t i = threadIdx.x; i < kSpreadTabBytes / 16; i += blockDim.x)
      ((uint4*)stab)[i] = ((const uint4*)g_spread_tab.e)[i];
    __syncthreads();
  }
  if constexpr (DIMS == 1) {
    // ... and the 64 bytes of spread table 1D reads (entries 0-15 of table 0:
    // r = x >> n < 2^4), behind the same barrier
    if (threadIdx.x < 4) ((uint4*)stab)[threadIdx.x] = ((const uint4*)g_spread_tab.e)[threadIdx.x];
    for (uint32_t i = threadIdx.x; i < sizeof(Pair1dLut) / 16; i += blockDim.x)
      ((uint4*)ptab)[i] = ((const uint4*)g_pair1d_lut.e)[i];
    __syncthreads();
  }
  lds_spread* p1d = (lds_spread*)ptab;
  if (!live_wave) return;
  // the plane coder's spread tables, written whole by every wave (see
  // g_spread_tab): their load is issued first so that storing them waits only
  // for it, not for the block's gathers
  constexpr uint32_t kTabPieces = kSpreadTabBytes / 16;  // two 16-byte pieces a lane
  // (1D: copied above, per workgroup; a per-lane staging array here was turned
  // into LDS by the compiler and made the 1D register-writer kernel 8x slower)
  uint4 tab16[kTabPieces / kLanes];
  if constexpr (!kGroupSpread) {
#pragma unroll
    for (uint32_t i = 0; i < kTabPieces / kLanes; i++) tab16[i] = ((const uint4*)g_spread_tab.e)[lane + i * kLanes];
  }
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);  // lowered through the plane loop (progress_priority)
  lds_spread* lut = (lds_spread*)stab;
  ZFP_STAMP_HWID();
  ZFP_STAMP_REAL(8);
  ZFP_STAMP(0);
  if constexpr (!ALIGNED) {
    for (uint32_t j = lane; j < g.maxbits + 2; j += kLanes) lds[j] = 0;
  }
  // ALIGNED: the wave's image is lane-interleaved, word j of lane l's block at
  // lds[64 j + l] (conflict-free ds_or_b64 whatever each lane's bit position),
  // W words per block plus kSlackWords rows
  const uint32_t W = g.maxbits >> 6;
  Scalar f[N];
  // (3D double rows staged through LDS like the decoder's stores measured
  // slower, round 4: 256^3 r16 encode 51.1 -> 54.5 us with non-temporal
  // loads, 50.9 -> 54.4 us with plain ones; non-temporal hints on these
  // strided row loads: 50.9 -> 55.6 us)
  // A wave of live blocks only (every wave but a partial last one) gathers
  // behind one wave-uniform test: with the per-lane test alone the compiler
  // zeroes the whole block first (64 v_mov a wave, on every wave) and then
  // loads over it under the lane mask.
  if ((wave + 1) * kLanes <= g.nblocks) {
    gather<Scalar, DIMS, FAST>(data, g, block_pos<DIMS>(g, b), f);
  } else if (b < g.nblocks) {
    gather<Scalar, DIMS, FAST>(data, g, block_pos<DIMS>(g, b), f);
  } else if constexpr (ALIGNED && !REG) {
    // a lane past the last block codes a zero block (see below)
#pragma unroll
    for (int i = 0; i < N; i++) f[i] = (Scalar)0;
  }
  // (one copy a workgroup behind a barrier measured slower: 28.0 -> 28.4 us at 256^3)
  if constexpr (!kGroupSpread) {
#pragma unroll
    for (uint32_t i = 0; i < kTabPieces / kLanes; i++) ((uint4*)stab)[lane + i * kLanes] = tab16[i];
  }
  if constexpr (REG) {
    wave_lds_sync();  // the spread tables
    uint64_t bits = 0;
    if (b < g.nblocks) {
      reg_writer<Scalar, PRIO, REG> wr{lut, p1d, 0, 0};
      if constexpr (REG == 2 || traits<Scalar>::is_int) wr.mb = g.maxbits;
      encode_block<Scalar, DIMS>(f, g.maxbits, wr);
      bits = wr.bits();
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);
    // block b is dword (maxbits 32) / word (64) b; with maxbits 32 and an odd
    // block count the lane after the last block writes the last word's zero half
    if constexpr (REG == 2) {
      if (b < g.nblocks) stream[b] = bits;
    } else {
      if (b < g.nblocks + (g.nblocks & 1u)) ((uint32_t*)stream)[b] = (uint32_t)bits;
    }
    return;
  }
  // ALIGNED: every lane of the wave codes (a lane past the last block holds a
  // zero block, which LdsOrWriter codes inline into its discarded slack), so
  // the coder runs outside any per-lane branch; the copy-out moves the live
  // blocks' words only
  if constexpr (ALIGNED) {
    uint64_t* mine = lds + lane;
    for (uint32_t j = 0; j < W + kSlackWords; j++) mine[j * 64] = 0;  // own column
    // The workgroup's waves (one on each SIMD of the CU) start coding
    // together, once every one of their blocks has landed: 256^3 r8 step
    // 46.04 / 45.80 -> 45.57 / 45.54 us (polynomial), 44.58 / 44.71 ->
    // 44.46 / 44.60 (splitmix), profiles/r06_ab_ebar.txt; the decoder's
    // barrier over its stream segments does the same (taking it away measured
    // +2 us, r06_ab_copyin.txt).  Only where every wave of the workgroup is
    // live (a wave-uniform test, the same on all of them): the others
    // returned above.
    if (g.wave0 + (bid + 1) * (blockDim.x >> 6) <= g.wave_end) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    wave_lds_sync();  // the tables
    LdsOrWriter<PRIO> wr{mine, lut, 0, 64 * W, p1d, uniform_const64(0x7fffu)};
    encode_block<Scalar, DIMS>(f, g.maxbits, wr);
  } else if (b < g.nblocks) {
    {
      wave_lds_sync();  // the tables and the zeroed image
      LdsBitWriter<PRIO> wr{lds, lut, lane * g.maxbits, (lane + 1) * g.maxbits, 0, 0, p1d, uniform_const64(0x7fffu)};
      encode_block<Scalar, DIMS>(f, g.maxbits, wr);
    }
  }
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);  // a wave out of the coder stores at once
  wave_lds_sync();
  const uint32_t nb = min((uint32_t)kLanes, g.nblocks - wave * kLanes);
  const uint32_t nwords = (nb * g.maxbits + 63) >> 6;
  uint64_t* out = stream + (size_t)wave * g.maxbits;
  if constexpr (ALIGNED) {
    if (nb == kLanes && g.vec_io && !(W & 1)) {
      // A full wave stores its 64 W words in lane order, each store covering
      // 1 KiB contiguously (non-temporal): store t covers words [128 t, 128 t
      // + 128), lane l's two at k = 128 t + 2 l, words j = k % W, j + 1 of
      // block s = k / W (column s of the image).  Each lane storing its own
      // W words instead puts every store instruction's 16-byte pieces W * 8
      // bytes apart: 256^3 r8 encode 27.4 -> 24.4 us, step 50.3 -> 49.2 us;
      // 1024^3 step -0.5 % (tools/xvar.py, r04_stream_stores; plain stores
      // here gave encode 26.5 us and a faster decode of the still-cached
      // stream at 256^3, step 48.8 us, but a cached stream is the bench's
      // artefact, not a decompressor's).
      uint32_t s, j, ds, dj;
      udivmod_uniform(2 * lane, W, s, j);
      udivmod_uniform(128u, W, ds, dj);
      for (uint32_t k = 2 * lane; k < kLanes * W; k += 128) {
        uint4 v;
        const uint64_t a0 = lds[j * 64 + s], a1 = lds[(j + 1) * 64 + s];
        __builtin_memcpy(&v.x, &a0, 8);
        __builtin_memcpy(&v.z, &a1, 8);
        st16<true>(&out[k], v);
        j += dj;
        s += ds;
        if (j >= W) { j -= W; s++; }
      }
      ZFP_STAMP(6);
      ZFP_STAMP_REAL(9);
      return;
    }
  }
  if constexpr (ALIGNED) {
    // each lane stores its own block: W words at out + lane * W
    if (b < g.nblocks) {
      const uint64_t* mine = lds + lane;
      uint64_t* dst = out + (size_t)lane * W;
      if (g.vec_io && !(W & 1)) {
        for (uint32_t j = 0; j < W; j += 2) {
          uint4 v;
          const uint64_t a0 = mine[j * 64], a1 = mine[(j + 1) * 64];
          __builtin_memcpy(&v.x, &a0, 8);
          __builtin_memcpy(&v.z, &a1, 8);
          st16<kNtStream>(&dst[j], v);
        }
      } else {
        for (uint32_t j = 0; j < W; j++) dst[j] = mine[j * 64];
      }
    }
  } else if (g.vec_io) {  // 16-byte aligned segment
    const uint32_t npairs = nwords >> 1;
    for (uint32_t j = lane; j < npairs; j += kLanes)
      ((uint4*)out)[j] = ((const uint4*)lds)[j];
    if ((nwords & 1) && lane == 0) out[nwords - 1] = lds[nwords - 1];
  } else {
    for (uint32_t j = lane; j < nwords; j += kLanes) out[j] = lds[j];
  }
  ZFP_STAMP(6);
  ZFP_STAMP_REAL(9);
}

// The kernel: the body above for workgroup blockIdx.x, with its tables in the
// kernel's static LDS.
template <typename Scalar, int DIMS, bool FAST, bool ALIGNED, bool PRIO = true, int REG = 0, int WPG = kEncWaves>
__global__ __launch_bounds__(kLanes * WPG, (occupancy<Scalar, DIMS, true>::value)) void zfp_encode(const Scalar* __restrict__ data,
                                                                      Geometry g,
                                                                      uint64_t* __restrict__ stream) {
  __shared__ __attribute__((aligned(16))) uint32_t stab[512];  // LDS address 0 (static)
  // 1D: the pair table (Pair1dLut, 4 KiB), one copy a workgroup: 16 bytes a lane
  __shared__ __attribute__((aligned(16))) uint32_t ptab[DIMS == 1 ? 1024 : 4];
  zfp_encode_body<Scalar, DIMS, FAST, ALIGNED, PRIO, REG, WPG>(data, g, stream, blockIdx.x, stab, ptab);
}

// WPG: waves per workgroup (16 for the 1D register-reader kernel, whose
// workgroup copies 20 KiB of tables for 1 KiB of output a wave)
// REG: 0 = the LDS image; 32 = a block of exactly 32 bits (one dword of the
// stream), 64 = of at most 64 bits, read into a register (RegReader)
template <typename Scalar, int DIMS, bool FAST, bool PRIO = true, int REG = 0, int WPG = kDecWaves>
__device__ __forceinline__ void zfp_decode_body(const uint64_t* __restrict__ stream, const Geometry& g,
                                                Scalar* __restrict__ data, uint32_t bid,
                                                uint32_t* ctab, uint16_t* dtab) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds_all[];
  constexpr int N = 1 << (2 * DIMS);
  const uint32_t wig = wave_in_group();
  const uint32_t wave = g.wave0 + bid * (blockDim.x >> 6) + wig;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t b = wave * kLanes + lane;
  const bool live = wave < g.wave_end && b < g.nblocks;
  uint64_t* lds = lds_all + (size_t)wig * g.lds_words;
  // Copy-in: each lane moves its own block into an LDS image stored
  // lane-interleaved -- dword j of lane l at dword j*64 + l -- so the plane
  // decoder's per-lane window reads hit 32 distinct banks whatever each lane's
  // read position (a contiguous image puts lanes maxbits/32 dwords apart, up
  // to 16 to a bank).  Rows D .. D+4 are zero slack for the reader.  The
  // block's loads are issued first, then the workgroup's copy of the chunk
  // tables, so both latencies overlap before the one barrier.
  // (the tables: ctab, the chunk tables at LDS address 0; dtab, 1D: the plane
  // table, Plane1dDecLut, 16 KiB -- the kernel's static LDS)
  uint32_t* lut = ctab;
  auto copy_dtab = [&]() {
    if constexpr (DIMS == 1)
      for (uint32_t i = threadIdx.x; i < sizeof(Plane1dDecLut) / 16; i += blockDim.x)
        ((uint4*)dtab)[i] = ((const uint4*)g_plane1d_lut.e)[i];
  };
  // (1D reads chunk-1 entries only: the state-2 table, the first kLutPairs entries)
  constexpr uint32_t kLutEnd = DIMS == 1 ? kLutPairs * 4 / 16 : sizeof(ChunkLut) / 16;
  const uint32_t* seg = (const uint32_t*)(stream + (size_t)wave * g.maxbits);
  uint32_t* L = (uint32_t*)lds + lane;
  uint64_t blk = 0;
  if constexpr (REG == 32) {
    // maxbits 32: the lane's block is dword `lane` of the wave's segment
    if (live) blk = seg[lane];  // (a non-temporal hint: 2D decode 63.1 -> 70.8 us, r04_regnt)
    for (uint32_t i = threadIdx.x; i < kLutEnd; i += blockDim.x)
      ((uint4*)lut)[i] = ((const uint4*)g_chunk_lut.e)[i];
    copy_dtab();
  } else if constexpr (REG) {
    // bits [s0, s0 + maxbits) of the wave's segment; dwords past its last one
    // read as zero
    if (live) {
      const uint32_t nb = min((uint32_t)kLanes, g.nblocks - wave * kLanes);
      const uint32_t lim = ((nb * g.maxbits + 63) >> 6) * 2;
      const uint32_t s0 = lane * g.maxbits, d0 = s0 >> 5;
      const uint32_t a0 = seg[d0];
      const uint32_t a1 = d0 + 1 < lim ? seg[d0 + 1] : 0u;
      const uint32_t a2 = d0 + 2 < lim ? seg[d0 + 2] : 0u;
      blk = ((uint64_t)__builtin_amdgcn_alignbit(a1, a0, s0) |
             ((uint64_t)__builtin_amdgcn_alignbit(a2, a1, s0) << 32)) & lowmask(g.maxbits);
    }
    for (uint32_t i = threadIdx.x; i < kLutEnd; i += blockDim.x)
      ((uint4*)lut)[i] = ((const uint4*)g_chunk_lut.e)[i];
    copy_dtab();
  } else {
    const uint32_t D = (g.maxbits + 31) >> 5;  // dwords per block
    const bool vec = (g.maxbits & 127) == 0 && g.vec_io;
    constexpr uint32_t kHeld = 8;  // 16-byte pieces held in registers (maxbits <= 1024)
    uint4 held[kHeld];
    // A full wave loads its segment in lane order, each load 1 KiB
    // contiguously with the non-temporal hint, and places the pieces in the
    // lanes' columns (the same LDS writes at other addresses).  Lane-owned
    // loads put each instruction's pieces D * 4 bytes apart.  256^3 r8
    // (tools/xvar.py, r04_stream_loads): step 48.9 -> 48.2 us (polynomial),
    // 46.2 -> 45.1 (splitmix); the decoder alone, replayed on one cached
    // stream, 23.4 -> 24.9 us (plain contiguous loads: unchanged).
    // (1024^3 r8, the same session: the step within +-0.5 % for contiguous
    // non-temporal, contiguous plain and lane-owned loads, r04_stream_loads)
    const bool cont = vec && wave < g.wave_end && g.nblocks - wave * kLanes >= kLanes && D <= 4 * kHeld;
    if (cont) {
      const uint4* src = (const uint4*)seg + lane;
#pragma unroll
      for (uint32_t q = 0; q < kHeld; q++)
        if (4 * q < D) held[q] = ld16<true>(&src[64 * q]);
    } else if (live && vec) {
      const uint4* src = (const uint4*)(seg + lane * D);
#pragma unroll
      for (uint32_t q = 0; q < kHeld; q++)
        if (4 * q < D) held[q] = ld16<kNtStream>(&src[q]);
    }
    for (uint32_t i = threadIdx.x; i < kLutEnd; i += blockDim.x)
      ((uint4*)lut)[i] = ((const uint4*)g_chunk_lut.e)[i];
    copy_dtab();
    if (cont) {
      // piece 64 q + lane: dwords j .. j + 3 of block s, 4 (64 q + lane) = s D + j
      uint32_t* L0 = (uint32_t*)lds;
      uint32_t sb, j, dsb, dj;
      udivmod_uniform(4 * lane, D, sb, j);
      udivmod_uniform(256u, D, dsb, dj);
#pragma unroll
      for (uint32_t q = 0; q < kHeld; q++)
        if (4 * q < D) {
          L0[(j) * 64 + sb] = held[q].x;
          L0[(j + 1) * 64 + sb] = held[q].y;
          L0[(j + 2) * 64 + sb] = held[q].z;
          L0[(j + 3) * 64 + sb] = held[q].w;
          j += dj;
          sb += dsb;
          if (j >= D) { j -= D; sb++; }
        }
    } else if (live) {
      if (vec) {
#pragma unroll
        for (uint32_t q = 0; q < kHeld; q++)
          if (4 * q < D) {
            L[(4 * q) * 64] = held[q].x;
            L[(4 * q + 1) * 64] = held[q].y;
            L[(4 * q + 2) * 64] = held[q].z;
            L[(4 * q + 3) * 64] = held[q].w;
          }
        const uint4* src = (const uint4*)(seg + lane * D);
        for (uint32_t q = 4 * kHeld; q < D; q += 4) {  // larger blocks
          const uint4 v = src[q >> 2];
          L[q * 64] = v.x;
          L[(q + 1) * 64] = v.y;
          L[(q + 2) * 64] = v.z;
          L[(q + 3) * 64] = v.w;
        }
      } else {
        // the block starts at bit lane*maxbits of the wave's segment; dwords
        // past the segment's last one read as zero
        const uint32_t nb = min((uint32_t)kLanes, g.nblocks - wave * kLanes);
        const uint32_t lim = ((nb * g.maxbits + 63) >> 6) * 2;
        const uint32_t s0 = lane * g.maxbits, d0 = s0 >> 5;
        uint32_t prev = seg[d0];
        for (uint32_t j = 0; j < D; j++) {
          const uint32_t nxt = d0 + j + 1 < lim ? seg[d0 + j + 1] : 0u;
          L[j * 64] = __builtin_amdgcn_alignbit(nxt, prev, s0);
          prev = nxt;
        }
        // the block reads as zeros past its last bit (the plane steps rely on it)
        if (g.maxbits & 31) L[(D - 1) * 64] &= (1u << (g.maxbits & 31)) - 1u;
      }
    } else if (wave < g.wave_end) {
      // a lane past the last block decodes a zero block (its stores are skipped)
      for (uint32_t j = 0; j < D; j++) L[j * 64] = 0;
    }
    if (wave < g.wave_end)
      for (uint32_t j = D; j < D + 5; j++) L[j * 64] = 0;
  }
  __syncthreads();
  if (wave >= g.wave_end) return;
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);  // lowered through the plane loop (progress_priority)
  ZFP_STAMP_HWID();
  ZFP_STAMP_REAL(8);
  ZFP_STAMP(0);
  wave_lds_sync();
  ZFP_STAMP(5);
  // Every lane of a live wave decodes (a lane past the last block reads a
  // zero block), so the coder runs outside any per-lane branch; only the
  // stores are guarded.
  {
    Scalar f[N];
    bool coded;  // false only for a wave of zero blocks (decode_block)
    if constexpr (REG) {
      RegReader<PRIO, REG == 32> rd;
      rd.lds32 = L;
      rd.lut32 = lut;
      rd.d1d = dtab;
      rd.set_block(blk);
      rd.init(0);
      coded = decode_block<Scalar, DIMS>(f, g.maxbits, rd);
    } else {
      LdsReader<PRIO> rd;
      rd.lds32 = L;
      rd.lut32 = lut;
      rd.d1d = dtab;
      rd.init(0);
      coded = decode_block<Scalar, DIMS>(f, g.maxbits, rd);
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);  // a wave out of the coder stores at once
    if constexpr (sizeof(Scalar) == 8 && DIMS == 3 && FAST && !REG) {
      // (row_stage != 0: every lane of the wave is here, see the launcher)
      if (g.row_stage) {
        const BlockPos bp = block_pos<DIMS>(g, b);
        if (g.row_stage == 4)
          scatter_f64_staged<4>((double*)data, g, bp, (const double*)f, coded, lds, lane);
        else if (g.row_stage == 2)
          scatter_f64_staged<2>((double*)data, g, bp, (const double*)f, coded, lds, lane);
        else
          scatter_f64_staged<1>((double*)data, g, bp, (const double*)f, coded, lds, lane);
        ZFP_STAMP(6);
        ZFP_STAMP_REAL(9);
        return;
      }
    }
    if (b < g.nblocks) {
      if (coded) {
        scatter<Scalar, DIMS, FAST>(data, g, block_pos<DIMS>(g, b), f);
      } else {  // a wave of zero blocks
        Scalar z[N];
#pragma unroll
        for (int i = 0; i < N; i++) z[i] = (Scalar)0;
        scatter<Scalar, DIMS, FAST>(data, g, block_pos<DIMS>(g, b), z);
      }
    }
  }
  ZFP_STAMP(6);
  ZFP_STAMP_REAL(9);
}

// The kernel: the body above for workgroup blockIdx.x, with its tables in the
// kernel's static LDS.
template <typename Scalar, int DIMS, bool FAST, bool PRIO = true, int REG = 0, int WPG = kDecWaves>
__global__ __launch_bounds__(kLanes * WPG, (occupancy<Scalar, DIMS>::value)) void zfp_decode(const uint64_t* __restrict__ stream,
                                                                      Geometry g,
                                                                      Scalar* __restrict__ data) {
  __shared__ __attribute__((aligned(16))) uint32_t ctab[chunk_lut_bytes<DIMS>() / 4];  // LDS address 0 (static)
  // 1D: the plane table (Plane1dDecLut, 16 KiB)
  __shared__ __attribute__((aligned(16))) uint16_t dtab[DIMS == 1 ? sizeof(Plane1dDecLut) / 2 : 8];
  zfp_decode_body<Scalar, DIMS, FAST, PRIO, REG, WPG>(stream, g, data, blockIdx.x, ctab, dtab);
}

// The register-writer encoder (1D/2D, maxbits 32 / 64) with K batches of 64
// blocks a wave: every batch's gathers are issued up front (K times the bytes
// in flight a wave: at 8 waves a SIMD, the hardware's cap, one batch a wave
// leaves HBM short of requests), then the batches are coded in order.
template <typename Scalar, int DIMS, bool PRIO, int REG, int WPG, int K>
__global__ __launch_bounds__(kLanes * WPG, (occupancy<Scalar, DIMS, true>::value)) void zfp_encode_regk(
    const Scalar* __restrict__ data, Geometry g, uint64_t* __restrict__ stream) {
  static_assert(DIMS <= 2 && (REG == 1 || REG == 2) && K >= 2 && K <= 8, "register-writer batches: 1D/2D");
  constexpr int N = 1 << (2 * DIMS);
  __shared__ __attribute__((aligned(16))) uint32_t stab[512];  // LDS address 0 (static)
  __shared__ __attribute__((aligned(16))) uint32_t ptab[DIMS == 1 ? 1024 : 4];
  const uint32_t wig = wave_in_group();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w0 = g.wave0 + (blockIdx.x * WPG + wig) * K;
  Scalar f[K][N];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const uint32_t b = (w0 + k) * kLanes + lane;
    if (w0 + k < g.wave_end && b < g.nblocks) gather<Scalar, DIMS, true>(data, g, block_pos<DIMS>(g, b), f[k]);
  }
  if constexpr (DIMS == 2) {
    for (uint32_t i = threadIdx.x; i < kSpreadTabBytes / 16; i += blockDim.x)
      ((uint4*)stab)[i] = ((const uint4*)g_spread_tab.e)[i];
  } else {
    if (threadIdx.x < 4) ((uint4*)stab)[threadIdx.x] = ((const uint4*)g_spread_tab.e)[threadIdx.x];
    for (uint32_t i = threadIdx.x; i < sizeof(Pair1dLut) / 16; i += blockDim.x)
      ((uint4*)ptab)[i] = ((const uint4*)g_pair1d_lut.e)[i];
  }
  __syncthreads();
  lds_spread* lut = (lds_spread*)stab;
  lds_spread* p1d = (lds_spread*)ptab;
#pragma unroll
  for (int k = 0; k < K; k++) {
    const uint32_t b = (w0 + k) * kLanes + lane;
    if (w0 + k >= g.wave_end) break;
    uint64_t bits = 0;
    if (b < g.nblocks) {
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);
      reg_writer<Scalar, PRIO, REG> wr{lut, p1d, 0, 0};
      if constexpr (REG == 2 || traits<Scalar>::is_int) wr.mb = g.maxbits;
      encode_block<Scalar, DIMS>(f[k], g.maxbits, wr);
      bits = wr.bits();
    }
    // block b is dword (maxbits 32) / word (64) b; with maxbits 32 and an odd
    // block count the lane after the last block writes the last word's zero half
    if constexpr (REG == 2) {
      if (b < g.nblocks) stream[b] = bits;
    } else {
      if (b < g.nblocks + (g.nblocks & 1u)) ((uint32_t*)stream)[b] = (uint32_t)bits;
    }
  }
}

// The register-reader decoder (1D/2D blocks of at most 64 bits) with K
// batches of 64 blocks a wave: the K batches' stream words are loaded up
// front, so a wave waits once for its loads (and once for its workgroup's
// table copy), and each batch's stores drain while the next batch decodes.
// Batches are taken in order, one at a time (a rolled loop: the decoder body
// is not replicated).  Logical wave w = g.wave0 + (physical wave) * K + k.
__device__ __forceinline__ uint64_t reg_block(const uint64_t* stream, const Geometry& g, uint32_t wave,
                                              uint32_t lane) {
  // bits [s0, s0 + maxbits) of the wave's segment; dwords past its last one
  // read as zero
  const uint32_t* seg = (const uint32_t*)(stream + (size_t)wave * g.maxbits);
  const uint32_t nb = min((uint32_t)kLanes, g.nblocks - wave * kLanes);
  const uint32_t lim = ((nb * g.maxbits + 63) >> 6) * 2;
  const uint32_t s0 = lane * g.maxbits, d0 = s0 >> 5;
  // clamped addresses and selects rather than guarded loads: no branch, so
  // the K batches' loads are all in flight before the first wait
  const uint32_t a0 = seg[d0];
  uint32_t a1 = seg[min(d0 + 1, lim - 1)];
  uint32_t a2 = seg[min(d0 + 2, lim - 1)];
  a1 = d0 + 1 < lim ? a1 : 0u;
  a2 = d0 + 2 < lim ? a2 : 0u;
  return ((uint64_t)__builtin_amdgcn_alignbit(a1, a0, s0) | ((uint64_t)__builtin_amdgcn_alignbit(a2, a1, s0) << 32)) &
         lowmask(g.maxbits);
}

template <typename Scalar, int DIMS, bool FAST, bool PRIO, int WPG, int K, int REG = 64>
__global__ __launch_bounds__(kLanes * WPG, (occupancy<Scalar, DIMS>::value)) void zfp_decode_regk(
    const uint64_t* __restrict__ stream, Geometry g, Scalar* __restrict__ data) {
  static_assert(DIMS <= 2 && K >= 2 && K <= 8, "register-reader batches: 1D/2D, 2-8 a wave");
  constexpr int N = 1 << (2 * DIMS);
  __shared__ __attribute__((aligned(16))) uint32_t ctab[chunk_lut_bytes<DIMS>() / 4];  // LDS address 0 (static)
  __shared__ __attribute__((aligned(16))) uint16_t dtab[DIMS == 1 ? sizeof(Plane1dDecLut) / 2 : 8];
  const uint32_t wig = wave_in_group();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w0 = g.wave0 + (blockIdx.x * WPG + wig) * K;
  uint64_t q[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const uint32_t w = w0 + k;
    if (w < g.wave_end && w * kLanes + lane < g.nblocks)
      q[k] = REG == 32 ? (uint64_t)((const uint32_t*)(stream + (size_t)w * g.maxbits))[lane] : reg_block(stream, g, w, lane);
    else
      q[k] = 0;
  }
  constexpr uint32_t kLutEnd = DIMS == 1 ? kLutPairs * 4 / 16 : sizeof(ChunkLut) / 16;
  for (uint32_t i = threadIdx.x; i < kLutEnd; i += blockDim.x) ((uint4*)ctab)[i] = ((const uint4*)g_chunk_lut.e)[i];
  if constexpr (DIMS == 1)
    for (uint32_t i = threadIdx.x; i < sizeof(Plane1dDecLut) / 16; i += blockDim.x)
      ((uint4*)dtab)[i] = ((const uint4*)g_plane1d_lut.e)[i];
  __syncthreads();
  const uint32_t nw = w0 < g.wave_end ? min((uint32_t)K, g.wave_end - w0) : 0u;
#pragma unroll 1
  for (uint32_t k = 0; k < nw; k++) {
    const uint64_t blk = q[0];
#pragma unroll
    for (int j = 0; j + 1 < K; j++) q[j] = q[j + 1];  // the next batch's words move up (static registers)
    const uint32_t b = (w0 + k) * kLanes + lane;
    // every lane decodes (a lane past the last block holds a zero block: its
    // word is 0); only the stores are guarded
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);  // lowered through the plane loop (progress_priority)
    Scalar f[N];
    RegReader<PRIO, REG == 32> rd;
    rd.lds32 = nullptr;
    rd.lut32 = ctab;
    rd.d1d = dtab;
    rd.set_block(blk);
    rd.init(0);
    const bool coded = decode_block<Scalar, DIMS>(f, g.maxbits, rd);  // false: a wave of zero blocks
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);
    if (!coded) {
#pragma unroll
      for (int i = 0; i < N; i++) f[i] = (Scalar)0;
    }
    if (b < g.nblocks) scatter<Scalar, DIMS, FAST>(data, g, block_pos<DIMS>(g, b), f);
  }
}

// ---------------------------------------------------------------------------
// Launchers

// The current device's LDS budget of one workgroup
// (hipDeviceAttributeMaxSharedMemoryPerBlock: 160 KiB on MI355X, where a single
// workgroup may use the whole CU's LDS), read once per device; 64 KiB if the
// runtime cannot say.  Thread-safe: each device's slot is an atomic written
// with the same value by whichever thread reads it first.
static inline size_t lds_cap_bytes() {
  // CUZFP_LDS_CAP_BYTES (read once a process) lowers the budget, so that the
  // launchers' refusal of a block image that cannot fit is testable on gfx950
  static const long forced = [] {
    const char* e = getenv("CUZFP_LDS_CAP_BYTES");
    return (e && *e) ? atol(e) : 0L;
  }();
  if (forced > 0) return (size_t)forced;
  static std::atomic<int> cap[kMaxDevices];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 65536;
  int c = cap[dev].load(std::memory_order_relaxed);
  if (!c) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || n <= 0)
      n = 65536;
    cap[dev].store(n, std::memory_order_relaxed);
    c = n;
  }
  return (size_t)c;
}

// waves per workgroup: as many as fit a workgroup's LDS budget (up to most)
static inline uint32_t waves_per_group(uint32_t lds_words, size_t shared_bytes, uint32_t most) {
  const size_t cap = lds_cap_bytes();
  uint32_t w = most;
  while (w > 1 && (size_t)w * lds_words * 8 + shared_bytes > cap) w >>= 1;
  return w;
}

// The plane-loop priority schedule (progress_priority) when the launch is at
// most `rounds` resident rounds of waves; without it beyond.  Measured
// (tools/prio_sweep.sh, profiles/r01_prio_sweep.txt, 3D f32 r8): with the
// schedule 256^3 (1 round) encode 33.3 / decode 29.7 us vs 35.2 / 33.4 us;
// 320^3 (1.95 rounds) the decoder still gains (57.5 vs 61.0 us) and the
// encoder no longer does (62.8 vs 61.3 us); from 384^3 (3.4 rounds) both lose,
// 768^3 by 14 % of the step.  CUZFP_PRIO=0/1 in the environment forces either.
// The environment is read once per process (a function-local static: thread-safe
// initialisation); the CU count once per device, as lds_cap_bytes.
static inline bool use_priority(uint32_t nwaves, int waves_per_simd, uint32_t rounds) {
  static const int forced = [] {
    const char* e = getenv("CUZFP_PRIO");
    return (e && *e) ? (atoi(e) != 0 ? 1 : 0) : -1;
  }();
  if (forced >= 0) return forced != 0;
  static std::atomic<int> cus[kMaxDevices];
  int dev = 0, c = 256;  // MI355X
  if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kMaxDevices) {
    c = cus[dev].load(std::memory_order_relaxed);
    if (!c) {
      int n = 0;
      if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
      cus[dev].store(n, std::memory_order_relaxed);
      c = n;
    }
  }
  return nwaves <= (uint32_t)c * 4u * (uint32_t)waves_per_simd * rounds;
}

#if defined(CUZFP_XVAR)  // tools/xvar.py builds: the fast-gather kernels only (compile time)
constexpr bool kFastOnly = true;
#else
constexpr bool kFastOnly = false;
#endif
#ifndef CUZFP_ENC_PRIO_ROUNDS  // A/B builds: 0 = the encoder never takes the schedule
#define CUZFP_ENC_PRIO_ROUNDS 1
#endif
template <typename Scalar, int DIMS>
int launch_encode_t(const void* data, const Geometry& g, bool fast, uint64_t* stream,
                           uint32_t wave0, uint32_t nwaves, hipStream_t st) {
  Geometry gg = g;
  gg.wave0 = wave0;
  gg.wave_end = wave0 + nwaves;
  gg.vec_io = (g.maxbits % 2 == 0) && ((uintptr_t)stream % 16 == 0);
  gg.lds_words = g.maxbits + kLanes * kSlackWords;  // + per-lane slack
  // the kernel's static LDS: the spread tables, and in 1D the pair table
  constexpr size_t kStatic = kSpreadTabBytes + (DIMS == 1 ? sizeof(Pair1dLut) : 16);
  const Scalar* d = (const Scalar*)data;
  if constexpr (DIMS <= 2) {
    // maxbits 32 or 64: the register writer, blocks stored straight from it
    if (g.maxbits == 32 || g.maxbits == 64) {
      gg.lds_words = 0;
      const dim3 grid((nwaves + kWavesPerGroup - 1) / kWavesPerGroup), block(kLanes * kWavesPerGroup);
      const bool prio = use_priority(nwaves, occupancy<Scalar, DIMS, true>::value, CUZFP_ENC_PRIO_ROUNDS);
#define ZFP_ENC_REG(FAST_, PRIO_)                                                                          \
  do {                                                                                                     \
    if (g.maxbits == 64)                                                                                   \
      hipLaunchKernelGGL((zfp_encode<Scalar, DIMS, FAST_, true, PRIO_, 2, kWavesPerGroup>), grid, block, 0, st, d, gg, stream); \
    else                                                                                                   \
      hipLaunchKernelGGL((zfp_encode<Scalar, DIMS, FAST_, true, PRIO_, 1, kWavesPerGroup>), grid, block, 0, st, d, gg, stream); \
  } while (0)
      if constexpr (DIMS == 1 && kRegEncBatch1d > 1) {
        if (fast && nwaves >= kRegBatchMinWaves) {
          constexpr int W = kWavesPerGroup, K = kRegEncBatch1d;
          const uint32_t phys = (nwaves + K - 1) / K;
          const dim3 kgrid((phys + W - 1) / W), kblock(kLanes * W);
          if (g.maxbits == 64)
            hipLaunchKernelGGL((zfp_encode_regk<Scalar, DIMS, false, 2, W, K>), kgrid, kblock, 0, st, d, gg, stream);
          else
            hipLaunchKernelGGL((zfp_encode_regk<Scalar, DIMS, false, 1, W, K>), kgrid, kblock, 0, st, d, gg, stream);
          const hipError_t e = hipGetLastError();
          t_last_hip = e;
          return e == hipSuccess ? CUZFP_SUCCESS : CUZFP_ERROR_HIP;
        }
      }
      if (fast && prio) ZFP_ENC_REG(true, true);
      else if (fast) ZFP_ENC_REG(true, false);
      else if (prio) ZFP_ENC_REG(false, true);
      else ZFP_ENC_REG(false, false);
#undef ZFP_ENC_REG
      const hipError_t e = hipGetLastError();
      t_last_hip = e;
      return e == hipSuccess ? CUZFP_SUCCESS : CUZFP_ERROR_HIP;
    }
  }
  // the word-aligned writer pads each lane with slack words; very large maxbits
  // (whose padded image would pass the workgroup's LDS) take the general writer
  const bool aligned = (g.maxbits & 63) == 0 && gg.lds_words * 8 + kStatic <= lds_cap_bytes();
  if (!aligned) gg.lds_words = g.maxbits + 2;
  gg.row_stage = 0;  // (the decoder's staged row stores only)
  // one wave's image beside the tables must fit the workgroup's LDS budget
  if (gg.lds_words * 8 + kStatic > lds_cap_bytes()) return CUZFP_ERROR_INVALID_ARGUMENT;
  const uint32_t wpg = waves_per_group(gg.lds_words, kStatic, kEncWaves);
  const dim3 grid((nwaves + wpg - 1) / wpg), block(kLanes * wpg);
  const size_t lds = (size_t)wpg * gg.lds_words * 8;
  if (fast && aligned && !use_priority(nwaves, occupancy<Scalar, DIMS, true>::value, CUZFP_ENC_PRIO_ROUNDS))
    hipLaunchKernelGGL((zfp_encode<Scalar, DIMS, true, true, false>), grid, block, lds, st, d, gg, stream);
  else if (fast && aligned)
    hipLaunchKernelGGL((zfp_encode<Scalar, DIMS, true, true>), grid, block, lds, st, d, gg, stream);
  else if (fast)
    hipLaunchKernelGGL((zfp_encode<Scalar, DIMS, true, false>), grid, block, lds, st, d, gg, stream);
  else if constexpr (kFastOnly)
    return CUZFP_ERROR_UNSUPPORTED_TYPE;
  else if (aligned)
    hipLaunchKernelGGL((zfp_encode<Scalar, DIMS, false, true>), grid, block, lds, st, d, gg, stream);
  else
    hipLaunchKernelGGL((zfp_encode<Scalar, DIMS, false, false>), grid, block, lds, st, d, gg, stream);
  const hipError_t e = hipGetLastError();
  t_last_hip = e;
  return e == hipSuccess ? CUZFP_SUCCESS : CUZFP_ERROR_HIP;
}

template <typename Scalar, int DIMS>
int launch_decode_t(const uint64_t* stream, const Geometry& g, bool fast, void* data,
                           uint32_t wave0, uint32_t nwaves, hipStream_t st) {
  Geometry gg = g;
  gg.wave0 = wave0;
  gg.wave_end = wave0 + nwaves;
  gg.vec_io = (g.maxbits % 2 == 0) && ((uintptr_t)stream % 16 == 0);
  gg.lds_words = ((g.maxbits + 31) / 32 + 5) * 32;  // (dwords per block + 5 slack rows) x 64 lanes
  // 3D double: stage the row stores through the wave's image when every wave
  // is a full x-row segment of 64 blocks (scatter_f64_staged), 4 / 2 / 1 rows
  // (2 KiB each) a pass as the image allows
  gg.row_stage = 0;
  if (sizeof(Scalar) == 8 && DIMS == 3 && fast && g.bx % kLanes == 0) {
    const size_t img = (size_t)gg.lds_words * 8;
    gg.row_stage = img >= 4 * 2048 ? 4 : img >= 2 * 2048 ? 2 : img >= 2048 ? 1 : 0;
  }
  // blocks of at most 64 bits are read into registers (RegReader): no LDS image
  const bool reg = DIMS <= 2 && g.maxbits <= 64;
  if (reg) gg.lds_words = 0;
  const size_t kStatic = chunk_lut_bytes<DIMS>() + (DIMS == 1 ? sizeof(Plane1dDecLut) : 16);
  // one wave's image beside the tables must fit the workgroup's LDS budget
  if (gg.lds_words * 8 + kStatic > lds_cap_bytes()) return CUZFP_ERROR_INVALID_ARGUMENT;
  const uint32_t wpg = waves_per_group(gg.lds_words, kStatic, kDecWaves);
  const dim3 grid((nwaves + wpg - 1) / wpg), block(kLanes * wpg);
  const size_t lds = (size_t)wpg * gg.lds_words * 8;  // (+ the static chunk tables)
  Scalar* d = (Scalar*)data;
  if constexpr (DIMS <= 2) {
    if (reg) {
      const bool prio = use_priority(nwaves, occupancy<Scalar, DIMS>::value, 2);
      if constexpr (DIMS == 1 && kRegDecBatch1d > 1) {
        if (fast && nwaves >= kRegBatchMinWaves) {
          constexpr int W = kRegBatchWaves1d, K = kRegDecBatch1d;
          const uint32_t phys = (nwaves + K - 1) / K;
          const dim3 kgrid((phys + W - 1) / W), kblock(kLanes * W);
          constexpr bool P = CUZFP_REG_BATCH_PRIO;
          if (g.maxbits == 32)
            hipLaunchKernelGGL((zfp_decode_regk<Scalar, DIMS, true, P, W, K, 32>), kgrid, kblock, 0, st, stream, gg, d);
          else
            hipLaunchKernelGGL((zfp_decode_regk<Scalar, DIMS, true, P, W, K, 64>), kgrid, kblock, 0, st, stream, gg, d);
          const hipError_t e = hipGetLastError();
          t_last_hip = e;
          return e == hipSuccess ? CUZFP_SUCCESS : CUZFP_ERROR_HIP;
        }
      }
      constexpr int W = DIMS == 1 ? kRegWaves1d : kRegWaves2d;
      const dim3 rgrid((nwaves + W - 1) / W), rblock(kLanes * W);
      auto go = [&](auto rb) {
        constexpr int RB = decltype(rb)::value;
        if (fast && prio)
          hipLaunchKernelGGL((zfp_decode<Scalar, DIMS, true, true, RB, W>), rgrid, rblock, 0, st, stream, gg, d);
        else if (fast)
          hipLaunchKernelGGL((zfp_decode<Scalar, DIMS, true, false, RB, W>), rgrid, rblock, 0, st, stream, gg, d);
        else if (prio)
          hipLaunchKernelGGL((zfp_decode<Scalar, DIMS, false, true, RB, W>), rgrid, rblock, 0, st, stream, gg, d);
        else
          hipLaunchKernelGGL((zfp_decode<Scalar, DIMS, false, false, RB, W>), rgrid, rblock, 0, st, stream, gg, d);
      };
      if (g.maxbits == 32)
        go(std::integral_constant<int, 32>{});
      else
        go(std::integral_constant<int, 64>{});
      const hipError_t e = hipGetLastError();
      t_last_hip = e;
      return e == hipSuccess ? CUZFP_SUCCESS : CUZFP_ERROR_HIP;
    }
  }
  // the decoder keeps the priority schedule up to two resident rounds; 3D
  // double (two waves a SIMD) up to one: at 256^3 r16 (two rounds) its decode
  // measured 56.6 -> 54.9 us without it (r04_f64prio)
  constexpr uint32_t kDecPrioRounds = (sizeof(Scalar) == 8 && DIMS == 3) ? 1 : 2;
  if (fast && !use_priority(nwaves, occupancy<Scalar, DIMS>::value, kDecPrioRounds))
    hipLaunchKernelGGL((zfp_decode<Scalar, DIMS, true, false>), grid, block, lds, st, stream, gg, d);
  else if (fast)
    hipLaunchKernelGGL((zfp_decode<Scalar, DIMS, true>), grid, block, lds, st, stream, gg, d);
  else if constexpr (!kFastOnly)
    hipLaunchKernelGGL((zfp_decode<Scalar, DIMS, false>), grid, block, lds, st, stream, gg, d);
  const hipError_t e = hipGetLastError();
  t_last_hip = e;
  return e == hipSuccess ? CUZFP_SUCCESS : CUZFP_ERROR_HIP;
}


// Per-type entry points (declared in launch.hpp).  tools/xvar.py's timing
// variants (never the product library) build the 3D fast-gather kernels alone
// from tools/xvar_launch.hpp instead.
#if defined(CUZFP_XVAR)
#include "../../tools/xvar_launch.hpp"
#else
template <typename Scalar>
int launch_encode_type(const Problem& p, const void* data, bool fast, uint64_t* stream,
                       uint32_t wave0, uint32_t nwaves, hipStream_t st) {
  switch (p.dims) {
    case 1: return launch_encode_t<Scalar, 1>(data, p.g, fast, stream, wave0, nwaves, st);
    case 2: return launch_encode_t<Scalar, 2>(data, p.g, fast, stream, wave0, nwaves, st);
    default: return launch_encode_t<Scalar, 3>(data, p.g, fast, stream, wave0, nwaves, st);
  }
}

template <typename Scalar>
int launch_decode_type(const Problem& p, const uint64_t* stream, bool fast, void* data,
                       uint32_t wave0, uint32_t nwaves, hipStream_t st) {
  switch (p.dims) {
    case 1: return launch_decode_t<Scalar, 1>(stream, p.g, fast, data, wave0, nwaves, st);
    case 2: return launch_decode_t<Scalar, 2>(stream, p.g, fast, data, wave0, nwaves, st);
    default: return launch_decode_t<Scalar, 3>(stream, p.g, fast, data, wave0, nwaves, st);
  }
}

#endif

}  // namespace cuzfp
