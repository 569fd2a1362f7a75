// tools/xvar_pad.hpp -- timing experiment for tools/xvar.py (never in the
// product library): force-included with -include, it defines the codec's phase
// hook ZFP_STAMP(i) (zfp_block.hpp; empty in the product) so that phase PAD_AT
// of every block runs PAD_N x 8 extra independent VALU instructions of kind
// PAD_KIND (1 v_add_u32, 2 v_bfi_b32, 3 v_lshlrev_b64, 4 v_min_u32, 5 v_bcnt).
// The kernel-time difference per instruction is the marginal issue cost of
// that kind in the real kernel's context.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#if defined(__HIP_DEVICE_COMPILE__)
#ifndef PAD_AT
#define PAD_AT 3
#endif
#ifndef PAD_N
#define PAD_N 8
#endif
#ifndef PAD_KIND
#define PAD_KIND 1
#endif
#if PAD_KIND == 1
#define XP_OP(r) "v_add_u32 " r ", " r ", %8\n"
#elif PAD_KIND == 2
#define XP_OP(r) "v_bfi_b32 " r ", %9, " r ", %8\n"
#elif PAD_KIND == 4
#define XP_OP(r) "v_min_u32 " r ", " r ", %8\n"
#elif PAD_KIND == 5
#define XP_OP(r) "v_bcnt_u32_b32 " r ", " r ", %8\n"
#endif
__device__ __forceinline__ void xvar_pad(uint32_t seed) {
#if PAD_KIND == 3
  uint64_t d0 = seed, d1 = seed + 1, d2 = seed + 2, d3 = seed + 3;
  asm volatile(".rept %c5\nv_lshlrev_b64 %0, %4, %0\nv_lshlrev_b64 %1, %4, %1\nv_lshlrev_b64 %2, %4, %2\n"
               "v_lshlrev_b64 %3, %4, %3\nv_lshlrev_b64 %0, %4, %0\nv_lshlrev_b64 %1, %4, %1\n"
               "v_lshlrev_b64 %2, %4, %2\nv_lshlrev_b64 %3, %4, %3\n.endr\n"
               : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3)
               : "v"(seed & 7), "i"(PAD_N));
#else
  uint32_t d0 = seed, d1 = seed + 1, d2 = seed + 2, d3 = seed + 3, d4 = seed + 4, d5 = seed + 5, d6 = seed + 6,
           d7 = seed + 7;
  asm volatile(".rept %c10\n" XP_OP("%0") XP_OP("%1") XP_OP("%2") XP_OP("%3") XP_OP("%4") XP_OP("%5") XP_OP("%6")
                   XP_OP("%7") ".endr\n"
               : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
               : "v"(seed * 3u), "s"(0x0f0f0f0fu), "i"(PAD_N));
#endif
}
#define ZFP_STAMP(i)                                 \
  do {                                               \
    if constexpr ((i) == PAD_AT) xvar_pad(threadIdx.x); \
  } while (0)
#endif
