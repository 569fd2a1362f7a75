// tools/ubench/opcost.hip -- SIMD cycles per wave64 instruction, by opcode
// (design measurement for the codec kernels, which are issue-bound).
//
// Each wave runs 8 independent chains of one opcode (no dependency stalls
// beyond the chain length) for ITERS x 32 instructions and stamps s_memtime
// (shader clock) around the loop.  Workgroups of 256 threads put one wave on
// each SIMD of a CU; the grid puts k = 1, 2, 4 workgroups on every CU, so a
// SIMD holds k waves.  Cycles per instruction = median wave duration /
// (k x instructions per wave).
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/opcost.hip -o build/opcost
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define ITERS 64

#define R4(x) x x x x
#define P4(op) op("%0") op("%1") op("%2") op("%3")
#define CH8(op) op("%0") op("%1") op("%2") op("%3") op("%4") op("%5") op("%6") op("%7")

// one instruction on chain register r, reading the other inputs from the
// loop-invariant operands %8 (VGPR) and %9 (SGPR)
#define OP_ADD(r) "v_add_u32 " r ", " r ", %8\n"
#define OP_ADD64E(r) "v_add_u32_e64 " r ", " r ", %8\n"
#define OP_ASHR(r) "v_ashrrev_i32 " r ", 1, " r "\n"
#define OP_SUB(r) "v_sub_u32 " r ", " r ", %8\n"
#define OP_XOR(r) "v_xor_b32 " r ", " r ", %8\n"
#define OP_BFI(r) "v_bfi_b32 " r ", %9, " r ", %8\n"
#define OP_PERM(r) "v_perm_b32 " r ", " r ", %8, %9\n"
#define OP_ALIGN(r) "v_alignbit_b32 " r ", " r ", %8, " r "\n"
#define OP_BFE(r) "v_bfe_u32 " r ", " r ", 3, 20\n"
#define OP_LSHLADD(r) "v_lshl_add_u32 " r ", " r ", 2, %8\n"
#define OP_ADD3(r) "v_add3_u32 " r ", " r ", %8, %9\n"
#define OP_BITOP3(r) "v_bitop3_b32 " r ", %9, " r ", %8 bitop3:0x35\n"
#define OP_LSHLOR(r) "v_lshl_or_b32 " r ", " r ", 1, %8\n"
#define OP_CNDMASK(r) "v_cndmask_b32 " r ", " r ", %8, vcc\n"
#define OP_BCNT(r) "v_bcnt_u32_b32 " r ", " r ", %8\n"
#define OP_FFBL(r) "v_ffbl_b32 " r ", " r "\n"
#define OP_CVTF(r) "v_cvt_f32_u32 " r ", " r "\n"
#define OP_FREXP(r) "v_frexp_exp_i32_f32 " r ", " r "\n"
#define OP_CVTI(r) "v_cvt_i32_f32 " r ", " r "\n"
#define OP_MULF(r) "v_mul_f32 " r ", " r ", %8\n"
#define OP_MAX3(r) "v_max3_f32 " r ", " r ", %8, %9\n"
#define OP_MOV(r) "v_mov_b32 " r ", %8\n"
#define OP_XAD(r) "v_xad_u32 " r ", " r ", %9, %8\n"
#define OP_MIN(r) "v_min_u32 " r ", " r ", %8\n"
#define OP_LSHR(r) "v_lshrrev_b32 " r ", 3, " r "\n"
#define OP_AND(r) "v_and_b32 " r ", " r ", %8\n"
#define OP_CNDS(r) "v_cndmask_b32_e64 " r ", " r ", %8, s[20:21]\n"
#define OP_SUBS(r) "v_sub_u32 " r ", %9, " r "\n"
#define OP_ADDK(r) "v_add_u32 " r ", 0x1234567, " r "\n"
#define OP_OR(r) "v_or_b32 " r ", " r ", %8\n"
#define OP_NOT(r) "v_not_b32 " r ", " r "\n"
#define OP_MAXU(r) "v_max_u32 " r ", " r ", %8\n"
#define OP_MULU24(r) "v_mul_u32_u24 " r ", " r ", %8\n"
#define OP_LSHL(r) "v_lshlrev_b32 " r ", %8, " r "\n"
#define OP_MIX(r) "v_add_u32 " r ", " r ", %8\nv_bfi_b32 " r ", %9, " r ", %8\n"
#define OP_MIX3(r) "v_add_u32 " r ", " r ", %8\nv_xor_b32 " r ", " r ", %8\nv_bfi_b32 " r ", %9, " r ", %8\n"
#define OP_CMP(r) "v_cmp_gt_u32 vcc, " r ", %8\n"
#define OP_CMPS(r) "v_cmp_gt_u32_e64 s[20:21], " r ", %8\n"
#define OP_SUBREV(r) "v_subrev_u32 " r ", " r ", %8\n"
#define OP_MINI(r) "v_min_i32 " r ", " r ", %8\n"
#define OP_MED3(r) "v_med3_u32 " r ", " r ", %8, %9\n"
#define OP_MADU24(r) "v_mad_u32_u24 " r ", " r ", %8, %9\n"
#define OP_DPP(r) "v_mov_b32_dpp " r ", " r " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define OP_LSHLREV16(r) "v_lshlrev_b16 " r ", 1, " r "\n"

template <int KIND>
__device__ __forceinline__ void body32(uint32_t (&c)[8], uint32_t v, uint32_t s) {
#define RUNS(OP)                                                                         \
  asm volatile(R4(CH8(OP))                                                               \
               : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), \
                 "+v"(c[6]), "+v"(c[7])                                                  \
               : "v"(v), "s"(s)                                                          \
               : "vcc", "s20", "s21")
#define RUN(OP)                                                                          \
  asm volatile(R4(CH8(OP))                                                               \
               : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), \
                 "+v"(c[6]), "+v"(c[7])                                                  \
               : "v"(v), "s"(s)                                                          \
               : "vcc")
  if constexpr (KIND == 0) RUN(OP_ADD);
  else if constexpr (KIND == 1) RUN(OP_ADD64E);
  else if constexpr (KIND == 2) RUN(OP_ASHR);
  else if constexpr (KIND == 3) RUN(OP_SUB);
  else if constexpr (KIND == 4) RUN(OP_XOR);
  else if constexpr (KIND == 5) RUN(OP_BFI);
  else if constexpr (KIND == 6) RUN(OP_PERM);
  else if constexpr (KIND == 7) RUN(OP_ALIGN);
  else if constexpr (KIND == 8) RUN(OP_BFE);
  else if constexpr (KIND == 9) RUN(OP_LSHLADD);
  else if constexpr (KIND == 10) RUN(OP_ADD3);
  else if constexpr (KIND == 11) RUN(OP_BITOP3);
  else if constexpr (KIND == 12) RUN(OP_LSHLOR);
  else if constexpr (KIND == 13) RUN(OP_CNDMASK);
  else if constexpr (KIND == 14) RUN(OP_BCNT);
  else if constexpr (KIND == 15) RUN(OP_FFBL);
  else if constexpr (KIND == 16) RUN(OP_CVTF);
  else if constexpr (KIND == 17) RUN(OP_FREXP);
  else if constexpr (KIND == 18) RUN(OP_CVTI);
  else if constexpr (KIND == 19) RUN(OP_MULF);
  else if constexpr (KIND == 20) RUN(OP_MAX3);
  else if constexpr (KIND == 21) RUN(OP_MOV);
  else if constexpr (KIND == 22) RUN(OP_XAD);
  else if constexpr (KIND == 23) RUN(OP_MIN);
  else if constexpr (KIND == 24) RUN(OP_LSHR);
  else if constexpr (KIND == 25) RUN(OP_AND);
  else if constexpr (KIND == 26) RUNS(OP_CNDS);
  else if constexpr (KIND == 27) RUN(OP_SUBS);
  else if constexpr (KIND == 28) RUN(OP_ADDK);
  else if constexpr (KIND == 29) RUN(OP_OR);
  else if constexpr (KIND == 30) RUN(OP_NOT);
  else if constexpr (KIND == 31) RUN(OP_MAXU);
  else if constexpr (KIND == 32) RUN(OP_MULU24);
  else if constexpr (KIND == 33) RUN(OP_LSHL);
  else if constexpr (KIND == 34) RUN(OP_MIX);
  else if constexpr (KIND == 35) RUN(OP_MIX3);
  else if constexpr (KIND == 36) RUN(OP_CMP);
  else if constexpr (KIND == 37) RUNS(OP_CMPS);
  else if constexpr (KIND == 38) RUN(OP_SUBREV);
  else if constexpr (KIND == 39) RUN(OP_MINI);
  else if constexpr (KIND == 40) RUN(OP_MED3);
  else if constexpr (KIND == 41) RUN(OP_MADU24);
  else if constexpr (KIND == 42) RUN(OP_DPP);
  else if constexpr (KIND == 43) RUN(OP_LSHLREV16);
  else if constexpr (KIND == 50) {  // VGPR-indexed read: s_set_gpr_idx_on / v_mov / off, + 3 fast ops
#define GI(r) "s_set_gpr_idx_on %9, gpr_idx(SRC0)\nv_mov_b32 " r ", v40\ns_set_gpr_idx_off\nv_add_u32 " r ", " r ", %8\nv_xor_b32 " r ", " r ", %8\nv_add_u32 " r ", " r ", %8\n"
    asm volatile(CH8(GI) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s & 7) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "m0");
#undef GI
  } else if constexpr (KIND == 51) {  // 4 fast ops only (baseline for 50)
#define GB(r) "v_mov_b32 " r ", %8\nv_add_u32 " r ", " r ", %8\nv_xor_b32 " r ", " r ", %8\nv_add_u32 " r ", " r ", %8\n"
    asm volatile(CH8(GB) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
#undef GB
  } else if constexpr (KIND == 52) {  // wave-uniform branch test: v_cmp + s_and + s_cbranch (not taken), + 3 fast ops
#define BR(r) "v_cmp_gt_u32 vcc, " r ", %8\ns_and_b64 vcc, exec, vcc\ns_cbranch_vccnz 1f\n1:\nv_add_u32 " r ", " r ", %8\nv_xor_b32 " r ", " r ", %8\nv_add_u32 " r ", " r ", %8\n"
    asm volatile(CH8(BR) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
#undef BR
  } else if constexpr (KIND == 53) {  // v_cmp only + 3 fast (baseline for 52)
#define BC(r) "v_cmp_gt_u32 vcc, " r ", %8\nv_add_u32 " r ", " r ", %8\nv_xor_b32 " r ", " r ", %8\nv_add_u32 " r ", " r ", %8\n"
    asm volatile(CH8(BC) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
#undef BC
  } else if constexpr (KIND == 54) {  // LDS round trip on the chain: ds_read_b32 at an address from the chain, wait, + 3 fast
#define LD(r) "v_and_b32 " r ", 0x3fc, " r "\nds_read_b32 " r ", " r "\ns_waitcnt lgkmcnt(0)\nv_add_u32 " r ", " r ", %8\nv_xor_b32 " r ", " r ", %8\n"
    asm volatile(CH8(LD) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc", "memory");
#undef LD
  } else if constexpr (KIND == 55) {  // 8 LDS reads in flight, one wait, + fast ops
#define LQ(r) "v_and_b32 " r ", 0x3fc, " r "\nds_read_b32 " r ", " r "\n"
#define LA(r) "v_add_u32 " r ", " r ", %8\nv_xor_b32 " r ", " r ", %8\n"
    asm volatile(CH8(LQ) "s_waitcnt lgkmcnt(0)\n" CH8(LA) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc", "memory");
#undef LQ
#undef LA
  } else if constexpr (KIND == 60) {  // v_cmp (VCC) then v_cndmask_b32 (VOP2, VCC) on each chain: 2 instructions
#define CV(r) "v_cmp_gt_u32 vcc, " r ", %8\nv_cndmask_b32 " r ", " r ", %8, vcc\n"
    asm volatile(CH8(CV) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
#undef CV
  } else if constexpr (KIND == 61) {  // the same with the VOP3 compare into an SGPR pair and v_cndmask_b32_e64
#define CS(r) "v_cmp_gt_u32_e64 s[20:21], " r ", %8\nv_cndmask_b32_e64 " r ", " r ", %8, s[20:21]\n"
    asm volatile(CH8(CS) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc", "s20", "s21");
#undef CS
  } else if constexpr (KIND == 62) {  // v_cndmask_b32 (VOP2) with VCC written once by a v_cmp before the block
    asm volatile("v_cmp_gt_u32 vcc, %0, %8\ns_nop 4\n" R4(CH8(OP_CNDMASK)) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
  } else if constexpr (KIND == 63) {  // one dependent chain of v_add_u32 (latency)
#define DA(r) "v_add_u32 %0, %0, %8\n"
    asm volatile(R4(CH8(DA)) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
#undef DA
  } else if constexpr (KIND == 64) {  // one dependent chain of v_bfi_b32
#define DB(r) "v_bfi_b32 %0, %9, %0, %8\n"
    asm volatile(R4(CH8(DB)) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
#undef DB
  } else if constexpr (KIND == 65) {  // two dependent chains of v_add_u32, interleaved
#define D2(r) "v_add_u32 %0, %0, %8\nv_add_u32 %1, %1, %8\n"
    asm volatile(R4(P4(D2)) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
#undef D2
  } else if constexpr (KIND == 66) {  // SDWA move into the high half, low half preserved
#define SD(r) "v_mov_b32_sdwa " r ", %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n"
    asm volatile(R4(CH8(SD)) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
#undef SD
  } else if constexpr (KIND == 67) {  // packed 16-bit add
#define PA(r) "v_pk_add_u16 " r ", " r ", %8\n"
    asm volatile(R4(CH8(PA)) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
#undef PA
  } else if constexpr (KIND == 68) {  // v_lshlrev_b32 by an inline constant
#define LC(r) "v_lshlrev_b32 " r ", 3, " r "\n"
    asm volatile(R4(CH8(LC)) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
#undef LC
  } else if constexpr (KIND == 69) {  // v_cndmask_b32_e64 with an inline-constant source
#define CK(r) "v_cndmask_b32_e64 " r ", 0, " r ", s[20:21]\n"
    asm volatile("s_mov_b64 s[20:21], -1\n" R4(CH8(CK)) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc", "s20", "s21");
#undef CK
  } else if constexpr (KIND == 70) {  // v_and_or_b32 (VOP3, SGPR mask)
#define AO(r) "v_and_or_b32 " r ", " r ", %9, %8\n"
    asm volatile(R4(CH8(AO)) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
#undef AO
  } else if constexpr (KIND == 71) {  // v_add_u32 with the literal and VGPR swapped to e64 with an SGPR
#define AS(r) "v_add_u32 " r ", %9, " r "\n"
    asm volatile(R4(CH8(AS)) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
#undef AS
  } else if constexpr (KIND == 72) {  // v_sub_u32 with a VGPR from another chain (two VGPR sources, both changing)
#define SV(r) "v_sub_u32 " r ", " r ", %0\n"
    asm volatile(R4(CH8(SV)) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc");
#undef SV
  } else if constexpr (KIND == 56) {  // readfirstlane + s_lshl + 3 fast
#define RF(r) "v_readfirstlane_b32 s20, " r "\ns_lshl_b32 s21, 1, s20\nv_add_u32 " r ", " r ", %8\nv_xor_b32 " r ", " r ", %8\nv_add_u32 " r ", " r ", %8\n"
    asm volatile(CH8(RF) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) : "v"(v), "s"(s) : "vcc", "s20", "s21", "scc");
#undef RF
  }
#undef RUN
#undef RUNS
}

// 64-bit kinds: 4 chains of register pairs
#define OP_SHL64(r) "v_lshlrev_b64 " r ", 1, " r "\n"
#define OP_SHR64(r) "v_lshrrev_b64 " r ", %4, " r "\n"
#define OP_LADD64(r) "v_lshl_add_u64 " r ", " r ", 1, %5\n"
#define OP_PKMUL(r) "v_pk_mul_f32 " r ", " r ", %5\n"
#define OP_PKADD(r) "v_pk_add_f32 " r ", " r ", %5\n"
#define OP_MOV64(r) "v_mov_b64 " r ", %5\n"

template <int KIND>
__device__ __forceinline__ void body64(uint64_t (&c)[4], uint32_t v, uint64_t w) {
#define RUN(OP)                                                                                   \
  asm volatile(R4(P4(OP)) R4(P4(OP)) : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]) : "v"(v), \
               "v"(w))
  if constexpr (KIND == 100) RUN(OP_SHL64);
  else if constexpr (KIND == 101) RUN(OP_SHR64);
  else if constexpr (KIND == 102) RUN(OP_LADD64);
  else if constexpr (KIND == 103) RUN(OP_PKMUL);
  else if constexpr (KIND == 104) RUN(OP_PKADD);
  else if constexpr (KIND == 105) RUN(OP_MOV64);
#undef RUN
}

template <int KIND>
__global__ __launch_bounds__(256) void work(uint32_t* out, uint64_t* cyc, uint32_t seed) {
  const uint32_t t = threadIdx.x;
  uint32_t v = seed * 7 + t, s = __builtin_amdgcn_readfirstlane(seed + 0x0c0d0e0fu);
  uint32_t c[8];
  uint64_t d[4];
  for (int i = 0; i < 8; i++) c[i] = seed + t * (i + 1);
  for (int i = 0; i < 4; i++) d[i] = ((uint64_t)(seed + i) << 32) | (t + i);
  __shared__ uint32_t sh[1024];  // the LDS kinds read dwords 0..255 of it
  for (int i = t; i < 1024; i += 256) sh[i] = i * 4;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; it++) {
    if constexpr (KIND < 100) body32<KIND>(c, v, s);
    else body64<KIND>(d, v & 7, ((uint64_t)v << 32) | v);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t r = 0;
  for (int i = 0; i < 8; i++) r ^= c[i];
  for (int i = 0; i < 4; i++) r ^= (uint32_t)d[i] ^ (uint32_t)(d[i] >> 32);
  out[blockIdx.x * 256 + t] = r ^ sh[(r >> 3) & 1023];
  if ((t & 63) == 0) cyc[blockIdx.x * 4 + (t >> 6)] = t1 - t0;
}

template <int KIND>
static void run(const char* name, uint32_t* d, uint64_t* c, int cus, int per_body = 32, double scale = 1.0) {
  printf("%-14s", name);
  for (int k : {1, 2, 4}) {
    const int groups = cus * k;
    double best = 1e30;
    for (int rep = 0; rep < 3; rep++) {
      hipLaunchKernelGGL(work<KIND>, dim3(groups), dim3(256), 0, 0, d, c, 1u);
      hipDeviceSynchronize();
      std::vector<uint64_t> h(groups * 4);
      hipMemcpy(h.data(), c, h.size() * 8, hipMemcpyDeviceToHost);
      std::sort(h.begin(), h.end());
      const double med = (double)h[h.size() / 2];
      if (med < best) best = med;
    }
    const double instr = (double)ITERS * per_body * k;  // per SIMD, while all k waves run
    printf("  k=%d %6.2f", k, best / instr);
  }
  printf(per_body == 32 ? "   cycles/instr (median wave, k waves per SIMD)\n" : "   cycles per sequence\n");
  (void)scale;
}

int main(int argc, char** argv) {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  uint32_t* d;
  uint64_t* c;
  hipMalloc(&d, (size_t)cus * 4 * 256 * 4);
  hipMalloc(&c, (size_t)cus * 4 * 4 * 8);
  if (argc > 1 && argv[1][0] == 'n') {  // the round-3 kinds only
    run<60>("cmp+cnd vcc", d, c, cus, 64);
    run<61>("cmp+cnd e64", d, c, cus, 64);
    run<62>("cnd vcc fixed", d, c, cus);
    run<13>("v_cndmask_b32", d, c, cus);
    run<26>("v_cndmask_e64 s", d, c, cus);
    run<69>("cnd e64 const", d, c, cus);
    run<63>("dep add x1", d, c, cus);
    run<65>("dep add x2", d, c, cus);
    run<0>("v_add_u32", d, c, cus);
    run<64>("dep bfi x1", d, c, cus);
    run<5>("v_bfi_b32", d, c, cus);
    run<66>("mov sdwa w1", d, c, cus);
    run<67>("v_pk_add_u16", d, c, cus);
    run<68>("lshl const", d, c, cus);
    run<33>("v_lshlrev_b32 v", d, c, cus);
    run<70>("v_and_or_b32", d, c, cus);
    run<71>("v_add_u32 sgpr", d, c, cus);
    run<72>("v_sub vv", d, c, cus);
    return 0;
  }
  run<0>("v_add_u32", d, c, cus);
  run<1>("v_add_u32_e64", d, c, cus);
  run<2>("v_ashrrev_i32", d, c, cus);
  run<3>("v_sub_u32", d, c, cus);
  run<4>("v_xor_b32", d, c, cus);
  run<23>("v_min_u32", d, c, cus);
  run<24>("v_lshrrev_b32", d, c, cus);
  run<25>("v_and_b32", d, c, cus);
  run<21>("v_mov_b32", d, c, cus);
  run<5>("v_bfi_b32", d, c, cus);
  run<6>("v_perm_b32", d, c, cus);
  run<7>("v_alignbit", d, c, cus);
  run<8>("v_bfe_u32", d, c, cus);
  run<9>("v_lshl_add_u32", d, c, cus);
  run<10>("v_add3_u32", d, c, cus);
  run<11>("v_bitop3_b32", d, c, cus);
  run<12>("v_lshl_or_b32", d, c, cus);
  run<22>("v_xad_u32", d, c, cus);
  run<13>("v_cndmask_b32", d, c, cus);
  run<14>("v_bcnt_u32", d, c, cus);
  run<15>("v_ffbl_b32", d, c, cus);
  run<16>("v_cvt_f32_u32", d, c, cus);
  run<17>("v_frexp_exp", d, c, cus);
  run<18>("v_cvt_i32_f32", d, c, cus);
  run<19>("v_mul_f32", d, c, cus);
  run<20>("v_max3_f32", d, c, cus);
  run<26>("v_cndmask_e64 s", d, c, cus);
  run<27>("v_sub_u32 sgpr", d, c, cus);
  run<28>("v_add_u32 lit", d, c, cus);
  run<29>("v_or_b32", d, c, cus);
  run<30>("v_not_b32", d, c, cus);
  run<31>("v_max_u32", d, c, cus);
  run<32>("v_mul_u32_u24", d, c, cus);
  run<33>("v_lshlrev_b32 v", d, c, cus);
  run<34>("mix add+bfi", d, c, cus);
  run<35>("mix 2fast+bfi", d, c, cus);
  run<36>("v_cmp vcc", d, c, cus);
  run<37>("v_cmp_e64 sgpr", d, c, cus);
  run<38>("v_subrev_u32", d, c, cus);
  run<39>("v_min_i32", d, c, cus);
  run<40>("v_med3_u32", d, c, cus);
  run<41>("v_mad_u32_u24", d, c, cus);
  run<42>("v_mov_dpp", d, c, cus);
  run<43>("v_lshlrev_b16", d, c, cus);
  run<50>("gpr_idx+3fast", d, c, cus, 8, 0.25);
  run<51>("mov+3fast", d, c, cus, 8, 0.25);
  run<52>("br-test+3fast", d, c, cus, 8, 0.25);
  run<53>("cmp+3fast", d, c, cus, 8, 0.25);
  run<54>("lds-rt+2fast", d, c, cus, 8, 0.25);
  run<55>("8lds,wait,16f", d, c, cus, 8, 0.25);
  run<56>("rfl+sl+3fast", d, c, cus, 8, 0.25);
  run<100>("v_lshlrev_b64", d, c, cus);
  run<101>("v_lshrrev_b64", d, c, cus);
  run<102>("v_lshl_add_u64", d, c, cus);
  run<103>("v_pk_mul_f32", d, c, cus);
  run<104>("v_pk_add_f32", d, c, cus);
  run<105>("v_mov_b64", d, c, cus);
  return 0;
}
