// Building blocks shared by the implicit-GEMM conv kernels (K1 conv_igemm.hip, K1c conv_chain.hip):
// LDS-DMA issue, counted vmcnt waits, the 64-B LDS row swizzle and the wave-uniform tap walk.
#pragma once
#include "common.h"

namespace ai4e_conv {

constexpr int BK = 32;  // K elements per LDS row (64 B)

// Physical 16-B chunk rotation of a 64-B LDS row: s = {0,2,3,1}[(row>>2)&3] makes every ds_read_b128
// fragment read conflict-free for the gfx950 lane groups (MI355X_MICROARCH.md §LDS).
__device__ __forceinline__ int swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

// One 16-B LDS-DMA per lane: global -> LDS at (wave-uniform M0 base + 16*lane). Inline asm so hipcc
// neither drains it with vmcnt(0) before every ds_read nor at barriers (cdna guide §5.7); completion is
// tracked by hand with counted vmcnt. The swizzle is applied to the per-lane SOURCE address.
// M0 is saved and restored around the DMA: hipcc treats M0 as a reserved register and ignores it in a clobber
// list (-Winline-asm), so a live M0 of its own (s_movrel indexing) would otherwise be corrupted silently.
// Streaming hints (default on; AI4E_STREAM_HINTS=0 builds the plain forms): activations read or written exactly once
// carry the non-temporal policy so they do not evict the weights every workgroup re-reads from L2.
#ifndef AI4E_STREAM_HINTS
#define AI4E_STREAM_HINTS 1
#endif
__device__ __forceinline__ void glds16_stream(const void* gsrc, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
#if AI4E_STREAM_HINTS
      "global_load_lds_dwordx4 %1, off nt\n\t"
#else
      "global_load_lds_dwordx4 %1, off\n\t"
#endif
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_base))
      : "memory");
}

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_stream(void* dst, const uint4& v) {
#if AI4E_STREAM_HINTS
  __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4_t*>(dst));
#else
  *reinterpret_cast<uint4*>(dst) = v;
#endif
}

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_base))
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// vmcnt wait with a count that is a compile-time constant after unrolling (folds to one s_waitcnt);
// counts above the 6-bit field clamp to 63 (a stronger wait, still correct).
__device__ __forceinline__ void wait_vmcnt_n(int n) {
#define AI4E_VMC(k) \
  case k:           \
    wait_vmcnt<k>(); \
    break;
  switch (n <= 0 ? 0 : (n > 63 ? 63 : n)) {
    AI4E_VMC(0) AI4E_VMC(1) AI4E_VMC(2) AI4E_VMC(3) AI4E_VMC(4) AI4E_VMC(5) AI4E_VMC(6) AI4E_VMC(7)
    AI4E_VMC(8) AI4E_VMC(9) AI4E_VMC(10) AI4E_VMC(11) AI4E_VMC(12) AI4E_VMC(13) AI4E_VMC(14) AI4E_VMC(15)
    AI4E_VMC(16) AI4E_VMC(17) AI4E_VMC(18) AI4E_VMC(19) AI4E_VMC(20) AI4E_VMC(21) AI4E_VMC(22) AI4E_VMC(23)
    AI4E_VMC(24) AI4E_VMC(25) AI4E_VMC(26) AI4E_VMC(27) AI4E_VMC(28) AI4E_VMC(29) AI4E_VMC(30) AI4E_VMC(31)
    AI4E_VMC(32) AI4E_VMC(33) AI4E_VMC(34) AI4E_VMC(35) AI4E_VMC(36) AI4E_VMC(37) AI4E_VMC(38) AI4E_VMC(39)
    AI4E_VMC(40) AI4E_VMC(41) AI4E_VMC(42) AI4E_VMC(43) AI4E_VMC(44) AI4E_VMC(45) AI4E_VMC(46) AI4E_VMC(47)
    default: wait_vmcnt<48>(); break;  // >= 48: a stronger wait is still correct
  }
#undef AI4E_VMC
}

// Wave-uniform (SGPR) walk over the taps of a conv whose K tiles never straddle a tap
// (C % step == 0): (kh, kw, channel base cb) and the element offset (kh*W + kw)*ldx + cb, kept up to
// date with adds only (no per-step multiplies or divisions on the scalar unit).
struct TapWalk {
  int kh = 0, kw = 0, cb = 0, off = 0;
  __device__ __forceinline__ void next(int step, int C, int KW, int ldx, int rowjump) {
    cb += step;
    off += step;
    if (cb == C) {
      cb = 0;
      off += ldx - C;
      if (++kw == KW) {
        kw = 0;
        ++kh;
        off += rowjump;  // (W - KW) * ldx
      }
    }
  }
};

}  // namespace ai4e_conv
