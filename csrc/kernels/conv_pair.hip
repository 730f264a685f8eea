// K1p — fused 1x1 pair of consecutive wide bottlenecks (ResNet layer3/4): block i's expand conv c3 with
// its residual and ReLU, and block i+1's reduce conv c1', in one launch:
//
//   Y   = relu(T2 . W3^T + b3 + R)        [BM x C4]    (HBM: block i+1's residual)
//   T1' = relu(Y . W1'^T + b1')           [BM x MIDN]  (HBM: block i+1's 3x3 input)
//
// Why: unfused, layer3 runs c3+res (reads T2 25 MB + R 100 MB, writes Y 100 MB at batch 250) and then the
// next c1 re-reads all of Y; both are short-K GEMMs whose tile grids leave HBM at 2-3 TB/s
// (profiles/r2_final/pmc_summary.txt: 58-70 us + 36-39 us per block). Fused, Y is read back from LDS.
//
// Structure: one 512-thread workgroup (8 wave64s) per BM-pixel tile; LDS holds the T2 tile [BM x MID] for
// the whole launch plus a double-buffered Y chunk [BM x CH]. The C4 output channels of c3 go in NP = C4/CH
// passes of CH = 128 channels:
//   B  accb[BM x 16 per wave] = b3 + T2 . W3[chunk rows]^T   (K = MID, v_mfma_f32_16x16x32_bf16)
//   epilogue: + residual (registers, prefetched a pass ahead), ReLU, bf16 -> Y chunk in LDS, one barrier
//   C  accn[BM x MIDN/8 per wave] += Y chunk . W1'[:, chunk]^T (persistent accumulators, seeded with b1')
//   copy-out of the Y chunk with 16-B row stores.
// Weights are pre-packed on the host into MFMA fragment order ([16-row block][32-wide K step][64 lanes][8]),
// so every weight fragment is ONE contiguous 1-KB wave load straight into registers: each wave streams only
// the rows it owns (no LDS ring, no per-step barriers), C fragments a B phase ahead, B fragments a C phase
// ahead. The residual is read in the accumulator layout (4 channels per lane), so the epilogue never
// shuffles. T1' leaves through the (then idle) T2 region with 16-B row stores.
#include "common.h"
#include "conv_common.h"

namespace {

constexpr int PR_CH = 128;     // c3 output channels per pass (Y chunk width)
constexpr int PR_WAVES = 8;

// swizzled 16-B chunk within a 64-B LDS row (same rotation as the K1/K1c operand tiles)
__device__ __forceinline__ int pswz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

// K-blocked tiles: [K/32 blocks][BM rows][64 B], the blocks padded by 128 B: BM * 64 is a multiple of the 256-B
// bank row, so unpadded the 16-B row-chunk copy-out reads conflict (a ds_read_b128 lane group {0-3, 12-15,
// 20-27} reads blocks 0 and 3 of row r and blocks 1-2 of row r+1); with block offsets of 128 B mod 256 the
// group's 16 chunks fall in distinct bank quads
template <int BM>
constexpr int kbs() { return BM * 64 + 128; }

// byte offset of the 8-byte group holding channels n..n+3 of row r in a K-blocked swizzled tile of BM rows
template <int BM>
__device__ __forceinline__ uint32_t poff(int r, int n) {
  const int kb = n >> 5, e = n & 31;
  return kb * kbs<BM>() + r * 64 + ((((e >> 3) ^ pswz(r)) << 4) | (((e >> 2) & 1) << 3));
}

// bias of the 4 channels blk[4 g .. 4 g + 3] (g = lane >> 4) from a wave-uniform 16-float block: scalar loads
// (lgkmcnt, outside the vector-memory waits) and a lane-group select on registers
typedef const float __attribute__((address_space(4)))* pconst_f32_ptr;
__device__ __forceinline__ f32x4_t pbias4(const float* blk, int g) {
  const pconst_f32_ptr b = reinterpret_cast<pconst_f32_ptr>(reinterpret_cast<uintptr_t>(blk));
  f32x4_t r;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float v0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(b[q])));
    const float v1 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(b[4 + q])));
    const float v2 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(b[8 + q])));
    const float v3 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(b[12 + q])));
    const float lo = g & 1 ? v1 : v0;
    const float hi = g & 1 ? v3 : v2;
    r[q] = g & 2 ? hi : lo;
  }
  return r;
}

__device__ __forceinline__ void pbarrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Diagnostic build (AI4E_PAIR_STAMPS=1): s_memtime stamps per wave, summed per segment: 0 = prologue (T2 tile,
// first operands, barrier), 1 = C-weight load issue + B phase (incl. the wait for its weights), 2 = residual wait +
// Y epilogue + barrier, 3 = next-pass load issue + Y copy-out, 4 = C phase (incl. the wait for its weights),
// 5 = T1' epilogue + stores (drained). Shares only: a stamp drains the wave's LDS reads.
#ifndef AI4E_PAIR_STAMPS
#define AI4E_PAIR_STAMPS 0
#endif
constexpr int PAIR_NSEG = 6, PAIR_MAXW = 32768;
#if AI4E_PAIR_STAMPS
__device__ unsigned long long g_pair_stamps[PAIR_MAXW * PAIR_NSEG];
#define PAIR_STAMP(k)                                                              \
  do {                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                             \
    unsigned long long _t;                                                         \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");     \
    __builtin_amdgcn_sched_barrier(0);                                             \
    ps_sum[k] += _t - ps_last;                                                     \
    ps_last = _t;                                                                  \
  } while (0)
#else
#define PAIR_STAMP(k) \
  do {                \
  } while (0)
#endif

struct PairParams {
  const uint16_t* t2;   // [M, MID]
  const uint16_t* w3p;  // packed [C4/16][MID/32][64][8]
  const float* b3;      // [C4]
  const uint16_t* res;  // [M, C4]
  uint16_t* y;          // [M, C4]
  const uint16_t* w1p;  // packed [MIDN/16][C4/32][64][8]
  const float* b1n;     // [MIDN]
  uint16_t* t1n;        // [M, MIDN]
  int M;
};

// SP (bm_cfg 98, the default for the layer3 pair): the residual loads of the next pass and this pass's Y copy-out are spread over the C-phase steps
// (one store chunk and FI / NKC residual loads after each step's MFMAs) instead of a burst between the Y barrier and
// the C phase: the stamps (profiles/r3_pair/) put 33 % of a wave's life in that burst (vector-memory issue backs up).
// (Spreading the next pass's B weight fragments over the C steps as well was measured slower: profiles/r3_pair/.)
// YW (bm_cfg 99): the Y epilogue pairs pixel fragments 16 rows apart with v_permlane16_swap (as the K1c chain's
// patch-mode T2 epilogue), so each lane adds a 16-B residual chunk and writes one 16-B Y chunk per fragment pair
// instead of 8 B per fragment.
__device__ __forceinline__ void pswap16(f32x4_t& a, f32x4_t& b) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[q]), __float_as_uint(b[q]), false, false);
    a[q] = __uint_as_float(r[0]);
    b[q] = __uint_as_float(r[1]);
  }
}

template <int MID, int C4, int MIDN, int BM, bool KF = true, bool SP = false, bool F16 = false, bool YW = false>
__global__ __launch_bounds__(512) void conv_pair_kernel(const PairParams p) {
  constexpr int FI = BM / 16;            // pixel fragments
  constexpr int NKB = MID / 32;          // B K steps
  constexpr int NKC = PR_CH / 32;        // C K steps per pass
  constexpr int NP = C4 / PR_CH;         // passes
  constexpr int JC = MIDN / 16 / PR_WAVES;  // C weight fragments (16-channel blocks) per wave
  constexpr int KBS = kbs<BM>();
  constexpr int T2_BYTES = MID / 32 * KBS;
  constexpr int Y_BYTES = PR_CH / 32 * KBS;
  static_assert(PR_CH == 16 * PR_WAVES, "B: one 16-channel block per wave");
  static_assert(JC >= 1 && MIDN == 16 * PR_WAVES * JC, "C: whole 16-channel blocks per wave");
  static_assert(T2_BYTES + 2 * Y_BYTES >= MIDN / 32 * KBS, "T1' staging fits the T2 + Y regions");
  extern __shared__ __attribute__((aligned(1024))) uint8_t smem[];
  uint8_t* const t2s = smem;
#if AI4E_PAIR_STAMPS
  unsigned long long ps_sum[PAIR_NSEG] = {0, 0, 0, 0, 0, 0}, ps_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ps_last)::"memory");
#endif

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lg = lane >> 4;
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BM;
  const int frow = lane & 15;
  const uint32_t fofs = frow * 64 + (((lg ^ pswz(frow)) << 4));

  // ---- T2 tile -> LDS (K-blocked, swizzled); 16-B loads, rows past M re-read row M-1 (never stored)
  {
    constexpr int N = BM * MID / 8 / 512;
    uint4 v[N];
#pragma unroll
    for (int e = 0; e < N; ++e) {
      const int g = tid + 512 * e;
      const int r = g / (MID / 8), cq = g % (MID / 8);
      v[e] = *reinterpret_cast<const uint4*>(p.t2 + static_cast<long>(min(m0 + r, p.M - 1)) * MID + 8 * cq);
    }
#pragma unroll
    for (int e = 0; e < N; ++e) {
      const int g = tid + 512 * e;
      const int r = g / (MID / 8), cq = g % (MID / 8);
      *reinterpret_cast<uint4*>(t2s + (cq >> 2) * KBS + r * 64 + (((cq & 3) ^ pswz(r)) << 4)) = v[e];
    }
  }

  // per-lane fragment pointers (elements): fragment (rb, ks) of a packed matrix with NK K steps is at
  // ((rb * NK + ks) * 64 + lane) * 8
  const uint16_t* const w3l = p.w3p + lane * 8;
  const uint16_t* const w1l = p.w1p + lane * 8;
  auto w3frag = [&](int pass, int ks) -> bf16x8_t {
    return *reinterpret_cast<const bf16x8_t*>(w3l + (static_cast<long>((pass * PR_WAVES + w) * NKB + ks) << 9));
  };
  auto w1frag = [&](int pass, int kc, int j) -> bf16x8_t {
    return *reinterpret_cast<const bf16x8_t*>(w1l + (static_cast<long>((w * JC + j) * (C4 / 32) + pass * NKC + kc) << 9));
  };
  // residual of pass `pass` in the accumulator layout: pixel 16i + frow, channels 128 pass + 16 w + 4 lg .. +3
  // (YW: in the swapped layout of fragment pair ip: pixel 32 ip + frow + 16 (lg & 1), channels 16 w + 8 (lg >> 1) ..
  // +7, i.e. entries 0 .. FI/2 - 1)
  static_assert(!YW || FI % 2 == 0, "YW: pairs of pixel fragments");
  constexpr int FR = YW ? FI / 2 : FI;  // residual loads per pass
  const uint16_t* resl[FI];
#pragma unroll
  for (int i = 0; i < FI; ++i)
    resl[i] = YW ? p.res + static_cast<long>(min(m0 + 32 * (i % FR) + frow + 16 * (lg & 1), p.M - 1)) * C4 + 16 * w +
                       8 * (lg >> 1)
                 : p.res + static_cast<long>(min(m0 + 16 * i + frow, p.M - 1)) * C4 + 16 * w + 4 * lg;

  // T1' accumulators seeded with b1'
  f32x4_t accn[FI][JC];
#pragma unroll
  for (int j = 0; j < JC; ++j) {
    const f32x4_t b = pbias4(p.b1n + (w * JC + j) * 16, lg);
#pragma unroll
    for (int i = 0; i < FI; ++i) accn[i][j] = b;
  }

  // pass-0 operands
  f32x4_t b3v = *reinterpret_cast<const f32x4_t*>(p.b3 + 16 * w + 4 * lg);
  bf16x8_t wb[NKB];
#pragma unroll
  for (int k = 0; k < NKB; ++k) wb[k] = w3frag(0, k);
  uint2 rr[FI];
  uint4 rr4[FR];
  if constexpr (YW) {
#pragma unroll
    for (int i = 0; i < FR; ++i) rr4[i] = *reinterpret_cast<const uint4*>(resl[i]);
  } else {
#pragma unroll
    for (int i = 0; i < FI; ++i) rr[i] = *reinterpret_cast<const uint2*>(resl[i]);
  }

  pbarrier();  // T2 tile visible
  PAIR_STAMP(0);

  constexpr int NS = BM * PR_CH / 8 / 512;  // Y copy-out: thread g -> (row g / 16, 16-B chunk g % 16)

#pragma unroll 1
  for (int pass = 0; pass < NP; ++pass) {
    uint8_t* const ybuf = smem + T2_BYTES + (pass & 1) * Y_BYTES;
    // C fragments of this pass (consumed after the B phase)
    bf16x8_t wc[NKC][JC];
#pragma unroll
    for (int k = 0; k < NKC; ++k)
#pragma unroll
      for (int j = 0; j < JC; ++j) wc[k][j] = w1frag(pass, k, j);
    __builtin_amdgcn_sched_barrier(0);  // keep these loads here, a whole B phase ahead of their use
    // ---- B: accb = b3 + T2 . W3[rows 128 pass + 16 w ..]^T; the pixel fragments of step k+1 are read from
    // LDS before the MFMAs of step k (the scheduler otherwise pairs each read with its MFMA)
    f32x4_t accb[FI];
#pragma unroll
    for (int i = 0; i < FI; ++i) accb[i] = b3v;
    bf16x8_t fx[2][FI];
#pragma unroll
    for (int i = 0; i < FI; ++i) fx[0][i] = *reinterpret_cast<const bf16x8_t*>(t2s + fofs + i * 1024);
#pragma unroll
    for (int k = 0; k < NKB; ++k) {
      if (k + 1 < NKB) {
        const uint8_t* x_ = t2s + (k + 1) * KBS + fofs;
#pragma unroll
        for (int i = 0; i < FI; ++i) fx[(k + 1) & 1][i] = *reinterpret_cast<const bf16x8_t*>(x_ + i * 1024);
      }
      if constexpr (KF) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < FI; ++i) accb[i] = mfma_16x16x32<F16>(wb[k], fx[k & 1][i], accb[i]);
      if constexpr (KF) __builtin_amdgcn_sched_barrier(0);
    }

    PAIR_STAMP(1);
    // ---- epilogue: + residual (registers), ReLU, bf16 -> Y chunk (LDS)
    if constexpr (YW) {
#pragma unroll
      for (int ip = 0; ip < FR; ++ip) {
        f32x4_t a = accb[2 * ip], b = accb[2 * ip + 1];
        pswap16(a, b);
        const int r = 32 * ip + frow + 16 * (lg & 1), n = 16 * w + 8 * (lg >> 1);
        const float f[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
        *reinterpret_cast<uint4*>(ybuf + (n >> 5) * KBS + r * 64 + ((((n & 31) >> 3) ^ pswz(r)) << 4)) =
            epilogue8<F16>(f, true, rr4[ip], true);
      }
    } else {
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        const uint2 rv = rr[i];
        *reinterpret_cast<uint2*>(ybuf + poff<BM>(16 * i + frow, 16 * w + 4 * lg)) =
            make_uint2(pack_relu2<F16>(add_lo<F16>(rv.x, accb[i][0]), add_hi<F16>(rv.x, accb[i][1])),
                       pack_relu2<F16>(add_lo<F16>(rv.y, accb[i][2]), add_hi<F16>(rv.y, accb[i][3])));
      }
    }
    pbarrier();  // Y chunk visible (and every wave is past the chunk buffer's previous readers)
    PAIR_STAMP(2);

    // next pass's bias and B fragments (waited for at the next B phase) and residual (waited for at the next
    // epilogue), issued in that order and ahead of this pass's Y stores: every wait is then a count of younger
    // operations that never has to drain the stores or, for the B phase, the residual loads
    const int pn = pass + 1 < NP ? pass + 1 : pass;
    b3v = *reinterpret_cast<const f32x4_t*>(p.b3 + pn * PR_CH + 16 * w + 4 * lg);
#pragma unroll
    for (int k = 0; k < NKB; ++k) wb[k] = w3frag(pn, k);
    auto copy_out = [&](int e) __attribute__((always_inline)) {  // ---- Y chunk -> HBM (16-B row stores)
      const int g = tid + 512 * e;
      const int r = g >> 4, cq = g & 15;
      const uint4 v = *reinterpret_cast<const uint4*>(ybuf + (cq >> 2) * KBS + r * 64 + (((cq & 3) ^ pswz(r)) << 4));
      if (m0 + r < p.M) ai4e_conv::st16_stream(p.y + static_cast<long>(m0 + r) * C4 + pass * PR_CH + 8 * cq, v);
    };
    if constexpr (!SP) {
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        if constexpr (YW) {
          if (i < FR) rr4[i] = *reinterpret_cast<const uint4*>(resl[i] + pn * PR_CH);
        } else {
          rr[i] = *reinterpret_cast<const uint2*>(resl[i] + pn * PR_CH);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int e = 0; e < NS; ++e) copy_out(e);
      __builtin_amdgcn_sched_barrier(0);
    }

    PAIR_STAMP(3);
    // ---- C: accn += Y chunk . W1'[:, chunk]^T (pixel fragments one K step ahead, as in B)
    bf16x8_t fy[2][FI];
#pragma unroll
    for (int i = 0; i < FI; ++i) fy[0][i] = *reinterpret_cast<const bf16x8_t*>(ybuf + fofs + i * 1024);
#pragma unroll
    for (int k = 0; k < NKC; ++k) {
      if (k + 1 < NKC) {
        const uint8_t* x_ = ybuf + (k + 1) * KBS + fofs;
#pragma unroll
        for (int i = 0; i < FI; ++i) fy[(k + 1) & 1][i] = *reinterpret_cast<const bf16x8_t*>(x_ + i * 1024);
      }
      if constexpr (KF) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < JC; ++j)
          accn[i][j] = mfma_16x16x32<F16>(wc[k][j], fy[k & 1][i], accn[i][j]);
      if constexpr (SP) {
        constexpr int RPS = (FR + NKC - 1) / NKC;  // residual loads per C step
        if (k < NS) copy_out(k);
#pragma unroll
        for (int i = k * RPS; i < (k + 1) * RPS && i < FR; ++i) {
          if constexpr (YW) rr4[i] = *reinterpret_cast<const uint4*>(resl[i] + pn * PR_CH);
          else rr[i] = *reinterpret_cast<const uint2*>(resl[i] + pn * PR_CH);
        }
        static_assert(NS <= NKC, "one Y store chunk per C step");
      }
      if constexpr (KF) __builtin_amdgcn_sched_barrier(0);
    }
    PAIR_STAMP(4);
  }

  // ---- T1' epilogue through the T2 region (every wave finished its last B phase before the last barrier);
  // a T1' wider than T2 (layer3 -> layer4's 512-wide c1) also spans the Y buffers: wait for every wave's C phase
  if constexpr (MIDN / 32 * KBS > T2_BYTES) pbarrier();
  if constexpr (YW && JC == 2) {
    // the wave's two 16-channel blocks form one 32-channel K block: swapped, each lane holds 8 consecutive channels
    // (16-B chunk ((lg & 1) << 1) | (lg >> 1) of the block) of one pixel and writes them with one 16-B store
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      f32x4_t a = accn[i][0], b = accn[i][1];
      pswap16(a, b);
      const int r = 16 * i + frow, q = ((lg & 1) << 1) | (lg >> 1);
      *reinterpret_cast<uint4*>(t2s + w * KBS + r * 64 + ((q ^ pswz(r)) << 4)) =
          make_uint4(pack_relu2<F16>(a[0], a[1]), pack_relu2<F16>(a[2], a[3]), pack_relu2<F16>(b[0], b[1]),
                     pack_relu2<F16>(b[2], b[3]));
    }
  } else {
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < JC; ++j)
        *reinterpret_cast<uint2*>(t2s + poff<BM>(16 * i + frow, (w * JC + j) * 16 + 4 * lg)) =
            make_uint2(pack_relu2<F16>(accn[i][j][0], accn[i][j][1]), pack_relu2<F16>(accn[i][j][2], accn[i][j][3]));
  }
  pbarrier();
  constexpr int NT = BM * MIDN / 8 / 512;
#pragma unroll
  for (int e = 0; e < NT; ++e) {
    const int g = tid + 512 * e;
    const int r = g / (MIDN / 8), cq = g % (MIDN / 8);
    const uint4 v = *reinterpret_cast<const uint4*>(t2s + (cq >> 2) * KBS + r * 64 + (((cq & 3) ^ pswz(r)) << 4));
    if (m0 + r < p.M) ai4e_conv::st16_stream(p.t1n + static_cast<long>(m0 + r) * MIDN + 8 * cq, v);
  }
#if AI4E_PAIR_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PAIR_STAMP(5);
  if (lane == 0 && blockIdx.x * PR_WAVES + w < PAIR_MAXW) {
#pragma unroll
    for (int k = 0; k < PAIR_NSEG; ++k) g_pair_stamps[(blockIdx.x * PR_WAVES + w) * PAIR_NSEG + k] = ps_sum[k];
  }
#endif
}

template <int MID, int C4, int MIDN, int BM, bool KF = true, bool SP = false, bool F16 = false, bool YW = false>
int launch_pair(const PairParams& p, hipStream_t s) {
  constexpr int LDS = (MID / 32 + 2 * PR_CH / 32 > MIDN / 32 ? MID / 32 + 2 * PR_CH / 32 : MIDN / 32) * kbs<BM>();
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(conv_pair_kernel<MID, C4, MIDN, BM, KF, SP, F16, YW>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, LDS) != hipSuccess)
      return AI4E_ELAUNCH;
    attr = true;
  }
  hipLaunchKernelGGL((conv_pair_kernel<MID, C4, MIDN, BM, KF, SP, F16, YW>), dim3(ai4e_cdiv(p.M, BM)), dim3(512), LDS, s, p);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

}  // namespace

// Fused 1x1 pair (see header). t2 [M, mid], res / y [M, c4], t1n [M, midn] bf16 row-major (contiguous);
// w3p / w1p packed by ops/conv.py pack_pair_weights; b3 [c4], b1n [midn] fp32.
// (mid, c4, midn) = (256, 1024, 256) (layer3), (128, 512, 256) (layer2 -> layer3), (256, 1024, 512) (layer3 -> layer4)
// or (512, 2048, 512) (layer4). bm_cfg: 0 = default tile,
// else the tile height in pixels (64 or 96 for layer3, 32 for layer4; taller tiles spill at 256 VGPRs).
#if AI4E_PAIR_STAMPS
// Diagnostic build only: per-wave segment cycle sums of the last K1p launch (32768 waves x 6).
AI4E_API int ai4e_pair_stamps_read(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pair_stamps), sizeof(g_pair_stamps)) == hipSuccess ? AI4E_OK
                                                                                                  : AI4E_ELAUNCH;
}
#endif

namespace {
PairParams pair_params(const void* t2, const void* w3p, const void* b3, const void* res, void* y, const void* w1p,
                       const void* b1n, void* t1n, int M) {
  PairParams p{};
  p.t2 = static_cast<const uint16_t*>(t2);
  p.w3p = static_cast<const uint16_t*>(w3p);
  p.b3 = static_cast<const float*>(b3);
  p.res = static_cast<const uint16_t*>(res);
  p.y = static_cast<uint16_t*>(y);
  p.w1p = static_cast<const uint16_t*>(w1p);
  p.b1n = static_cast<const float*>(b1n);
  p.t1n = static_cast<uint16_t*>(t1n);
  p.M = M;
  return p;
}
}  // namespace

// fp16 form (the ensemble's crop classifier: f16 MFMA, fp32 accumulation): the default layer3 pair only.
AI4E_API int ai4e_conv_pair_f16_fwd(const void* t2, const void* w3p, const void* b3, const void* res, void* y,
                                    const void* w1p, const void* b1n, void* t1n, int M, int mid, int c4, int midn,
                                    int bm_cfg, hipStream_t stream) {
  if (!t2 || !w3p || !b3 || !res || !y || !w1p || !b1n || !t1n || M < 0) return AI4E_EINVAL;
  if (mid != 256 || c4 != 1024 || midn != 256 || (bm_cfg != 0 && bm_cfg != 98)) return AI4E_EINVAL;
  if (M == 0) return AI4E_OK;
  // 16-B Y writes (YW) as the bf16 default: epilogue8<true> runs the same fp16 dot2 residual adds, cvt and sign-bit
  // ReLU as the 8-B form, so the bits are the same
  return launch_pair<256, 1024, 256, 96, true, true, true, true>(pair_params(t2, w3p, b3, res, y, w1p, b1n, t1n, M),
                                                                 stream);
}

AI4E_API int ai4e_conv_pair_fwd(const void* t2, const void* w3p, const void* b3, const void* res, void* y,
                                const void* w1p, const void* b1n, void* t1n, int M, int mid, int c4, int midn,
                                int bm_cfg, hipStream_t stream) {
  if (!t2 || !w3p || !b3 || !res || !y || !w1p || !b1n || !t1n || M < 0) return AI4E_EINVAL;
  PairParams p{};
  p.t2 = static_cast<const uint16_t*>(t2);
  p.w3p = static_cast<const uint16_t*>(w3p);
  p.b3 = static_cast<const float*>(b3);
  p.res = static_cast<const uint16_t*>(res);
  p.y = static_cast<uint16_t*>(y);
  p.w1p = static_cast<const uint16_t*>(w1p);
  p.b1n = static_cast<const float*>(b1n);
  p.t1n = static_cast<uint16_t*>(t1n);
  p.M = M;
  if (M == 0) return AI4E_OK;
  if (mid == 256 && c4 == 1024 && midn == 256) {
    switch (bm_cfg) {
      case 0:   // default: loads + stores spread over the C phase (profiles/r3_pair/), 16-B Y writes (round 6:
      case 99:  // -0.7 % of the serial forward, bit-identical, profiles/r6_pair_yw/)
        return launch_pair<256, 1024, 256, 96, true, true, false, true>(p, stream);
      case 98: return launch_pair<256, 1024, 256, 96, true, true>(p, stream);  // A/B reference: 8-B Y writes
      case 96: return launch_pair<256, 1024, 256, 96>(p, stream);  // A/B reference: the burst after the Y barrier
      case 64: return launch_pair<256, 1024, 256, 64>(p, stream);
      case 97: return launch_pair<256, 1024, 256, 96, false>(p, stream);  // A/B: scheduler-placed fragment reads
      default: return AI4E_EINVAL;
    }
  }
  if (mid == 128 && c4 == 512 && midn == 256) {  // last layer2 block -> layer3's first c1
    switch (bm_cfg) {
      case 96: return launch_pair<128, 512, 256, 96>(p, stream);
      case 0:
      case 98: return launch_pair<128, 512, 256, 96, true, true>(p, stream);  // spread loads/stores (A/B)
      case 64: return launch_pair<128, 512, 256, 64>(p, stream);
      default: return AI4E_EINVAL;
    }
  }
  if (mid == 256 && c4 == 1024 && midn == 512) {  // last layer3 block -> layer4's first c1 (BM 64: 241 VGPRs at 96)
    switch (bm_cfg) {
      case 64: return launch_pair<256, 1024, 512, 64>(p, stream);
      case 0:
      case 98: return launch_pair<256, 1024, 512, 64, true, true>(p, stream);  // spread loads/stores (A/B)
      default: return AI4E_EINVAL;
    }
  }
  if (mid == 512 && c4 == 2048 && midn == 512) {
    switch (bm_cfg) {
      case 0:
      case 32: return launch_pair<512, 2048, 512, 32>(p, stream);
      case 98: return launch_pair<512, 2048, 512, 32, true, true>(p, stream);  // spread loads/stores (A/B)
      default: return AI4E_EINVAL;
    }
  }
  return AI4E_EINVAL;
}
