// K1 — NHWC bf16 conv2d as an implicit GEMM on CDNA4 MFMA, with a fused epilogue.
//
//   Y[m, n] = act( sum_k X~[m, k] * W[n, k] + bias[n] (+ R[m, n]) )
//   m = (img, oh, ow) output pixel   (M = N*OH*OW)
//   n = output channel               (Kout)
//   k = (kh, kw, c) filter tap x input channel, c innermost (K = KH*KW*C, padded to Kpad)
//
// BatchNorm is folded into W/bias on the host, so conv + BN + ReLU (+ residual add) of a ResNet
// bottleneck is ONE kernel and the activations make one HBM round trip per layer.
//
// Design (MI355X-first, see docs/KERNELS.md):
// * 256-thread workgroups (4 wave64s), every wave owns a 64(pixels) x 64(channels) output tile =
//   4 x 4 fragments of v_mfma_f32_16x16x32_bf16; workgroup tile = WAVES_M*64 x WAVES_N*64
//   (128x128 for wide layers, 256x64 for Cout=64 layers).
// * Operands are swapped (A = weights, B = activations) so each lane's accumulator holds 4
//   consecutive output CHANNELS of one pixel. Epilogue (EPI_LDS, the default when the output and
//   residual row strides are multiples of 8 channels): acc + bias is staged through the now idle
//   LDS ring as an fp32 tile, then every thread reads back whole 16-B row chunks, adds the 16-B
//   residual chunk, applies ReLU and writes 16 B — fully coalesced rows instead of 8-B fragments.
//   The fallback (odd strides, Cout < 8) stores 8 B per lane straight from the accumulators.
// * A/B tiles (BK = 32) stream global -> LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR staging)
//   into a 4-deep ring: 3 K-steps stay in flight across the one raw s_barrier per step, retired by a
//   counted vmcnt (cdna guide §5 "Pipelining across barriers", T3/T4) — one K-step of MFMA work is
//   far shorter than an HBM round trip, so depth, not a 2-buffer swap, is what hides latency.
//   Each 64-B LDS row (32 bf16) is XOR-swizzled per 16-B chunk with s = {0,2,3,1}[(row>>2)&3],
//   which makes every ds_read_b128 fragment read conflict-free for the gfx950 lane groups
//   {0-3,12-15,20-27},{4-11,16-19,28-31},... (MI355X_MICROARCH.md §LDS). Since an LDS-DMA writes
//   base + 16*lane, the swizzle is applied to the per-lane SOURCE address (rule 21).
// * The activation gather handles padding/stride/any KHxKW with one 16-B DMA per (pixel, tap,
//   8-channel chunk); padding taps read a zero chunk. C must be a multiple of 8 (the stem is fed C=8
//   by the preprocess kernel). The residual tile is prefetched into registers before the K loop.
// * XCD-aware tile order: tiles that share an activation panel (same m-tile, different n-tiles)
//   land on one XCD's L2 (common.h xcd_remap).
#include <type_traits>

#include "conv_common.h"

namespace {

constexpr int BK = ai4e_conv::BK;
using ai4e_conv::glds16;
using ai4e_conv::swz;
using ai4e_conv::TapWalk;
using ai4e_conv::wait_vmcnt;
using ai4e_conv::wait_vmcnt_n;

// Source of the zero 16-B chunks the DMA gather reads for padding / out-of-range taps.
__device__ __attribute__((aligned(64))) uint16_t g_zero_chunk[32];

// Diagnostic build (AI4E_K256_STAMPS=1): s_memtime stamps in the 256-wide kernel's 4-phase loop, per wave, summed per
// segment: 0 = LDS fragment reads + DMA issue, 1 = counted vmcnt wait, 2 = the two barriers of a phase (+ the
// lgkmcnt drain), 3 = MFMAs, 4 = prologue, 5 = epilogue. Written to g_k256_stamps (read SHARES: a stamp drains the
// wave's LDS reads, moving their latency into segment 0).
#ifndef AI4E_K256_STAMPS
#define AI4E_K256_STAMPS 0
#endif
constexpr int K256_NSEG = 6, K256_MAXW = 32768;
#if AI4E_K256_STAMPS
__device__ unsigned long long g_k256_stamps[K256_MAXW * K256_NSEG];
#define K256_STAMP(k)                                                              \
  do {                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                             \
    unsigned long long _t;                                                         \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");     \
    __builtin_amdgcn_sched_barrier(0);                                             \
    k_sum[k] += _t - k_last;                                                       \
    k_last = _t;                                                                   \
  } while (0)
#else
#define K256_STAMP(k) \
  do {                \
  } while (0)
#endif

struct ConvParams {
  const uint16_t* x;
  const uint16_t* w;
  const float* bias;
  const uint16_t* res;
  uint16_t* y;
  int N, H, W, C, ldx, xcoff;
  int KH, KW, stride, pad;
  int OH, OW;
  int Kout, Kpad;
  int ldy, ycoff, ldres;
  int relu;
  int M;
  int ntiles_n;
  const uint16_t* zero;  // >= 16 zero bytes: source of the DMA gather for padding taps
  // GroupNorm statistics of the stored (bf16) output, fused into the EPI_LDS epilogue (null = off): per
  // (image, BM-pixel chunk, group) shifted sum, sum of squares and the shift (norm_resample.hip) ->
  // gnp[((img * (OH*OW/BM) + chunk) * gn_groups + g) * 4 + {0, 1, 2}]
  float* gnp;
  int gn_groups;
  // a 1x1 conv to 16 channels fused after this one (256-wide configs, Kout == 256; null = off): hy [M, 16] =
  // (the stored bf16 output) . hw^T + hb, hw [16 rows, ld hw_ld >= 256]; y may then be null (output not stored)
  const uint16_t* hw;
  const float* hb;
  uint16_t* hy;
  int hw_ld;
  // split-K (256-wide configs only; ksplit 1 = off, 2 = on): the K tiles of an output tile are split over two
  // workgroups; the first to finish parks its fp32 accumulators in skw, the other adds them and runs the epilogue.
  // sks [2 x tiles] int32 (zero at launch, zero again when the launch ends): arrivals, then parked partials
  int ksplit;
  float* skw;
  int* sks;
  int skdiag;  // 1 = split-K without the parked traffic (timing only; wrong sums)
};

// Row of the residual tensor for output pixel m: m itself, or (relu flag bit 1) the pixel (oh/2, ow/2) of a
// half-resolution residual [N, OH/2, OW/2, ldres]: the FPN top-down nearest-neighbour 2x upsample fused into
// the lateral conv's residual read (no upsampled tensor is materialized).
__device__ __forceinline__ long res_row(const ConvParams& p, int m) {
  if (!(p.relu & 2)) return m;
  const int ohw = p.OH * p.OW;
  const int img = m / ohw, rem = m - img * ohw;
  const int oh = rem / p.OW, ow = rem - oh * p.OW;
  return (static_cast<long>(img) * (p.OH >> 1) + (oh >> 1)) * (p.OW >> 1) + (ow >> 1);
}

// Gather modes of the activation operand.
enum { GATHER_GENERAL = 0,  // any C % 8: a 32-wide K chunk may span taps -> per-lane tap walk
       GATHER_POINTWISE = 1,  // 1x1, pad 0 (any stride): K is the channel axis of one input pixel
       GATHER_TAP = 2 };      // C % 32 == 0: a K chunk lies in ONE tap -> the tap walk is wave-uniform (SGPRs)

// OCC = workgroups per CU the config is built for (waves per SIMD): 2 for the 4-stage ring (64 KB of
// LDS), 3 for the 3-stage ring (48 KB) — the register budget (<= 512/OCC VGPRs) must let that many
// resident, which is what lets a 766-tile layer3 grid run as ONE balanced round on 256 CUs.
// Epilogue LDS handoffs between the waves (the staged fp32 tile, the GroupNorm reduction): wait for this wave's LDS
// operations, then the barrier. Not __syncthreads(): its workgroup release fence makes the compiler drain vmcnt (on
// gfx9 it counts loads and stores together) at every handoff, so each pass waited for the previous pass's output
// stores and its residual loads, and the last pass for all its stores before the workgroup could retire. The ring's
// LDS-DMA loads are drained explicitly (wait_vmcnt<0>) before the epilogue. AI4E_EPI_FENCE=1 builds the old form
// (A/B library variant).
#ifndef AI4E_EPI_FENCE
#define AI4E_EPI_FENCE 0
#endif
#if AI4E_EPI_FENCE
#define EPI_BARRIER() __syncthreads()
#else
#define EPI_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")
#endif

template <int WAVES_M, int WAVES_N, int STAGES, int GATHER, bool EPI_LDS, int OCC = 2, bool F16 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC > 2 ? OCC : 1, OCC))) void conv_igemm_kernel(const ConvParams p) {
  static_assert(WAVES_M * WAVES_N == 4, "4 waves per workgroup");
  static_assert(STAGES >= 3, "fragment prefetch needs >= 3 ring stages");
  constexpr int BM = WAVES_M * 64;  // pixels per workgroup
  constexpr int BN = WAVES_N * 64;  // channels per workgroup
  constexpr int CA = BM / 64;       // A (activation) DMA instructions per wave per stage
  constexpr int CB = BN / 64;       // B (weight) DMA instructions per wave per stage
  constexpr int PER_STAGE = CA + CB;
  constexpr int STAGE_ELEMS = (BM + BN) * BK;
  __shared__ __attribute__((aligned(1024))) uint16_t smem[STAGES * STAGE_ELEMS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WAVES_M;
  const int wn = wave / WAVES_M;

  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = t / p.ntiles_n;
  const int nt = t - mt * p.ntiles_n;
  const int m0 = mt * BM;
  const int n0 = nt * BN;

  // ---- residual prefetch (issued first: the first stage wait also retires it)
  const int pm = m0 + wm * 64 + (lane & 15);
  const int pn = n0 + wn * 64 + 4 * (lane >> 4);
  // EPI_LDS layout: thread handles 16-B output chunks g = tid + 256*e of the row-major tile
  constexpr int CPR = BN / 8;                 // 16-B chunks per tile row
  constexpr int EPI_CHUNKS = BM * CPR / 256;  // chunks per thread
  uint2 rres[4][4];
  uint4 rres16[EPI_CHUNKS];
  // occupancy-3 configs cannot hold the residual tile in registers across the K loop (168-VGPR budget):
  // they load it per epilogue pass instead, with the other resident workgroups covering the latency
  constexpr bool EARLY_RES = OCC <= 2;
  if (p.res) {  // unconditional loads (clamped rows/cols) so hipcc keeps one counted wait for all
    if constexpr (EPI_LDS) {
      if constexpr (EARLY_RES) {
#pragma unroll
        for (int e = 0; e < EPI_CHUNKS; ++e) {
          const int g = tid + 256 * e;
          const int m = min(m0 + g / CPR, p.M - 1), n = min(n0 + 8 * (g % CPR), p.Kout - 8);
          rres16[e] = *reinterpret_cast<const uint4*>(p.res + res_row(p, m) * p.ldres + n);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = min(pm + 16 * i, p.M - 1), n = min(pn + 16 * j, p.Kout - 4);
          rres[i][j] = *reinterpret_cast<const uint2*>(p.res + res_row(p, m) * p.ldres + n);
        }
    }
  }

  // ---- DMA lane mapping: lane writes LDS slot 16*lane of a 16-row x 64-B block, i.e. row lane>>2,
  //      physical chunk lane&3, which holds logical k-chunk c = (lane&3) ^ swz(row).
  const int rin = lane >> 2;
  const int c = (lane & 3) ^ swz(rin);
  const int OHW = p.OH * p.OW;
  int ih0[CA], iw0[CA];
  long xbase[CA];
  const uint16_t* rowp[CA];  // the pixel's (ih0, iw0) channel row (+ the lane's 8-channel chunk for
                             // GATHER_TAP), nullptr past M
#pragma unroll
  for (int i = 0; i < CA; ++i) {
    const int m = m0 + 16 * (wave + 4 * i) + rin;
    if (m < p.M) {
      const int img = m / OHW;
      const int rem = m - img * OHW;
      const int oh = rem / p.OW;
      const int ow = rem - oh * p.OW;
      ih0[i] = oh * p.stride - p.pad;
      iw0[i] = ow * p.stride - p.pad;
      xbase[i] = static_cast<long>(img) * p.H * p.W * p.ldx + p.xcoff;
      rowp[i] = p.x + xbase[i] + (static_cast<long>(ih0[i]) * p.W + iw0[i]) * p.ldx +
                (GATHER == GATHER_TAP ? 8 * c : 0);
    } else {
      ih0[i] = -(1 << 28);  // fails the bounds check -> zero chunk
      iw0[i] = 0;
      xbase[i] = 0;
      rowp[i] = nullptr;
    }
  }
  int cc, kh, kw;  // GATHER_GENERAL: per-lane tap walk
  {
    const int k = 8 * c;
    const int tap = k / p.C;
    cc = k - tap * p.C;
    kh = tap / p.KW;
    kw = tap - kh * p.KW;
  }
  TapWalk tw;  // GATHER_TAP: wave-uniform tap walk
  const int rowjump = (p.W - p.KW) * p.ldx;
  const uint16_t* const wsrc = p.w + static_cast<long>(n0 + 16 * wave + rin) * p.Kpad + 8 * c;
  const long wstep = 64L * p.Kpad;  // rows 16*(wave+4i)
  const uint32_t smem_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem));
  const uint16_t* const zero = p.zero;
  const int nk = p.Kpad / BK;

  auto issue_stage = [&](int kt) {
    const uint32_t sbase = smem_base + (kt % STAGES) * STAGE_ELEMS * 2;
    if constexpr (GATHER == GATHER_POINTWISE) {
      const int k = kt * BK + 8 * c;
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const void* src = (rowp[i] != nullptr && k < p.C) ? static_cast<const void*>(rowp[i] + k) : zero;
        glds16(src, sbase + (16 * (wave + 4 * i)) * BK * 2);
      }
    } else if constexpr (GATHER == GATHER_TAP) {
      // one tap per K chunk: offset and the padding test's tap part are scalar; per lane only the
      // two unsigned bounds compares and a pointer select remain
      const int toff = tw.off;
      const bool tap_ok = tw.kh < p.KH;
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const bool ok = tap_ok && static_cast<unsigned>(ih0[i] + tw.kh) < static_cast<unsigned>(p.H) &&
                        static_cast<unsigned>(iw0[i] + tw.kw) < static_cast<unsigned>(p.W);
        glds16(ok ? static_cast<const void*>(rowp[i] + toff) : zero, sbase + (16 * (wave + 4 * i)) * BK * 2);
      }
      tw.next(BK, p.C, p.KW, p.ldx, rowjump);
    } else {
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const int ih = ih0[i] + kh, iw = iw0[i] + kw;
        const void* src = zero;
        if (kh < p.KH && static_cast<unsigned>(ih) < static_cast<unsigned>(p.H) &&
            static_cast<unsigned>(iw) < static_cast<unsigned>(p.W))
          src = p.x + xbase[i] + (static_cast<long>(ih) * p.W + iw) * p.ldx + cc;
        glds16(src, sbase + (16 * (wave + 4 * i)) * BK * 2);
      }
      cc += BK;
      while (cc >= p.C) {
        cc -= p.C;
        if (++kw == p.KW) {
          kw = 0;
          ++kh;
        }
      }
    }
    // past the end of K (the stray stages of the unconditional loop) every source is the zero chunk
    const bool live = kt < nk;
#pragma unroll
    for (int i = 0; i < CB; ++i)
      glds16(live ? static_cast<const void*>(wsrc + i * wstep + kt * BK) : zero,
             sbase + (BM + 16 * (wave + 4 * i)) * BK * 2);
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15;
  const int fofs = frow * BK + (((lane >> 4) ^ swz(frow)) << 3);

  // Software pipeline, per K step kt (fragments of step kt already in registers):
  //   wait stage kt+1 + barrier -> ds_read fragments of kt+1 (async) -> 16 MFMAs on step kt
  //   (hide the LDS latency) -> DMA-issue stage kt+STAGES-1 into the slot of step kt-1, which every
  //   wave finished reading before this step's barrier.
  bf16x8_t fw0[4], fx0[4], fw1[4], fx1[4];
#define K1_READ(FW, FX, KT)                                                                     \
  {                                                                                             \
    const uint16_t* st_ = smem + ((KT) % STAGES) * STAGE_ELEMS;                                 \
    const uint16_t* x_ = st_ + (wm * 64) * BK + fofs;                                           \
    const uint16_t* w_ = st_ + (BM + wn * 64) * BK + fofs;                                      \
    _Pragma("unroll") for (int j = 0; j < 4; ++j) FW[j] = *reinterpret_cast<const bf16x8_t*>(w_ + j * 16 * BK); \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) FX[i] = *reinterpret_cast<const bf16x8_t*>(x_ + i * 16 * BK); \
  }
// Every step waits, reads the next stage and issues stage kt+STAGES-1 unconditionally: past the
// end of K the DMA re-reads the last weight columns / the zero chunk into a ring slot nobody reads
// again, which keeps the loop free of scalar tail checks (and of the AGPR<->VGPR accumulator
// shuffling hipcc emits around a second, checked loop). The stray DMAs drain before the epilogue.
#define K1_STEP(KT, FWC, FXC, FWN, FXN)                                                         \
  {                                                                                             \
    const int kt_ = (KT);                                                                       \
    wait_vmcnt<(STAGES - 3) * PER_STAGE>();                                                     \
    __builtin_amdgcn_s_barrier();                                                               \
    K1_READ(FWN, FXN, kt_ + 1)                                                                  \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                               \
      _Pragma("unroll") for (int j = 0; j < 4; ++j)                                             \
        acc[i][j] = mfma_16x16x32<F16>(FWC[j], FXC[i], acc[i][j]);                                \
    issue_stage(kt_ + STAGES - 1);                                                              \
  }

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) issue_stage(s);
  wait_vmcnt<(STAGES - 2) * PER_STAGE>();
  __builtin_amdgcn_s_barrier();
  K1_READ(fw0, fx0, 0)
  // unrolled by two so the fragment buffers alternate without register copies; the MFMAs sit
  // outside any branch (a conditional MFMA block makes hipcc shuttle the accumulators AGPR<->VGPR),
  // hence K is padded to whole pairs of steps
  // (nk is even: the host pads K to a multiple of 2*BK)
  for (int kt = 0; kt < nk; kt += 2) {
    K1_STEP(kt, fw0, fx0, fw1, fx1)
    K1_STEP(kt + 1, fw1, fx1, fw0, fx0)
  }
  wait_vmcnt<0>();  // the stray tail DMAs land before any LDS reuse
#undef K1_STEP
#undef K1_READ

  // ---- fused epilogue: lane holds channels n..n+3 of pixel m for each (i, j) fragment.
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float4 b = *reinterpret_cast<const float4*>(p.bias + min(pn + 16 * j, p.Kout - 4));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[i][j][0] += b.x; acc[i][j][1] += b.y; acc[i][j][2] += b.z; acc[i][j][3] += b.w;
    }
  }
  const float lo = (p.relu & 1) ? 0.f : -INFINITY;
  if constexpr (EPI_LDS) {
    // Stage the fp32 tile through LDS (the now idle stage ring: BM*BN*4 bytes) so every lane
    // reads/writes 16 contiguous bytes: a wave instruction then covers whole 256-B+ pixel rows,
    // halving store instructions and giving the residual read the same full-line shape.
    // Row-major [BM][BN] fp32 with the 16-B chunk index XOR-swizzled by (row & 7): the 8-lane
    // ds_write_b128 groups (8 rows, one column) hit 8 different bank quads.
    // A ring smaller than the fp32 tile (the 3-stage configs) stages it in two row halves: the waves
    // owning rows [0, BM/2) write first, every thread stores those rows, then the other half.
    constexpr int EPI_PASSES = (BM * BN * 4 <= STAGES * STAGE_ELEMS * 2) ? 1 : 2;
    static_assert(EPI_PASSES == 1 || (WAVES_M % 2 == 0 && BM * BN * 2 <= STAGES * STAGE_ELEMS * 2),
                  "epilogue tile (or half of it) must fit the stage ring");
    constexpr int PASS_ROWS = BM / EPI_PASSES;
    float* tile = reinterpret_cast<float*>(smem);
    float gs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, gq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float gk[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, kout = 0.f;  // GN shifts (norm_resample.hip)
    __builtin_amdgcn_s_barrier();  // all waves finished reading the last stage
#pragma unroll
    for (int pass = 0; pass < EPI_PASSES; ++pass) {
    if (pass) EPI_BARRIER();  // the first half is stored before the second overwrites it
    constexpr int PC = EPI_CHUNKS / EPI_PASSES;
    uint4 rlate[PC];
    if constexpr (!EARLY_RES) {
      if (p.res) {
#pragma unroll
        for (int k = 0; k < PC; ++k) {
          const int g = tid + 256 * (pass * PC + k);
          const int m = min(m0 + g / CPR, p.M - 1), n = min(n0 + 8 * (g % CPR), p.Kout - 8);
          rlate[k] = *reinterpret_cast<const uint4*>(p.res + res_row(p, m) * p.ldres + n);
        }
      }
    }
    if (wm * 64 / PASS_ROWS == pass) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + 16 * i + (lane & 15) - pass * PASS_ROWS;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = (wn * 64 + 16 * j + 4 * (lane >> 4)) >> 2;  // fp32 16-B chunk in the row
          *reinterpret_cast<f32x4_t*>(tile + r * BN + 4 * (q ^ (r & 7))) = acc[i][j];
        }
      }
    }
    EPI_BARRIER();
    if (p.gnp && pass == 0) {
      // GN shift per channel slot: the tile's first pixel (row 0, unswizzled) at the group's first channel
      const int cg = p.Kout / p.gn_groups;
      const int c8 = 8 * (tid % CPR);
      if ((cg & (cg - 1)) == 0) {  // power-of-two group width (every model here): mask, no division
#pragma unroll
        for (int k = 0; k < 8; ++k) gk[k] = fmaxf(tile[(c8 + k) & -cg], lo);
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) gk[k] = fmaxf(tile[(c8 + k) / cg * cg], lo);
      }
      if (tid < BN / cg) kout = fmaxf(tile[tid * cg], lo);
    }
#pragma unroll
    for (int e = pass * EPI_CHUNKS / EPI_PASSES; e < (pass + 1) * EPI_CHUNKS / EPI_PASSES; ++e) {
      const int g = tid + 256 * e;
      const int r = g / CPR, cq = g % CPR;
      const int m = m0 + r, n = n0 + 8 * cq;
      const int rl = r - pass * PASS_ROWS;  // row within the staged half
      const float4 v0 = *reinterpret_cast<const float4*>(tile + rl * BN + 4 * ((2 * cq) ^ (rl & 7)));
      const float4 v1 = *reinterpret_cast<const float4*>(tile + rl * BN + 4 * ((2 * cq + 1) ^ (rl & 7)));
      const float f[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      const uint4 o = epilogue8<F16>(f, p.res != nullptr, EARLY_RES ? rres16[e] : rlate[e - pass * PC],
                                     (p.relu & 1) != 0);
      if (p.gnp && m < p.M && n < p.Kout) {  // GN statistics of the values as stored (bf16)
        const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float a, b;
          unpack2<F16>(ow[q], a, b);
          a -= gk[2 * q];
          b -= gk[2 * q + 1];
          gs[2 * q] += a; gq[2 * q] += a * a;
          gs[2 * q + 1] += b; gq[2 * q + 1] += b * b;
        }
      }
      if (m < p.M && n < p.Kout) {
        uint16_t* dst = p.y + static_cast<long>(m) * p.ldy + p.ycoff + n;
        if (n + 8 <= p.Kout) {
          ai4e_conv::st16_stream(dst, o);
        } else {
          *reinterpret_cast<uint2*>(dst) = make_uint2(o.x, o.y);  // Kout % 8 == 4 tail
        }
      }
    }
    }  // pass
    if (p.gnp) {
      // (1) in-thread: fold this lane's 8 channels into their groups (cgm = min(channels per group, 8) adjacent
      // channels per slot); (2) lanes sharing the 8-channel column (lane % CPR) reduce by xor shuffles; (3) the
      // 4 waves and each group's slots meet in LDS (the staged tile is dead by then)
      const int cg = p.Kout / p.gn_groups;
      const int cgm = cg < 8 ? cg : 8;
      auto reduce = [&](auto cgc) __attribute__((always_inline)) {
        constexpr int CG = decltype(cgc)::value;
#pragma unroll
        for (int w = 1; w < CG; w <<= 1)
#pragma unroll
          for (int k = 0; k < 8; k += 2 * w) {
            gs[k] += gs[k + w];
            gq[k] += gq[k + w];
          }
#pragma unroll
        for (int off = CPR; off < 64; off <<= 1)
#pragma unroll
          for (int k = 0; k < 8; k += CG) {
            gs[k] += __shfl_xor(gs[k], off);
            gq[k] += __shfl_xor(gq[k], off);
          }
      };
      switch (cgm) {
        case 1: reduce(std::integral_constant<int, 1>{}); break;
        case 2: reduce(std::integral_constant<int, 2>{}); break;
        case 4: reduce(std::integral_constant<int, 4>{}); break;
        default: reduce(std::integral_constant<int, 8>{}); break;
      }
      EPI_BARRIER();
      float* red = tile;  // [4 waves][BN channel slots][2]; slot c holds channels c .. c + cgm - 1
      if (lane < CPR) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (k % cgm == 0) {
            red[(wave * BN + lane * 8 + k) * 2] = gs[k];
            red[(wave * BN + lane * 8 + k) * 2 + 1] = gq[k];
          }
        }
      }
      EPI_BARRIER();
      const int ng = min(BN, p.Kout - n0) / cg;  // host: BN % cg == 0, Kout % cg == 0
      if (tid < ng) {
        float S = 0.f, Q = 0.f;
        for (int w = 0; w < 4; ++w)
          for (int c = 0; c < cg; c += cgm) {
            S += red[(w * BN + tid * cg + c) * 2];
            Q += red[(w * BN + tid * cg + c) * 2 + 1];
          }
        const int ohw = p.OH * p.OW;  // host: ohw % BM == 0, so a tile never straddles images
        const int img = m0 / ohw, chunk = (m0 - img * ohw) / BM;
        float* o = p.gnp + ((static_cast<long>(img) * (ohw / BM) + chunk) * p.gn_groups + n0 / cg + tid) * 4;
        *reinterpret_cast<float4*>(o) = make_float4(S, Q, kout, 0.f);  // shifted sums, shift
      }
    }
  } else {
    if (p.res) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float a0, a1, a2, a3;
          unpack2<F16>(rres[i][j].x, a0, a1);
          unpack2<F16>(rres[i][j].y, a2, a3);
          acc[i][j][0] += a0; acc[i][j][1] += a1; acc[i][j][2] += a2; acc[i][j][3] += a3;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = pn + 16 * j;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = pm + 16 * i;
        if (m < p.M && n < p.Kout)
          *reinterpret_cast<uint2*>(p.y + static_cast<long>(m) * p.ldy + p.ycoff + n) =
              make_uint2(pack2<F16>(fmaxf(acc[i][j][0], lo), fmaxf(acc[i][j][1], lo)),
                         pack2<F16>(fmaxf(acc[i][j][2], lo), fmaxf(acc[i][j][3], lo)));
      }
    }
  }
}

// ============================================================================================
// K1 "256" variant: 256x256 workgroup tile, 8 waves (2 pixel groups x 4 channel groups, each wave
// 128 pixels x 64 channels), BK = 64, LDS-DMA staging of 16-KB "units", and a ping-pong phase
// schedule: the two wave groups are offset by one barrier, so on every SIMD one wave issues its
// LDS reads / DMA while the other runs its 16-MFMA phase (cdna guide §5 "The 256² 8-phase
// template": 8 waves, BK 64, counted vmcnt never 0 in the loop, raw s_barrier, setprio around the
// MFMAs). One workgroup per CU (128 KB LDS).
//
// Units (128 rows x 128 B each; LDS = 2 buffers x 4 units):
//   u0 XQ0: pixel rows {wr*128 + 0..63}     u3 XQ1: pixel rows {wr*128 + 64..127}   (wr = 0, 1)
//   u1 WQ0: channel rows {wc*64 + 0..31}    u2 WQ1: channel rows {wc*64 + 32..63}   (wc = 0..3)
// Per K tile (4 phases) a wave computes its 2x2 quadrants (mq = pixel half, nq = channel half):
//   phase 1 (0,0): ds_read XQ0 + WQ0 | phase 2 (0,1): ds_read WQ1 | phase 3 (1,1): ds_read XQ1 |
//   phase 4 (1,0): no reads (WQ0 fragments kept in registers since phase 1).
// So within a tile u0/u1 are last read in phase 1, u2 in phase 2, u3 in phase 3.
// Staging (one unit per phase g = 4t+p): phase g stages unit (g-3) mod 4 of tile (g-3) div 4 + 2
// into the buffer of tile t: u0 at p=3, u1 at p=4, u2 at p=1 and u3 at p=2 of the NEXT tile — every
// slot is overwritten >= 2 phases after its last read (WAR with the one-barrier stagger), and
// read >= 4 phases after it was staged. At phase g each wave waits until its DMAs of phases <= g-3
// have landed (vmcnt = loads of phases g-2..g, at most 6), before that phase's first barrier; the
// readers of phase g+1 pass that barrier first (RAW).
// ============================================================================================
constexpr int U_ROWS = 128, U_BYTES = U_ROWS * 128;

// BM = 192 (tile config 9) keeps the schedule with 96-pixel wave groups: u0 holds pixel rows
// {wr*96 + 0..63} (still 128 unit rows), u3 only {wr*96 + 64..95} (64 rows: one DMA per lane, two
// fragments, 8-MFMA phases 3 and 4). A 14x14 layer of 250 images (M = 49000) is then 256 tiles —
// one per CU — instead of 192 256-row tiles that leave a quarter of the chip idle.
//
// PH3 (BM 192 only, tile config 10): three 16-MFMA phases per K tile instead of 16/16/8/8 — quadrants (1,1) and
// (1,0) of the 64-row XQ1 half share one phase — so 6 barriers instead of 8 per K tile. Staging (phase g = 3t+p):
// p = 0 stages u2 of tile t+1, p = 1 u3 of tile t+1, p = 2 u0 and u1 of tile t+2. Last reads within tile t:
// u0/u1 at p = 0, u2 at p = 1, u3 at p = 2, so every slot is again overwritten >= 2 phases after its last read
// and read >= 4 phases after it was staged, and the per-phase wait is the same rule (own DMAs of phases <= g-3).
// Measured and removed (profiles/r3_ph3/, profiles/r3_k256/; the code is in the git history up to commit bc1ff0a):
// a static priority for the trailing wave group (config 11), the staging DMAs inside the MFMA segment (12 / 13),
// 32x32x16 MFMAs (14 / 15) and priority on the load segment instead of the MFMAs (16 / 17) — all slower.
template <int GATHER, int BM, bool F16 = false, bool PH3 = false, bool SK = false>
__global__ __launch_bounds__(512) void conv_igemm256_kernel(const ConvParams p) {
  static_assert(GATHER == GATHER_TAP || GATHER == GATHER_POINTWISE, "256 tile needs C % 64 == 0");
  static_assert(BM == 256 || BM == 192, "wave groups of 128 or 96 pixels");
  static_assert(!PH3 || BM == 192, "the 3-phase schedule is the 192-pixel tile's");
  constexpr int WROWS = BM / 2;    // pixels per wave group
  constexpr int X1 = WROWS - 64;   // u3 rows per wave group
  constexpr int L3 = X1 / 32;      // DMAs per lane for u3
  constexpr int MF1 = X1 / 16;     // u3 fragments per wave
  constexpr int MFR = 4 + MF1;     // accumulator rows
  __shared__ __attribute__((aligned(1024))) uint8_t smem[2 * 4 * U_BYTES];  // the ring, then the epilogue tile
  // fused head only (p.hy): its 16 x 256 weights, 8 KB of dynamic LDS past the ring (still one workgroup per CU),
  // row r's 16-B chunk c at chunk c ^ r (the head's 16 lanes of a K chunk read 16 different chunks)
  extern __shared__ __attribute__((aligned(16))) uint8_t hsm[];
#if AI4E_K256_STAMPS
  unsigned long long k_sum[K256_NSEG] = {0, 0, 0, 0, 0, 0}, k_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(k_last)::"memory");
#endif

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  // split-K (SK): the two workgroups of one output tile are consecutive logical tiles (one XCD's L2 holds the
  // parked partial), each running K tiles [kb, kb + nk) of the nk_all
  int t = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int ksp = SK ? 2 : 1;
  const int ks = t % ksp;
  t /= ksp;
  const int mt = t / p.ntiles_n;
  const int nt = t - mt * p.ntiles_n;
  const int m0 = mt * BM;
  const int n0 = nt * 256;
  const int nk_all = p.Kpad / 64;
  const int kb = ks * nk_all / ksp;
  const int nk = (ks + 1) * nk_all / ksp - kb;
  const uint32_t sbase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem));
  if (p.hy) {
    // the oldest DMA of the launch, so every counted ring wait below also covers it; thread tid fills slot tid
    const int hr = tid >> 5, hc = (tid & 31) ^ hr;
    glds16(p.hw + hr * p.hw_ld + 8 * hc, static_cast<uint32_t>(reinterpret_cast<uintptr_t>(hsm)) + wave * 1024);
  }

  // ---- DMA sources. Lane writes unit row R_i = 16*wave + 8*i + (lane>>3) (u3 of BM 192: 8*wave +
  //      (lane>>3)), physical 16-B chunk lane&7, holding logical chunk q_i = (lane&7) ^ ((R_i >> 1) & 7).
  const int OHW = p.OH * p.OW;
  const uint16_t* xrow[2][2];  // [i][xq] pixel row pointer (+ 8*q_i), nullptr past M
  int ih0[2][2], iw0[2][2];
  const uint16_t* wrow[2];     // [i] weight row pointer (+ 8*q_i) for WQ0; WQ1 = +32 rows
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int R = 16 * wave + 8 * i + (lane >> 3);
    const int q = (lane & 7) ^ ((R >> 1) & 7);
#pragma unroll
    for (int xq = 0; xq < 2; ++xq) {
      const int RG = xq ? X1 : 64;  // unit rows per wave group
      const int Rx = (xq && L3 == 1) ? 8 * wave + (lane >> 3) : R;
      const int qx = (lane & 7) ^ ((Rx >> 1) & 7);
      const int m = m0 + (Rx / RG) * WROWS + (xq ? 64 : 0) + (Rx % RG);
      if (m < p.M && !(xq && L3 == 1 && i == 1)) {
        const int img = m / OHW;
        const int rem = m - img * OHW;
        const int oh = rem / p.OW;
        const int ow = rem - oh * p.OW;
        ih0[i][xq] = oh * p.stride - p.pad;
        iw0[i][xq] = ow * p.stride - p.pad;
        xrow[i][xq] = p.x + static_cast<long>(img) * p.H * p.W * p.ldx + p.xcoff +
                      (static_cast<long>(ih0[i][xq]) * p.W + iw0[i][xq]) * p.ldx + 8 * qx;
      } else {
        ih0[i][xq] = -(1 << 28);
        iw0[i][xq] = 0;
        xrow[i][xq] = nullptr;
      }
    }
    wrow[i] = p.w + static_cast<long>(n0 + (R >> 5) * 64 + (R & 31)) * p.Kpad + kb * 64 + 8 * q;
  }
  const uint16_t* const zero = p.zero;
  // X units are staged tile by tile (XQ0 and XQ1 at different phases): one tap walk per unit kind, started at
  // K element kb * 64 (tap (kh, kw), channel cb: element offset (kh * W + kw) * ldx + cb)
  TapWalk wx[2];
  const int kx0 = kb * 64;  // pointwise: channel offset of this split's first K tile
  if (GATHER == GATHER_TAP && kb > 0) {
    const int tap = kx0 / p.C, cb = kx0 - tap * p.C;
    const int kh = tap / p.KW, kw = tap - kh * p.KW;
#pragma unroll
    for (int xq = 0; xq < 2; ++xq) {
      wx[xq].kh = kh;
      wx[xq].kw = kw;
      wx[xq].cb = cb;
      wx[xq].off = (kh * p.W + kw) * p.ldx + cb;
    }
  }
  const int rowjump = (p.W - p.KW) * p.ldx;

  // stage unit u of K tile kt into buffer kt&1 (2 DMAs per lane); X units must be staged in tile order

  // X unit xq (compile-time, so each tap walk stays in registers) of the K tile at k0
  auto stage_x = [&](auto XQ, uint32_t ubase, int k0) {
    constexpr int xq = decltype(XQ)::value;
    constexpr int nl = xq ? L3 : 2;
    const uint32_t xb = (xq && L3 == 1) ? ubase - (8 * wave) * 128 : ubase;
    if constexpr (GATHER == GATHER_POINTWISE) {
      const bool kok = kx0 + k0 < p.C;
#pragma unroll
      for (int i = 0; i < nl; ++i) {
        const void* src = (kok && xrow[i][xq] != nullptr) ? static_cast<const void*>(xrow[i][xq] + kx0 + k0) : zero;
        glds16(src, xb + i * 8 * 128);
      }
    } else {
      // a 64-wide K tile lies in one tap (C % 64 == 0): wave-uniform walk
      TapWalk& tw = wx[xq];
      const bool tok = tw.kh < p.KH;
#pragma unroll
      for (int i = 0; i < nl; ++i) {
        const bool ok = tok && static_cast<unsigned>(ih0[i][xq] + tw.kh) < static_cast<unsigned>(p.H) &&
                        static_cast<unsigned>(iw0[i][xq] + tw.kw) < static_cast<unsigned>(p.W);
        glds16(ok ? static_cast<const void*>(xrow[i][xq] + tw.off) : zero, xb + i * 8 * 128);
      }
      tw.next(64, p.C, p.KW, p.ldx, rowjump);
    }
  };
  auto stage = [&](int kt, int u) {
    const uint32_t ubase = sbase + ((kt & 1) * 4 + u) * U_BYTES + (16 * wave) * 128;
    const int k0 = kt * 64;
    if (u == 1 || u == 2) {
      const long roff = (u == 2 ? 32L * p.Kpad : 0L) + k0;
#pragma unroll
      for (int i = 0; i < 2; ++i) glds16(wrow[i] + roff, ubase + i * 8 * 128);
    } else if (u == 3) {
      stage_x(std::integral_constant<int, 1>{}, ubase, k0);
    } else {
      stage_x(std::integral_constant<int, 0>{}, ubase, k0);
    }
  };
  // phase g stages unit (g-3) mod 4 of tile (g-3) div 4 + 2 (g may be <= 0: the prologue)
  auto phase_tile = [&](int g) { return ((g + 5) >> 2); };  // floor((g-3)/4)+2 for g >= -5
  auto phase_unit = [&](int g) { return (g + 5) & 3; };
  auto stage_phase = [&](int g) {
    const int kt = phase_tile(g);
    if (kt < nk) stage(kt, phase_unit(g));
  };
  auto loads_of = [&](int g) { return phase_tile(g) < nk ? (phase_unit(g) == 3 ? L3 : 2) : 0; };
  // wait until this wave's DMAs of phases <= g-3 have landed
  auto wait_phase = [&](int g) { wait_vmcnt_n(loads_of(g - 2) + loads_of(g - 1) + loads_of(g)); };

  f32x4_t acc[MFR][4];
#pragma unroll
  for (int i = 0; i < MFR; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets: row (lane&15) of a 16-row block, logical chunk 4s + (lane>>4)
  const int frow = lane & 15;
  const int fsw = frow >> 1;
  const uint32_t fofs0 = frow * 128 + (((lane >> 4) ^ fsw) << 4);        // s = 0
  const uint32_t fofs1 = frow * 128 + (((4 + (lane >> 4)) ^ fsw) << 4);  // s = 1
  bf16x8_t xr[4][2], w0r[2][2], w1r[2][2];

#define K256_READ_X(XQ, KT)                                                                        \
  {                                                                                                \
    const uint8_t* b_ = smem + (((KT) & 1) * 4 + ((XQ) ? 3 : 0)) * U_BYTES + (wr * ((XQ) ? X1 : 64)) * 128; \
    _Pragma("unroll") for (int i = 0; i < ((XQ) ? MF1 : 4); ++i) {                                 \
      xr[i][0] = *reinterpret_cast<const bf16x8_t*>(b_ + i * 16 * 128 + fofs0);                    \
      xr[i][1] = *reinterpret_cast<const bf16x8_t*>(b_ + i * 16 * 128 + fofs1);                    \
    }                                                                                              \
  }
#define K256_READ_W(WR, NQ, KT)                                                                    \
  {                                                                                                \
    const uint8_t* b_ = smem + (((KT) & 1) * 4 + 1 + (NQ)) * U_BYTES + (wc * 32) * 128;            \
    _Pragma("unroll") for (int j = 0; j < 2; ++j) {                                                \
      WR[j][0] = *reinterpret_cast<const bf16x8_t*>(b_ + j * 16 * 128 + fofs0);                    \
      WR[j][1] = *reinterpret_cast<const bf16x8_t*>(b_ + j * 16 * 128 + fofs1);                    \
    }                                                                                              \
  }
#define K256_MFMA(MQ, NQ, WR)                                                                      \
  {                                                                                                \
    __builtin_amdgcn_s_setprio(1);                                                                 \
    _Pragma("unroll") for (int s = 0; s < 2; ++s)                                                  \
      _Pragma("unroll") for (int i = 0; i < ((MQ) ? MF1 : 4); ++i)                                 \
        _Pragma("unroll") for (int j = 0; j < 2; ++j)                                              \
          acc[4 * (MQ) + i][2 * (NQ) + j] =                                                        \
              mfma_16x16x32<F16>(WR[j][s], xr[i][s], acc[4 * (MQ) + i][2 * (NQ) + j]);             \
    __builtin_amdgcn_s_setprio(0);                                                                 \
  }
// CHECKED = 0: steady state (kt + 2 < nk): every phase stages a unit, 3 phases of DMAs in flight
// (NS = this wave's DMAs of those 3 phases: 6 at phase 1, 4 + L3 at phases 2-4, which stage u3 or follow it)
#define K256_SYNC_LOADS(G, CHECKED, NS)                                                            \
  if (CHECKED) {                                                                                   \
    stage_phase(G);                                                                                \
    K256_STAMP(0);                                                                                 \
    wait_phase(G);                                                                                 \
  } else {                                                                                         \
    stage(phase_tile(G), phase_unit(G));                                                           \
    K256_STAMP(0);                                                                                 \
    wait_vmcnt<NS>();                                                                              \
  }                                                                                                \
  K256_STAMP(1);                                                                                   \
  __builtin_amdgcn_s_barrier();                                                                    \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                               \
  K256_STAMP(2);
#define K256_TILE(KT, CHECKED)                                                                     \
  {                                                                                                \
    const int g = 4 * (KT);                                                                        \
    /* phase 1: quadrant (0,0) */                                                                  \
    K256_READ_W(w0r, 0, KT)                                                                        \
    K256_READ_X(0, KT)                                                                             \
    K256_SYNC_LOADS(g + 1, CHECKED, 6)                                                                \
    K256_MFMA(0, 0, w0r)                                                                           \
    K256_STAMP(3);                                                                                 \
    __builtin_amdgcn_s_barrier();                                                                  \
    K256_STAMP(2);                                                                                 \
    /* phase 2: quadrant (0,1) */                                                                  \
    K256_READ_W(w1r, 1, KT)                                                                        \
    K256_SYNC_LOADS(g + 2, CHECKED, 4 + L3)                                                                \
    K256_MFMA(0, 1, w1r)                                                                           \
    K256_STAMP(3);                                                                                 \
    __builtin_amdgcn_s_barrier();                                                                  \
    K256_STAMP(2);                                                                                 \
    /* phase 3: quadrant (1,1) */                                                                  \
    K256_READ_X(1, KT)                                                                             \
    K256_SYNC_LOADS(g + 3, CHECKED, 4 + L3)                                                                \
    K256_MFMA(1, 1, w1r)                                                                           \
    K256_STAMP(3);                                                                                 \
    __builtin_amdgcn_s_barrier();                                                                  \
    K256_STAMP(2);                                                                                 \
    /* phase 4: quadrant (1,0), fragments already in registers */                                  \
    K256_SYNC_LOADS(g + 4, CHECKED, 4 + L3)                                                                \
    K256_MFMA(1, 0, w0r)                                                                           \
    K256_STAMP(3);                                                                                 \
    __builtin_amdgcn_s_barrier();                                                                  \
    K256_STAMP(2);                                                                                 \
  }

  // 3-phase schedule (PH3): phase g = 3t + p, g >= -6 (the prologue is g = -4 .. -1)
  auto ph3_tile = [&](int g) { return (g + 6) / 3 - 2; };
  auto stage3 = [&](int g) {
    const int t = ph3_tile(g), q = g - 3 * t;
    if (q == 0) {
      if (t + 1 < nk) stage(t + 1, 2);
    } else if (q == 1) {
      if (t + 1 < nk) stage(t + 1, 3);
    } else if (t + 2 < nk) {
      stage(t + 2, 0);
      stage(t + 2, 1);
    }
  };
  auto loads3 = [&](int g) {
    const int t = ph3_tile(g), q = g - 3 * t;
    return q == 0 ? (t + 1 < nk ? 2 : 0) : q == 1 ? (t + 1 < nk ? L3 : 0) : (t + 2 < nk ? 4 : 0);
  };
#define K256_SYNC3(G, CHECKED, STAGE_UNCHECKED)                                                       \
  if (CHECKED) {                                                                                   \
    stage3(G);                                                                                     \
    wait_vmcnt_n(loads3((G) - 2) + loads3((G) - 1) + loads3(G));                                   \
  } else {                                                                                         \
    STAGE_UNCHECKED;                                                                               \
    wait_vmcnt<6 + L3>();                                                                          \
  }                                                                                                \
  __builtin_amdgcn_s_barrier();                                                                    \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#define K256_TILE3(KT, CHECKED)                                                                    \
  {                                                                                                \
    const int g = 3 * (KT);                                                                        \
    K256_READ_W(w0r, 0, KT)                                                                        \
    K256_READ_X(0, KT)                                                                             \
    K256_SYNC3(g, CHECKED, stage((KT) + 1, 2))                                                     \
    K256_MFMA(0, 0, w0r)                                                                           \
    __builtin_amdgcn_s_barrier();                                                                  \
    K256_READ_W(w1r, 1, KT)                                                                        \
    K256_SYNC3(g + 1, CHECKED, stage((KT) + 1, 3))                                                 \
    K256_MFMA(0, 1, w1r)                                                                           \
    __builtin_amdgcn_s_barrier();                                                                  \
    K256_READ_X(1, KT)                                                                             \
    K256_SYNC3(g + 2, CHECKED, (stage((KT) + 2, 0), stage((KT) + 2, 1)))                           \
    K256_MFMA(1, 1, w1r)                                                                           \
    K256_MFMA(1, 0, w0r)                                                                           \
    __builtin_amdgcn_s_barrier();                                                                  \
  }

  int kt = 0;
  if constexpr (PH3) {
    // ---- prologue: tile 0 (phases -4 .. -2) and tile 1's u0, u1 (phase -1); tile 0's u0/u1 must have landed
#pragma unroll
    for (int g = -4; g <= -1; ++g) stage3(g);
    wait_vmcnt_n(loads3(-3) + loads3(-2) + loads3(-1));
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();  // the stagger: group 1 trails by one barrier
    for (; kt + 2 < nk; ++kt) K256_TILE3(kt, 0)
    for (; kt < nk; ++kt) K256_TILE3(kt, 1)
  } else {
    // ---- prologue: tile 0 (virtual phases -5..-2) and tile 1's u0, u1 (phases -1, 0)
#pragma unroll
    for (int g = -5; g <= 0; ++g) stage_phase(g);
    if (loads_of(-1) + loads_of(0) == 4) wait_vmcnt<4>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();  // the stagger: group 1 trails by one barrier
    K256_STAMP(4);
    for (; kt + 2 < nk; ++kt) K256_TILE(kt, 0)
    for (; kt < nk; ++kt) K256_TILE(kt, 1)
  }
#undef K256_TILE3
#undef K256_SYNC3
#undef K256_TILE
#undef K256_SYNC_LOADS
#undef K256_MFMA
#undef K256_READ_W
#undef K256_READ_X
  if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the two groups
  wait_vmcnt<0>();
  __syncthreads();

  if constexpr (SK) {
    // split-K hand-off. Arrival order decides the roles, so nobody waits on a workgroup that has not started: the
    // first arrival parks its accumulators and counts itself ready; the second waits for that count (the first is
    // already past its arrival, only its stores are outstanding), adds the parked partial (fp32 addition commutes:
    // the same bits whichever split arrived last), resets both counters for the next launch and runs the epilogue.
    // The parked values move with agent-coherent (sc1) 16-B buffer stores and loads, ordered by vmcnt and the
    // barrier: a release / acquire fence would write back / invalidate the whole L2 of the XCD (buffer_wbl2 /
    // buffer_inv) and every workgroup on it would refetch its operands (measured 1.6-6x slower), and sc1 dword
    // atomics cost 2x the 16-B form (profiles/r6_splitk/). p.skdiag = 1 (timing only): no parked traffic.
    __shared__ int sk_arrival;
    const int ntl = gridDim.x / 2;
    constexpr int PSZ = MFR * 4 * 512;  // f32x4 per parked partial: [i][j][thread]
    if (tid == 0) sk_arrival = atomicAdd(p.sks + t, 1);
    __syncthreads();
    const bool traffic = p.skdiag != 1;
    const __amdgpu_buffer_rsrc_t park =
        __builtin_amdgcn_make_buffer_rsrc(p.skw + static_cast<long>(t) * 2 * PSZ * 4, 0, 2 * PSZ * 16, 0x00020000);
    constexpr int SC1 = 16;  // cache policy: agent coherent
    if (sk_arrival == 0) {
      if (traffic) {
#pragma unroll
        for (int i = 0; i < MFR; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ai4e_conv::u32x4_t, acc[i][j]), park,
                                                   (ks * PSZ + tid) * 16, (i * 4 + j) * 512 * 16, SC1);
      }
      wait_vmcnt<0>();  // this thread's partial has reached the coherence point
      __syncthreads();
      if (tid == 0) atomicAdd(p.sks + ntl + t, 1);
      return;
    }
    if (tid == 0) {
      while (__hip_atomic_load(p.sks + ntl + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 1)
        __builtin_amdgcn_s_sleep(2);
      __hip_atomic_store(p.sks + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p.sks + ntl + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (traffic) {
      // two accumulator rows (8 loads) in flight at a time (the offsets of a row in SGPRs: VGPR offsets spilled
      // the 256-pixel tile)
#ifndef AI4E_SK_RB
#define AI4E_SK_RB 2
#endif
      constexpr int RB = AI4E_SK_RB < MFR ? AI4E_SK_RB : MFR;
#pragma unroll
      for (int i = 0; i < MFR; i += RB) {
#pragma unroll
        for (int ii = i; ii < i + RB && ii < MFR; ++ii)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[ii][j] += __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                          park, ((1 - ks) * PSZ + tid) * 16, (ii * 4 + j) * 512 * 16, SC1));
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }

  // ---- epilogue, one pixel group at a time: fp32 [WROWS][256] tile in LDS (16-B chunk index
  //      XOR (row & 7)), then every thread handles 16-B output chunks: + bias (+ residual), ReLU.
  //      With p.gnp: the GroupNorm statistics of the stored values as well (the K1 epilogue's shifted partial sums,
  //      one [BM-pixel chunk, group] record each), so a GroupNorm after a 256-wide conv needs no statistics pass. A
  //      thread always owns the same 8 channels (c8 = tid % 32) of every row it stores.
  float* tile = reinterpret_cast<float*>(smem);
  float gs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, gq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float gk[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, kout = 0.f;  // GN shifts: the tile's first pixel, per group
  const float lo_gn = (p.relu & 1) ? 0.f : -INFINITY;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (wr == pass) {
#pragma unroll
      for (int i = 0; i < MFR; ++i) {
        const int r = 16 * i + (lane & 15);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c4 = (wc * 64 + 16 * j) / 4 + (lane >> 4);
          *reinterpret_cast<f32x4_t*>(tile + r * 256 + 4 * (c4 ^ (r & 7))) = acc[i][j];
        }
      }
    }
    EPI_BARRIER();
    if (p.gnp && pass == 0) {
      // shift per channel slot: row 0 (unswizzled) + bias at the group's first channel (host: power-of-two groups)
      const int cg = p.Kout / p.gn_groups;
      const int c8 = 8 * (tid & 31);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = (c8 + k) & -cg;
        gk[k] = fmaxf(tile[c] + p.bias[min(n0 + c, p.Kout - 1)], lo_gn);
      }
      if (tid < 256 / cg) kout = fmaxf(tile[tid * cg] + p.bias[min(n0 + tid * cg, p.Kout - 1)], lo_gn);
    }
    if (p.hy) {
      // the fused 16-channel 1x1 (the FPN RPN head after its 3x3 conv): each wave takes 16-pixel blocks of this pass;
      // the B operand is the epilogue's bf16 output (bias, ReLU, same rounding as the stored tensor) built from the
      // staged fp32 tile, the A operand the head weights (row = lane & 15) from the 8 KB of dynamic LDS they were
      // DMA'd into at kernel start
      const uint4 nores = make_uint4(0u, 0u, 0u, 0u);
      for (int blk = wave; blk < WROWS / 16; blk += 8) {
        const int r = 16 * blk + (lane & 15);
        f32x4_t hacc = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const int c8 = 4 * s + (lane >> 4);  // 8-channel chunk of K
          const float4 v0 = *reinterpret_cast<const float4*>(tile + r * 256 + 4 * ((2 * c8) ^ (r & 7)));
          const float4 v1 = *reinterpret_cast<const float4*>(tile + r * 256 + 4 * ((2 * c8 + 1) ^ (r & 7)));
          const float4 b0 = *reinterpret_cast<const float4*>(p.bias + 8 * c8);
          const float4 b1 = *reinterpret_cast<const float4*>(p.bias + 8 * c8 + 4);
          const float f[8] = {v0.x + b0.x, v0.y + b0.y, v0.z + b0.z, v0.w + b0.w,
                              v1.x + b1.x, v1.y + b1.y, v1.z + b1.z, v1.w + b1.w};
          const uint4 o = epilogue8<F16>(f, false, nores, (p.relu & 1) != 0);
          const int hr = lane & 15;
          const bf16x8_t wb = *reinterpret_cast<const bf16x8_t*>(hsm + hr * 512 + ((c8 ^ hr) << 4));
          hacc = mfma_16x16x32<F16>(wb, __builtin_bit_cast(bf16x8_t, o), hacc);
        }
        // lane: pixel r, head channels 4 * (lane >> 4) + 0..3
        const int m = m0 + WROWS * pass + r;
        if (m < p.M) {
          const int hc = 4 * (lane >> 4);
          const float4 hb = *reinterpret_cast<const float4*>(p.hb + hc);
          const uint2 ho = make_uint2(pack2<F16>(hacc[0] + hb.x, hacc[1] + hb.y), pack2<F16>(hacc[2] + hb.z, hacc[3] + hb.w));
          *reinterpret_cast<uint2*>(p.hy + static_cast<long>(m) * 16 + hc) = ho;
        }
      }
    }
    constexpr int EP = WROWS / 16;  // 16-B output chunks per thread and pass
    uint4 rv[EP];
    if (!p.y) {  // head only: the conv's own output is not stored
      EPI_BARRIER();
      continue;
    }
    if (p.res) {
#pragma unroll
      for (int e = 0; e < EP; ++e) {
        const int g = tid + 512 * e;
        const int m = min(m0 + WROWS * pass + (g >> 5), p.M - 1), n = min(n0 + 8 * (g & 31), p.Kout - 8);
        rv[e] = *reinterpret_cast<const uint4*>(p.res + res_row(p, m) * p.ldres + n);
      }
    }
#pragma unroll
    for (int e = 0; e < EP; ++e) {
      const int g = tid + 512 * e;
      const int r = g >> 5, c8 = g & 31;
      const int m = m0 + WROWS * pass + r, n = n0 + 8 * c8;
      // the lane's two fp32 chunks (2 c8, 2 c8 + 1), the odd one first in the upper half of the row (c8 >= 16): a
      // ds_read_b128 lane group ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}: 16 lanes of one row) then covers 16
      // distinct bank quads; reading both halves even-first put every group's 16 lanes on 8 quads (2-way conflicts
      // on every epilogue read: profiles/r5_pmc/ ldsconf 9-14 % on the 1x1 configs)
      const int hi = (c8 >> 4) & 1;
      const float4 va = *reinterpret_cast<const float4*>(tile + r * 256 + 4 * ((2 * c8 + hi) ^ (r & 7)));
      const float4 vb = *reinterpret_cast<const float4*>(tile + r * 256 + 4 * ((2 * c8 + 1 - hi) ^ (r & 7)));
      const float4 v0 = hi ? vb : va, v1 = hi ? va : vb;
      const int nb = min(n, p.Kout - 8);
      const float4 b0 = *reinterpret_cast<const float4*>(p.bias + nb);
      const float4 b1 = *reinterpret_cast<const float4*>(p.bias + nb + 4);
      const float f[8] = {v0.x + b0.x, v0.y + b0.y, v0.z + b0.z, v0.w + b0.w,
                          v1.x + b1.x, v1.y + b1.y, v1.z + b1.z, v1.w + b1.w};
      const uint4 o = epilogue8<F16>(f, p.res != nullptr, rv[e], (p.relu & 1) != 0);
      if (m < p.M && n < p.Kout && p.y) ai4e_conv::st16_stream(p.y + static_cast<long>(m) * p.ldy + p.ycoff + n, o);
      if (p.gnp && m < p.M && n < p.Kout) {  // statistics of the values as stored (bf16)
        const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float a, b;
          unpack2<F16>(ow[q], a, b);
          a -= gk[2 * q];
          b -= gk[2 * q + 1];
          gs[2 * q] += a; gq[2 * q] += a * a;
          gs[2 * q + 1] += b; gq[2 * q + 1] += b * b;
        }
      }
    }
    EPI_BARRIER();
  }
  if (p.gnp) {
    // (1) in-thread: this thread's 8 channels into their groups (cgm = min(channels per group, 8) adjacent channels
    // per slot); (2) the two lanes of a wave that own the same channels (lane, lane ^ 32) by one xor shuffle; (3) the
    // 8 waves and each group's slots meet in LDS (the staged tile is dead after the last pass's barrier)
    const int cg = p.Kout / p.gn_groups;
    const int cgm = cg < 8 ? cg : 8;
    auto reduce = [&](auto cgc) __attribute__((always_inline)) {
      constexpr int CG = decltype(cgc)::value;
#pragma unroll
      for (int w = 1; w < CG; w <<= 1)
#pragma unroll
        for (int k = 0; k < 8; k += 2 * w) {
          gs[k] += gs[k + w];
          gq[k] += gq[k + w];
        }
#pragma unroll
      for (int k = 0; k < 8; k += CG) {
        gs[k] += __shfl_xor(gs[k], 32);
        gq[k] += __shfl_xor(gq[k], 32);
      }
    };
    switch (cgm) {
      case 1: reduce(std::integral_constant<int, 1>{}); break;
      case 2: reduce(std::integral_constant<int, 2>{}); break;
      case 4: reduce(std::integral_constant<int, 4>{}); break;
      default: reduce(std::integral_constant<int, 8>{}); break;
    }
    float* red = tile;  // [8 waves][256 channel slots][2]; slot c holds channels c .. c + cgm - 1
    if (lane < 32) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (k % cgm == 0) {
          red[(wave * 256 + lane * 8 + k) * 2] = gs[k];
          red[(wave * 256 + lane * 8 + k) * 2 + 1] = gq[k];
        }
      }
    }
    EPI_BARRIER();
    const int ng = min(256, p.Kout - n0) / cg;  // host: 256 % cg == 0, Kout % cg == 0
    if (tid < ng) {
      float S = 0.f, Q = 0.f;
      for (int w = 0; w < 8; ++w)
        for (int c = 0; c < cg; c += cgm) {
          S += red[(w * 256 + tid * cg + c) * 2];
          Q += red[(w * 256 + tid * cg + c) * 2 + 1];
        }
      const int ohw = p.OH * p.OW;  // host: ohw % BM == 0, so a tile never straddles images
      const int img = m0 / ohw, chunk = (m0 - img * ohw) / BM;
      float* o = p.gnp + ((static_cast<long>(img) * (ohw / BM) + chunk) * p.gn_groups + n0 / 256 * (256 / cg) + tid) * 4;
      *reinterpret_cast<float4*>(o) = make_float4(S, Q, kout, 0.f);  // shifted sums, shift
    }
  }
#if AI4E_K256_STAMPS
  wait_vmcnt<0>();
  K256_STAMP(5);
  if (lane == 0 && blockIdx.x * 8 + wave < K256_MAXW) {
#pragma unroll
    for (int k = 0; k < K256_NSEG; ++k) g_k256_stamps[(blockIdx.x * 8 + wave) * K256_NSEG + k] = k_sum[k];
  }
#endif
}

}  // namespace

namespace {

const uint16_t* zero_chunk_ptr() {
  static const uint16_t* ptr = nullptr;
  if (!ptr) {
    void* a = nullptr;
    if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_zero_chunk)) == hipSuccess) ptr = static_cast<const uint16_t*>(a);
  }
  return ptr;
}

template <int WM, int WN, int STAGES, int OCC = 2, bool F16 = false>
int launch(const ConvParams& p0, hipStream_t s) {
  ConvParams p = p0;
  const int mt = ai4e_cdiv(p.M, WM * 64);
  p.ntiles_n = ai4e_cdiv(p.Kout, WN * 64);
  const int nb = mt * p.ntiles_n;
  p.zero = zero_chunk_ptr();
  if (!p.zero) return AI4E_ELAUNCH;
  const int g = (p.KH == 1 && p.KW == 1 && p.pad == 0) ? GATHER_POINTWISE
                : (p.C % BK == 0)                          ? GATHER_TAP
                                                           : GATHER_GENERAL;
  // coalesced LDS epilogue needs 16-B aligned output/residual rows
  const bool epi = !(p.ldy % 8 || p.ycoff % 8 || (p.res && p.ldres % 8) || p.Kout < 8);
#define K1_LAUNCH(G, E) \
  hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, STAGES, G, E, OCC, F16>), dim3(nb), dim3(256), 0, s, p)
  if (g == GATHER_POINTWISE) {
    if (epi) K1_LAUNCH(GATHER_POINTWISE, true); else K1_LAUNCH(GATHER_POINTWISE, false);
  } else if (g == GATHER_TAP) {
    if (epi) K1_LAUNCH(GATHER_TAP, true); else K1_LAUNCH(GATHER_TAP, false);
  } else {
    if (epi) K1_LAUNCH(GATHER_GENERAL, true); else K1_LAUNCH(GATHER_GENERAL, false);
  }
#undef K1_LAUNCH
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

template <int BM, bool F16 = false, bool PH3 = false>
int launch256(const ConvParams& p0, hipStream_t s) {
  ConvParams p = p0;
  // 256 tile: C % 64 (one tap per 64-wide K tile), 16-B output/residual rows, Kout % 8
  if (p.C % 64 || p.Kpad % 64 || p.ldy % 8 || p.ycoff % 8 || (p.res && p.ldres % 8) || p.Kout % 8)
    return AI4E_EINVAL;
  const int mt = ai4e_cdiv(p.M, BM);
  p.ntiles_n = ai4e_cdiv(p.Kout, 256);
  const int nb = mt * p.ntiles_n * (p.ksplit > 1 ? p.ksplit : 1);
  p.zero = zero_chunk_ptr();
  if (!p.zero) return AI4E_ELAUNCH;
  const unsigned dyn = p.hy ? 16u * 512u : 0u;  // the fused head's weights
  const bool pw = p.KH == 1 && p.KW == 1 && p.pad == 0;
  if (p.ksplit > 1) {
    if (pw)
      hipLaunchKernelGGL((conv_igemm256_kernel<GATHER_POINTWISE, BM, F16, PH3, true>), dim3(nb), dim3(512), dyn, s, p);
    else
      hipLaunchKernelGGL((conv_igemm256_kernel<GATHER_TAP, BM, F16, PH3, true>), dim3(nb), dim3(512), dyn, s, p);
  } else if (pw) {
    hipLaunchKernelGGL((conv_igemm256_kernel<GATHER_POINTWISE, BM, F16, PH3>), dim3(nb), dim3(512), dyn, s, p);
  } else {
    hipLaunchKernelGGL((conv_igemm256_kernel<GATHER_TAP, BM, F16, PH3>), dim3(nb), dim3(512), dyn, s, p);
  }
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

}  // namespace

// tile_cfg (pixels x channels per workgroup, LDS ring depth): 0 = auto, 1 = 128x128 (2x2 waves),
// 2 = 256x64 (4x1), 3 = 64x256 (1x4) with 4 stages; 4 = 128x128 with 5 stages (80 KB: still two
// workgroups per CU), 5 = 256x64 with 5 stages (100 KB: one workgroup per CU), 6 = 256x256, 8 waves,
// ping-pong phases (needs C % 64 == 0, Kout % 8 == 0); 7/8 = the 128x128 / 256x64 tiles with a 3-stage
// ring (48 KB, two-pass LDS epilogue) built for three workgroups per CU; 9 = the 256x256 schedule with
// 192-pixel tiles (one tile per CU for 250-image 14x14 layers); 10 = config 9 with three 16-MFMA phases per K tile.
// relu: bit 0 = ReLU; bit 1 = `res` is on the half-resolution grid [N, OH/2, OW/2, ldres] (nearest 2x
// upsample of the residual, OH and OW even).
namespace {
template <bool F16>
int conv2d_impl(const void* x, const void* w, const void* bias, const void* res, void* y, int N, int H, int W, int C,
                int ldx, int xcoff, int KH, int KW, int stride, int pad, int OH, int OW, int Kout, int Kpad, int ldy,
                int ycoff, int ldres, int relu, int tile_cfg, float* gnp, int gn_groups, hipStream_t stream,
                const void* hw = nullptr, int hw_ld = 0, const void* hb = nullptr, void* hy = nullptr,
                int ksplit = 1, void* skw = nullptr, void* sks = nullptr) {
  if (C % 8 || ldx % 8 || xcoff % 8 || Kpad % (2 * BK) || Kout % 4 || ldy % 4 || ycoff % 4 || (res && ldres % 4) ||
      Kpad < KH * KW * C)
    return AI4E_EINVAL;
  ConvParams p{};
  p.x = static_cast<const uint16_t*>(x);
  p.w = static_cast<const uint16_t*>(w);
  p.bias = static_cast<const float*>(bias);
  p.res = static_cast<const uint16_t*>(res);
  p.y = static_cast<uint16_t*>(y);
  p.N = N; p.H = H; p.W = W; p.C = C; p.ldx = ldx; p.xcoff = xcoff;
  p.KH = KH; p.KW = KW; p.stride = stride; p.pad = pad; p.OH = OH; p.OW = OW;
  p.Kout = Kout; p.Kpad = Kpad; p.ldy = ldy; p.ycoff = ycoff; p.ldres = ldres; p.relu = relu;
  p.M = N * OH * OW;
  if ((relu & 2) && (!res || (OH & 1) || (OW & 1))) return AI4E_EINVAL;  // half-resolution residual grid
  if (hy) {
    // fused 16-channel head: the 256-wide configs with the whole Kout = 256 in one channel tile
    if (!hw || !hb || hw_ld < 256 || hw_ld % 8 || Kout != 256 || gnp || (relu & 2) ||
        !(tile_cfg == 6 || tile_cfg == 9 || tile_cfg == 10))
      return AI4E_EINVAL;
    p.hw = static_cast<const uint16_t*>(hw);
    p.hw_ld = hw_ld;
    p.hb = static_cast<const float*>(hb);
    p.hy = static_cast<uint16_t*>(hy);
  } else if (!y) {
    return AI4E_EINVAL;
  }
  if (ksplit > 1) {
    // split-K: the 256-wide configs, plain epilogue (no GroupNorm statistics, no fused head), >= 1 K tile per split
    p.skdiag = ksplit >> 8;  // diagnostic hand-off variant (timing only)
    ksplit &= 255;
    if (ksplit != 2 || !skw || !sks || hy || !(tile_cfg == 6 || tile_cfg == 9 || tile_cfg == 10) || Kpad / 64 < ksplit)
      return AI4E_EINVAL;
    p.ksplit = ksplit;
    p.skw = static_cast<float*>(skw);
    p.sks = static_cast<int*>(sks);
  }
  if (p.M <= 0) return AI4E_OK;
  if (tile_cfg == 0) tile_cfg = Kout <= 64 ? 2 : 1;
  if (gnp) {
    // fused GroupNorm statistics: the LDS-epilogue tiles (configs 1, 2, 4, 5, 7, 8) and the 256-wide ones (6, 9,
    // 10), whole groups per channel tile, power-of-two group widths, tiles that never straddle images, full 16-B
    // output rows
    const bool tall = tile_cfg == 2 || tile_cfg == 5 || tile_cfg == 8;
    const bool wide = tile_cfg == 6 || tile_cfg == 9 || tile_cfg == 10;
    const int bm = tall ? 256 : wide ? (tile_cfg == 6 ? 256 : 192) : 128, bn = tall ? 64 : wide ? 256 : 128;
    const int cgw = gn_groups > 0 ? Kout / gn_groups : 0;
    if (tile_cfg == 3 || gn_groups <= 0 || Kout % gn_groups || (OH * OW) % bm || Kout % 8 || ldy % 8 || ycoff % 8 ||
        (res && ldres % 8) || bn % cgw || (wide && (cgw & (cgw - 1))))
      return AI4E_EINVAL;
    if (ksplit > 1) return AI4E_EINVAL;
    p.gnp = gnp;
    p.gn_groups = gn_groups;
  }
  switch (tile_cfg) {
    case 1: return launch<2, 2, 4, 2, F16>(p, stream);
    case 2: return launch<4, 1, 4, 2, F16>(p, stream);
    case 3: return launch<1, 4, 4, 2, F16>(p, stream);
    case 4: return launch<2, 2, 5, 2, F16>(p, stream);
    case 5: return launch<4, 1, 5, 2, F16>(p, stream);
    case 6: return launch256<256, F16>(p, stream);
    case 7: return launch<2, 2, 3, 3, F16>(p, stream);
    case 8: return launch<4, 1, 3, 3, F16>(p, stream);
    case 9: return launch256<192, F16>(p, stream);
    case 10: return launch256<192, F16, true>(p, stream);
    default: return AI4E_EINVAL;
  }
}

}  // namespace

AI4E_API int ai4e_conv2d_fwd(const void* x, const void* w, const void* bias, const void* res, void* y, int N, int H,
                             int W, int C, int ldx, int xcoff, int KH, int KW, int stride, int pad, int OH, int OW,
                             int Kout, int Kpad, int ldy, int ycoff, int ldres, int relu, int tile_cfg,
                             hipStream_t stream) {
  return conv2d_impl<false>(x, w, bias, res, y, N, H, W, C, ldx, xcoff, KH, KW, stride, pad, OH, OW, Kout, Kpad, ldy,
                            ycoff, ldres, relu, tile_cfg, nullptr, 0, stream);
}

// The same conv on fp16 activations and weights (f16 MFMA, fp32 accumulate; bias fp32).
AI4E_API int ai4e_conv2d_f16_fwd(const void* x, const void* w, const void* bias, const void* res, void* y, int N, int H,
                                 int W, int C, int ldx, int xcoff, int KH, int KW, int stride, int pad, int OH, int OW,
                                 int Kout, int Kpad, int ldy, int ycoff, int ldres, int relu, int tile_cfg,
                                 hipStream_t stream) {
  return conv2d_impl<true>(x, w, bias, res, y, N, H, W, C, ldx, xcoff, KH, KW, stride, pad, OH, OW, Kout, Kpad, ldy,
                           ycoff, ldres, relu, tile_cfg, nullptr, 0, stream);
}

// Same conv, plus the GroupNorm statistics of its output (gn_groups groups over Kout channels) written as
// per-(image, tile-row chunk, group) shifted partial sums (sum(x - K), sum((x - K)^2), K, pad) into gn_partials
// [N, OH*OW / BM, gn_groups, 4] fp32 (BM = 256 for tile configs 2, 5, 6 and 8, 192 for 9 and 10, else 128). Config 3
// and shapes whose tiles would straddle images are refused (EINVAL) before anything is launched.
AI4E_API int ai4e_conv2d_gn_fwd(const void* x, const void* w, const void* bias, const void* res, void* y, int N,
                                int H, int W, int C, int ldx, int xcoff, int KH, int KW, int stride, int pad, int OH,
                                int OW, int Kout, int Kpad, int ldy, int ycoff, int ldres, int relu, int tile_cfg,
                                void* gn_partials, int gn_groups, hipStream_t stream) {
  if (!gn_partials) return AI4E_EINVAL;
  return conv2d_impl<false>(x, w, bias, res, y, N, H, W, C, ldx, xcoff, KH, KW, stride, pad, OH, OW, Kout, Kpad, ldy,
                            ycoff, ldres, relu, tile_cfg, static_cast<float*>(gn_partials), gn_groups, stream);
}

// Same conv (a 256-wide tile config: 6, 9 or 10; Kout == 256, no residual upsample, no GroupNorm) with a 1x1 conv
// to 16 channels fused into its epilogue: head [N*OH*OW, 16] = (the conv's stored bf16 output) . hw^T + hb, hw
// [16 rows, ld hw_ld] bf16, hb [16] fp32. y may be null: the conv's output is then never written (the FPN RPN conv,
// whose only consumer is its 16-channel head).
AI4E_API int ai4e_conv2d_head_fwd(const void* x, const void* w, const void* bias, const void* res, void* y, int N,
                                  int H, int W, int C, int ldx, int xcoff, int KH, int KW, int stride, int pad, int OH,
                                  int OW, int Kout, int Kpad, int ldy, int ycoff, int ldres, int relu, int tile_cfg,
                                  const void* hw, int hw_ld, const void* hb, void* head, hipStream_t stream) {
  if (!head) return AI4E_EINVAL;
  return conv2d_impl<false>(x, w, bias, res, y, N, H, W, C, ldx, xcoff, KH, KW, stride, pad, OH, OW, Kout, Kpad, ldy,
                            ycoff, ldres, relu, tile_cfg, nullptr, 0, stream, hw, hw_ld, hb, head);
}

// Same conv with split-K over ksplit (= 2) workgroups per output tile, for grids too small to fill the chip (a 256-wide
// tile config 6, 9 or 10; e.g. ResNet-50 layer4's 3x3 convs: 128 tiles of K = 4608 -> 256 workgroups of 2304).
// skw: fp32 workspace of tiles * ksplit * BM * 256 floats (BM = 256 for config 6, else 192; tiles =
// ceil(M / BM) * ceil(Kout / 256)); sks: 2 * tiles int32, zero at launch (the launch leaves them zero again).
AI4E_API int ai4e_conv2d_sk_fwd(const void* x, const void* w, const void* bias, const void* res, void* y, int N, int H,
                                int W, int C, int ldx, int xcoff, int KH, int KW, int stride, int pad, int OH, int OW,
                                int Kout, int Kpad, int ldy, int ycoff, int ldres, int relu, int tile_cfg, int ksplit,
                                void* skw, void* sks, hipStream_t stream) {
  if (ksplit < 2) return AI4E_EINVAL;
  return conv2d_impl<false>(x, w, bias, res, y, N, H, W, C, ldx, xcoff, KH, KW, stride, pad, OH, OW, Kout, Kpad, ldy,
                            ycoff, ldres, relu, tile_cfg, nullptr, 0, stream, nullptr, 0, nullptr, nullptr, ksplit, skw,
                            sks);
}

#if AI4E_K256_STAMPS
// Diagnostic build only: per-wave segment cycle sums of the last 256-wide K1 launch (32768 waves x 6).
AI4E_API int ai4e_k256_stamps_read(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_k256_stamps), sizeof(g_k256_stamps)) == hipSuccess ? AI4E_OK
                                                                                                    : AI4E_ELAUNCH;
}
#endif

// Weight rows must be padded to this multiple (tile height in the channel dimension).
AI4E_API int ai4e_conv2d_weight_row_align() { return 256; }
