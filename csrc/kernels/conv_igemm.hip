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
#include "common.h"

namespace {

constexpr int BK = 32;

// Source of the zero 16-B chunks the DMA gather reads for padding / out-of-range taps.
__device__ __attribute__((aligned(64))) uint16_t g_zero_chunk[32];

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
};

__device__ __forceinline__ int swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

// One 16-B LDS-DMA per lane: global -> LDS at (wave-uniform M0 base + 16*lane). Inline asm so hipcc
// neither drains it with vmcnt(0) before every ds_read nor at barriers (cdna guide §5.7, §5 "Pipelining
// across barriers"); completion is tracked by hand with counted vmcnt.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_base)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Gather modes of the activation operand.
enum { GATHER_GENERAL = 0,  // any C % 8: a 32-wide K chunk may span taps -> per-lane tap walk
       GATHER_POINTWISE = 1,  // 1x1, pad 0 (any stride): K is the channel axis of one input pixel
       GATHER_TAP = 2 };      // C % 32 == 0: a K chunk lies in ONE tap -> the tap walk is wave-uniform (SGPRs)

template <int WAVES_M, int WAVES_N, int STAGES, int GATHER, bool EPI_LDS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void conv_igemm_kernel(const ConvParams p) {
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
  if (p.res) {  // unconditional loads (clamped rows/cols) so hipcc keeps one counted wait for all
    if constexpr (EPI_LDS) {
#pragma unroll
      for (int e = 0; e < EPI_CHUNKS; ++e) {
        const int g = tid + 256 * e;
        const int m = min(m0 + g / CPR, p.M - 1), n = min(n0 + 8 * (g % CPR), p.Kout - 8);
        rres16[e] = *reinterpret_cast<const uint4*>(p.res + static_cast<long>(m) * p.ldres + n);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = min(pm + 16 * i, p.M - 1), n = min(pn + 16 * j, p.Kout - 4);
          rres[i][j] = *reinterpret_cast<const uint2*>(p.res + static_cast<long>(m) * p.ldres + n);
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
  int tkh = 0, tkw = 0, tcb = 0;  // GATHER_TAP: wave-uniform tap (kh, kw) and channel base
  const uint16_t* const wsrc = p.w + static_cast<long>(n0 + 16 * wave + rin) * p.Kpad + 8 * c;
  const long wstep = 64L * p.Kpad;  // rows 16*(wave+4i)
  const uint32_t smem_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem));
  const uint16_t* const zero = p.zero;

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
      const long toff = (static_cast<long>(tkh) * p.W + tkw) * p.ldx + tcb;
      const bool tap_ok = tkh < p.KH;
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const bool ok = tap_ok && static_cast<unsigned>(ih0[i] + tkh) < static_cast<unsigned>(p.H) &&
                        static_cast<unsigned>(iw0[i] + tkw) < static_cast<unsigned>(p.W);
        glds16(ok ? static_cast<const void*>(rowp[i] + toff) : zero, sbase + (16 * (wave + 4 * i)) * BK * 2);
      }
      tcb += BK;
      if (tcb == p.C) {
        tcb = 0;
        if (++tkw == p.KW) {
          tkw = 0;
          ++tkh;
        }
      }
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
#pragma unroll
    for (int i = 0; i < CB; ++i) glds16(wsrc + i * wstep + kt * BK, sbase + (BM + 16 * (wave + 4 * i)) * BK * 2);
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15;
  const int fofs = frow * BK + (((lane >> 4) ^ swz(frow)) << 3);
  const int nk = p.Kpad / BK;

  // Wait until ring stage `kt` has landed for this wave: the stages issued after it (at most
  // min(ahead, nk-1-kt) of them, PER_STAGE DMAs each) may stay in flight.
  auto wait_stage = [&](int kt, int ahead) {
    const int younger = min(ahead, nk - 1 - kt);
    if (younger >= 3) wait_vmcnt<3 * PER_STAGE>();
    else if (younger == 2) wait_vmcnt<2 * PER_STAGE>();
    else if (younger == 1) wait_vmcnt<PER_STAGE>();
    else wait_vmcnt<0>();
  };

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
#define K1_STEP(KT, FWC, FXC, FWN, FXN)                                                         \
  {                                                                                             \
    const int kt_ = (KT);                                                                       \
    if (kt_ + 1 < nk) {                                                                         \
      wait_stage(kt_ + 1, STAGES - 3); /* issued so far: up to kt+STAGES-2 */                   \
      __builtin_amdgcn_s_barrier();                                                             \
      K1_READ(FWN, FXN, kt_ + 1)                                                                \
    }                                                                                           \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                               \
      _Pragma("unroll") for (int j = 0; j < 4; ++j)                                             \
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FWC[j], FXC[i], acc[i][j], 0, 0, 0); \
    if (kt_ + STAGES - 1 < nk) issue_stage(kt_ + STAGES - 1);                                   \
  }

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue_stage(s);
  wait_stage(0, STAGES - 2);
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
  const float lo = p.relu ? 0.f : -INFINITY;
  if constexpr (EPI_LDS) {
    // Stage the fp32 tile through LDS (the now idle stage ring: BM*BN*4 bytes) so every lane
    // reads/writes 16 contiguous bytes: a wave instruction then covers whole 256-B+ pixel rows,
    // halving store instructions and giving the residual read the same full-line shape.
    // Row-major [BM][BN] fp32 with the 16-B chunk index XOR-swizzled by (row & 7): the 8-lane
    // ds_write_b128 groups (8 rows, one column) hit 8 different bank quads.
    static_assert(BM * BN * 4 <= STAGES * STAGE_ELEMS * 2, "epilogue tile must fit the stage ring");
    float* tile = reinterpret_cast<float*>(smem);
    __builtin_amdgcn_s_barrier();  // all waves finished reading the last stage
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wm * 64 + 16 * i + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = (wn * 64 + 16 * j + 4 * (lane >> 4)) >> 2;  // fp32 16-B chunk in the row
        *reinterpret_cast<f32x4_t*>(tile + r * BN + 4 * (q ^ (r & 7))) = acc[i][j];
      }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < EPI_CHUNKS; ++e) {
      const int g = tid + 256 * e;
      const int r = g / CPR, cq = g % CPR;
      const int m = m0 + r, n = n0 + 8 * cq;
      const float4 v0 = *reinterpret_cast<const float4*>(tile + r * BN + 4 * ((2 * cq) ^ (r & 7)));
      const float4 v1 = *reinterpret_cast<const float4*>(tile + r * BN + 4 * ((2 * cq + 1) ^ (r & 7)));
      float f[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      if (p.res) {
        float a[8];
        unpack_bf16x2(rres16[e].x, a[0], a[1]);
        unpack_bf16x2(rres16[e].y, a[2], a[3]);
        unpack_bf16x2(rres16[e].z, a[4], a[5]);
        unpack_bf16x2(rres16[e].w, a[6], a[7]);
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] += a[k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = fmaxf(f[k], lo);
      if (m < p.M && n < p.Kout) {
        uint16_t* dst = p.y + static_cast<long>(m) * p.ldy + p.ycoff + n;
        const uint2 lo4 = make_uint2(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]));
        if (n + 8 <= p.Kout) {
          *reinterpret_cast<uint4*>(dst) = make_uint4(lo4.x, lo4.y, pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7]));
        } else {
          *reinterpret_cast<uint2*>(dst) = lo4;  // Kout % 8 == 4 tail
        }
      }
    }
  } else {
    if (p.res) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float a0, a1, a2, a3;
          unpack_bf16x2(rres[i][j].x, a0, a1);
          unpack_bf16x2(rres[i][j].y, a2, a3);
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
              make_uint2(pack_bf16x2(fmaxf(acc[i][j][0], lo), fmaxf(acc[i][j][1], lo)),
                         pack_bf16x2(fmaxf(acc[i][j][2], lo), fmaxf(acc[i][j][3], lo)));
      }
    }
  }
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

template <int WM, int WN, int STAGES>
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
  hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, STAGES, G, E>), dim3(nb), dim3(256), 0, s, p)
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

}  // namespace

// tile_cfg (pixels x channels per workgroup, LDS ring depth): 0 = auto, 1 = 128x128 (2x2 waves),
// 2 = 256x64 (4x1), 3 = 64x256 (1x4) with 4 stages; 4 = 128x128 with 5 stages (80 KB: still two
// workgroups per CU), 5 = 256x64 with 5 stages (100 KB: one workgroup per CU).
AI4E_API int ai4e_conv2d_fwd(const void* x, const void* w, const void* bias, const void* res, void* y, int N, int H,
                             int W, int C, int ldx, int xcoff, int KH, int KW, int stride, int pad, int OH, int OW,
                             int Kout, int Kpad, int ldy, int ycoff, int ldres, int relu, int tile_cfg,
                             hipStream_t stream) {
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
  if (p.M <= 0) return AI4E_OK;
  if (tile_cfg == 0) tile_cfg = Kout <= 64 ? 2 : 1;
  switch (tile_cfg) {
    case 1: return launch<2, 2, 4>(p, stream);
    case 2: return launch<4, 1, 4>(p, stream);
    case 3: return launch<1, 4, 4>(p, stream);
    case 4: return launch<2, 2, 5>(p, stream);
    case 5: return launch<4, 1, 5>(p, stream);
    default: return AI4E_EINVAL;
  }
}

// Weight rows must be padded to this multiple (tile height in the channel dimension).
AI4E_API int ai4e_conv2d_weight_row_align() { return 256; }
