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
//   consecutive output CHANNELS of one pixel: the epilogue stores 8 contiguous bytes per lane
//   straight from registers (bias float4, residual 8-B loads) with no LDS round trip.
// * A/B tiles (BK = 32) are register-staged into a 2-deep LDS ring with one barrier per K-step;
//   the global loads of step k+1 are issued before the MFMAs of step k (cdna guide T14).
//   Each 64-B LDS row (32 bf16) is XOR-swizzled per 16-B chunk with s = {0,2,3,1}[(row>>2)&3],
//   which makes every ds_read_b128 fragment read conflict-free for the gfx950 lane groups
//   {0-3,12-15,20-27},{4-11,16-19,28-31},... (MI355X_MICROARCH.md §LDS).
// * The activation gather handles padding/stride/any KHxKW with 16-B loads per (pixel, tap,
//   8-channel chunk); C must be a multiple of 8 (the stem is fed C=8 by the preprocess kernel).
// * XCD-aware tile order: tiles that share an activation panel (same m-tile, different n-tiles)
//   land on one XCD's L2 (common.h xcd_remap).
#include "common.h"

namespace {

constexpr int BK = 32;

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
};

__device__ __forceinline__ int swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

template <int WAVES_M, int WAVES_N>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, WAVES_N > 1 ? 2 : 3))) void conv_igemm_kernel(const ConvParams p) {
  constexpr int BM = WAVES_M * 64;  // pixels per workgroup
  constexpr int BN = WAVES_N * 64;  // channels per workgroup
  constexpr int CA = BM / 64;       // A (activation) 16-B chunks per thread per K-step
  constexpr int CB = BN / 64;       // B (weight) chunks per thread per K-step
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * (BM + BN) * BK];
  uint16_t* const sX = smem;                // [2][BM][BK]
  uint16_t* const sW = smem + 2 * BM * BK;  // [2][BN][BK]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WAVES_M;
  const int wn = wave / WAVES_M;

  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = t / p.ntiles_n;
  const int nt = t - mt * p.ntiles_n;
  const int m0 = mt * BM;
  const int n0 = nt * BN;

  // ---- per-thread load assignment: chunk column c fixed, rows (tid>>2) + 64*i
  const int c = tid & 3;
  const int r0 = tid >> 2;
  const int OHW = p.OH * p.OW;
  int ih0[CA], iw0[CA];
  long xbase[CA];
#pragma unroll
  for (int i = 0; i < CA; ++i) {
    const int m = m0 + r0 + 64 * i;
    if (m < p.M) {
      const int img = m / OHW;
      const int rem = m - img * OHW;
      const int oh = rem / p.OW;
      const int ow = rem - oh * p.OW;
      ih0[i] = oh * p.stride - p.pad;
      iw0[i] = ow * p.stride - p.pad;
      xbase[i] = static_cast<long>(img) * p.H * p.W * p.ldx + p.xcoff;
    } else {
      ih0[i] = -(1 << 28);  // forces the bounds check to fail -> zeros
      iw0[i] = 0;
      xbase[i] = 0;
    }
  }
  // k-state of this thread's chunk: k = kt*BK + 8c  ->  (kh, kw, cc)
  int cc, kh, kw;
  {
    const int k = 8 * c;
    const int tap = k / p.C;
    cc = k - tap * p.C;
    kh = tap / p.KW;
    kw = tap - kh * p.KW;
  }
  const uint16_t* const wbase = p.w + static_cast<long>(n0 + r0) * p.Kpad + 8 * c;
  const long wstride64 = 64L * p.Kpad;

  uint4 ra[CA], rb[CB];
  // Issue the global loads of K-tile kt into registers, then advance the k-state by BK.
#define AI4E_LOAD_TILE(kt)                                                                                   \
  do {                                                                                                       \
    _Pragma("unroll") for (int i = 0; i < CA; ++i) {                                                         \
      const int ih = ih0[i] + kh, iw = iw0[i] + kw;                                                          \
      uint4 v = make_uint4(0, 0, 0, 0);                                                                      \
      if (kh < p.KH && static_cast<unsigned>(ih) < static_cast<unsigned>(p.H) &&                             \
          static_cast<unsigned>(iw) < static_cast<unsigned>(p.W))                                            \
        v = *reinterpret_cast<const uint4*>(p.x + xbase[i] + (static_cast<long>(ih) * p.W + iw) * p.ldx + cc); \
      ra[i] = v;                                                                                             \
    }                                                                                                        \
    _Pragma("unroll") for (int i = 0; i < CB; ++i) rb[i] =                                                   \
        *reinterpret_cast<const uint4*>(wbase + i * wstride64 + (kt) * BK);                                  \
    cc += BK;                                                                                                \
    while (cc >= p.C) {                                                                                      \
      cc -= p.C;                                                                                             \
      if (++kw == p.KW) {                                                                                    \
        kw = 0;                                                                                              \
        ++kh;                                                                                                \
      }                                                                                                      \
    }                                                                                                        \
  } while (0)
  // Write the staged registers into LDS buffer `buf` (swizzled 16-B chunks).
#define AI4E_STORE_TILE(buf)                                                                                 \
  do {                                                                                                       \
    uint16_t* sx_ = sX + (buf) * BM * BK;                                                                    \
    uint16_t* sw_ = sW + (buf) * BN * BK;                                                                    \
    _Pragma("unroll") for (int i = 0; i < CA; ++i) {                                                         \
      const int row = r0 + 64 * i;                                                                           \
      *reinterpret_cast<uint4*>(sx_ + row * BK + ((c ^ swz(row)) << 3)) = ra[i];                              \
    }                                                                                                        \
    _Pragma("unroll") for (int i = 0; i < CB; ++i) {                                                         \
      const int row = r0 + 64 * i;                                                                           \
      *reinterpret_cast<uint4*>(sw_ + row * BK + ((c ^ swz(row)) << 3)) = rb[i];                              \
    }                                                                                                        \
  } while (0)

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // fragment read offset (elements) inside a 16-row block: row = lane&15, chunk = lane>>4 swizzled
  const int frow = lane & 15;
  const int fofs = frow * BK + (((lane >> 4) ^ swz(frow)) << 3);
  const int nk = p.Kpad / BK;

  AI4E_LOAD_TILE(0);
  AI4E_STORE_TILE(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) AI4E_LOAD_TILE(kt + 1);
    const uint16_t* x = sX + cur * BM * BK + (wm * 64) * BK + fofs;
    const uint16_t* w = sW + cur * BN * BK + (wn * 64) * BK + fofs;
    bf16x8_t bw[4], bx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bw[j] = *reinterpret_cast<const bf16x8_t*>(w + j * 16 * BK);
#pragma unroll
    for (int i = 0; i < 4; ++i) bx[i] = *reinterpret_cast<const bf16x8_t*>(x + i * 16 * BK);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], bx[i], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) AI4E_STORE_TILE(cur ^ 1);
    __syncthreads();
  }

#undef AI4E_LOAD_TILE
#undef AI4E_STORE_TILE

  // ---- fused epilogue: lane holds channels n..n+3 of pixel m for each (i, j) fragment
  const int pm = m0 + wm * 64 + (lane & 15);
  const int pn = n0 + wn * 64 + 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = pn + 16 * j;
    if (n >= p.Kout) continue;
    const float4 b = *reinterpret_cast<const float4*>(p.bias + n);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = pm + 16 * i;
      if (m >= p.M) continue;
      float v0 = acc[i][j][0] + b.x, v1 = acc[i][j][1] + b.y, v2 = acc[i][j][2] + b.z, v3 = acc[i][j][3] + b.w;
      if (p.res) {
        const uint2 r = *reinterpret_cast<const uint2*>(p.res + static_cast<long>(m) * p.ldres + n);
        float a0, a1, a2, a3;
        unpack_bf16x2(r.x, a0, a1);
        unpack_bf16x2(r.y, a2, a3);
        v0 += a0; v1 += a1; v2 += a2; v3 += a3;
      }
      if (p.relu) {
        v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
      }
      *reinterpret_cast<uint2*>(p.y + static_cast<long>(m) * p.ldy + p.ycoff + n) =
          make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
    }
  }
}

template <int WM, int WN>
int launch(const ConvParams& p0, hipStream_t s) {
  ConvParams p = p0;
  const int mt = ai4e_cdiv(p.M, WM * 64);
  p.ntiles_n = ai4e_cdiv(p.Kout, WN * 64);
  const int nb = mt * p.ntiles_n;
  hipLaunchKernelGGL((conv_igemm_kernel<WM, WN>), dim3(nb), dim3(256), 0, s, p);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

}  // namespace

// tile_cfg (pixels x channels per workgroup): 0 = auto, 1 = 128x128 (2x2 waves), 2 = 256x64 (4x1),
// 3 = 64x256 (1x4), 4 = 128x64 (2x1).
AI4E_API int ai4e_conv2d_fwd(const void* x, const void* w, const void* bias, const void* res, void* y, int N, int H,
                             int W, int C, int ldx, int xcoff, int KH, int KW, int stride, int pad, int OH, int OW,
                             int Kout, int Kpad, int ldy, int ycoff, int ldres, int relu, int tile_cfg,
                             hipStream_t stream) {
  if (C % 8 || ldx % 8 || xcoff % 8 || Kpad % BK || Kout % 4 || ldy % 4 || ycoff % 4 || (res && ldres % 4) ||
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
    case 1: return launch<2, 2>(p, stream);
    case 2: return launch<4, 1>(p, stream);
    case 3: return launch<1, 4>(p, stream);
    case 4: return launch<2, 1>(p, stream);
    default: return AI4E_EINVAL;
  }
}

// Weight rows must be padded to this multiple (tile height in the channel dimension).
AI4E_API int ai4e_conv2d_weight_row_align() { return 256; }
