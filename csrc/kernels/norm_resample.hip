// K2 GroupNorm (+ReLU) and K3 bilinear 2x upsample — NHWC bf16, memory-bound, 16-B vectors per lane.
//
// GroupNorm is two launches: (1) per-(image, pixel-chunk) partial sums per group, reduced in-register
// then across the workgroup in LDS in a fixed order and written as fp32 partials (no atomics: bitwise
// reproducible); (2) a finalize
// workgroup per image combines the partials (fp64) into mean / rstd, then the normalize pass applies
// (x - mean) * rstd * gamma + beta (+ReLU) and writes bf16 — optionally into a channel slice of a
// wider buffer (U-Net concat).
// Partials are SHIFTED sums: chunk k of group g stores (S, Q, K) = (sum(x - K), sum((x - K)^2), K) with
// K one of the chunk's own values of that group, so a group whose mean is far from 0 relative to its
// spread (e.g. 50 + 0.05 * noise) does not cancel in E[x^2] - mean^2; the finalize re-bases every chunk
// on chunk 0's K in fp64 (GN_PARTIAL floats per (chunk, group); the conv epilogue writes the same form).
// The upsample writes straight into a concat slice as well, so the decoder's "upsample + concat" never
// materialises a separate tensor.
#include "common.h"

namespace {

// pixels per statistics chunk (one workgroup each). 256, not 1024: the U-Net's deep levels (64^2 and 32^2 maps of
// 512-1024 channels, 16 tiles) then still launch 256 / 64 workgroups instead of 64 / 16, which ran the statistics
// pass at 1.06 TB/s (profiles/r4h_unet/pmc_by_kernel.txt). ops/norm.py sizes the workspace from ai4e_gn_chunk_px().
#ifndef AI4E_UPSAMPLE_QUAD
#define AI4E_UPSAMPLE_QUAD 1  // 0: the per-output-vector upsample kernel (A/B library variant)
#endif
#ifndef AI4E_GN_CHUNK
#define AI4E_GN_CHUNK 256
#endif
constexpr int GN_PIX_PER_BLOCK = AI4E_GN_CHUNK;
constexpr int GN_PARTIAL = 4;  // floats per (chunk, group) partial: S, Q, K, pad

// x: [N, HW, C] (row stride ldx, channel offset xcoff); partials: [N, nchunks, G, 2]
__global__ __launch_bounds__(256) void gn_stats_kernel(const uint16_t* __restrict__ x, float* __restrict__ partials,
                                                       int HW, int C, int G, int ldx, int xcoff, int nchunks) {
  const int n = blockIdx.y;
  const int chunk = blockIdx.x;
  const int C8 = C >> 3;
  const int cg = C / G;  // channels per group (multiple of 8 or a divisor of 8)
  // each lane owns one 8-channel vector column (c8) and strides over pixels
  const int lanes_per_pix = C8;
  const int pix_per_iter = 256 / lanes_per_pix;  // requires C8 <= 256 and 256 % C8 == 0 (host checks)
  const int c8 = threadIdx.x % lanes_per_pix;
  const int p0 = threadIdx.x / lanes_per_pix;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int pbeg = chunk * GN_PIX_PER_BLOCK, pend = min(HW, pbeg + GN_PIX_PER_BLOCK);
  // the chunk's shift per group: its first pixel's value of the group's first channel
  __shared__ float gk[64];
  if (static_cast<int>(threadIdx.x) < G) {
    const uint16_t v = x[static_cast<long>(n) * HW * ldx + xcoff + static_cast<long>(pbeg) * ldx + threadIdx.x * cg];
    gk[threadIdx.x] = __uint_as_float(static_cast<uint32_t>(v) << 16);
  }
  __syncthreads();
  float k[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) k[j] = gk[min((8 * c8 + j) / cg, G - 1)];
  if (p0 < pix_per_iter) {
    const uint16_t* const xb = x + static_cast<long>(n) * HW * ldx + xcoff + 8 * c8;
    auto acc = [&](const uint4& v) __attribute__((always_inline)) {
      float a, b;
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        unpack_bf16x2(w[h], a, b);
        a -= k[2 * h];
        b -= k[2 * h + 1];
        s[2 * h] += a; q[2 * h] += a * a; s[2 * h + 1] += b; q[2 * h + 1] += b * b;
      }
    };
    int p = pbeg + p0;
    // four independent 16-B loads in flight per lane, then the accumulation
    for (; p + 3 * pix_per_iter < pend; p += 4 * pix_per_iter) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4*>(xb + static_cast<long>(p + u * pix_per_iter) * ldx);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc(v[u]);
    }
    for (; p < pend; p += pix_per_iter) acc(*reinterpret_cast<const uint4*>(xb + static_cast<long>(p) * ldx));
  }
  // every lane's 8 channel sums go to LDS; one thread per group then adds its group's (pixel row, channel)
  // terms in a fixed order, so the partials (and everything normalized by them) are bitwise reproducible
  // run to run (LDS float atomics would add in arrival order). Layout [channel-in-vector j][thread], rows padded
  // to 257 floats: the stores are lane-contiguous (conflict-free; [thread][j] put 8 lanes on each bank, 73 % of the
  // kernel's LDS cycles were bank conflicts, profiles/r4_unet/pmc_by_kernel.txt) and a group's reads fall <= 2 lanes
  // per bank for every C this kernel takes. Same addition order as before: bitwise-identical partials.
  constexpr int RS = 257;
  __shared__ float rs[8 * RS], rq[8 * RS];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    rs[j * RS + threadIdx.x] = s[j];
    rq[j * RS + threadIdx.x] = q[j];
  }
  __syncthreads();
  if (static_cast<int>(threadIdx.x) < G) {
    const int g = threadIdx.x;
    float S = 0.f, Q = 0.f;
    for (int pp = 0; pp < pix_per_iter; ++pp)
      for (int ch = g * cg; ch < (g + 1) * cg; ++ch) {
        const int t = pp * lanes_per_pix + (ch >> 3);
        S += rs[(ch & 7) * RS + t];
        Q += rq[(ch & 7) * RS + t];
      }
    float* o = partials + ((static_cast<long>(n) * nchunks + chunk) * G + g) * GN_PARTIAL;
    *reinterpret_cast<float4*>(o) = make_float4(S, Q, gk[g], 0.f);
  }
}

// One workgroup per image: combine the image's chunk partials (fp64) into per-group mean / rstd, then fold
// gamma / beta into a per-channel affine: ss[n, c] = (a, b) with y = x * a + b, a = rstd_g * gamma_c,
// b = beta_c - mean_g * a. (Done once per image instead of in every normalize workgroup.) Chunk k holds
// chunk_px pixels (the last one possibly fewer); its shifted sums are re-based on chunk 0's shift K0:
// sum(x - K0) = S + n d, sum((x - K0)^2) = Q + 2 d S + n d^2 with d = K - K0.
constexpr int GN_FIN_THREADS = 512;
constexpr int GN_FIN_GROUPS = 8;  // groups per finalize workgroup (gridDim.y = G / 8 when it divides)

// One workgroup per (image, slice of GL groups): reading an image's partials is per-CU-bandwidth bound, so the
// groups of an image are spread over several workgroups (groups are independent).
__global__ __launch_bounds__(GN_FIN_THREADS) void gn_finalize_kernel(const float* __restrict__ partials,
                                                                     const float* __restrict__ gamma,
                                                                     const float* __restrict__ beta,
                                                                     float2* __restrict__ ss, int HW, int C, int G,
                                                                     float eps, int nchunks, int chunk_px) {
  const int n = blockIdx.x;
  const int GL = G / gridDim.y;      // groups of this workgroup
  const int g0 = blockIdx.y * GL;
  __shared__ double red_s[GN_FIN_THREADS], red_q[GN_FIN_THREADS];
  __shared__ float mean_s[64], rstd_s[64];
  const int lpg = GN_FIN_THREADS / GL;  // threads per group (GL <= 64; a GL that does not divide leaves some idle)
  const int gl = threadIdx.x % GL, l = threadIdx.x / GL;
  const int cg = C / G;
  const float4* pp = reinterpret_cast<const float4*>(partials) + static_cast<long>(n) * nchunks * G + g0 + gl;
  const double k0 = pp[0].z;
  double s0 = 0, q0 = 0;
  if (l < lpg) {
    // 8 independent loads in flight per lane
    for (int k = l; k < nchunks; k += 8 * lpg) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k + u * lpg < nchunks) v[u] = pp[static_cast<long>(k + u * lpg) * G];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int kk = k + u * lpg;
        if (kk >= nchunks) break;
        const double cnt = static_cast<double>(min(chunk_px, HW - kk * chunk_px)) * cg;
        const double d = static_cast<double>(v[u].z) - k0;
        s0 += v[u].x + cnt * d;
        q0 += v[u].y + (2.0 * v[u].x + cnt * d) * d;
      }
    }
  }
  red_s[threadIdx.x] = s0;
  red_q[threadIdx.x] = q0;
  __syncthreads();
  if (static_cast<int>(threadIdx.x) < GL) {
    double s = 0, q = 0;
    for (int k = 0; k < lpg; ++k) {
      s += red_s[k * GL + threadIdx.x];
      q += red_q[k * GL + threadIdx.x];
    }
    const double cnt = static_cast<double>(HW) * cg;
    const double m = s / cnt;  // mean relative to K0
    const double var = fmax(q / cnt - m * m, 0.0);
    mean_s[threadIdx.x] = static_cast<float>(k0 + m);
    rstd_s[threadIdx.x] = static_cast<float>(1.0 / sqrt(var + eps));
  }
  __syncthreads();
  for (int c = threadIdx.x; c < GL * cg; c += GN_FIN_THREADS) {
    const int cc = g0 * cg + c;
    const float a = rstd_s[c / cg] * gamma[cc];
    ss[static_cast<long>(n) * C + cc] = make_float2(a, beta[cc] - mean_s[c / cg] * a);
  }
}

inline dim3 gn_finalize_grid(int N, int G) { return dim3(N, G % GN_FIN_GROUPS == 0 ? G / GN_FIN_GROUPS : 1); }

// y = x * a_c + b_c (+ReLU), 16-B vectors. C8 = C/8 divides 256, so with a grid stride that is a multiple of
// 256 every lane keeps one 8-channel column: its 8 affine pairs load once, the loop is unpack + FMA + cvt.
__global__ __launch_bounds__(256) void gn_apply_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                       const float2* __restrict__ ss, int HW, int C, int relu, int ldx,
                                                       int xcoff, int ldy, int ycoff) {
  const int n = blockIdx.y;
  const int C8 = C >> 3;
  const int sh = __builtin_ctz(C8);  // C8 is a power of two (divides 256)
  const int c8 = threadIdx.x & (C8 - 1);
  float a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float2 v = ss[static_cast<long>(n) * C + 8 * c8 + j];
    a[j] = v.x;
    b[j] = v.y;
  }
  const uint16_t* xn = x + static_cast<long>(n) * HW * ldx + xcoff + 8 * c8;
  uint16_t* yn = y + static_cast<long>(n) * HW * ldy + ycoff + 8 * c8;
  const int total = HW * C8;
  const int S = gridDim.x * 256;
  // the launch gives each lane ~4 vectors: issue their 4 loads together, then normalize and store
  for (int i0 = blockIdx.x * 256 + threadIdx.x; i0 < total; i0 += 4 * S) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * S;
      if (i < total) v[u] = *reinterpret_cast<const uint4*>(xn + static_cast<long>(i >> sh) * ldx);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * S;
      if (i >= total) break;
      float f[8];
      unpack_bf16x2(v[u].x, f[0], f[1]);
      unpack_bf16x2(v[u].y, f[2], f[3]);
      unpack_bf16x2(v[u].z, f[4], f[5]);
      unpack_bf16x2(v[u].w, f[6], f[7]);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fmaf(f[j], a[j], b[j]);
      uint4 o = make_uint4(cvt_bf16x2(f[0], f[1]), cvt_bf16x2(f[2], f[3]), cvt_bf16x2(f[4], f[5]),
                           cvt_bf16x2(f[6], f[7]));
      if (relu) {
        o.x = relu_bf16x2(o.x); o.y = relu_bf16x2(o.y); o.z = relu_bf16x2(o.z); o.w = relu_bf16x2(o.w);
      }
      *reinterpret_cast<uint4*>(yn + static_cast<long>(i >> sh) * ldy) = o;
    }
  }
}

// U-Net head: logits = conv1x1(relu(GroupNorm(z))) + bias, 64 -> 8 channels, in ONE pass over z (instead of an apply
// pass that writes the normalized tensor and a 1x1 conv that reads it back: ~2x the HBM traffic of the full-resolution
// 64-channel tensor). The norm arrives as the per-(image, channel) affine of ai4e_groupnorm_finalize. 8 lanes per
// pixel: lane = 8-channel column (one coalesced 16-B load; a wave covers 8 whole pixels), the normalized values are
// rounded to bf16 and ReLU'd exactly as the apply pass stores them, each lane forms the 8 outputs' partial dot
// products over its 8 channels, and a transpose-reduce over the 8 lanes (xor 4, 2, 1: 4 + 2 + 1 shuffles) leaves lane
// c8 with output channel c8, so a wave stores 8 pixels x 8 bf16 = 128 contiguous bytes. Host: HW % 32 == 0, so every
// block iteration covers 32 whole pixels and all lanes run the same trip count (full shuffle groups).
__global__ __launch_bounds__(256) void gn_relu_head8_kernel(const uint16_t* __restrict__ z, int ldz,
                                                            const float2* __restrict__ ss,
                                                            const uint16_t* __restrict__ w, int kpad,
                                                            const float* __restrict__ bias, uint16_t* __restrict__ y,
                                                            int HW) {
  const int n = blockIdx.y;
  const int c8 = threadIdx.x & 7;
  float a[8], b[8], wt[8][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float2 v = ss[n * 64 + 8 * c8 + j];
    a[j] = v.x;
    b[j] = v.y;
  }
#pragma unroll
  for (int o = 0; o < 8; ++o)
#pragma unroll
    for (int j = 0; j < 8; ++j) wt[o][j] = bf16_to_f32(w[o * kpad + 8 * c8 + j]);
  const float bo = bias[c8];
  const bool h4 = (c8 & 4) != 0, h2 = (c8 & 2) != 0, h1 = (c8 & 1) != 0;
  const uint16_t* const zn = z + static_cast<long>(n) * HW * ldz + 8 * c8;
  uint16_t* const yn = y + static_cast<long>(n) * HW * 8;
  const int S = gridDim.x * 32;  // pixels per grid stride
  for (int p0 = blockIdx.x * 32; p0 < HW; p0 += 4 * S) {  // block-uniform bounds (HW % 32 == 0)
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)  // the lane's loads first, then the math
      if (p0 + u * S < HW) v[u] = *reinterpret_cast<const uint4*>(zn + static_cast<long>(p0 + u * S + (threadIdx.x >> 3)) * ldz);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (p0 + u * S >= HW) break;
      const uint32_t q[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
      float f[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float lo, hi;
        unpack_bf16x2(q[k], lo, hi);
        unpack_bf16x2(relu_bf16x2(cvt_bf16x2(fmaf(lo, a[2 * k], b[2 * k]), fmaf(hi, a[2 * k + 1], b[2 * k + 1]))),
                      f[2 * k], f[2 * k + 1]);
      }
      float s8[8];
#pragma unroll
      for (int o = 0; o < 8; ++o) {
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc = fmaf(wt[o][j], f[j], acc);
        s8[o] = acc;
      }
      float t[4], r2[2];
#pragma unroll
      for (int k = 0; k < 4; ++k) t[k] = (h4 ? s8[k + 4] : s8[k]) + __shfl_xor(h4 ? s8[k] : s8[k + 4], 4);
#pragma unroll
      for (int k = 0; k < 2; ++k) r2[k] = (h2 ? t[k + 2] : t[k]) + __shfl_xor(h2 ? t[k] : t[k + 2], 2);
      const float r = (h1 ? r2[1] : r2[0]) + __shfl_xor(h1 ? r2[0] : r2[1], 1);  // output channel 4 h4 + 2 h2 + h1
      yn[static_cast<long>(p0 + u * S + (threadIdx.x >> 3)) * 8 + c8] = f32_to_bf16(r + bo);
    }
  }
}

// GN apply (+ReLU) that also emits the 2x2/2 max-pool of its output (the U-Net encoder's skip tensor and the
// next level's input from one pass: the pool never re-reads the skip). One lane = one 8-channel column of a
// 2x2 pixel quad; H, W even; pooled [N, H/2, W/2, C] contiguous.
__global__ __launch_bounds__(256) void gn_apply_pool_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                            uint16_t* __restrict__ pooled, const float2* __restrict__ ss,
                                                            int H, int W, int C, int relu, int ldx, int xcoff, int ldy,
                                                            int ycoff) {
  const int n = blockIdx.y;
  const int C8 = C >> 3;
  const int sh = __builtin_ctz(C8);
  const int c8 = threadIdx.x & (C8 - 1);
  float a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float2 v = ss[static_cast<long>(n) * C + 8 * c8 + j];
    a[j] = v.x;
    b[j] = v.y;
  }
  const int PW = W >> 1, PH = H >> 1;
  const uint16_t* xn = x + static_cast<long>(n) * H * W * ldx + xcoff + 8 * c8;
  uint16_t* yn = y + static_cast<long>(n) * H * W * ldy + ycoff + 8 * c8;
  uint16_t* pn = pooled + static_cast<long>(n) * PH * PW * C + 8 * c8;
  const int total = PH * PW * C8;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int q = i >> sh;
    const int qh = q / PW, qw = q - qh * PW;
    uint4 v[4];
#pragma unroll
    for (int d = 0; d < 4; ++d)
      v[d] = *reinterpret_cast<const uint4*>(xn + static_cast<long>((2 * qh + (d >> 1)) * W + 2 * qw + (d & 1)) * ldx);
    float m[8];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      float f[8];
      unpack_bf16x2(v[d].x, f[0], f[1]);
      unpack_bf16x2(v[d].y, f[2], f[3]);
      unpack_bf16x2(v[d].z, f[4], f[5]);
      unpack_bf16x2(v[d].w, f[6], f[7]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f[j] = fmaf(f[j], a[j], b[j]);
        if (relu) f[j] = fmaxf(f[j], 0.f);
        m[j] = d == 0 ? f[j] : fmaxf(m[j], f[j]);
      }
      *reinterpret_cast<uint4*>(yn + static_cast<long>((2 * qh + (d >> 1)) * W + 2 * qw + (d & 1)) * ldy) =
          make_uint4(cvt_bf16x2(f[0], f[1]), cvt_bf16x2(f[2], f[3]), cvt_bf16x2(f[4], f[5]), cvt_bf16x2(f[6], f[7]));
    }
    // max of the rounded values == rounded max (rounding is monotonic)
    *reinterpret_cast<uint4*>(pn + static_cast<long>(q) * C) =
        make_uint4(cvt_bf16x2(m[0], m[1]), cvt_bf16x2(m[2], m[3]), cvt_bf16x2(m[4], m[5]), cvt_bf16x2(m[6], m[7]));
  }
}

// Bilinear 2x upsample, align_corners=False (PyTorch semantics): src = (dst + 0.5) / 2 - 0.5, clamped.
// IDX = int when the element count fits (32-bit index math instead of a 64-bit div/mod chain per vector)
template <typename IDX>
__global__ __launch_bounds__(256) void upsample2x_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                         int N, int H, int W, int C, int ldy, int ycoff) {
  const int C8 = C >> 3;
  const int OH = 2 * H, OW = 2 * W;
  const IDX total = static_cast<IDX>(N) * OH * OW * C8;
  for (IDX i = static_cast<IDX>(blockIdx.x) * 256 + threadIdx.x; i < total; i += static_cast<IDX>(gridDim.x) * 256) {
    const IDX pix0 = i / C8;
    const int c8 = static_cast<int>(i - pix0 * C8);
    const IDX pix1 = pix0 / OW;
    const int ox = static_cast<int>(pix0 - pix1 * OW);
    const int n = static_cast<int>(pix1 / OH);
    const int oy = static_cast<int>(pix1 - static_cast<IDX>(n) * OH);
    const float sy = fmaxf((oy + 0.5f) * 0.5f - 0.5f, 0.f), sx = fmaxf((ox + 0.5f) * 0.5f - 0.5f, 0.f);
    const int y0 = static_cast<int>(sy), x0 = static_cast<int>(sx);
    const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
    const float ly = sy - y0, lx = sx - x0;
    const float w00 = (1 - ly) * (1 - lx), w01 = (1 - ly) * lx, w10 = ly * (1 - lx), w11 = ly * lx;
    const uint4* base = reinterpret_cast<const uint4*>(x) + static_cast<long>(n) * H * W * C8 + c8;
    const uint4 a = base[(static_cast<long>(y0) * W + x0) * C8], b = base[(static_cast<long>(y0) * W + x1) * C8];
    const uint4 c = base[(static_cast<long>(y1) * W + x0) * C8], d = base[(static_cast<long>(y1) * W + x1) * C8];
    uint32_t out[4];
    const uint32_t* pa = &a.x;
    const uint32_t* pb = &b.x;
    const uint32_t* pc = &c.x;
    const uint32_t* pd = &d.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float a0, a1, b0, b1, c0, c1, d0, d1;
      unpack_bf16x2(pa[k], a0, a1);
      unpack_bf16x2(pb[k], b0, b1);
      unpack_bf16x2(pc[k], c0, c1);
      unpack_bf16x2(pd[k], d0, d1);
      out[k] = pack_bf16x2(w00 * a0 + w01 * b0 + w10 * c0 + w11 * d0, w00 * a1 + w01 * b1 + w10 * c1 + w11 * d1);
    }
    *reinterpret_cast<uint4*>(y + ((static_cast<long>(n) * OH + oy) * OW + ox) * ldy + ycoff + 8 * c8) =
        make_uint4(out[0], out[1], out[2], out[3]);
  }
}

// The same upsample, one thread per INPUT pixel and 8-channel column: its 2x2 output quad (2i .. 2i + 1, 2j .. 2j + 1)
// reads only the 3x3 neighbourhood (rows i - 1 .. i + 1, columns j - 1 .. j + 1, clamped), loaded once: 9 gathers for
// 4 outputs instead of 16, and the index math (divisions by C8, W, H) once per quad. With align_corners=False the
// even output row uses rows (i - 1, i) at ly = 0.75 (at i = 0: rows (0, min(1, H - 1)) at ly = 0), the odd one rows
// (i, min(i + 1, H - 1)) at ly = 0.25; columns alike. Rows and columns are chosen by register selects (a runtime-
// indexed register array would live in scratch); the weights and the sum are formed exactly as upsample2x_kernel's.
template <typename IDX>
__global__ __launch_bounds__(256) void upsample2x_quad_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                              int N, int H, int W, int C, int ldy, int ycoff) {
  const int C8 = C >> 3;
  const IDX total = static_cast<IDX>(N) * H * W * C8;
  for (IDX t = static_cast<IDX>(blockIdx.x) * 256 + threadIdx.x; t < total; t += static_cast<IDX>(gridDim.x) * 256) {
    const IDX pix = t / C8;
    const int c8 = static_cast<int>(t - pix * C8);
    const IDX row = pix / W;
    const int j = static_cast<int>(pix - row * W);
    const int n = static_cast<int>(row / H);
    const int i = static_cast<int>(row - static_cast<IDX>(n) * H);
    const int r0 = i > 0 ? i - 1 : 0, r2 = i + 1 < H ? i + 1 : H - 1;
    const int q0 = j > 0 ? j - 1 : 0, q2 = j + 1 < W ? j + 1 : W - 1;
    const uint4* base = reinterpret_cast<const uint4*>(x) + static_cast<long>(n) * H * W * C8 + c8;
    const int rr[3] = {r0, i, r2}, qq[3] = {q0, j, q2};
    uint4 v[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) v[a][b] = base[(static_cast<long>(rr[a]) * W + qq[b]) * C8];
    const bool top = i > 0, left = j > 0;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      const int oy = 2 * i + dy;
      const float sy = fmaxf((oy + 0.5f) * 0.5f - 0.5f, 0.f);
      const float ly = sy - static_cast<int>(sy);
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int ox = 2 * j + dx;
        const float sx = fmaxf((ox + 0.5f) * 0.5f - 0.5f, 0.f);
        const float lx = sx - static_cast<int>(sx);
        const float w00 = (1 - ly) * (1 - lx), w01 = (1 - ly) * lx, w10 = ly * (1 - lx), w11 = ly * lx;
        // (y0, y1) window rows: even row (0, 1) when i > 0 else (1, 2); odd row (1, 2). Columns alike.
        uint4 a, b, c, d;
        auto pick = [&](const uint4& p0, const uint4& p1, bool s1) __attribute__((always_inline)) {
          return s1 ? p0 : p1;
        };
        if (dy == 0) {
          if (dx == 0) {
            a = pick(pick(v[0][0], v[0][1], left), pick(v[1][0], v[1][1], left), top);
            b = pick(pick(v[0][1], v[0][2], left), pick(v[1][1], v[1][2], left), top);
            c = pick(pick(v[1][0], v[1][1], left), pick(v[2][0], v[2][1], left), top);
            d = pick(pick(v[1][1], v[1][2], left), pick(v[2][1], v[2][2], left), top);
          } else {
            a = pick(v[0][1], v[1][1], top);
            b = pick(v[0][2], v[1][2], top);
            c = pick(v[1][1], v[2][1], top);
            d = pick(v[1][2], v[2][2], top);
          }
        } else {
          if (dx == 0) {
            a = pick(v[1][0], v[1][1], left);
            b = pick(v[1][1], v[1][2], left);
            c = pick(v[2][0], v[2][1], left);
            d = pick(v[2][1], v[2][2], left);
          } else {
            a = v[1][1];
            b = v[1][2];
            c = v[2][1];
            d = v[2][2];
          }
        }
        uint32_t out[4];
        const uint32_t pa[4] = {a.x, a.y, a.z, a.w}, pb[4] = {b.x, b.y, b.z, b.w};
        const uint32_t pc[4] = {c.x, c.y, c.z, c.w}, pd[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float a0, a1, b0, b1, c0, c1, d0, d1;
          unpack_bf16x2(pa[k], a0, a1);
          unpack_bf16x2(pb[k], b0, b1);
          unpack_bf16x2(pc[k], c0, c1);
          unpack_bf16x2(pd[k], d0, d1);
          out[k] = pack_bf16x2(w00 * a0 + w01 * b0 + w10 * c0 + w11 * d0, w00 * a1 + w01 * b1 + w10 * c1 + w11 * d1);
        }
        *reinterpret_cast<uint4*>(y + ((static_cast<long>(n) * 2 * H + oy) * 2 * W + ox) * ldy + ycoff + 8 * c8) =
            make_uint4(out[0], out[1], out[2], out[3]);
      }
    }
  }
}

inline int grid_for(long work) {
  long g = (work + 255) / 256;
  return static_cast<int>(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace

// partials (workspace) must hold N * ceil(HW / GN_PIX_PER_BLOCK (256)) * G * 4 + N * C * 2 floats (chunk partials, then the
// per-channel affine). HW * C / 8 < 2^31.
AI4E_API int ai4e_groupnorm_nhwc(const void* x, void* y, const void* gamma, const void* beta, void* partials, int N,
                                 int HW, int C, int G, float eps, int relu, int ldx_ldy_pack, int coff_pack,
                                 hipStream_t s) {
  // ldx_ldy_pack = ldx | (ldy << 16), coff_pack = xcoff | (ycoff << 16) (channel strides/offsets < 65536)
  const int ldx = ldx_ldy_pack & 0xffff, ldy = (ldx_ldy_pack >> 16) & 0xffff;
  const int xcoff = coff_pack & 0xffff, ycoff = (coff_pack >> 16) & 0xffff;
  if (C % 8 || G > 64 || C % G || (C / 8) > 256 || 256 % (C / 8) || ldx % 8 || ldy % 8 || xcoff % 8 || ycoff % 8)
    return AI4E_EINVAL;
  if ((C / G) % 8 && 8 % (C / G)) return AI4E_EINVAL;
  if (static_cast<long>(HW) * (C / 8) >= (1L << 31) - 4 * 8192L * 256) return AI4E_EINVAL;
  const int nchunks = (HW + GN_PIX_PER_BLOCK - 1) / GN_PIX_PER_BLOCK;
  hipLaunchKernelGGL(gn_stats_kernel, dim3(nchunks, N), dim3(256), 0, s, static_cast<const uint16_t*>(x),
                     static_cast<float*>(partials), HW, C, G, ldx, xcoff, nchunks);
  float2* ss =
      reinterpret_cast<float2*>(static_cast<float*>(partials) + static_cast<long>(N) * nchunks * G * GN_PARTIAL);
  hipLaunchKernelGGL(gn_finalize_kernel, gn_finalize_grid(N, G), dim3(GN_FIN_THREADS), 0, s, static_cast<const float*>(partials),
                     static_cast<const float*>(gamma), static_cast<const float*>(beta), ss, HW, C, G, eps, nchunks,
                     GN_PIX_PER_BLOCK);
  // ~4 vectors per lane; at most 8192 workgroups per image
  const int gx = grid_for(static_cast<long>(HW) * (C / 8) / 4 + 1);
  hipLaunchKernelGGL(gn_apply_kernel, dim3(gx, N), dim3(256), 0, s, static_cast<const uint16_t*>(x),
                     static_cast<uint16_t*>(y), ss, HW, C, relu, ldx, xcoff, ldy, ycoff);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

// GroupNorm when the statistics were already produced (e.g. by the conv epilogue, ai4e_conv2d_gn_fwd):
// partials [N, nchunks, G, 4] shifted chunk sums (HW / nchunks pixels per chunk), followed by room for the
// per-channel affine (N * C * 2 floats).
AI4E_API int ai4e_groupnorm_apply_nhwc(const void* x, void* y, const void* gamma, const void* beta, void* partials,
                                       int N, int HW, int C, int G, float eps, int relu, int ldx_ldy_pack,
                                       int coff_pack, int nchunks, hipStream_t s) {
  const int ldx = ldx_ldy_pack & 0xffff, ldy = (ldx_ldy_pack >> 16) & 0xffff;
  const int xcoff = coff_pack & 0xffff, ycoff = (coff_pack >> 16) & 0xffff;
  if (C % 8 || G > 64 || C % G || (C / 8) > 256 || 256 % (C / 8) || ldx % 8 || ldy % 8 || xcoff % 8 || ycoff % 8 ||
      nchunks <= 0)
    return AI4E_EINVAL;
  if (static_cast<long>(HW) * (C / 8) >= (1L << 31) - 4 * 8192L * 256) return AI4E_EINVAL;
  if (HW % nchunks) return AI4E_EINVAL;  // conv-epilogue partials: whole tiles per image
  float2* ss =
      reinterpret_cast<float2*>(static_cast<float*>(partials) + static_cast<long>(N) * nchunks * G * GN_PARTIAL);
  hipLaunchKernelGGL(gn_finalize_kernel, gn_finalize_grid(N, G), dim3(GN_FIN_THREADS), 0, s, static_cast<const float*>(partials),
                     static_cast<const float*>(gamma), static_cast<const float*>(beta), ss, HW, C, G, eps, nchunks,
                     HW / nchunks);
  const int gx = grid_for(static_cast<long>(HW) * (C / 8) / 4 + 1);
  hipLaunchKernelGGL(gn_apply_kernel, dim3(gx, N), dim3(256), 0, s, static_cast<const uint16_t*>(x),
                     static_cast<uint16_t*>(y), ss, HW, C, relu, ldx, xcoff, ldy, ycoff);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

// GroupNorm statistics -> per-(image, channel) affine only (no apply pass): partials [N, nchunks, G, 4] from a conv
// epilogue, the affine (a, b) written after them as float2 [N, C] (y = x * a + b). For a consumer that applies the norm
// itself while loading its input (conv_tile3x3.hip's prologue).
AI4E_API int ai4e_groupnorm_finalize(void* partials, const void* gamma, const void* beta, int N, int HW, int C, int G,
                                     float eps, int nchunks, hipStream_t s) {
  if (!partials || !gamma || !beta || N <= 0 || G <= 0 || G > 64 || C % G || nchunks <= 0 || HW % nchunks)
    return AI4E_EINVAL;
  float2* ss =
      reinterpret_cast<float2*>(static_cast<float*>(partials) + static_cast<long>(N) * nchunks * G * GN_PARTIAL);
  hipLaunchKernelGGL(gn_finalize_kernel, gn_finalize_grid(N, G), dim3(GN_FIN_THREADS), 0, s, static_cast<const float*>(partials),
                     static_cast<const float*>(gamma), static_cast<const float*>(beta), ss, HW, C, G, eps, nchunks,
                     HW / nchunks);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

// GN (precomputed statistics, as ai4e_groupnorm_apply_nhwc) that also writes the 2x2/2 max-pool of its output
// into pooled [N, H/2, W/2, C] (contiguous); H and W even.
AI4E_API int ai4e_groupnorm_apply_pool_nhwc(const void* x, void* y, const void* gamma, const void* beta, void* partials,
                                            void* pooled, int N, int H, int W, int C, int G, float eps, int relu,
                                            int ldx_ldy_pack, int coff_pack, int nchunks, hipStream_t s) {
  const int ldx = ldx_ldy_pack & 0xffff, ldy = (ldx_ldy_pack >> 16) & 0xffff;
  const int xcoff = coff_pack & 0xffff, ycoff = (coff_pack >> 16) & 0xffff;
  if (!pooled || (H & 1) || (W & 1) || C % 8 || G > 64 || C % G || (C / 8) > 256 || 256 % (C / 8) || ldx % 8 ||
      ldy % 8 || xcoff % 8 || ycoff % 8 || nchunks <= 0)
    return AI4E_EINVAL;
  const int HW = H * W;
  if (static_cast<long>(HW) * (C / 8) >= (1L << 31) - 4 * 8192L * 256) return AI4E_EINVAL;
  if (HW % nchunks) return AI4E_EINVAL;  // conv-epilogue partials: whole tiles per image
  float2* ss =
      reinterpret_cast<float2*>(static_cast<float*>(partials) + static_cast<long>(N) * nchunks * G * GN_PARTIAL);
  hipLaunchKernelGGL(gn_finalize_kernel, gn_finalize_grid(N, G), dim3(GN_FIN_THREADS), 0, s, static_cast<const float*>(partials),
                     static_cast<const float*>(gamma), static_cast<const float*>(beta), ss, HW, C, G, eps, nchunks,
                     HW / nchunks);
  const int gx = grid_for(static_cast<long>(HW / 4) * (C / 8) / 2 + 1);
  hipLaunchKernelGGL(gn_apply_pool_kernel, dim3(gx, N), dim3(256), 0, s, static_cast<const uint16_t*>(x),
                     static_cast<uint16_t*>(y), static_cast<uint16_t*>(pooled), ss, H, W, C, relu, ldx, xcoff, ldy,
                     ycoff);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

AI4E_API int ai4e_upsample2x_bilinear(const void* x, void* y, int N, int H, int W, int C, int ldy, int ycoff, int unused,
                                      hipStream_t s) {
  (void)unused;
  if (C % 8 || ldy % 8 || ycoff % 8) return AI4E_EINVAL;
  const long total = static_cast<long>(N) * 4 * H * W * (C / 8);
#if AI4E_UPSAMPLE_QUAD
  const long quads = total / 4;
  if (quads < (1L << 31) - 4 * 8192L * 256)
    hipLaunchKernelGGL(upsample2x_quad_kernel<int>, dim3(grid_for(quads)), dim3(256), 0, s,
                       static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), N, H, W, C, ldy, ycoff);
  else
    hipLaunchKernelGGL(upsample2x_quad_kernel<long>, dim3(grid_for(quads)), dim3(256), 0, s,
                       static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), N, H, W, C, ldy, ycoff);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
#endif
  if (total < (1L << 31) - 4 * 8192L * 256)
    hipLaunchKernelGGL(upsample2x_kernel<int>, dim3(grid_for(total)), dim3(256), 0, s, static_cast<const uint16_t*>(x),
                       static_cast<uint16_t*>(y), N, H, W, C, ldy, ycoff);
  else
    hipLaunchKernelGGL(upsample2x_kernel<long>, dim3(grid_for(total)), dim3(256), 0, s, static_cast<const uint16_t*>(x),
                       static_cast<uint16_t*>(y), N, H, W, C, ldy, ycoff);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

// logits [N, HW, 8] = conv1x1(relu(z * a + b)) + bias: z [N, HW, ldz] bf16, channels [zoff, zoff + 64); ss float2
// [N, 64] (ai4e_groupnorm_finalize); w bf16 [>= 8 rows, kpad >= 64] (row o = output channel o, K = input channel);
// bias fp32 [>= 8]. HW % 32 == 0.
AI4E_API int ai4e_gn_relu_head8(const void* z, int ldz, int zoff, const void* ss, const void* w, int kpad,
                                const void* bias, void* y, int N, int HW, hipStream_t s) {
  if (!z || !ss || !w || !bias || !y || N <= 0 || HW <= 0 || HW % 32 || ldz % 8 || zoff % 8 || zoff + 64 > ldz ||
      kpad < 64 || N > 65535)
    return AI4E_EINVAL;
  if (static_cast<long>(HW) * ldz >= (1L << 40)) return AI4E_EINVAL;
  const int blocks = HW / 32;
  const int gx = blocks < 4 * 1024 ? (blocks + 3) / 4 : 1024;  // ~4 pixels per lane
  hipLaunchKernelGGL(gn_relu_head8_kernel, dim3(gx, N), dim3(256), 0, s, static_cast<const uint16_t*>(z) + zoff, ldz,
                     static_cast<const float2*>(ss), static_cast<const uint16_t*>(w), kpad,
                     static_cast<const float*>(bias), static_cast<uint16_t*>(y), HW);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

// pixels per GroupNorm statistics chunk (the workspace of ai4e_groupnorm_nhwc is sized from it)
AI4E_API int ai4e_gn_chunk_px() { return GN_PIX_PER_BLOCK; }
