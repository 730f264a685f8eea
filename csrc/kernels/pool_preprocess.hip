// K7 preprocess, max-pool, global-avg-pool — memory-bound NHWC bf16 (or fp16: F16) kernels, 16-B vectors per lane.
#include "common.h"

namespace {

// uint8 [N,H,W,Cin] (Cin<=8, e.g. decoded RGB / RGB+NIR) -> bf16 [N,H,W,8], (x*scale - mean)/std,
// channels >= Cin zero-filled so the stem conv sees C = 8 (one 16-B vector per pixel).
__global__ __launch_bounds__(256) void preprocess_u8_kernel(const uint8_t* __restrict__ in, uint16_t* __restrict__ out,
                                                            long npix, int cin, float4 mean_lo, float4 mean_hi,
                                                            float4 istd_lo, float4 istd_hi, float scale) {
  const float mean[8] = {mean_lo.x, mean_lo.y, mean_lo.z, mean_lo.w, mean_hi.x, mean_hi.y, mean_hi.z, mean_hi.w};
  const float istd[8] = {istd_lo.x, istd_lo.y, istd_lo.z, istd_lo.w, istd_hi.x, istd_hi.y, istd_hi.z, istd_hi.w};
  for (long p = blockIdx.x * 256L + threadIdx.x; p < npix; p += static_cast<long>(gridDim.x) * 256) {
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = c < cin ? (in[p * cin + c] * scale - mean[c]) * istd[c] : 0.f;
    uint4 o = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                         pack_bf16x2(v[6], v[7]));
    reinterpret_cast<uint4*>(out)[p] = o;
  }
}

// Space-to-depth preprocess for the 7x7/2 stem (see ops/conv.py pack_stem_s2d):
// uint8 [N,H,W,cin<=4] -> bf16 [N,H/2,W/2,16], out[i,j,(dy*2+dx)*cin+c] = norm(x[2i+dy-1, 2j+dx-1, c])
// (zero outside the image = the conv's zero padding of the normalized input).
// CIN > 0: channel count known at compile time (fully unrolled, the 16 outputs stay in registers) and
// 32-bit pixel indexing (IDX = int when N*H/2*W/2 < 2^31); CIN = 0: runtime cin, 64-bit indexing.
template <int CIN, typename IDX, bool F16 = false>
__global__ __launch_bounds__(256) void preprocess_s2d_kernel(const uint8_t* __restrict__ in, uint16_t* __restrict__ out,
                                                             int N, int H, int W, int cin_rt, float4 mean, float4 istd,
                                                             float scale) {
  const int cin = CIN > 0 ? CIN : cin_rt;
  const int OH = H >> 1, OW = W >> 1;
  const float m[4] = {mean.x, mean.y, mean.z, mean.w};
  const float is[4] = {istd.x, istd.y, istd.z, istd.w};
  const IDX total = static_cast<IDX>(N) * OH * OW;
  for (IDX p = static_cast<IDX>(blockIdx.x) * 256 + threadIdx.x; p < total; p += static_cast<IDX>(gridDim.x) * 256) {
    const IDX t = p / OW;
    const int j = static_cast<int>(p - t * OW);
    const IDX n = t / OH;
    const int i = static_cast<int>(t - n * OH);
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      const int y = 2 * i + dy - 1;
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int x = 2 * j + dx - 1;
        if (y < 0 || y >= H || x < 0 || x >= W) continue;
        const uint8_t* src = in + ((static_cast<long>(n) * H + y) * W + x) * cin;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (c < cin) v[(dy * 2 + dx) * cin + c] = (src[c] * scale - m[c]) * is[c];
      }
    }
    uint4* o = reinterpret_cast<uint4*>(out) + 2 * static_cast<long>(p);
    o[0] = make_uint4(pack2<F16>(v[0], v[1]), pack2<F16>(v[2], v[3]), pack2<F16>(v[4], v[5]), pack2<F16>(v[6], v[7]));
    o[1] = make_uint4(pack2<F16>(v[8], v[9]), pack2<F16>(v[10], v[11]), pack2<F16>(v[12], v[13]),
                      pack2<F16>(v[14], v[15]));
  }
}

// Max pool NHWC bf16; one lane = 8 channels of one output pixel. Padding ignored (= -inf).
// IDX = int when the element count fits (32-bit index math: the 64-bit div/mod chain cost more than the loads)
template <typename IDX, bool F16 = false>
__global__ __launch_bounds__(256) void maxpool_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int N,
                                                      int H, int W, int C, int OH, int OW, int k, int s, int pad,
                                                      int ldx8) {
  const int C8 = C >> 3;
  const IDX total = static_cast<IDX>(N) * OH * OW * C8;
  for (IDX i = static_cast<IDX>(blockIdx.x) * 256 + threadIdx.x; i < total; i += static_cast<IDX>(gridDim.x) * 256) {
    const IDX pix0 = i / C8;
    const int c8 = static_cast<int>(i - pix0 * C8);
    const IDX pix1 = pix0 / OW;
    const int ow = static_cast<int>(pix0 - pix1 * OW);
    const int n = static_cast<int>(pix1 / OH);
    const int oh = static_cast<int>(pix1 - static_cast<IDX>(n) * OH);
    float m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
    for (int dh = 0; dh < k; ++dh) {
      const int ih = oh * s - pad + dh;
      if (ih < 0 || ih >= H) continue;
      for (int dw = 0; dw < k; ++dw) {
        const int iw = ow * s - pad + dw;
        if (iw < 0 || iw >= W) continue;
        const uint4 v = reinterpret_cast<const uint4*>(x)[((static_cast<long>(n) * H + ih) * W + iw) * ldx8 + c8];
        float a, b;
        unpack2<F16>(v.x, a, b); m[0] = fmaxf(m[0], a); m[1] = fmaxf(m[1], b);
        unpack2<F16>(v.y, a, b); m[2] = fmaxf(m[2], a); m[3] = fmaxf(m[3], b);
        unpack2<F16>(v.z, a, b); m[4] = fmaxf(m[4], a); m[5] = fmaxf(m[5], b);
        unpack2<F16>(v.w, a, b); m[6] = fmaxf(m[6], a); m[7] = fmaxf(m[7], b);
      }
    }
    reinterpret_cast<uint4*>(y)[i] =
        make_uint4(pack2<F16>(m[0], m[1]), pack2<F16>(m[2], m[3]), pack2<F16>(m[4], m[5]), pack2<F16>(m[6], m[7]));
  }
}

// Global average pool [N, HW, C] -> [N, C] (bf16 out, fp32 accumulate). One lane = 8 channels.
template <bool F16 = false>
__global__ __launch_bounds__(256) void avgpool_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int N,
                                                      int HW, int C) {
  const int C8 = C >> 3;
  const long total = static_cast<long>(N) * C8;
  const float inv = 1.f / HW;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += static_cast<long>(gridDim.x) * 256) {
    const int c8 = static_cast<int>(i % C8);
    const long n = i / C8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint4* p = reinterpret_cast<const uint4*>(x) + n * HW * C8 + c8;
    auto add = [&](const uint4& v) __attribute__((always_inline)) {
      float a, b;
      unpack2<F16>(v.x, a, b); acc[0] += a; acc[1] += b;
      unpack2<F16>(v.y, a, b); acc[2] += a; acc[3] += b;
      unpack2<F16>(v.z, a, b); acc[4] += a; acc[5] += b;
      unpack2<F16>(v.w, a, b); acc[6] += a; acc[7] += b;
    };
    int j = 0;
    for (; j + 7 <= HW; j += 7) {  // seven independent 16-B loads in flight (7x7 maps: one batch per row)
      uint4 v[7];
#pragma unroll
      for (int u = 0; u < 7; ++u) v[u] = p[static_cast<long>(j + u) * C8];
#pragma unroll
      for (int u = 0; u < 7; ++u) add(v[u]);
    }
    for (; j < HW; ++j) add(p[static_cast<long>(j) * C8]);
    reinterpret_cast<uint4*>(y)[i] = make_uint4(pack2<F16>(acc[0] * inv, acc[1] * inv), pack2<F16>(acc[2] * inv, acc[3] * inv),
                                                pack2<F16>(acc[4] * inv, acc[5] * inv), pack2<F16>(acc[6] * inv, acc[7] * inv));
  }
}

inline int grid_for(long work) {
  long g = (work + 255) / 256;
  return static_cast<int>(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace

AI4E_API int ai4e_preprocess_u8(const void* in, void* out, long npix, int cin, const float* mean8, const float* std8,
                                float scale, hipStream_t s) {
  if (cin < 1 || cin > 8) return AI4E_EINVAL;
  float4 ml = make_float4(mean8[0], mean8[1], mean8[2], mean8[3]), mh = make_float4(mean8[4], mean8[5], mean8[6], mean8[7]);
  float4 il = make_float4(1.f / std8[0], 1.f / std8[1], 1.f / std8[2], 1.f / std8[3]);
  float4 ih = make_float4(1.f / std8[4], 1.f / std8[5], 1.f / std8[6], 1.f / std8[7]);
  hipLaunchKernelGGL(preprocess_u8_kernel, dim3(grid_for(npix)), dim3(256), 0, s, static_cast<const uint8_t*>(in),
                     static_cast<uint16_t*>(out), npix, cin, ml, mh, il, ih, scale);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

namespace {

template <bool F16>
int preprocess_s2d_impl(const void* in, void* out, int N, int H, int W, int cin, const float* mean4, const float* std4,
                        float scale, hipStream_t s) {
  if (cin < 1 || cin > 4 || (H & 1) || (W & 1)) return AI4E_EINVAL;
  float4 m = make_float4(mean4[0], mean4[1], mean4[2], mean4[3]);
  float4 is = make_float4(1.f / std4[0], 1.f / std4[1], 1.f / std4[2], 1.f / std4[3]);
  const long total = static_cast<long>(N) * (H / 2) * (W / 2);
  const dim3 grid(grid_for(total));
  const uint8_t* i8 = static_cast<const uint8_t*>(in);
  uint16_t* o16 = static_cast<uint16_t*>(out);
  const bool small = total < (1L << 31) - 65536L * 256;
  if (small && cin == 3) {
    hipLaunchKernelGGL((preprocess_s2d_kernel<3, int, F16>), grid, dim3(256), 0, s, i8, o16, N, H, W, cin, m, is, scale);
  } else if (small && cin == 4) {
    hipLaunchKernelGGL((preprocess_s2d_kernel<4, int, F16>), grid, dim3(256), 0, s, i8, o16, N, H, W, cin, m, is, scale);
  } else {
    hipLaunchKernelGGL((preprocess_s2d_kernel<0, long, F16>), grid, dim3(256), 0, s, i8, o16, N, H, W, cin, m, is, scale);
  }
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

template <bool F16>
int maxpool_impl(const void* x, void* y, int N, int H, int W, int C, int OH, int OW, int k, int stride, int pad, int ldx,
                 hipStream_t s) {
  if (C % 8 || ldx % 8 || ldx < C) return AI4E_EINVAL;
  const long total = static_cast<long>(N) * OH * OW * (C / 8);
  if (total < (1L << 31) - 8192L * 256)
    hipLaunchKernelGGL((maxpool_kernel<int, F16>), dim3(grid_for(total)), dim3(256), 0, s,
                       static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), N, H, W, C, OH, OW, k, stride, pad,
                       ldx / 8);
  else
    hipLaunchKernelGGL((maxpool_kernel<long, F16>), dim3(grid_for(total)), dim3(256), 0, s,
                       static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), N, H, W, C, OH, OW, k, stride, pad,
                       ldx / 8);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

template <bool F16>
int avgpool_impl(const void* x, void* y, int N, int HW, int C, hipStream_t s) {
  if (C % 8) return AI4E_EINVAL;
  hipLaunchKernelGGL((avgpool_kernel<F16>), dim3(grid_for(static_cast<long>(N) * (C / 8))), dim3(256), 0, s,
                     static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), N, HW, C);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

}  // namespace

// uint8 [N,H,W,cin<=4] -> s2d [N,H/2,W/2,16] bf16 (f16 != 0: fp16).
AI4E_API int ai4e_preprocess_s2d_u8(const void* in, void* out, int N, int H, int W, int cin, const float* mean4,
                                    const float* std4, float scale, hipStream_t s) {
  return preprocess_s2d_impl<false>(in, out, N, H, W, cin, mean4, std4, scale, s);
}
AI4E_API int ai4e_preprocess_s2d_u8_dt(const void* in, void* out, int N, int H, int W, int cin, const float* mean4,
                                       const float* std4, float scale, int f16, hipStream_t s) {
  return f16 ? preprocess_s2d_impl<true>(in, out, N, H, W, cin, mean4, std4, scale, s)
             : preprocess_s2d_impl<false>(in, out, N, H, W, cin, mean4, std4, scale, s);
}

// x may be a channel slice of a wider NHWC buffer: row stride ldx (elements), x points at the slice start.
AI4E_API int ai4e_maxpool2d(const void* x, void* y, int N, int H, int W, int C, int OH, int OW, int k, int stride,
                            int pad, int ldx, hipStream_t s) {
  return maxpool_impl<false>(x, y, N, H, W, C, OH, OW, k, stride, pad, ldx, s);
}
AI4E_API int ai4e_maxpool2d_dt(const void* x, void* y, int N, int H, int W, int C, int OH, int OW, int k, int stride,
                               int pad, int ldx, int f16, hipStream_t s) {
  return f16 ? maxpool_impl<true>(x, y, N, H, W, C, OH, OW, k, stride, pad, ldx, s)
             : maxpool_impl<false>(x, y, N, H, W, C, OH, OW, k, stride, pad, ldx, s);
}

AI4E_API int ai4e_global_avgpool(const void* x, void* y, int N, int HW, int C, hipStream_t s) {
  return avgpool_impl<false>(x, y, N, HW, C, s);
}
AI4E_API int ai4e_global_avgpool_dt(const void* x, void* y, int N, int HW, int C, int f16, hipStream_t s) {
  return f16 ? avgpool_impl<true>(x, y, N, HW, C, s) : avgpool_impl<false>(x, y, N, HW, C, s);
}
