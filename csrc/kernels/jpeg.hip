// On-GPU JPEG reconstruction for camera-trap ingest (survey §5.8(4) / §7.5.4): a batch of baseline JPEG frames goes
// from the prepared scan (csrc/core/jpeg_coef.h prepare(): headers, lookup tables, unstuffed entropy-coded bits) to the
// model's uint8 HWC input with no CPU work beyond that copy:
//
//   huff_sync x (1 + N) / huff_fixup / huff_prefix / huff_write   parallel Huffman decoding (csrc/core/jpeg_span.h);
//               huff_fixup finishes, one wave per frame, the spans the N sync passes left unsettled (usually none)
//   idct        dequantisation + libjpeg's scaled IDCT per 8x8 block (8x8 ISLOW, 4x4 / 2x2 / 1x1 reduced), clearing
//               the coefficients it read (the array stays zero between batches)
//   color_h     YCbCr -> RGB (libjpeg's fixed-point tables) fused into PIL's horizontal bilinear pass
//   resize_v    PIL's vertical bilinear pass, into the model input
//
// Every step reproduces the CPU path bit for bit: PIL's draft decode (libjpeg-turbo, DCT-domain 1/2..1/8 scaling, the
// chroma IDCT scaled up instead of upsampled) followed by Image.resize(BILINEAR) with its 22-bit fixed-point
// coefficients (runtime/decode.py decode_image; runtime/jpeg_gpu.py builds the coefficient tables on the host).
// Frames are independent: blockIdx.y is the frame of the batch (JpegFrameDesc).
#define AI4E_HD __host__ __device__
#define AI4E_GAS __attribute__((address_space(1)))
#include "common.h"
#include "../core/jpeg_span.h"

namespace {

using ai4e::GpuHuff;
using ai4e::JpegFrameDesc;
using ai4e::JpegScanHeader;
using ai4e::JSpanResult;
using ai4e::JSpanTables;
using ai4e::kGpuLook;

__device__ const uint8_t kNatural[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
    6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
    39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

constexpr int kThreads = 256;

// zigzag -> natural, as a compile-time table (the IDCT's unrolled de-zigzag keeps every index constant)
constexpr uint8_t kNat64[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                                41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                                30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct SpanLds {
  uint32_t lut[4 << kGpuLook];  // 16 KB: the frame's 2 DC + 2 AC lookahead tables
  uint8_t natural[80];
  uint8_t btab[16];
};

// Stage the frame's lookup tables in LDS (every thread of the block) and build the span decoder's view of the frame.
__device__ __forceinline__ JSpanTables stage_tables(const JpegFrameDesc& D, SpanLds& L) {
  const auto* H = reinterpret_cast<const JpegScanHeader*>(D.scan);
  const uint4* src_dc = reinterpret_cast<const uint4*>(H->dc[0].fast);
  constexpr int kPerTab = (1 << kGpuLook) / 4;                 // uint4 per fast table
  constexpr int kStride = sizeof(GpuHuff) / sizeof(uint4);     // uint4 per GpuHuff
  uint4* dst = reinterpret_cast<uint4*>(L.lut);
  for (int i = threadIdx.x; i < 4 * kPerTab; i += blockDim.x) {
    const int t = i / kPerTab, j = i - t * kPerTab;
    dst[i] = src_dc[t * kStride + j];
  }
  for (int i = threadIdx.x; i < 80; i += blockDim.x) L.natural[i] = kNatural[i];
  if (threadIdx.x < 16) {
    const uint32_t k = threadIdx.x;
    const int c = k < H->bpm ? min(static_cast<int>(H->blk_comp[k]), 2) : 0;
    L.btab[k] = static_cast<uint8_t>((H->comp[c][6] & 1) | ((H->comp[c][7] & 1) << 2) | (c << 4));
  }
  __syncthreads();
  JSpanTables T;
  T.lut = L.lut;
  T.huff = (const AI4E_GAS GpuHuff*)(H->dc);  // (generic -> global: a C-style address-space cast)
  T.blk_tab = L.btab;
  T.natural = L.natural;
  T.words = (const AI4E_GAS uint32_t*)(reinterpret_cast<const uint8_t*>(H) + sizeof(JpegScanHeader));
  T.nwords = static_cast<uint32_t>((H->scan_bytes + ai4e::kJpegScanPad) / 4);
  T.bpm = static_cast<int>(H->bpm);
  return T;
}

__device__ __forceinline__ uint32_t span_end(const JpegFrameDesc& D, int t) {
  const auto* H = reinterpret_cast<const JpegScanHeader*>(D.scan);
  const uint64_t e = static_cast<uint64_t>(t + 1) * static_cast<uint32_t>(D.span_bits);
  return e < H->total_bits ? static_cast<uint32_t>(e) : H->total_bits;
}

__device__ __forceinline__ void store_counts(const JpegFrameDesc& D, int t, const JSpanResult& r) {
  reinterpret_cast<int4*>(D.counts)[t] = make_int4(r.nblk, r.dc[0], r.dc[1], r.dc[2]);
}

// pass 0 (pass == 0): every span from a guessed state; pass k: re-decode span t from span t-1's exit state of pass k-1
// when that state changed in pass k-1 (pass 1: always).
__global__ __launch_bounds__(kThreads) void huff_sync_kernel(const JpegFrameDesc* __restrict__ descs, int pass) {
  const JpegFrameDesc& D = descs[blockIdx.y];
  const int t = blockIdx.x * kThreads + threadIdx.x;
  const int in = (pass - 1) & 1, out = pass & 1;
  auto* ex_in = reinterpret_cast<const uint64_t*>(D.exit[in]);
  auto* ex_out = reinterpret_cast<uint64_t*>(D.exit[out]);
  auto* chg_in = reinterpret_cast<const uint32_t*>(D.chg[in]);
  auto* chg_out = reinterpret_cast<uint32_t*>(D.chg[out]);
  bool work = t < D.nthreads;
  if (pass > 0 && work) {
    if (t == 0 || (pass >= 2 && !chg_in[t - 1])) {  // same entry state as last pass: same exit
      ex_out[t] = ex_in[t];
      chg_out[t] = 0;
      work = false;
    }
  }
  if (!__syncthreads_or(work)) return;  // the whole workgroup is settled: skip staging the tables
  __shared__ SpanLds L;
  const JSpanTables T = stage_tables(D, L);
  if (!work) return;
  uint32_t pos;
  int z, cp;
  if (pass == 0) {
    pos = static_cast<uint32_t>(t) * static_cast<uint32_t>(D.span_bits);
    z = cp = 0;
  } else {
    const uint64_t s = ex_in[t - 1];
    pos = ai4e::jspan_pos(s);
    z = ai4e::jspan_z(s);
    cp = ai4e::jspan_cp(s);
  }
  JSpanResult r;
  ai4e::jspan_decode<false>(T, pos, z, cp, span_end(D, t), r);
  ex_out[t] = r.exit;
  chg_out[t] = pass == 0 ? 1u : static_cast<uint32_t>(r.exit != ex_in[t]);
  store_counts(D, t, r);
}

// After the sync passes: walk the frame's spans in order and re-decode, sequentially, every span whose entry state is
// still stale (the predecessor changed in the last pass, or was re-decoded here with a new exit). One wave per frame;
// the wave skips 64 settled spans per step, so a settled frame costs ~nthreads / 64 loads. Makes every valid frame's
// states exact however slowly its spans synchronise.
__global__ __launch_bounds__(64) void huff_fixup_kernel(const JpegFrameDesc* __restrict__ descs, int last) {
  const JpegFrameDesc& D = descs[blockIdx.y];
  auto* ex = reinterpret_cast<uint64_t*>(D.exit[last & 1]);
  auto* chg = reinterpret_cast<uint32_t*>(D.chg[last & 1]);
  const int n = D.nthreads;
  int first = -1;
  for (int b = 0; b < n - 1 && first < 0; b += 64) {
    const int i = b + static_cast<int>(threadIdx.x);
    const uint64_t m = __ballot(i < n - 1 && chg[i] != 0);
    if (m) first = b + __ffsll(static_cast<long long>(m)) - 1;
  }
  if (first < 0) return;  // settled (wave-uniform)
  __shared__ SpanLds L;
  const JSpanTables T = stage_tables(D, L);
  if (threadIdx.x != 0) return;
  bool dirty = false;  // span t-1 was re-decoded here with a different exit
  for (int t = first + 1; t < n; ++t) {
    if (!dirty && !chg[t - 1]) continue;
    chg[t - 1] = 0;
    const uint64_t s = ex[t - 1];
    JSpanResult r;
    ai4e::jspan_decode<false>(T, ai4e::jspan_pos(s), ai4e::jspan_z(s), ai4e::jspan_cp(s), span_end(D, t), r);
    dirty = r.exit != ex[t];
    ex[t] = r.exit;
    store_counts(D, t, r);
  }
  if (n >= 1) chg[n - 1] = 0;
}

// Exclusive prefix over the frame's spans of (blocks completed, DC sums): one workgroup per frame.
__global__ __launch_bounds__(kThreads) void huff_prefix_kernel(const JpegFrameDesc* __restrict__ descs) {
  const JpegFrameDesc& D = descs[blockIdx.y];
  int4* cnt = reinterpret_cast<int4*>(D.counts);
  const int n = D.nthreads;
  const int per = (n + kThreads - 1) / kThreads;
  const int b = threadIdx.x * per, e = min(n, b + per);
  int4 s = make_int4(0, 0, 0, 0);
  for (int i = b; i < e; ++i) {
    const int4 v = cnt[i];
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  __shared__ int4 part[kThreads];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < kThreads; off <<= 1) {  // inclusive Hillis-Steele scan
    const int4 o = threadIdx.x >= off ? part[threadIdx.x - off] : make_int4(0, 0, 0, 0);
    __syncthreads();
    int4 v = part[threadIdx.x];
    v.x += o.x;
    v.y += o.y;
    v.z += o.z;
    v.w += o.w;
    part[threadIdx.x] = v;
    __syncthreads();
  }
  int4 acc = threadIdx.x ? part[threadIdx.x - 1] : make_int4(0, 0, 0, 0);
  for (int i = b; i < e; ++i) {
    const int4 v = cnt[i];
    cnt[i] = acc;
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  if (threadIdx.x == kThreads - 1) {
    const auto* H = reinterpret_cast<const JpegScanHeader*>(D.scan);
    if (part[kThreads - 1].x < static_cast<int>(H->nblocks)) atomicOr(reinterpret_cast<uint32_t*>(D.status), 2u);
  }
}

// Final pass: decode each span from its exact entry state into the dense coefficient array.
__global__ __launch_bounds__(kThreads) void huff_write_kernel(const JpegFrameDesc* __restrict__ descs, int last) {
  const JpegFrameDesc& D = descs[blockIdx.y];
  const int t = blockIdx.x * kThreads + threadIdx.x;
  const bool work = t < D.nthreads;
  if (!__syncthreads_or(work)) return;
  __shared__ SpanLds L;
  const JSpanTables T = stage_tables(D, L);
  if (!work) return;
  const auto* H = reinterpret_cast<const JpegScanHeader*>(D.scan);
  auto* ex = reinterpret_cast<const uint64_t*>(D.exit[last & 1]);
  auto* chg = reinterpret_cast<const uint32_t*>(D.chg[last & 1]);
  uint32_t* status = reinterpret_cast<uint32_t*>(D.status);
  if (t > 0 && chg[t - 1]) atomicOr(status, 1u);  // (cannot happen after the fix-up: kept as a guard)
  const uint64_t s = t ? ex[t - 1] : ai4e::jspan_pack(0, 0, 0);
  const int4 base = reinterpret_cast<const int4*>(D.counts)[t];
  const int32_t pred[3] = {base.y, base.z, base.w};
  JSpanResult r;
  ai4e::jspan_decode<true>(T, ai4e::jspan_pos(s), ai4e::jspan_z(s), ai4e::jspan_cp(s), span_end(D, t), r,
                           reinterpret_cast<AI4E_GAS int16_t*>(D.coef), base.x, pred, static_cast<int32_t>(H->nblocks),
                           reinterpret_cast<AI4E_GAS uint8_t*>(D.blen));
  if (r.bad) atomicOr(status, 2u);
}

// ---- scaled IDCTs (libjpeg jidctint.c / jidctred.c integer arithmetic; inputs dequantised) ----
constexpr int kConstBits = 13, kPass1Bits = 2;
__device__ __forceinline__ int descale(int64_t x, int n) { return static_cast<int>((x + (1ll << (n - 1))) >> n); }
__device__ __forceinline__ uint8_t range_limit(int x) {  // libjpeg's sample_range_limit[(x + 128) & 1023]
  const int y = (x + 128) & 1023;
  return static_cast<uint8_t>(y < 256 ? y : (y < 640 ? 255 : 0));
}

// 1-D 8-point ISLOW butterfly (jidctint.c); `shift` = the pass's descale
__device__ __forceinline__ void islow_1d(const int (&x)[8], int shift, int (&o)[8]) {
  int z2 = x[2], z3 = x[6];
  int z1 = (z2 + z3) * 4433;
  const int tmp2 = z1 - z3 * 15137, tmp3 = z1 + z2 * 6270;
  const int tmp0 = (x[0] + x[4]) * (1 << kConstBits), tmp1 = (x[0] - x[4]) * (1 << kConstBits);
  const int t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
  int o0 = x[7], o1 = x[5], o2 = x[3], o3 = x[1];
  z1 = o0 + o3;
  z2 = o1 + o2;
  z3 = o0 + o2;
  int z4 = o1 + o3;
  const int z5 = (z3 + z4) * 9633;
  o0 *= 2446;
  o1 *= 16819;
  o2 *= 25172;
  o3 *= 12299;
  z1 *= -7373;
  z2 *= -20995;
  z3 = z3 * -16069 + z5;
  z4 = z4 * -3196 + z5;
  o0 += z1 + z3;
  o1 += z2 + z4;
  o2 += z2 + z3;
  o3 += z1 + z4;
  o[0] = descale(t10 + o3, shift);
  o[7] = descale(t10 - o3, shift);
  o[1] = descale(t11 + o2, shift);
  o[6] = descale(t11 - o2, shift);
  o[2] = descale(t12 + o1, shift);
  o[5] = descale(t12 - o1, shift);
  o[3] = descale(t13 + o0, shift);
  o[4] = descale(t13 - o0, shift);
}

__device__ void idct8(const int (&d)[64], uint8_t* out, int pitch) {
  int ws[64];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    int x[8], o[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) x[r] = d[r * 8 + c];
    if ((x[1] | x[2] | x[3] | x[4] | x[5] | x[6] | x[7]) == 0) {
#pragma unroll
      for (int r = 0; r < 8; ++r) ws[r * 8 + c] = x[0] * (1 << kPass1Bits);
    } else {
      islow_1d(x, kConstBits - kPass1Bits, o);
#pragma unroll
      for (int r = 0; r < 8; ++r) ws[r * 8 + c] = o[r];
    }
  }
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    int x[8], o[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = ws[r * 8 + c];
    if ((x[1] | x[2] | x[3] | x[4] | x[5] | x[6] | x[7]) == 0) {
      const uint8_t v = range_limit(descale(x[0], kPass1Bits + 3));
#pragma unroll
      for (int c = 0; c < 8; ++c) o[c] = v;
    } else {
      islow_1d(x, kConstBits + kPass1Bits + 3, o);
#pragma unroll
      for (int c = 0; c < 8; ++c) o[c] = range_limit(o[c]);
    }
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      lo |= static_cast<uint32_t>(o[c] & 0xFF) << (8 * c);
      hi |= static_cast<uint32_t>(o[c + 4] & 0xFF) << (8 * c);
    }
    *reinterpret_cast<uint2*>(out + r * pitch) = make_uint2(lo, hi);
  }
}

// jidctred.c 4x4 (rows / columns 0-3, 5-7 of the 8x8 input)
__device__ __forceinline__ void red4_1d(const int (&x)[8], int s_even, int s_out, int (&o)[4]) {
  const int64_t tmp0 = static_cast<int64_t>(x[0]) << (kConstBits + 1);
  const int64_t tmp2 = static_cast<int64_t>(x[2]) * 15137 + static_cast<int64_t>(x[6]) * -6270;
  const int64_t t10 = tmp0 + tmp2, t12 = tmp0 - tmp2;
  const int64_t z1 = x[7], z2 = x[5], z3 = x[3], z4 = x[1];
  const int64_t e0 = z1 * -1730 + z2 * 11893 + z3 * -17799 + z4 * 8697;
  const int64_t e2 = z1 * -4176 + z2 * -4926 + z3 * 7373 + z4 * 20995;
  (void)s_even;
  o[0] = descale(t10 + e2, s_out);
  o[3] = descale(t10 - e2, s_out);
  o[1] = descale(t12 + e0, s_out);
  o[2] = descale(t12 - e0, s_out);
}

__device__ void idct4(const int (&d)[64], uint8_t* out, int pitch) {
  int ws[4 * 8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    if (c == 4) continue;
    int x[8], o[4];
#pragma unroll
    for (int r = 0; r < 8; ++r) x[r] = d[r * 8 + c];
    if ((x[1] | x[2] | x[3] | x[5] | x[6] | x[7]) == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) ws[r * 8 + c] = x[0] * (1 << kPass1Bits);
    } else {
      red4_1d(x, 0, kConstBits - kPass1Bits + 1, o);
#pragma unroll
      for (int r = 0; r < 4; ++r) ws[r * 8 + c] = o[r];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    int x[8], o[4];
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = c == 4 ? 0 : ws[r * 8 + c];
    if ((x[1] | x[2] | x[3] | x[5] | x[6] | x[7]) == 0) {
      const int v = descale(x[0], kPass1Bits + 3);
      o[0] = o[1] = o[2] = o[3] = v;
    } else {
      red4_1d(x, 0, kConstBits + kPass1Bits + 3 + 1, o);
    }
    uint32_t w = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) w |= static_cast<uint32_t>(range_limit(o[c])) << (8 * c);
    *reinterpret_cast<uint32_t*>(out + r * pitch) = w;
  }
}

// jidctred.c 2x2 (rows / columns 0, 1, 3, 5, 7)
__device__ void idct2(const int (&d)[64], uint8_t* out, int pitch) {
  int ws[2 * 8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    if (c == 2 || c == 4 || c == 6) continue;
    const int x0 = d[c], x1 = d[8 + c], x3 = d[24 + c], x5 = d[40 + c], x7 = d[56 + c];
    if ((x1 | x3 | x5 | x7) == 0) {
      ws[c] = ws[8 + c] = x0 * (1 << kPass1Bits);
      continue;
    }
    const int64_t t10 = static_cast<int64_t>(x0) << (kConstBits + 2);
    const int64_t t0 = static_cast<int64_t>(x7) * -5906 + static_cast<int64_t>(x5) * 6967 +
                       static_cast<int64_t>(x3) * -10426 + static_cast<int64_t>(x1) * 29692;
    ws[c] = descale(t10 + t0, kConstBits - kPass1Bits + 2);
    ws[8 + c] = descale(t10 - t0, kConstBits - kPass1Bits + 2);
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int* w = ws + r * 8;
    int a, b;
    if ((w[1] | w[3] | w[5] | w[7]) == 0) {
      a = b = descale(w[0], kPass1Bits + 3);
    } else {
      const int64_t t10 = static_cast<int64_t>(w[0]) << (kConstBits + 2);
      const int64_t t0 = static_cast<int64_t>(w[7]) * -5906 + static_cast<int64_t>(w[5]) * 6967 +
                         static_cast<int64_t>(w[3]) * -10426 + static_cast<int64_t>(w[1]) * 29692;
      a = descale(t10 + t0, kConstBits + kPass1Bits + 3 + 2);
      b = descale(t10 - t0, kConstBits + kPass1Bits + 3 + 2);
    }
    out[r * pitch] = range_limit(a);
    out[r * pitch + 1] = range_limit(b);
  }
}

// One thread per 8x8 block, planar order (a wave stays on one component: one IDCT size, contiguous plane rows).
__global__ __launch_bounds__(kThreads) void idct_kernel(const JpegFrameDesc* __restrict__ descs) {
  const JpegFrameDesc& D = descs[blockIdx.y];
  const auto* H = reinterpret_cast<const JpegScanHeader*>(D.scan);
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= static_cast<int>(H->nblocks)) return;
  const int ncomp = static_cast<int>(H->ncomp);
  const int c = (ncomp > 1 && i >= static_cast<int>(H->comp[1][4])) + (ncomp > 2 && i >= static_cast<int>(H->comp[2][4]));
  const uint32_t* C = H->comp[c];
  const int h = static_cast<int>(C[0]), v = static_cast<int>(C[1]), bw = static_cast<int>(C[2]);
  const int li = i - static_cast<int>(C[4]);
  const int row = li / bw, col = li - row * bw;
  const int m = (row / v) * static_cast<int>(H->mcux) + col / h;
  const int kb = c == 0 ? 0 : (c == 1 ? D.kbase1 : D.kbase2);
  const int k = kb + (row % v) * h + (col % h);
  const int64_t q = static_cast<int64_t>(m) * static_cast<int64_t>(H->bpm) + k;
  // the block's zigzag prefix only (a frame flagged corrupt: all 64, whatever its spans wrote); cleared behind us
  uint4* src = reinterpret_cast<uint4*>(reinterpret_cast<int16_t*>(D.coef) + q * 64);
  uint8_t* bl = reinterpret_cast<uint8_t*>(D.blen) + q;
  const int len = *reinterpret_cast<const uint32_t*>(D.status) ? 64 : *bl;
  const int nchunk = (len + 7) >> 3;
  *bl = 0;
  const uint16_t* qt = H->quant[C[5]];
  int zz[64];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint4 w = make_uint4(0, 0, 0, 0);
    if (j < nchunk) {
      w = src[j];
      src[j] = make_uint4(0, 0, 0, 0);
    }
    const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int h2 = 0; h2 < 4; ++h2) {
      zz[8 * j + 2 * h2] = static_cast<int16_t>(ww[h2] & 0xFFFF);
      zz[8 * j + 2 * h2 + 1] = static_cast<int16_t>(ww[h2] >> 16);
    }
  }
  int d[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) d[kNat64[k]] = zz[k] * static_cast<int>(qt[kNat64[k]]);
  const int ss = D.ssize[c];
  uint8_t* out = reinterpret_cast<uint8_t*>(D.planes) + D.plane_off[c] + static_cast<int64_t>(row) * ss * D.plane_pitch[c] +
                 col * ss;
  if (ss == 8) {
    idct8(d, out, D.plane_pitch[c]);
  } else if (ss == 4) {
    idct4(d, out, D.plane_pitch[c]);
  } else if (ss == 2) {
    idct2(d, out, D.plane_pitch[c]);
  } else {
    out[0] = range_limit(descale(d[0], 3));
  }
}

// libjpeg ycc_rgb_convert (jdcolor.c tables, SCALEBITS 16)
__device__ __forceinline__ void ycc_rgb(int y, int cb, int cr, int& r, int& g, int& b) {
  cb -= 128;
  cr -= 128;
  r = y + ((91881 * cr + 32768) >> 16);
  g = y + ((-22554 * cb - 46802 * cr + 32768) >> 16);
  b = y + ((116130 * cb + 32768) >> 16);
  r = min(max(r, 0), 255);
  g = min(max(g, 0), 255);
  b = min(max(b, 0), 255);
}

__device__ __forceinline__ uint8_t clip22(int acc) {  // PIL clip8 (PRECISION_BITS 22)
  const int v = acc >> 22;
  return static_cast<uint8_t>(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// rows[y][xo] = PIL horizontal bilinear pass over the RGB (or grey) pixels of source row y.
__global__ __launch_bounds__(kThreads) void color_h_kernel(const JpegFrameDesc* __restrict__ descs) {
  const JpegFrameDesc& D = descs[blockIdx.y];
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (idx >= static_cast<int64_t>(D.src_h) * D.out_w) return;
  const int y = static_cast<int>(idx / D.out_w), xo = static_cast<int>(idx - static_cast<int64_t>(y) * D.out_w);
  const auto* H = reinterpret_cast<const JpegScanHeader*>(D.scan);
  const int* hb = reinterpret_cast<const int*>(D.hb) + 2 * xo;
  const int* hk = reinterpret_cast<const int*>(D.hk) + xo * D.hks;
  const uint8_t* P = reinterpret_cast<const uint8_t*>(D.planes);
  const uint8_t* py = P + D.plane_off[0] + static_cast<int64_t>(y) * D.plane_pitch[0];
  const bool color = H->ncomp == 3;
  const uint8_t* pcb = P + D.plane_off[1] + static_cast<int64_t>(y) * D.plane_pitch[1];
  const uint8_t* pcr = P + D.plane_off[2] + static_cast<int64_t>(y) * D.plane_pitch[2];
  int a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21;
  const int x0 = hb[0], n = hb[1];
  uint8_t* o = reinterpret_cast<uint8_t*>(D.rows) + idx * D.out_c;
  if (D.out_c == 1 || !color) {
    for (int j = 0; j < n; ++j) a0 += hk[j] * static_cast<int>(py[x0 + j]);
    const uint8_t v = clip22(a0);
    o[0] = v;
    if (D.out_c == 3) {
      o[1] = v;
      o[2] = v;
    }
    return;
  }
  for (int j = 0; j < n; ++j) {
    int r, g, b;
    ycc_rgb(py[x0 + j], pcb[x0 + j], pcr[x0 + j], r, g, b);
    const int k = hk[j];
    a0 += k * r;
    a1 += k * g;
    a2 += k * b;
  }
  o[0] = clip22(a0);
  o[1] = clip22(a1);
  o[2] = clip22(a2);
}

// PIL's vertical pass: 4 output bytes per thread (one 32-bit load per tap per lane, the bytes being independent
// channels / pixels with the same row weights) when a row is a multiple of 4 bytes, else one byte per thread.
__global__ __launch_bounds__(kThreads) void resize_v_kernel(const JpegFrameDesc* __restrict__ descs) {
  const JpegFrameDesc& D = descs[blockIdx.y];
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  const int64_t per_row = static_cast<int64_t>(D.out_w) * D.out_c;
  const bool quad = (per_row & 3) == 0;
  const int64_t units = quad ? per_row >> 2 : per_row;
  if (idx >= static_cast<int64_t>(D.out_h) * units) return;
  const int yo = static_cast<int>(idx / units);
  const int64_t xu = idx - yo * units;
  const int* vb = reinterpret_cast<const int*>(D.vb) + 2 * yo;
  const int* vk = reinterpret_cast<const int*>(D.vk) + yo * D.vks;
  const int y0 = vb[0], n = vb[1];
  if (quad) {
    const uint32_t* rows = reinterpret_cast<const uint32_t*>(D.rows) + xu;
    const int64_t pitch = per_row >> 2;
    int a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21, a3 = 1 << 21;
    for (int j = 0; j < n; ++j) {
      const uint32_t v = rows[static_cast<int64_t>(y0 + j) * pitch];
      const int k = vk[j];
      a0 += k * static_cast<int>(v & 0xFF);
      a1 += k * static_cast<int>((v >> 8) & 0xFF);
      a2 += k * static_cast<int>((v >> 16) & 0xFF);
      a3 += k * static_cast<int>(v >> 24);
    }
    // (the empty asm keeps the clamp + pack from being matched to v_ashr_pk_u8_i32: measured, that packing left
    // the upper half of the word holding stale register bits, i.e. bytes 2-3 of every output word garbage)
    uint32_t b0 = clip22(a0), b1 = clip22(a1), b2 = clip22(a2), b3 = clip22(a3);
    asm volatile("" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));
    reinterpret_cast<uint32_t*>(D.out)[static_cast<int64_t>(yo) * pitch + xu] = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    return;
  }
  const uint8_t* rows = reinterpret_cast<const uint8_t*>(D.rows) + xu;
  int acc = 1 << 21;
  for (int j = 0; j < n; ++j) acc += vk[j] * static_cast<int>(rows[static_cast<int64_t>(y0 + j) * per_row]);
  reinterpret_cast<uint8_t*>(D.out)[static_cast<int64_t>(yo) * per_row + xu] = clip22(acc);
}

}  // namespace

// descs: device array of `nframes` JpegFrameDesc. max_threads / max_blocks / max_rows_px (src_h * out_w) / max_out
// (out_h * out_w * out_c): maxima over the frames (grid sizes). sync_passes: parallel re-decode passes after the
// speculative one; what they leave unsettled the fix-up kernel finishes sequentially.
AI4E_API int ai4e_jpeg_decode(const void* descs, int nframes, int max_threads, int max_blocks, long max_rows_px,
                              long max_out, int sync_passes, hipStream_t stream) {
  if (nframes <= 0 || nframes > 65535 || max_threads <= 0 || max_blocks <= 0 || sync_passes < 1 || sync_passes > 64)
    return AI4E_EINVAL;
  const auto* d = static_cast<const JpegFrameDesc*>(descs);
  const dim3 blk(kThreads);
  const dim3 gs((max_threads + kThreads - 1) / kThreads, nframes);
  for (int p = 0; p <= sync_passes; ++p) hipLaunchKernelGGL(huff_sync_kernel, gs, blk, 0, stream, d, p);
  hipLaunchKernelGGL(huff_fixup_kernel, dim3(1, nframes), dim3(64), 0, stream, d, sync_passes);
  hipLaunchKernelGGL(huff_prefix_kernel, dim3(1, nframes), blk, 0, stream, d);
  hipLaunchKernelGGL(huff_write_kernel, gs, blk, 0, stream, d, sync_passes);
  hipLaunchKernelGGL(idct_kernel, dim3((max_blocks + kThreads - 1) / kThreads, nframes), blk, 0, stream, d);
  hipLaunchKernelGGL(color_h_kernel, dim3(static_cast<unsigned>((max_rows_px + kThreads - 1) / kThreads), nframes),
                     blk, 0, stream, d);
  hipLaunchKernelGGL(resize_v_kernel, dim3(static_cast<unsigned>((max_out + kThreads - 1) / kThreads), nframes), blk,
                     0, stream, d);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}
