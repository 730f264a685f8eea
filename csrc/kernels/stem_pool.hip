// K1s — ResNet stem: the space-to-depth 4x4/1 conv (BN folded, + bias, ReLU) fused with the 3x3/2 pad-1
// max-pool that follows it. The 112x112x64 stem activation (411 MB at batch 256) never reaches HBM.
//
// Each workgroup owns a 7 x 8 tile of POOLED outputs of one image; the conv region that tile's pooling
// windows cover is 15 x 17 = 255 conv pixels (recompute factor 255/224 = 1.14 over the unfused conv).
// Those 255 (+1 idle) pixels are the M rows of one 256 x 64 implicit-GEMM tile on MFMA
// (v_mfma_f32_16x16x32_bf16, 4 wave64s x 64 pixels, the K1 LDS-DMA ring with counted vmcnt). The
// epilogue writes relu(acc + b) as bf16 into LDS (conv pixels outside the image write 0: post-ReLU
// values are >= 0, so a 0 never wins a max over a window that always holds a real pixel), then every
// thread max-reduces 3x3 windows of 16-B channel chunks (integer max on the bf16 bits: non-negative bf16
// order like unsigned integers) and stores 16-B pooled chunks.
//
// Input: the s2d layout of preprocess_s2d (ops/pool.py) [N, H, W, 16] bf16, K = (kh, kw, c) = 4x4x16 = 256
// padded top/left 1 (bottom/right 2: bounds-checked). Output [N, PH, PW, 64], PH = ceil(H/2).
#include <cstdlib>

#include "conv_common.h"

namespace {

using ai4e_conv::BK;
using ai4e_conv::glds16;
using ai4e_conv::swz;
using ai4e_conv::wait_vmcnt;

__device__ __attribute__((aligned(64))) uint16_t g_stem_zero[32];

constexpr int SP_TR = 7, SP_TC = 8;                        // pooled tile
constexpr int SP_RR = 2 * SP_TR + 1, SP_RC = 2 * SP_TC + 1;  // conv region 15 x 17
constexpr int SP_STAGES = 4;
constexpr int SP_BM = 256, SP_BN = 64, SP_C = 16, SP_NK = 256 / BK;  // 8 K steps

struct StemParams {
  const uint16_t* x;   // [N, H, W, 16]
  const uint16_t* w;   // [>= 64 rows, kpad >= 256]
  const float* bias;   // [64]
  uint16_t* y;         // [N, PH, PW, 64]
  const uint16_t* zero;
  int H, W, PH, PW, kpad, tiles_r, tiles_c;
  // fused next 1x1 (the first bottleneck's c1, 64 -> 64, + bias, ReLU) on the pooled tile (null = off):
  // t1 [N, PH, PW, 64] = relu(y . W1^T + b1), W1 [>= 64 rows, kpad1 >= 64]
  const uint16_t* w1;
  const float* b1;
  uint16_t* t1;
  int kpad1;
  // U8 (direct kernel): the footprint is built from the uint8 RGB images [N, 2H, 2W, 3] instead of the s2d tensor:
  // s2d channel (dy * 2 + dx) * 3 + c of pixel (i, j) = (x8[2i + dy - 1, 2j + dx - 1, c] * scale - mean_c) * istd_c
  // (zero outside the image), the preprocess_s2d_kernel's arithmetic, so the preprocess launch and its 100 MB bf16
  // round trip disappear; pixels i = H / j = W are built as well (the exact 7x7/2 conv at the bottom / right edge)
  const uint8_t* x8;
  float pm[3], pis[3], pscale;
};

typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t max_bf16x2(uint32_t a, uint32_t b) {
  // both halves non-negative bf16: unsigned 16-bit max per half, one v_pk_max_u16
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2_t, a), __builtin_bit_cast(u16x2_t, b)));
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void stem_pool_kernel(const StemParams p) {
  constexpr int STAGE_ELEMS = (SP_BM + SP_BN) * BK;
  __shared__ __attribute__((aligned(1024))) uint16_t smem[SP_STAGES * STAGE_ELEMS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int per_img = p.tiles_r * p.tiles_c;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int img = t / per_img;
  const int tr = (t - img * per_img) / p.tiles_c;
  const int tc = t - img * per_img - tr * p.tiles_c;
  const int ph0 = tr * SP_TR, pw0 = tc * SP_TC;
  const int oh0 = 2 * ph0 - 1, ow0 = 2 * pw0 - 1;  // conv region origin

  // DMA lanes: row rin of a 16-row block, logical 8-element chunk c of the 32-wide K step
  const int rin = lane >> 2;
  const int c = (lane & 3) ^ swz(rin);
  int ihb[4], iwb[4];
  const uint16_t* const xi = p.x + static_cast<long>(img) * p.H * p.W * SP_C;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = 16 * (wave + 4 * i) + rin;
    const int r = m / SP_RC, cc = m - r * SP_RC;
    // conv pixel (oh0 + r, ow0 + cc); its tap (kh, kw) reads input (oh - 1 + kh, ow - 1 + kw)
    const bool live = m < SP_RR * SP_RC && oh0 + r >= 0 && oh0 + r < p.H && ow0 + cc >= 0 && ow0 + cc < p.W;
    ihb[i] = live ? oh0 + r - 1 : -(1 << 28);
    iwb[i] = ow0 + cc - 1;
  }
  const uint16_t* const wsrc = p.w + static_cast<long>(16 * wave + rin) * p.kpad + 8 * c;
  const uint32_t smem_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem));

  // K step kt: kh = kt / 2, the chunk's tap kw = 2 * (kt % 2) + (c >> 1), channels 8 * (c & 1)
  auto issue_stage = [&](int kt) {
    const uint32_t sbase = smem_base + (kt % SP_STAGES) * STAGE_ELEMS * 2;
    const int kh = kt >> 1, kw = 2 * (kt & 1) + (c >> 1);
    const bool kt_ok = kt < SP_NK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ih = ihb[i] + kh, iw = iwb[i] + kw;
      const bool ok = kt_ok && static_cast<unsigned>(ih) < static_cast<unsigned>(p.H) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(p.W);
      glds16(ok ? static_cast<const void*>(xi + (static_cast<long>(ih) * p.W + iw) * SP_C + 8 * (c & 1)) : p.zero,
             sbase + (16 * (wave + 4 * i)) * BK * 2);
    }
    glds16(kt_ok ? static_cast<const void*>(wsrc + kt * BK) : p.zero, sbase + (SP_BM + 16 * wave) * BK * 2);
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int frow = lane & 15;
  const int fofs = frow * BK + (((lane >> 4) ^ swz(frow)) << 3);
  constexpr int PER_STAGE = 5;

#pragma unroll
  for (int s = 0; s < SP_STAGES - 1; ++s) issue_stage(s);
#pragma unroll
  for (int kt = 0; kt < SP_NK; ++kt) {
    // stage kt landed: the younger stages in flight are kt+1 .. min(kt+2, NK-1)
    ai4e_conv::wait_vmcnt_n(PER_STAGE * min(SP_STAGES - 2, SP_NK - 1 - kt));
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const uint16_t* st = smem + (kt % SP_STAGES) * STAGE_ELEMS;
    bf16x8_t fw[4], fx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) fw[j] = *reinterpret_cast<const bf16x8_t*>(st + (SP_BM + 16 * j) * BK + fofs);
#pragma unroll
    for (int i = 0; i < 4; ++i) fx[i] = *reinterpret_cast<const bf16x8_t*>(st + (wave * 64 + 16 * i) * BK + fofs);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[j], fx[i], acc[i][j], 0, 0, 0);
    if (kt + SP_STAGES - 1 < SP_NK) issue_stage(kt + SP_STAGES - 1);
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // ring idle

  // ---- epilogue: bf16 relu(acc + b) -> LDS [256 px][64 ch] (128-B rows, 16-B chunk ^= px & 7)
  uint8_t* const tile = reinterpret_cast<uint8_t*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = wave * 64 + 16 * i + (lane & 15);
    const int r = m / SP_RC, cc = m - r * SP_RC;
    const bool live = m < SP_RR * SP_RC && oh0 + r >= 0 && oh0 + r < p.H && ow0 + cc >= 0 && ow0 + cc < p.W;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = 16 * j + 4 * (lane >> 4);
      const float4 b = *reinterpret_cast<const float4*>(p.bias + n);
      uint2 v = make_uint2(0u, 0u);
      if (live)
        v = make_uint2(pack_bf16x2(fmaxf(acc[i][j][0] + b.x, 0.f), fmaxf(acc[i][j][1] + b.y, 0.f)),
                       pack_bf16x2(fmaxf(acc[i][j][2] + b.z, 0.f), fmaxf(acc[i][j][3] + b.w, 0.f)));
      *reinterpret_cast<uint2*>(tile + m * 128 + ((((n >> 3) ^ (m & 7)) << 4) | (((n >> 2) & 1) << 3))) = v;
    }
  }
  __syncthreads();
  // ---- 3x3/2 max over the region: task = (pooled pixel q, 8-channel chunk k8)
  for (int task = tid; task < SP_TR * SP_TC * 8; task += 256) {
    const int q = task >> 3, k8 = task & 7;
    const int py = q / SP_TC, px = q - py * SP_TC;
    const int ph = ph0 + py, pw = pw0 + px;
    if (ph >= p.PH || pw >= p.PW) continue;
    uint4 mx = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int m = (2 * py + dy) * SP_RC + 2 * px + dx;
        const uint4 v = *reinterpret_cast<const uint4*>(tile + m * 128 + ((k8 ^ (m & 7)) << 4));
        mx.x = max_bf16x2(mx.x, v.x);
        mx.y = max_bf16x2(mx.y, v.y);
        mx.z = max_bf16x2(mx.z, v.z);
        mx.w = max_bf16x2(mx.w, v.w);
      }
    ai4e_conv::st16_stream(p.y + ((static_cast<long>(img) * p.PH + ph) * p.PW + pw) * SP_BN + 8 * k8, mx);
  }
}


// ---- v2: direct conv from the input footprint in LDS (persistent workgroups).
// The 15x17 conv region of a tile reads an 18x20 input footprint (the 4x4 taps overlap 16-fold), so
// instead of gathering 16 taps x 255 pixels through the DMA ring (128 KB per tile) the footprint is
// DMA'd once (360 pixels x 32 B = 11.25 KB, zero outside the image) and every MFMA operand fragment is
// read straight from it: the K step kt covers taps 2kt, 2kt+1 of filter row kt/2, a lane group g reads
// the 8 channels 8(g&1) of tap 2kt + (g>>1) of its pixel. The footprint is stored as two channel planes
// (channels 0-7 | 8-15, 16 B per pixel) so 16 lanes reading 16 consecutive pixels hit 16 distinct bank
// quads. The 64 x 256 weights (32 KB) stay in LDS for the whole persistent loop, each 512-B row with its
// 16-B chunk index XOR (row & 31) so the 16 rows of a fragment read hit distinct bank quads.
// Footprint 18 x 20 pixels stored with a row stride of FP_C = 21 slots (column 20 unused). The MFMA fragments
// cover the 15 x 17 conv region as 15 row fragments (row r, columns 0..15: 16 consecutive slots) plus one column
// fragment (column 16 of rows 0..14: slots 21 r, and 21 = 5 (mod 16) is odd, so 16 rows hit 16 distinct bank
// quads). Every fragment read of the main loop is then conflict-free for the gfx950 ds_read_b128 lane groups
// (round 2's row-major fragments of 16 consecutive region pixels crossed a region row almost every time and
// jumped 3 slots there: 42.5 % SQ_LDS_BANK_CONFLICT, profiles/r2_final/pmc_summary.txt).
constexpr int FP_R = SP_RR + 3, FP_C = SP_RC + 4, FP_PIX = FP_R * FP_C;  // 18 x 21 slots
// plane stride padded to a multiple of 16 slots: a ds_read_b128 lane group {0-3, 12-15, 20-27} reads lanes of
// both planes, which must then sit at the same bank offset
constexpr int FP_STRIDE = (FP_PIX + 15) / 16 * 16;                      // 384
// Epilogue tile [256 px][64 ch] bf16 for the pooling (direct kernel): pixels 2t and 2t+1 share one 256-B bank row,
// pixel m in half h(m) = (m ^ m >> 1) & 1 (so pooled neighbours px, px+1 -- whose window pixels differ by 2 --
// always sit in opposite halves), 16-B chunk k at k ^ (m & 7) within the half, and the two 8-B halves of a chunk
// swapped when bit 3 of m is set (the 16 consecutive pixels of an epilogue ds_write_b64 group then cover all 32
// banks). Byte address of chunk k of pixel m:
__device__ __forceinline__ int ptile(int m, int k) {
  return (m >> 1) * 256 + ((((m ^ (m >> 1)) & 1) << 3) | (k ^ (m & 7))) * 16;
}
constexpr int FP_SLOTS = 2 * FP_STRIDE;                                 // 736 16-B slots (2 planes + pad)
constexpr int FP_DMA = (FP_SLOTS + 255) / 256;                          // DMA instrs per wave (3)
constexpr int D_W = 0, D_FP = 64 * 512, D_TILE = D_FP + FP_DMA * 4 * 1024, D_LDS = D_TILE + SP_BM * 128;

// Diagnostic build (AI4E_STEM_STAMPS=1): s_memtime stamps between the loop's phases, summed per wave and
// written once per wave to g_stem_stamps (read by ai4e_stem_stamps_read). Never used for timing: read SHARES.
#ifndef AI4E_STEM_STAMPS
#define AI4E_STEM_STAMPS 0
#endif

constexpr int STEM_NSEG = 8;
#if AI4E_STEM_STAMPS
__device__ unsigned long long g_stem_stamps[2048 * 4 * STEM_NSEG];
#define STEM_STAMP(k)                                                                          \
  do {                                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    unsigned long long _t;                                                                     \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");               \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    st_sum[k] += _t - st_last;                                                                 \
    st_last = _t;                                                                              \
  } while (0)
#else
#define STEM_STAMP(k) \
  do {                \
  } while (0)
#endif

template <bool C1 = false, bool F16 = false, bool U8 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void stem_pool_direct_kernel(const StemParams p, int ntiles) {
#if AI4E_STEM_STAMPS
  unsigned long long st_sum[STEM_NSEG] = {0, 0, 0, 0, 0, 0, 0, 0}, st_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
#endif
  extern __shared__ __attribute__((aligned(1024))) uint8_t dsm[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t sb = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(dsm));
  // weights -> LDS once: row n (512 B), chunk q stored at chunk q ^ (n & 31)
  for (int e = tid; e < 64 * 32; e += 256) {
    const int n = e >> 5, q = e & 31;
    *reinterpret_cast<uint4*>(dsm + D_W + n * 512 + ((q ^ (n & 31)) << 4)) =
        *reinterpret_cast<const uint4*>(p.w + static_cast<long>(n) * p.kpad + 8 * q);
  }
  float4 bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bias[j] = *reinterpret_cast<const float4*>(p.bias + 16 * j + 4 * (lane >> 4));
  const int per_img = p.tiles_r * p.tiles_c;
  const int g = lane >> 4;
  // this lane's 4 pixels (one per fragment f = 4 wave + i): row fragments f < 15 hold region row f, columns
  // lane&15; fragment 15 holds column 16 of rows lane&15 (lane 15 idle: reads footprint slot 0, writes tile row 255,
  // which no pooling window covers). rm = the pixel's region index r * 17 + cc (the epilogue tile row).
  int fpb[4], rmi[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int f = 4 * wave + i;
    const int r = f < SP_RR ? f : (lane & 15), cc = f < SP_RR ? (lane & 15) : SP_RC - 1;
    const bool v = r < SP_RR;
    fpb[i] = v ? r * FP_C + cc : 0;
    rmi[i] = v ? r * SP_RC + cc : SP_BM - 1;
  }
  uint8_t* const tile = dsm + D_TILE;

  // footprint DMA of tile t: slot s = plane * FP_STRIDE + pixel (pixels >= FP_PIX are padding, zero-filled);
  // footprint pixel (a, b) is input (oh0-1+a, ow0-1+b). Issued one tile ahead: the next tile's footprint lands
  // while this tile's epilogue, pooling and fused c1 run (the MFMA loop is the footprint's only reader).
  auto issue_fp = [&](int tt) __attribute__((always_inline)) {
    const int im = tt / per_img;
    const int r0 = (tt - im * per_img) / p.tiles_c;
    const int c0 = tt - im * per_img - r0 * p.tiles_c;
    const int oh = 2 * r0 * SP_TR - 1, ow = 2 * c0 * SP_TC - 1;
    const uint16_t* const xs = p.x + static_cast<long>(im) * p.H * p.W * SP_C;
#pragma unroll
    for (int q = 0; q < FP_DMA; ++q) {
      const int s = (wave + 4 * q) * 64 + lane;
      const int h = s >= FP_STRIDE ? 1 : 0, pix = s - h * FP_STRIDE;
      const int a = pix / FP_C, b = pix - a * FP_C;
      const int ih = oh - 1 + a, iw = ow - 1 + b;
      const bool ok = s < FP_SLOTS && pix < FP_PIX && b < SP_RC + 3 && static_cast<unsigned>(ih) < static_cast<unsigned>(p.H) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(p.W);
      glds16(ok ? static_cast<const void*>(xs + (static_cast<long>(ih) * p.W + iw) * SP_C + 8 * h) : p.zero,
             sb + D_FP + (wave + 4 * q) * 1024);
    }
  };
  // U8: the footprint slots from the uint8 images, one byte load per s2d channel (s2d channel k = 8 * plane + e of
  // footprint pixel (ih, iw) is byte c of image pixel (2 ih + dy - 1, 2 iw + dx - 1), (dy * 2 + dx) * 3 + c = k), then
  // normalized, packed and written with 16-B LDS stores at the slot the DMA would have filled. Loaded and written in
  // one go after the epilogue (accumulators dead, footprint free): bytes held in registers across the epilogue, as
  // the DMA form's prefetch distance would need, spill (24 VGPRs over the 250 the kernel uses)
  auto build_fp8 = [&](int tt) __attribute__((always_inline)) {
    const int im = tt / per_img;
    const int r0 = (tt - im * per_img) / p.tiles_c;
    const int c0 = tt - im * per_img - r0 * p.tiles_c;
    const int oh = 2 * r0 * SP_TR - 1, ow = 2 * c0 * SP_TC - 1;
    const int H8 = 2 * p.H, W8 = 2 * p.W;
    const uint8_t* const xs = p.x8 + static_cast<long>(im) * H8 * W8 * 3;
    uint32_t u8r[FP_DMA][8];
    int u8m[FP_DMA], u8h[FP_DMA];
    // an opaque zero: the slot geometry below is loop-invariant, and hoisted out of the persistent loop it stays live
    // across the MFMA loop and spills; recomputed per tile it costs a few VALU ops
    int opq;
    asm volatile("v_mov_b32 %0, 0" : "=v"(opq));
#pragma unroll
    for (int q = 0; q < FP_DMA; ++q) {
      const int s = (wave + 4 * q) * 64 + lane + opq;
      const int h = s >= FP_STRIDE ? 1 : 0, pix = s - h * FP_STRIDE;
      const int a = pix / FP_C, b = pix - a * FP_C;
      const int ih = oh - 1 + a, iw = ow - 1 + b;
      // s2d pixels 0..H (W): pixel H holds image rows 2H - 1 (real) and 2H (outside), so the last image row / column
      // reaches the conv's last output row / column as in the 7x7/2 conv (the [N, H/2, W/2, 16] s2d tensor of the
      // two-launch path ends at pixel H - 1 and leaves image row / column 2H - 1 out)
      const bool ok = s < FP_SLOTS && pix < FP_PIX && b < SP_RC + 3 && static_cast<unsigned>(ih) <= static_cast<unsigned>(p.H) &&
                      static_cast<unsigned>(iw) <= static_cast<unsigned>(p.W);
      // byte offsets of image rows 2 ih - 1 (o0) and 2 ih (o1) at pixel 2 iw - 1. Plane 0 (channels 0-7) = row o0
      // bytes 0-5, row o1 bytes 0-1; plane 1 (channels 8-11) = row o1 bytes 2-5: so e < 6 reads ra + e with ra = o0
      // (plane 0) or o1 + 2 (plane 1), e = 6, 7 read o1 + e - 6 (plane 0 only)
      const int o0 = ((2 * ih - 1) * W8 + 2 * iw - 1) * 3, o1 = o0 + 3 * W8;
      const int ra = h ? o1 + 2 : o0;
      // row 2 ih - 1 / 2 ih and pixel 2 iw - 1 / 2 iw inside the image (ih and iw run over 0..H / 0..W)
      const bool y0 = ih > 0, y1 = ih < p.H, x0 = iw > 0, x1 = iw < p.W;
      int m = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = 8 * h + e, blk = k / 3;
        const bool v = ok && k < 12 && ((blk >> 1) ? y1 : y0) && ((blk & 1) ? x1 : x0);
        // unconditional loads (a masked-off byte reads the image's first byte): a conditional load becomes a branch
        // per byte with its own wait
        const int off = v ? (e < 6 ? ra + e : o1 + e - 6) : 0;
        u8r[q][e] = xs[off];
        m |= v ? 1 << e : 0;
      }
      u8m[q] = m;
      u8h[q] = h;
    }
#pragma unroll
    for (int q = 0; q < FP_DMA; ++q) {
      const int h = u8h[q];
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = (8 * h + e) % 3;
        const float mc = c == 0 ? p.pm[0] : c == 1 ? p.pm[1] : p.pm[2];
        const float ic = c == 0 ? p.pis[0] : c == 1 ? p.pis[1] : p.pis[2];
        v[e] = (u8m[q] >> e) & 1 ? (static_cast<float>(u8r[q][e]) * p.pscale - mc) * ic : 0.f;
      }
      *reinterpret_cast<uint4*>(dsm + D_FP + (wave + 4 * q) * 1024 + 16 * (lane + opq)) =
          make_uint4(pack2<F16>(v[0], v[1]), pack2<F16>(v[2], v[3]), pack2<F16>(v[4], v[5]), pack2<F16>(v[6], v[7]));
    }
  };
  if (static_cast<int>(blockIdx.x) < ntiles) {
    if constexpr (U8) build_fp8(blockIdx.x);
    else issue_fp(blockIdx.x);
  }

  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int img = t / per_img;
    const int tr = (t - img * per_img) / p.tiles_c;
    const int tc = t - img * per_img - tr * p.tiles_c;
    const int ph0 = tr * SP_TR, pw0 = tc * SP_TC;
    const int oh0 = 2 * ph0 - 1, ow0 = 2 * pw0 - 1;
    // this tile's footprint landed. From the second tile on (C1) the DMA is already complete: the previous
    // iteration waited for its c1 weight loads, issued after the DMA (vmcnt retires in issue order), so only the
    // previous tile's stores can be outstanding (<= 2 pooled-row + 4 t1 stores per wave): they may stay in flight
    STEM_STAMP(7);  // loop overhead
    if (C1 && t != static_cast<int>(blockIdx.x)) {
      wait_vmcnt<6>();
    } else {
      wait_vmcnt<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // footprint (and weights) visible
    STEM_STAMP(0);  // footprint wait + barrier

    f32x4_t acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < SP_NK; ++kt) {
      const int kh = kt >> 1, kw = 2 * (kt & 1) + (g >> 1);
      const int plane = (g & 1) * FP_STRIDE * 16;
      bf16x8_t fw[4], fx[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 16 * j + (lane & 15);
        fw[j] = *reinterpret_cast<const bf16x8_t*>(dsm + D_W + n * 512 + (((4 * kt + g) ^ (n & 31)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fx[i] = *reinterpret_cast<const bf16x8_t*>(dsm + D_FP + plane + (fpb[i] + kh * FP_C + kw) * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = mfma_16x16x32<F16>(fw[j], fx[i], acc[i][j]);
    }
    STEM_STAMP(1);  // MFMA loop
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave finished reading the footprint
    if (!U8 && t + static_cast<int>(gridDim.x) < ntiles) issue_fp(t + gridDim.x);
    STEM_STAMP(2);  // barrier + next footprint DMA issue
    // epilogue: bf16 relu(acc + b) -> tile [256 px][64 ch] (ptile layout)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = rmi[i];
      const int r = m / SP_RC, cc = m - r * SP_RC;
      const bool live = m < SP_RR * SP_RC && oh0 + r >= 0 && oh0 + r < p.H && ow0 + cc >= 0 && ow0 + cc < p.W;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 16 * j + 4 * (lane >> 4);
        const float4 b = bias[j];
        uint2 v = make_uint2(0u, 0u);
        if (live)
          v = make_uint2(pack2<F16>(fmaxf(acc[i][j][0] + b.x, 0.f), fmaxf(acc[i][j][1] + b.y, 0.f)),
                         pack2<F16>(fmaxf(acc[i][j][2] + b.z, 0.f), fmaxf(acc[i][j][3] + b.w, 0.f)));
        *reinterpret_cast<uint2*>(tile + ptile(m, n >> 3) + ((((n >> 2) ^ (m >> 3)) & 1) << 3)) = v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // U8: the next tile's footprint, built here where the accumulators are dead (the MFMA loop's last footprint
    // read is behind the barrier above it)
    if (U8 && t + static_cast<int>(gridDim.x) < ntiles) build_fp8(t + gridDim.x);
    STEM_STAMP(3);  // epilogue tile writes + barrier
    // fused c1 operands, issued now so the L2 latency hides under the pooling: W1 fragments (output-channel
    // rows 16j + lane&15, k-chunk lane>>4 of k-step ks; 8 KB, L2-resident) and the bias
    bf16x8_t w1f[4][2];
    float4 b1v[4];
    if constexpr (C1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          w1f[j][ks] = *reinterpret_cast<const bf16x8_t*>(p.w1 + static_cast<long>(16 * j + (lane & 15)) * p.kpad1 +
                                                          32 * ks + 8 * (lane >> 4));
        b1v[j] = *reinterpret_cast<const float4*>(p.b1 + 16 * j + 4 * (lane >> 4));
      }
    }
    // one pooled row (8 pixels x 8 chunks) per wave instruction; the lanes of each ds_read_b128 group
    // {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32) read the 8 chunks of two neighbouring pooled pixels, which
    // ptile puts in opposite bank-row halves: conflict-free for every window offset
    const int sub = lane & 31;
    const int pxl = sub < 4 ? 0 : sub < 12 ? 2 : sub < 16 ? 0 : sub < 20 ? 3 : sub < 28 ? 1 : 3;
    const int k8 = sub < 4 ? sub : sub < 12 ? sub - 4 : sub < 16 ? sub - 8 : sub < 20 ? sub - 16 : sub < 28 ? sub - 20 : sub - 24;
    const int px = pxl + 4 * (lane >> 5);
    uint4 mxs[2] = {make_uint4(0u, 0u, 0u, 0u), make_uint4(0u, 0u, 0u, 0u)};  // pooled rows wave, wave + 4 (c1)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int py = wave + 4 * e;
      if (py >= SP_TR) break;
      const int ph = ph0 + py, pw = pw0 + px;
      if (ph >= p.PH || pw >= p.PW) continue;
      uint4 mx = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int m = (2 * py + dy) * SP_RC + 2 * px + dx;
          uint4 v = *reinterpret_cast<const uint4*>(tile + ptile(m, k8));
          if ((m >> 3) & 1) v = make_uint4(v.z, v.w, v.x, v.y);  // the chunk's 8-B halves are stored swapped
          mx.x = max_bf16x2(mx.x, v.x);
          mx.y = max_bf16x2(mx.y, v.y);
          mx.z = max_bf16x2(mx.z, v.z);
          mx.w = max_bf16x2(mx.w, v.w);
        }
      ai4e_conv::st16_stream(p.y + ((static_cast<long>(img) * p.PH + ph) * p.PW + pw) * SP_BN + 8 * k8, mx);
      mxs[e] = mx;
    }
    STEM_STAMP(4);  // c1 operand loads issue + pooling + pooled stores
    if constexpr (C1) {
      // pooled rows q as the c1 B operand [k-block k8/4][64 rows][4 x 16-B chunks ^ swz(q)], staged in the tile
      // region once every wave has finished pooling from it (the footprint region holds the next tile's DMA)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int q = (wave + 4 * e) * SP_TC + px;
        if (wave + 4 * e < SP_TR)
          *reinterpret_cast<uint4*>(tile + (k8 >> 2) * 64 * 64 + q * 64 + (((k8 & 3) ^ swz(q)) << 4)) = mxs[e];
      }
    }
    // the next tile's epilogue overwrites what this tile's readers still use
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    STEM_STAMP(5);  // c1 operand staging + barriers
    if constexpr (C1) {
      // t1 = relu(W1 . pooled + b1) for the tile's 56 pooled pixels (wave w: rows 16w..16w+15; rows >= 56 and
      // pooled pixels outside the image are computed from stale LDS and never stored)
      const int r = 16 * wave + (lane & 15);
      f32x4_t a1[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) a1[j] = f32x4_t{b1v[j].x, b1v[j].y, b1v[j].z, b1v[j].w};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8_t fx = *reinterpret_cast<const bf16x8_t*>(tile + ks * 64 * 64 + r * 64 +
                                                               (((lane >> 4) ^ swz(r)) << 4));
#pragma unroll
        for (int j = 0; j < 4; ++j) a1[j] = mfma_16x16x32<F16>(w1f[j][ks], fx, a1[j]);
      }
      const int py = r / SP_TC, px = r - py * SP_TC;
      const int ph = ph0 + py, pw = pw0 + px;
      if (r < SP_TR * SP_TC && ph < p.PH && pw < p.PW) {
        uint16_t* dst = p.t1 + ((static_cast<long>(img) * p.PH + ph) * p.PW + pw) * 64 + 4 * (lane >> 4);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<uint2*>(dst + 16 * j) =
              make_uint2(pack_relu2<F16>(a1[j][0], a1[j][1]), pack_relu2<F16>(a1[j][2], a1[j][3]));
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // pooled rows read before the next epilogue
    }
    STEM_STAMP(6);  // c1 MFMA + t1 stores + barrier
  }
#if AI4E_STEM_STAMPS
  if (lane == 0 && blockIdx.x < 2048) {
    const int w = static_cast<int>(blockIdx.x) * 4 + wave;
#pragma unroll
    for (int k = 0; k < STEM_NSEG; ++k) g_stem_stamps[w * STEM_NSEG + k] = st_sum[k];
  }
#endif
}

template <bool C1 = false, bool F16 = false, bool U8 = false>
int launch_direct(const StemParams& p, long nb, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(stem_pool_direct_kernel<C1, F16, U8>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, D_LDS) != hipSuccess)
      return AI4E_ELAUNCH;
    attr = true;
  }
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  // persistent workgroups per CU (AI4E_STEM_WPC, default 2): each strides over the tiles, so a workgroup that
  // starts late (CUs held by the other serving stream's kernels) delays the whole launch by its full share
  static const long wpc = [] {
    const char* e = getenv("AI4E_STEM_WPC");
    const long v = e ? atol(e) : 2;
    return v < 1 ? 1L : v;
  }();
  const long grid = nb < wpc * cus ? nb : wpc * cus;
  hipLaunchKernelGGL((stem_pool_direct_kernel<C1, F16, U8>), dim3(static_cast<unsigned>(grid)), dim3(256), D_LDS, stream, p,
                     static_cast<int>(nb));
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

const uint16_t* stem_zero_ptr() {
  static const uint16_t* zero = nullptr;
  if (!zero) {
    void* a = nullptr;
    if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_stem_zero)) == hipSuccess) zero = static_cast<const uint16_t*>(a);
  }
  return zero;
}

}  // namespace

// Stem + pool + the first bottleneck's 1x1 c1 (64 -> 64, bias, ReLU) in one launch: y as ai4e_stem_pool_fwd,
// plus t1 [N, PH, PW, 64] = relu(y . W1^T + b1) (w1 [>= 64 rows, kpad1 >= 64] bf16, b1 [>= 64] fp32), computed
// from the pooled tile while it is still in LDS (no re-read of y, no separate launch).
namespace {
int stem_c1(bool f16, const void* x, const void* w, const void* bias, void* y, const void* w1, const void* b1, void* t1,
            int kpad1, int N, int H, int W, int kpad, hipStream_t stream) {
  if (!x || !w || !bias || !y || !w1 || !b1 || !t1 || kpad < 256 || kpad % 8 || kpad1 < 64 || kpad1 % 8 || H <= 0 ||
      W <= 0)
    return AI4E_EINVAL;
  StemParams p{};
  p.x = static_cast<const uint16_t*>(x);
  p.w = static_cast<const uint16_t*>(w);
  p.bias = static_cast<const float*>(bias);
  p.y = static_cast<uint16_t*>(y);
  p.zero = stem_zero_ptr();
  if (!p.zero) return AI4E_ELAUNCH;
  p.w1 = static_cast<const uint16_t*>(w1);
  p.b1 = static_cast<const float*>(b1);
  p.t1 = static_cast<uint16_t*>(t1);
  p.kpad1 = kpad1;
  p.H = H; p.W = W;
  p.PH = (H - 1) / 2 + 1;
  p.PW = (W - 1) / 2 + 1;
  p.kpad = kpad;
  p.tiles_r = ai4e_cdiv(p.PH, SP_TR);
  p.tiles_c = ai4e_cdiv(p.PW, SP_TC);
  const long nb = static_cast<long>(N) * p.tiles_r * p.tiles_c;
  if (nb <= 0) return AI4E_OK;
  return f16 ? launch_direct<true, true>(p, nb, stream) : launch_direct<true>(p, nb, stream);
}
}  // namespace

// The same from uint8 RGB images [N, H8, W8, 3] (H8, W8 even; the s2d stem input is their normalized 2x2 space-to-depth,
// built in the kernel: mean3 / std3 / scale as ai4e_preprocess_s2d_u8), bf16. y, t1: [N, ceil(H8/4), ceil(W8/4), 64].
AI4E_API int ai4e_stem_pool_c1_u8_fwd(const void* x8, const float* mean3, const float* std3, float scale, const void* w,
                                      const void* bias, void* y, const void* w1, const void* b1, void* t1, int kpad1,
                                      int N, int H8, int W8, int kpad, hipStream_t stream) {
  if (!x8 || !mean3 || !std3 || !w || !bias || !y || !w1 || !b1 || !t1 || kpad < 256 || kpad % 8 || kpad1 < 64 ||
      kpad1 % 8 || H8 <= 0 || W8 <= 0 || (H8 & 1) || (W8 & 1))
    return AI4E_EINVAL;
  StemParams p{};
  p.x8 = static_cast<const uint8_t*>(x8);
  for (int c = 0; c < 3; ++c) {
    p.pm[c] = mean3[c];
    p.pis[c] = 1.f / std3[c];  // as the preprocess launcher: the same fp32 reciprocal
  }
  p.pscale = scale;
  p.w = static_cast<const uint16_t*>(w);
  p.bias = static_cast<const float*>(bias);
  p.y = static_cast<uint16_t*>(y);
  p.zero = stem_zero_ptr();
  if (!p.zero) return AI4E_ELAUNCH;
  p.w1 = static_cast<const uint16_t*>(w1);
  p.b1 = static_cast<const float*>(b1);
  p.t1 = static_cast<uint16_t*>(t1);
  p.kpad1 = kpad1;
  p.H = H8 / 2; p.W = W8 / 2;
  p.PH = (p.H - 1) / 2 + 1;
  p.PW = (p.W - 1) / 2 + 1;
  p.kpad = kpad;
  p.tiles_r = ai4e_cdiv(p.PH, SP_TR);
  p.tiles_c = ai4e_cdiv(p.PW, SP_TC);
  const long nb = static_cast<long>(N) * p.tiles_r * p.tiles_c;
  if (nb <= 0) return AI4E_OK;
  return launch_direct<true, false, true>(p, nb, stream);
}

AI4E_API int ai4e_stem_pool_c1_fwd(const void* x, const void* w, const void* bias, void* y, const void* w1,
                                   const void* b1, void* t1, int kpad1, int N, int H, int W, int kpad,
                                   hipStream_t stream) {
  return stem_c1(false, x, w, bias, y, w1, b1, t1, kpad1, N, H, W, kpad, stream);
}

// The same on fp16 input / weights / outputs (f16 MFMA, fp32 accumulation; the max-pool's unsigned 16-bit max
// orders non-negative fp16 exactly as it does bf16).
AI4E_API int ai4e_stem_pool_c1_f16_fwd(const void* x, const void* w, const void* bias, void* y, const void* w1,
                                       const void* b1, void* t1, int kpad1, int N, int H, int W, int kpad,
                                       hipStream_t stream) {
  return stem_c1(true, x, w, bias, y, w1, b1, t1, kpad1, N, H, W, kpad, stream);
}

// x: s2d stem input [N, H, W, 16] bf16; w: packed 4x4x16 stem weights [>= 64 rows, kpad >= 256] (pad 1/2,
// ops/conv.py pack_stem_s2d); bias [>= 64] fp32; y: [N, ceil(H/2), ceil(W/2), 64] bf16.
// variant: 0 = direct conv from the LDS input footprint (persistent, default), 1 = DMA-gather implicit GEMM.
AI4E_API int ai4e_stem_pool_fwd(const void* x, const void* w, const void* bias, void* y, int N, int H, int W, int kpad,
                                int variant, hipStream_t stream) {
  if (!x || !w || !bias || !y || kpad < 256 || kpad % 8 || H <= 0 || W <= 0) return AI4E_EINVAL;
  static const uint16_t* zero = nullptr;
  if (!zero) {
    void* a = nullptr;
    if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_stem_zero)) != hipSuccess) return AI4E_ELAUNCH;
    zero = static_cast<const uint16_t*>(a);
  }
  StemParams p{};
  p.x = static_cast<const uint16_t*>(x);
  p.w = static_cast<const uint16_t*>(w);
  p.bias = static_cast<const float*>(bias);
  p.y = static_cast<uint16_t*>(y);
  p.zero = zero;
  p.H = H; p.W = W;
  p.PH = (H - 1) / 2 + 1;
  p.PW = (W - 1) / 2 + 1;
  p.kpad = kpad;
  p.tiles_r = ai4e_cdiv(p.PH, SP_TR);
  p.tiles_c = ai4e_cdiv(p.PW, SP_TC);
  const long nb = static_cast<long>(N) * p.tiles_r * p.tiles_c;
  if (nb <= 0) return AI4E_OK;
  if (variant == 0) return launch_direct<>(p, nb, stream);
  hipLaunchKernelGGL(stem_pool_kernel, dim3(static_cast<unsigned>(nb)), dim3(256), 0, stream, p);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

#if AI4E_STEM_STAMPS
// Diagnostic build only: per-wave phase cycle sums of the last direct-stem launch (2048 x 4 waves x 8).
AI4E_API int ai4e_stem_stamps_read(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stem_stamps), sizeof(g_stem_stamps)) == hipSuccess ? AI4E_OK
                                                                                                    : AI4E_ELAUNCH;
}
#endif
