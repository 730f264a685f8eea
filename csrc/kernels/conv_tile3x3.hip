// K1t: 3x3 / stride 1 / pad 1 convolution, NHWC bf16, for wide feature maps: 64 / 128 -> 64 channels (the U-Net's
// full-resolution level, 512^2 tiles). At level 0 the K1 implicit GEMM gathers every tap of every pixel through the
// LDS-DMA ring (nine 16-B gathers per pixel and 32-channel step) and ran at 23 % MFMA / 1.3 TB/s
// (profiles/r4_unet/pmc_by_kernel.txt).
//
// Each 8 x 32 output tile is computed by one workgroup (4 waves):
// * the (TH + 2) x 34 x 64 input patch (halo 1, zero outside the image) is loaded ONCE into LDS (16-B chunks of a
//   pixel slot XOR-swizzled for the real ds_read_b128 lane groups), optionally through a prologue: x * a[c] + b[c]
//   (+ ReLU) per (image, channel) — the previous layer's GroupNorm apply, so that the normalized tensor is never
//   written (its statistics came from the previous conv's epilogue);
// * the nine taps then run as LDS-read + MFMA steps (v_mfma_f32_16x16x32_bf16; weights as the A operand, pixels as
//   B; per wave 64 px x 64 ch: 32 MFMAs per stage), the next tap's weights loaded from L2 during
//   the current tap into the other half of a two-tap LDS buffer;
// * epilogue: + bias, bf16 store, and the GroupNorm statistics of the stored values per (image, tile, group) in the
//   K1 conv-epilogue format (shifted sums S, Q and the shift K: norm_resample.hip gn_finalize_kernel).
// CIN > 64: the same tiles, run as CIN / 64 k-slices through one 64-channel patch buffer (accumulators carried over).
// Measured and removed in round 5 (patches in profiles/r5_pruned/): 128-output-channel instances (-1.4 % on the
// U-Net, profiles/r4_k1t/cout128/), weight stages by LDS-DMA (-2 %, profiles/r4_k1t/wdma/) and the 2x upsample formed
// in LDS for the decoder c1 (neutral, profiles/r4_k1t/ups/).
// Persistent: min(tiles, 2 x CUs) workgroups walk the tiles with stride gridDim.x. The next (tile, slice)'s patch is
// loaded into registers while the current taps run (spread over the stages, so every vmcnt wait stays exact), and its
// first weight stage while the epilogue runs, then stored into LDS (through the prologue) behind one barrier.
// Every global address is inside its tensor by construction (host: H % TH == 0, W % 32 == 0; tile t < ntiles; patch
// loads clamped to in-tensor pixels, out-of-image chunks zeroed in LDS).
#include <type_traits>

#include "common.h"
#include "conv_common.h"

namespace {

constexpr int T_W = 32, P_W = T_W + 2;           // output tile width; patch width with halo

// 8 x 32 output tiles from a 10 x 34 x 64-channel input patch (43.5 KB). CIN = 128 (decoder c1s reading a
// [skip | upsampled] concat) runs each tile as 2 k-slices through the same patch buffer: the accumulators carry over,
// the epilogue runs once, and the next slice's patch is prefetched under the current slice's taps like the next tile's.
// LDS: patch + CIN x 8 B affine + two 64 x 128 B weight stages + the bias; two workgroups per CU.
template <int CIN, int COUT = 64>
struct TileCfg {
  static constexpr int TH = 8;                          // output tile rows
  static constexpr int P_SLOTS = (TH + 2) * P_W;
  static constexpr int NCH = 8;                         // 16-B chunks per 64-channel pixel slot
  static constexpr int SLOT_B = 128;
  static constexpr int L_PATCH = P_SLOTS * SLOT_B;
  static constexpr int L_AFF = CIN * 8;                 // prologue affine of this image: CIN x (a, b)
  static constexpr int L_W = COUT * 128;                // one weight stage: COUT rows x 64 input channels of one tap
  static constexpr int NWB = 2;                         // weight stage buffers
  static constexpr int L_TOTAL = L_PATCH + L_AFF + NWB * L_W + COUT * 4;  // + the bias
  static constexpr int P_CHUNKS = P_SLOTS * NCH;
  static constexpr int P_ITERS = (P_CHUNKS + 255) / 256;
  static constexpr int KS = CIN / 64;                   // 64-channel k-slices per tile
  static constexpr int NST = 9;                         // weight stages (taps) per k-slice
  static constexpr int FPW = TH / 2;                    // pixel fragments per wave (TH / 4 rows x 2 half-rows)
  static constexpr int NJ = COUT / 16;                  // 16-channel output blocks per wave
  static constexpr int NWV = COUT / 32;                 // 16-B weight chunks per thread per stage
  static constexpr int L_ALL = L_TOTAL;
  static_assert(CIN == 64 || CIN == 128, "K1t: 64 or 128 input channels");
  static_assert(COUT == 64, "K1t: 64 output channels");
  static_assert(L_TOTAL <= 80 * 1024, "two workgroups per CU");
  static_assert((COUT + 4 * COUT * 2) * 4 <= L_W, "GroupNorm scratch (shift + 4-wave sums) fits a weight stage");
};

struct TileParams {
  const uint16_t* x;
  int ldx, xcoff;          // input [N, H, W, ldx], channels [xcoff, xcoff + CIN)
  const uint16_t* w;
  int kpad;                // packed weights [COUT rows, kpad >= 9 CIN], K = (kh, kw, c)
  const float* bias;       // [COUT]
  const float2* pro;       // prologue (a, b) per (image, channel) [N, CIN]; null = none
  int pro_relu;
  uint16_t* y;
  int ldy, ycoff;          // output [N, H, W, ldy], channels [ycoff, ycoff + COUT)
  float* gnp;              // GroupNorm partials [N, tiles per image, G, 4]; null = off
  int gn_groups;
  int H, W, tiles_w, tiles_per_img;
};

// Byte offset within its row of 16-B chunk c of row `row` (M = 8 chunks per row). ds_read_b128 is serviced in four
// 16-lane groups that are NOT contiguous: {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same +32
// (MI355X_MICROARCH.md, LDS). A fragment read (16 consecutive rows, chunk 4 s + lane / 16) therefore puts in one group
// all 16 rows, 8 of them at chunk c and 8 at chunk c ^ 1 (c even). The chunk's bank group is
// 8 (row & 1) + (c ^ key(row)), so for every window of 16 rows the keys of each row parity, with the middle pixels'
// extra ^ 1, must be distinct: key = row & 6 is (tests/test_tile_layout.py searches and checks this). The earlier key
// (row >> 1) & 7 was conflict-free only for contiguous 16-lane groups, and measured 16-18 % bank conflicts.
template <int M>
__device__ __forceinline__ uint32_t swz(int row, int c) {
  static_assert(M == 8, "8 chunks per row");
  return static_cast<uint32_t>((c ^ (row & 6)) << 4);
}

// LDS handoff between the waves: wait for this wave's LDS operations, then the barrier. Not __syncthreads(): its
// workgroup release fence makes the compiler drain vmcnt (which on gfx9 counts loads and stores together) before
// every barrier, so the weight and next-patch loads in flight would be waited for at each of the 9 stages. Nothing
// in this kernel passes data between waves through global memory.
__device__ __forceinline__ void tile_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int CIN, int COUT = 64>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv3x3_tile_kernel(
    const TileParams p, int ntiles) {
  using Cfg = TileCfg<CIN, COUT>;
  constexpr int NJ = Cfg::NJ, L_W = Cfg::L_W;
  constexpr int TH = Cfg::TH, P_CHUNKS = Cfg::P_CHUNKS, P_ITERS = Cfg::P_ITERS, NCH = Cfg::NCH, SLOT_B = Cfg::SLOT_B;
  constexpr int KS = Cfg::KS, NST = Cfg::NST, FPW = Cfg::FPW;
  static_assert(P_ITERS <= 32, "in-image mask bits");
  constexpr int PPS = (P_ITERS + NST - 2) / (NST - 1);  // next-patch chunk loads per stage (stages 0 .. NST - 2)
  extern __shared__ __attribute__((aligned(1024))) uint8_t sm[];
  uint8_t* const patch = sm;
  float2* const aff = reinterpret_cast<float2*>(sm + Cfg::L_PATCH);
  uint8_t* const wbuf = sm + Cfg::L_PATCH + Cfg::L_AFF;
  constexpr int NWB = Cfg::NWB;
  float* const sbias = reinterpret_cast<float*>(wbuf + NWB * L_W);  // [COUT]: epilogue reads stay off the vmcnt queue
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g4 = lane >> 4;

  // one weight stage in flight: rows n = tid / 8 + 32 e (e < NWV), 16-B chunk tid % 8 (named registers: an array
  // indexed inside these lambdas was kept in scratch)
  uint4 wv0, wv1;
  auto load_w = [&](int tap, int ks) __attribute__((always_inline)) {  // stage = (tap, 64-channel k-slice)
    const int tq = tid;  // (the hoisted per-stage addresses: 3-4 % faster than per-call address math)
    const uint16_t* const src = p.w + static_cast<long>(tq >> 3) * p.kpad + tap * CIN + ks * 64 + 8 * (tq & 7);
    wv0 = *reinterpret_cast<const uint4*>(src);
    wv1 = *reinterpret_cast<const uint4*>(src + 32L * p.kpad);
  };
  auto store_w = [&](int buf) __attribute__((always_inline)) {
    const int n = tid >> 3, c = tid & 7;
    uint8_t* const b = wbuf + buf * L_W;
    *reinterpret_cast<uint4*>(b + n * 128 + swz<8>(n, c)) = wv0;
    *reinterpret_cast<uint4*>(b + (n + 32) * 128 + swz<8>(n + 32, c)) = wv1;
  };
  // the patch of one tile: global -> registers (pv, in-image chunks in pmask), later registers -> LDS
  uint4 pv[P_ITERS];
  uint32_t pmask = 0;
  auto load_patch = [&](int img, int h0, int w0, int ks, int k0, int k1) __attribute__((always_inline)) {
    const uint16_t* const xi = p.x + static_cast<long>(img) * p.H * p.W * p.ldx + p.xcoff + 64 * ks;
    int tq = tid;
    asm volatile("" : "+v"(tq));  // recompute the chunk address math per tile (hoisted, it spills)
#pragma unroll
    for (int k = k0; k < k1; ++k) {
      const int e = tq + 256 * k;
      const int slot = e / NCH, c = e - slot * NCH;
      const int pr = slot / P_W, pc = slot - pr * P_W;
      const int ih = h0 - 1 + pr, iw = w0 - 1 + pc;
      const bool in = e < P_CHUNKS && static_cast<unsigned>(ih) < static_cast<unsigned>(p.H) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(p.W);
      pmask |= in ? (1u << k) : 0u;
      // unconditional load from the nearest in-image pixel (no branch around it, so the vmcnt waits stay exact);
      // store_patch zeroes the chunks outside the image
      const int ihc = min(max(ih, 0), p.H - 1), iwc = min(max(iw, 0), p.W - 1);
      const uint16_t* src = xi + (static_cast<long>(ihc) * p.W + iwc) * p.ldx + 8 * (c & 7);
      pv[k] = *reinterpret_cast<const uint4*>(src);
    }
  };
  auto store_patch = [&](int ks) __attribute__((always_inline)) {
    int tq = tid;
    asm volatile("" : "+v"(tq));
#pragma unroll
    for (int k = 0; k < P_ITERS; ++k) {
      const int e = tq + 256 * k;
      if (e >= P_CHUNKS) continue;
      const int slot = e / NCH, c = e - slot * NCH;
      const bool in = (pmask >> k) & 1u;
      uint4 v = in ? pv[k] : make_uint4(0u, 0u, 0u, 0u);
      if (p.pro != nullptr && in) {  // padding stays zero: the conv pads the normalized tensor
        // packed math per channel pair: one v_pk_fma_f32, one v_cvt_pk_bf16_f32 and (ReLU) one v_pk_max_i16 on the
        // packed bf16 (relu(round(x)) == round(relu(x))), instead of two FMAs, two max and a pack
        uint32_t wds[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float lo, hi;
          unpack_bf16x2(wds[q], lo, hi);
          const float4 ab = *reinterpret_cast<const float4*>(aff + 64 * ks + 8 * c + 2 * q);  // (a0, b0, a1, b1)
          const f32x2_t x2 = {lo, hi}, a2 = {ab.x, ab.z}, b2 = {ab.y, ab.w};
          const f32x2_t y2 = __builtin_elementwise_fma(x2, a2, b2);
          const uint32_t packed = __builtin_bit_cast(uint32_t, __builtin_convertvector(y2, bf16x2_t));
          wds[q] = p.pro_relu ? relu_bf16x2(packed) : packed;
        }
        v = make_uint4(wds[0], wds[1], wds[2], wds[3]);
      }
      *reinterpret_cast<uint4*>(patch + slot * SLOT_B + swz<NCH>(slot, c)) = v;
    }
  };
  auto coords = [&](int t, int& img, int& tin, int& h0, int& w0) __attribute__((always_inline)) {
    img = t / p.tiles_per_img;
    tin = t - img * p.tiles_per_img;
    const int tr = tin / p.tiles_w, tc = tin - tr * p.tiles_w;
    h0 = tr * TH;
    w0 = tc * T_W;
  };

  // persistent: tiles blockIdx.x, + gridDim.x, ... (host: gridDim.x <= ntiles), each as KS k-slices. The next
  // (tile, slice)'s patch is loaded into registers under the current slice's taps and stored into the patch buffer
  // after it (and after the tile's epilogue).
  int t = blockIdx.x, ks = 0, img, tin, h0, w0;
  coords(t, img, tin, h0, w0);
  load_w(0, 0);
  if (p.pro != nullptr && tid < CIN) aff[tid] = p.pro[img * CIN + tid];
  if (tid < COUT) sbias[tid] = p.bias[tid];
  pmask = 0;
  load_patch(img, h0, w0, 0, 0, P_ITERS);
  store_w(0);
  tile_barrier();  // the affine is in LDS
  store_patch(0);
  tile_barrier();

  // GroupNorm scratch: the weight buffer 0 (its next stage is stored behind the next barrier)
  float* const kshift = reinterpret_cast<float*>(wbuf);  // [COUT] the tile's first pixel, as stored
  float* const red = kshift + COUT;                                    // [4 waves][COUT channels][2]

  f32x4_t acc[FPW][NJ];  // carried over the k-slices of a tile; zeroed here and after each tile's epilogue
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int f = 0; f < FPW; ++f)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[f][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();
  for (;;) {
    // the next (tile, slice): workgroup-uniform
    const bool last_slice = ks == KS - 1;
    const int tn = last_slice ? t + static_cast<int>(gridDim.x) : t;
    const int ksn = last_slice ? 0 : ks + 1;
    const bool has_next = tn < ntiles;
    // without a next item the "next" coordinates stay the current ones: the loads below are then issued anyway (to
    // valid addresses, their data unused) — a branch around them would make every later vmcnt wait a full drain
    int imgn = img, tinn = tin, h0n = h0, w0n = w0;
    if (has_next && last_slice) coords(tn, imgn, tinn, h0n, w0n);
    pmask = 0;
    // ---- weight stages (9 taps x CIN / 64 halves) x two 32-channel steps
    int l16 = lane & 15;
    asm volatile("" : "+v"(l16));  // per-tile fragment offsets (hoisted out of the tile loop, they spill)
    // slot of tap (0, 0) for this lane's pixel in fragment f: tile row (TH / 4) wave + f / 2, column 16 (f & 1) + l16
    int sbase[FPW];
#pragma unroll
    for (int f = 0; f < FPW; ++f) sbase[f] = ((TH / 4) * wave + (f >> 1)) * P_W + 16 * (f & 1) + l16;
#pragma unroll
    for (int st = 0; st < NST; ++st) {  // stage = tap
      // issue order is the wait order (vmcnt retires in order): this stage's weight chunks first, then PPS chunks
      // of the next (tile, slice)'s patch, which the waits of later stages cover; pinned against the scheduler,
      // which otherwise sinks the weight loads to their use at the end of the stage
      if (st + 1 < NST) load_w(st + 1, ks);
      load_patch(imgn, h0n, w0n, ksn, st * PPS < P_ITERS ? st * PPS : P_ITERS,
                 (st + 1) * PPS < P_ITERS ? (st + 1) * PPS : P_ITERS);
      __builtin_amdgcn_sched_barrier(0);
      const int kh = st / 3, kw = st - 3 * kh;
      const uint8_t* const wb = wbuf + (st & 1) * L_W;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int wc = 4 * s + g4;  // chunk within the stage's 64 channels
        bf16x8_t fx[FPW], fw[NJ];
#pragma unroll
        for (int f = 0; f < FPW; ++f) {
          const int slot = sbase[f] + kh * P_W + kw;
          fx[f] = *reinterpret_cast<const bf16x8_t*>(patch + slot * SLOT_B + swz<NCH>(slot, wc));
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int n = 16 * j + l16;
          fw[j] = *reinterpret_cast<const bf16x8_t*>(wb + n * 128 + swz<8>(n, wc));
        }
#pragma unroll
        for (int f = 0; f < FPW; ++f)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[f][j] = mfma_16x16x32<false>(fw[j], fx[f], acc[f][j]);
      }
      if (st + 1 < NST) store_w((st + 1) & 1);  // that buffer was last read at stage st - 1 (before the previous barrier)
      tile_barrier();
    }
    load_w(0, ksn);  // the next slice's first weight stage, in flight under the epilogue

    // ---- epilogue (after the tile's last slice): lane holds channels 16 j + 4 g4 + v of pixel (lane % 16) of
    // each fragment
    if (last_slice) {
      uint2 ov[FPW][NJ];
  #pragma unroll
      for (int f = 0; f < FPW; ++f) {
        const int oh = h0 + (TH / 4) * wave + (f >> 1), ow = w0 + 16 * (f & 1) + (lane & 15);
        uint16_t* const dst = p.y + ((static_cast<long>(img) * p.H + oh) * p.W + ow) * p.ldy + p.ycoff;
  #pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const float4 bv = *reinterpret_cast<const float4*>(sbias + 16 * j + 4 * g4);  // LDS: frees 16 VGPRs
          ov[f][j] = make_uint2(pack_bf16x2(acc[f][j][0] + bv.x, acc[f][j][1] + bv.y),
                                pack_bf16x2(acc[f][j][2] + bv.z, acc[f][j][3] + bv.w));
          *reinterpret_cast<uint2*>(dst + 16 * j + 4 * g4) = ov[f][j];
        }
      }
      if (p.gnp != nullptr) {
        // GroupNorm statistics of the stored values (cg = COUT / G channels per group, cg in {1, 2, 4}: a lane's 4
        // channels of one j hold whole groups), shifted by the tile's first pixel at each group's first channel
        if (wave == 0 && (lane & 15) == 0) {
  #pragma unroll
          for (int j = 0; j < NJ; ++j) {
            float a, b, c, d;
            unpack_bf16x2(ov[0][j].x, a, b);
            unpack_bf16x2(ov[0][j].y, c, d);
            kshift[16 * j + 4 * g4] = a;
            kshift[16 * j + 4 * g4 + 1] = b;
            kshift[16 * j + 4 * g4 + 2] = c;
            kshift[16 * j + 4 * g4 + 3] = d;
          }
        }
        tile_barrier();
        const int cg = COUT / p.gn_groups;
  #pragma unroll
        for (int j = 0; j < NJ; ++j) {  // one 16-channel block at a time (register pressure)
          float gs[4], gq[4];
  #pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int ch = 16 * j + 4 * g4 + v;
            const float K = kshift[ch - ch % cg];
            float s = 0.f, q = 0.f;
  #pragma unroll
            for (int f = 0; f < FPW; ++f) {
              float a, b;
              unpack_bf16x2(v < 2 ? ov[f][j].x : ov[f][j].y, a, b);
              const float d = ((v & 1) ? b : a) - K;
              s += d;
              q += d * d;
            }
            gs[v] = s;
            gq[v] = q;
          }
  #pragma unroll
          for (int off = 1; off < 16; off <<= 1)  // over the 16 pixels of a fragment row (lanes sharing g4)
  #pragma unroll
            for (int v = 0; v < 4; ++v) {
              gs[v] += __shfl_xor(gs[v], off);
              gq[v] += __shfl_xor(gq[v], off);
            }
          if ((lane & 15) == 0) {
  #pragma unroll
            for (int v = 0; v < 4; ++v) {
              const int ch = 16 * j + 4 * g4 + v;
              red[(wave * COUT + ch) * 2] = gs[v];
              red[(wave * COUT + ch) * 2 + 1] = gq[v];
            }
          }
        }
        tile_barrier();
        if (tid < p.gn_groups) {
          float S = 0.f, Q = 0.f;
          for (int w = 0; w < 4; ++w)
            for (int c = 0; c < cg; ++c) {
              S += red[(w * COUT + tid * cg + c) * 2];
              Q += red[(w * COUT + tid * cg + c) * 2 + 1];
            }
          float* const o = p.gnp + ((static_cast<long>(img) * p.tiles_per_img + tin) * p.gn_groups + tid) * 4;
          *reinterpret_cast<float4*>(o) = make_float4(S, Q, kshift[tid * cg], 0.f);
        }
      }
      zero_acc();  // (not at the next slice's start: that keeps the old values live through the epilogue)
    }  // last_slice
    if (!has_next) break;
    tile_barrier();  // this slice's patch, weight stages and statistics scratch are read
    if (last_slice && p.pro != nullptr && tid < CIN) aff[tid] = p.pro[imgn * CIN + tid];
    store_w(0);
    tile_barrier();  // the next tile's affine is in LDS
    store_patch(ksn);
    tile_barrier();
    t = tn;
    ks = ksn;
    img = imgn;
    tin = tinn;
    h0 = h0n;
    w0 = w0n;
  }
}

}  // namespace

namespace {

template <int CIN>
int launch_tile(const TileParams& p, int N, hipStream_t stream) {
  constexpr int L = TileCfg<CIN>::L_ALL;
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(conv3x3_tile_kernel<CIN>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, L) == hipSuccess;
  }();
  if (!attr) return AI4E_ELAUNCH;
  // persistent grid: two workgroups per CU (LDS), never more workgroups than tiles
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    return AI4E_ELAUNCH;
  const int ntiles = N * p.tiles_per_img;
  const int grid = ntiles > 2 * cus ? 2 * cus : ntiles;
  hipLaunchKernelGGL((conv3x3_tile_kernel<CIN>), dim3(static_cast<unsigned>(grid)), dim3(256), L, stream, p, ntiles);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

}  // namespace

// y = conv3x3(pro(x)) + bias (cin 64 / 128 -> 64 channels; stride 1, pad 1) with GroupNorm partials of y
// (gn_groups > 0): [N, (H / 8) * (W / 32), G, 4]. pro: null or float2 [N, cin] (x * a + b, then ReLU if pro_relu).
AI4E_API int ai4e_conv3x3_tile_fwd(const void* x, const void* w, const void* bias, const void* pro, int pro_relu,
                                   void* y, int N, int H, int W, int cin, int cout, int ldx, int xcoff, int kpad,
                                   int ldy, int ycoff, void* gn_partials, int gn_groups, hipStream_t stream) {
  const bool ok_c = cout == 64 && (cin == 64 || cin == 128);
  const int th = TileCfg<64>::TH;
  if (!x || !w || !bias || !y || N <= 0 || !ok_c || H % th || W % T_W || kpad < 9 * cin || ldx % 8 || xcoff % 8 ||
      xcoff + cin > ldx || ldy % 8 || ycoff % 8 || ycoff + cout > ldy)
    return AI4E_EINVAL;
  if (reinterpret_cast<uintptr_t>(bias) % 16) return AI4E_EINVAL;  // float4 reads in the epilogue
  if (gn_partials && (gn_groups <= 0 || gn_groups > 64 || cout % gn_groups || cout / gn_groups > 4))
    return AI4E_EINVAL;
  if (static_cast<long>(N) * H * W * (ldx > ldy ? ldx : ldy) >= (1L << 40)) return AI4E_EINVAL;
  TileParams p;
  p.x = static_cast<const uint16_t*>(x);
  p.ldx = ldx;
  p.xcoff = xcoff;
  p.w = static_cast<const uint16_t*>(w);
  p.kpad = kpad;
  p.bias = static_cast<const float*>(bias);
  p.pro = static_cast<const float2*>(pro);
  p.pro_relu = pro_relu;
  p.y = static_cast<uint16_t*>(y);
  p.ldy = ldy;
  p.ycoff = ycoff;
  p.gnp = static_cast<float*>(gn_partials);
  p.gn_groups = gn_partials ? gn_groups : 1;
  p.H = H;
  p.W = W;
  p.tiles_w = W / T_W;
  p.tiles_per_img = (H / th) * p.tiles_w;
  return cin == 64 ? launch_tile<64>(p, N, stream) : launch_tile<128>(p, N, stream);
}
