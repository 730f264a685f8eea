// K1c — fused ResNet bottleneck chain: 3x3 conv (c2) -> 1x1 expand (c3) + residual -> [next block's
// 1x1 reduce (c1')], one kernel per pixel tile, intermediates kept in LDS.
//
//   T2  = relu(conv3x3_s(T1; W2) + b2)                    [BM x MID]   (LDS only)
//   Y   = relu(T2 . W3^T + b3 + R)                        [BM x 4MID]  (HBM: next block's residual)
//   T1' = relu(Y . W1'^T + b1')          (NEXT only)      [BM x MID]   (HBM: next block's c2 input)
//
// Why: at batch 256 a layer1 bottleneck moves 1.6 GB through HBM as three separate convs (c1 reads the
// 256-channel input, c3 re-reads T2 and the residual). Chained, a block reads T1 (+3x3 halo, L2) and R
// once and writes Y and T1' once: 1.0 GB for layer1, and c1 of every identity block disappears as a
// launch. BatchNorm is folded into W/b on the host (ops/conv.py).
//
// Structure (4 wave64s, every wave a 64-pixel x 64-channel MFMA tile of v_mfma_f32_16x16x32_bf16,
// workgroup tile BM x MID with BM = 16384 / MID, i.e. 256x64, 128x128, 64x256):
// * phase A: the K1 implicit-GEMM main loop (LDS-DMA ring, counted vmcnt, fragment double-buffering)
//   over the 9*MID-long K of the 3x3 conv; epilogue writes bf16 T2 into LDS in the K-blocked,
//   chunk-swizzled layout the MFMA operand reads expect ([MID/32][BM][32], 64-B rows).
// * phases B/C, four passes p over the 4*MID output channels of c3: the residual chunk R_p is DMA'd into
//   the Y buffer (coalesced 16-B rows), B_p = T2 . W3[p]^T, the epilogue adds b3 + R_p, applies ReLU and
//   writes bf16 Y_p in place, C_p accumulates Y_p . W1'[:, p]^T into the persistent T1' accumulators,
//   and Y_p is copied out to HBM with 16-B stores. Weights of B/C stream through a weights-only LDS ring
//   (one continuous DMA stream across passes); every wait is a counted vmcnt whose count is a constant
//   after unrolling (the wave's own DMA/store bookkeeping below).
// LDS: max(phase-A pixel ring, T2 + Y buffer) + weight ring (48 KB for the 128-pixel MID-64 tile: 3 workgroups
// per CU; 80 KB for MID 128: 2). c3 biases seed the B accumulators (MID 64: staged in LDS; MID 128: carried in
// the weight ring); the T2 bias comes through scalar loads. Epilogues add the residual from packed bf16 (dot2),
// convert with v_cvt_pk_bf16_f32 and apply ReLU on the packed bf16 (v_pk_max_i16).
#include <type_traits>

#include "conv_common.h"

namespace {

using ai4e_conv::BK;
using ai4e_conv::glds16;
using ai4e_conv::swz;
using ai4e_conv::TapWalk;
using ai4e_conv::wait_vmcnt;
using ai4e_conv::wait_vmcnt_n;

__device__ __attribute__((aligned(64))) uint16_t g_chain_zero[32];
// target of the masked-off tail stores: a row base (+ column offsets up to 4*128) must stay inside it
__device__ __attribute__((aligned(64))) uint16_t g_chain_sink[512 + 64];

// LDS-ordering barrier: own LDS reads/writes retired, then s_barrier; an asm statement with a memory
// clobber so hipcc moves no LDS access across it (the raw builtin is not a compiler memory barrier).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Conflict-free chain layout (round 4; profiles/r4_chain_cf/: neutral in time against the round-3 layout, which was
// 2-way conflicted on every epilogue write and on the patch reads of fragments that wrap an image row):
// * the T2 / Y / T1' tiles use the 16-B chunk swizzle swt(r) = gray((r >> 1) & 3), chosen (exhaustive search over
//   per-row chunk rotations of a 64-B row) so that BOTH the MFMA fragment reads (ds_read_b128, 4 x 16 lane groups,
//   rows 0-3 / 12-15 at chunk c and rows 4-11 at c ^ 1) AND the epilogue's 16-B row writes (ds_write_b128, 8 x 8
//   contiguous lanes = 8 consecutive rows, banks mod 32) hit every bank once. The epilogues first regroup two 16-channel
//   accumulator blocks with v_permlane16_swap so each lane writes 8 consecutive channels (one ds_write_b128 instead of
//   two 2-way-conflicted ds_write_b64; the same for the residual read);
// * patch rows are padded to W + 8 slots (row stride = W mod 8), so 16 consecutive pixels read 16 consecutive slots mod 8
//   even where a fragment wraps to the next image row, and a masked tap reads a zero slot of the same residue mod 8
//   instead of slot 0 (both were 2-way conflicts on the patch reads of phase A).
// phase-A weight K steps prefetched into registers (patch mode): 4 (6 / 8 were neutral on the MID-64 chains,
// profiles/r4_chain_pd/; deeper MID-128 prefetch spills)
constexpr int CHAIN_PD = 4;
__device__ __forceinline__ int swt(int r) {
  const int x = (r >> 1) & 3;
  return x ^ (x >> 1);
}

// Regroup two accumulator blocks of one 32-channel K block: a = this lane's 4 values of channels 4*lg.. of block j,
// b = the same of block j + 1 (j even). After the row swaps (lanes 16-31 of a <-> lanes 0-15 of b, and 48-63 <-> 32-47)
// the lane holds 8 consecutive channels [a | b] of 16-B chunk swap_chunk(lg) of that K block. With a, b = one block of
// two fragments 16 rows apart instead, the lane holds row + 16 * (lg & 1), chunk of the block + (lg >> 1).
__device__ __forceinline__ void swap16(f32x4_t& a, f32x4_t& b) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[q]), __float_as_uint(b[q]), false, false);
    a[q] = __uint_as_float(r[0]);
    b[q] = __uint_as_float(r[1]);
  }
}
__device__ __forceinline__ int swap_chunk(int lg) { return ((lg & 1) << 1) | (lg >> 1); }
// 8 values -> 8 x bf16 / fp16 with ReLU (the sign-bit ReLU of relu_bf16x2 holds for fp16 bits too)
template <bool F16>
__device__ __forceinline__ uint4 relu8(const f32x4_t& a, const f32x4_t& b) {
  return make_uint4(relu_bf16x2(pack2<F16>(a[0], a[1])), relu_bf16x2(pack2<F16>(a[2], a[3])),
                    relu_bf16x2(pack2<F16>(b[0], b[1])), relu_bf16x2(pack2<F16>(b[2], b[3])));
}

// Diagnostic build (AI4E_CHAIN_STAMPS=1): s_memtime stamps at the phase boundaries (phase A, B/C setup + T2
// epilogue, the passes, the T1' epilogue + copy-out), per wave, written to g_chain_stamps (read SHARES only).
#ifndef AI4E_CHAIN_STAMPS
#define AI4E_CHAIN_STAMPS 0
#endif
// Diagnostic what-if builds (wrong numerics, timing only; tools/chain_stamps.py): 1 = phase A without its per-step
// weight loads (the K-loop reuses the first PD prefetched steps), 2 = no patch DMA (phase A reads whatever is in LDS)
#ifndef AI4E_CHAIN_WHATIF
#define AI4E_CHAIN_WHATIF 0
#endif
constexpr int CHAIN_NSEG = 5, CHAIN_MAXW = 65536;
#if AI4E_CHAIN_STAMPS
__device__ unsigned long long g_chain_stamps[CHAIN_MAXW * CHAIN_NSEG];
#define CHAIN_STAMP(k)                                                             \
  do {                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                             \
    unsigned long long _t;                                                         \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");  \
    __builtin_amdgcn_sched_barrier(0);                                             \
    ch_sum[k] += _t - ch_last;                                                     \
    ch_last = _t;                                                                  \
  } while (0)
#else
#define CHAIN_STAMP(k) \
  do {                 \
  } while (0)
#endif

// Bias of the 4 channels n0 + 4*(lane>>4) + 0..3 from a wave-uniform 16-float block: read through the
// constant address space (s_load: lgkmcnt, outside the hand-counted vmcnt bookkeeping), then a
// lane-group select on registers.
typedef const float __attribute__((address_space(4)))* const_f32_ptr;
__device__ __forceinline__ f32x4_t bias4(const float* blk, int g) {
  const const_f32_ptr b = reinterpret_cast<const_f32_ptr>(reinterpret_cast<uintptr_t>(blk));
  f32x4_t r;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    // readfirstlane pins each value to an SGPR so the selects below stay register selects (without it
    // hipcc folds select(load, load) into a per-lane vector load)
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

struct ChainParams {
  const uint16_t* x;  // T1 [N, H, W, ldx], MID channels at offset 0
  const uint16_t* w2;
  const float* b2;
  const uint16_t* w3;
  const float* b3;
  const uint16_t* res;  // [M, 4*MID]
  uint16_t* y;          // [M, 4*MID]
  const uint16_t* w1n;  // [MID rows, kpad1n >= 4*MID]   (NEXT)
  const float* b1n;
  uint16_t* t1n;        // [M, MID]                      (NEXT)
  const uint16_t* zero;
  int H, W, ldx, stride, OH, OW, M;
  int kpad2, kpad3, kpad1n;
  uint16_t* sink;
  const uint16_t* x0;   // DOWN: the block input [M, ldx0] (64 channels) whose 1x1 projection is the residual
  int ldx0;
  int pw2;              // patch mode: slots per patch row (W + 8 where it fits, else W + 2)
};

// Phase A "patch" mode (PATCH, stride 1): instead of gathering every 3x3 tap of every pixel through the
// LDS-DMA ring (nine 16-B gathers per pixel and channel chunk, 18-36 short dependent K steps), the workgroup
// DMAs the input rows its BM pixels touch, plus one halo row above and below, ONCE into LDS as a padded
// patch [rows][W + 2 slots][MID] (a zero slot at each row end = the left/right padding), waits once, and
// then runs the nine taps as pure LDS-read + MFMA steps: tap (kh, kw) of pixel (r, ow) is slot
// (r - r_lo + kh) * (W + 2) + ow + kw. A tap above / below the image (the row belongs to the neighbouring
// image in the flattened row order, or lies outside the tensor) reads the zero slot instead. The 16-B
// chunks of a slot are XOR-swizzled by the slot index (psw) so the 16 consecutive pixels of a fragment
// read conflict-free. Weights come straight from global memory (L2-resident, 4 K steps prefetched in
// registers). The 4 waves split the channels. The patch lives in the same LDS as phases B/C
// (the host only picks this mode when the patch fits the config's LDS).
template <int MID>
__device__ __forceinline__ int psw(int slot) {
  return MID == 64 ? ((slot >> 1) & 3) << 1 : (slot & 7) << 1;
}

template <int MID, int BM_, int MIDN = 0, bool DOWN = false, int ST = 4, bool BL = true>
struct ChainCfg {
  static constexpr int BM = BM_;              // pixels per workgroup
  static constexpr bool NEXT = MIDN > 0;      // chained 1x1 c1' (output width MIDN)
  static constexpr int WN = MID / 64;         // phase A / C: waves along channels
  static constexpr int WM = 4 / WN;           // phase A / C: waves along pixels
  static constexpr int WPX = BM / WM;         // phase A / C: pixels per wave
  static constexpr int FI = WPX / 16;         // phase A / C: pixel fragments per wave
  static constexpr int STAGES = ST;           // DMA ring depth (phase A pixel/weight ring, B/C weight ring)
  static constexpr int CA = BM / 64;          // phase A pixel-row DMAs per wave per stage
  static constexpr int CB = MID / 64;         // phase A / C weight-row DMAs per wave per stage
  static constexpr int A_PX = STAGES * BM * 64;           // phase A: pixel ring, then the weight ring
  static constexpr int A_BYTES = A_PX + STAGES * MID * 64;
  // B operand [T2 | X0] [BM x KB] (K-blocked; X0 = the 64-channel block input in DOWN mode, where the
  // downsample 1x1 is folded into c3 as extra K: W3' = [W3 | Wd], b3' = b3 + bd), later T1' staging
  static constexpr int KB = MID + (DOWN ? 64 : 0);
  static constexpr int T2_BYTES = BM * KB * 2;
  static constexpr int Y_BYTES = BM * 64 * 2;             // one 64-channel chunk [BM x 64] of R -> Y
  static constexpr int RING = T2_BYTES + Y_BYTES;         // B/C weight ring: STAGES x SLOT rows x 64 B
  static constexpr int SLOT = NEXT ? (MID > MIDN ? MID : MIDN) : MID;  // >= 64 (B) and MIDN (C) rows
  static constexpr int BC_BYTES = RING + STAGES * SLOT * 64;
  // phase C layout over the [BM x MIDN] T1' tile (4 waves, 64-channel wave columns)
  static constexpr int WNC = NEXT ? MIDN / 64 : 1;
  static constexpr int WMC = 4 / WNC;
  static constexpr int WPXC = BM / WMC;
  static constexpr int FIC = WPXC / 16;
  static constexpr int CBC = NEXT ? MIDN / 64 : 1;  // C weight-row DMAs per wave per stage
  static constexpr int LDS = A_BYTES > BC_BYTES ? A_BYTES : BC_BYTES;
  // MID 64: the c3 / c1' biases are staged in LDS past everything else (<= 1.5 KB, same occupancy) and read
  // back as one ds_read_b128 per 16-channel block: they seed the B accumulators (no epilogue add) and
  // replace the SGPR lane-group select of bias4 (~20 VALU per block). MID 128 has no LDS to spare (80 KB).
  static constexpr bool BIAS_LDS = BL && MID == 64 && LDS + (4 * MID + MIDN) * 4 <= 80 * 1024;
  static constexpr int NBIAS = 4 * MID + (NEXT ? MIDN : 0);  // floats: b3 then b1'
  static constexpr int LDS_ALL = LDS + (BIAS_LDS ? NBIAS * 4 : 0);
  // Otherwise (MID 128), when a weight-ring slot has >= 128 rows: B steps fill only its first 64 rows, so the
  // pass's c3 bias chunk (64 floats) rides in the free half of the pass's first B slot (one extra DMA per
  // wave per pass) and seeds the accumulators the same way.
  static constexpr bool BIAS_RING = !BIAS_LDS && BL && SLOT >= 128;
  static constexpr int NP = 4 * MID / 64;     // 64-channel passes over c3's output
  static constexpr int NB = KB / 32;          // B steps
  static constexpr int NC = 2;                // C steps (K = 64)
  static constexpr int SP = NB + NC;
  static constexpr int BPW = BM / 4;          // B: pixels per wave (all 64 channels of the chunk)
  static constexpr int BFI = BPW / 16;        // B: pixel fragments per wave
  static constexpr int NR = Y_BYTES / 1024 / 4;   // residual-chunk DMAs per wave
  static constexpr int NS = Y_BYTES / 16 / 256;   // 16-B Y copy-out stores per thread
  static_assert(!NEXT || BM * MIDN * 2 <= RING, "T1' staging fits below the weight ring");
  static constexpr int MINW = LDS_ALL <= 160 * 1024 / 3 ? 3 : 2;  // workgroups (= waves per SIMD) per CU
  static_assert(LDS_ALL <= 80 * 1024, "two workgroups per CU");
  static_assert(!BIAS_LDS || NBIAS <= 512, "bias staging: two values per thread");
  static_assert(FI >= 1 && FI <= 4 && BFI >= 1 && FIC >= 1 && FIC <= 4, "tile");
};

// byte offset of 16-B chunk c (channels 8c .. 8c + 7) of row r in the same tile
template <int BM>
__device__ __forceinline__ uint32_t tile_off16(int r, int c) {
  return (c >> 2) * BM * 64 + r * 64 + (((c & 3) ^ swt(r)) << 4);
}

// Measured and removed (profiles/r3_rreg/; code in the git history up to commit bc1ff0a): the residual chunk
// prefetched into registers a pass ahead (tile configs 9 / 11), bit-identical but -2 % end to end.
// Phase A in patch mode: every wave computes all BM pixels x MID/4 output channels (PWN = 4 waves along the channels).
// Measured and removed in round 5 (patches in profiles/r5_pruned/): a 2 x 2 phase-A split (PWN 2, neutral,
// profiles/r3_pw2/), padded unswizzled patch slots (neutral, profiles/r3_pad/), the SGPR lane-select biases of the
// round-2 kernel (the A/B reference of the LDS / ring-borne biases) and 256-pixel MID-64 ring tiles.
template <int MID, int BM_, int MIDN, bool DOWN, int ST, bool BL, bool PATCH, bool F16 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ChainCfg<MID, BM_, MIDN, DOWN, ST, BL>::MINW,
                                                                     ChainCfg<MID, BM_, MIDN, DOWN, ST, BL>::MINW)))
void conv_chain_kernel(const ChainParams p) {
  using Cfg = ChainCfg<MID, BM_, MIDN, DOWN, ST, BL>;
  static_assert(BM_ == 128, "128-pixel tiles (patch mode: 4 waves x all pixels; ring: 2 x 2 waves of 64 pixels)");
  constexpr bool NEXT = Cfg::NEXT;
  constexpr int FIC = Cfg::FIC, WPXC = Cfg::WPXC, CBC = Cfg::CBC;
  constexpr int WM = Cfg::WM, BM = Cfg::BM, STAGES = Cfg::STAGES, CA = Cfg::CA, CB = Cfg::CB;
  constexpr int FI = Cfg::FI, WPX = Cfg::WPX;
  constexpr int NB = Cfg::NB, NC = Cfg::NC, SP = Cfg::SP, BFI = Cfg::BFI;
  constexpr int C4 = 4 * MID;
  extern __shared__ __attribute__((aligned(1024))) uint8_t smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#if AI4E_CHAIN_STAMPS
  unsigned long long ch_sum[CHAIN_NSEG] = {0, 0, 0, 0, 0}, ch_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ch_last)::"memory");
#endif
  const int wm = wave % WM;
  const int wn = wave / WM;
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BM;
  const uint32_t sb = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem));
  const uint32_t PX = sb;
  uint8_t* const t2buf = smem;                      // [BM x MID] T2 (then T1' staging)
  uint8_t* const ybuf = smem + Cfg::T2_BYTES;       // [BM x 64] residual chunk -> Y chunk
  const uint32_t RING = sb + Cfg::RING;
  const uint16_t* const zero = p.zero;
  const int lg = lane >> 4;

  const int rin = lane >> 2;
  const int c = (lane & 3) ^ swz(rin);
  const int frow = lane & 15;
  const uint32_t fofs = frow * 64 + ((((lane >> 4) ^ swz(frow)) << 4));  // fragment byte offset in a 16-row block
  const uint32_t tofs = frow * 64 + ((((lane >> 4) ^ swt(frow)) << 4));  // the same in the T2 / Y / T1' tiles
  const int ct = (lane & 3) ^ swt(rin);  // logical chunk of a tile DMA lane (rows rin, physical chunk lane & 3)

  // bias values this thread stages into LDS once phase A has drained (loaded now, ahead of the DMA asm)
  float bstage[2] = {0.f, 0.f};
  if constexpr (Cfg::BIAS_LDS) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int idx = tid + 256 * e;
      if (idx < C4) bstage[e] = p.b3[idx];
      else if (NEXT && idx < Cfg::NBIAS) bstage[e] = p.b1n[idx - C4];
    }
  }

  // ================= phase A: T2 = relu(conv3x3(T1) + b2), K1 main loop (GATHER_TAP) =================
  f32x4_t acc[FI][4];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // patch mode: the 4 waves split the channels (each all BM pixels = PFI fragments x MID/4 channels = CF
  // fragments), so every weight element is loaded by exactly one wave
  constexpr int PWN = 4, PWM = 1;
  constexpr int PFI = PATCH ? BM_ / 16 / PWM : 1, CF = PATCH ? MID / 16 / PWN : 1;
  const int pwm = wave % PWM, pwn = wave / PWM;
  f32x4_t pacc[PFI][CF];
#pragma unroll
  for (int i = 0; i < PFI; ++i)
#pragma unroll
    for (int j = 0; j < CF; ++j) pacc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  if constexpr (PATCH) {
    constexpr int RB = MID * 2;    // bytes per pixel slot
    constexpr int CPS = RB / 16;   // 16-B chunks per slot
    const int W = p.W, W2 = p.pw2;
    const int NZ = W2 - W;   // zero slots per patch row: slot 0 and W + 1 .. W2 - 1
    const int r_lo = m0 / W;                          // flattened (image, row) index of the first pixel
    const int r_hi = (min(m0 + BM, p.M) - 1) / W;
    const int prows = r_hi - r_lo + 3;                // + one halo row above and below
    const int nrows = p.M / W;                        // N * H
    const int ipr = W * RB / 1024;                    // 1-KB DMA pieces per patch row (host: W * RB % 1024 == 0)
    {
      // the patch: row j = flattened row r_lo - 1 + j, data in slots 1..W (one contiguous 1-KB piece per wave DMA)
      for (int I = wave; I < prows * ipr; I += 4) {
        const int j = I / ipr, piece = I - j * ipr;
        const int R = r_lo - 1 + j;
        const int o = piece * 1024 + 16 * lane;
        const int s1 = o / RB;                          // data slot in the row (0-based)
        const int slot = j * W2 + 1 + s1;
        const int q = ((o % RB) >> 4) ^ psw<MID>(slot);  // logical chunk that belongs at this physical chunk
        const bool ok = R >= 0 && R < nrows;
        if (AI4E_CHAIN_WHATIF != 2)
          glds16(ok ? static_cast<const void*>(p.x + (static_cast<long>(R) * W + s1) * p.ldx + 8 * q) : zero,
                 sb + (j * W2 + 1) * RB + piece * 1024);
      }
      // zero pad slots (left / right of every row; with NZ = 8 the slots W + 1 .. W + 8 (= slot 0 of the next row)
      // hold one zero slot per residue mod 8, the source of masked taps; else slot 0)
      for (int g = tid; g < prows * NZ * CPS; g += 256) {
        const int j = g / (NZ * CPS), e = g - j * NZ * CPS;
        const int z = e / CPS;
        const int slot = j * W2 + (z == 0 ? 0 : W + z);
        *reinterpret_cast<uint4*>(smem + slot * RB + (e - z * CPS) * 16) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    // per pixel fragment: slot of tap (0, 0) and the row-validity bits of kh = 0, 1, 2
    int sbase[PFI], vmask[PFI];
#pragma unroll
    for (int i = 0; i < PFI; ++i) {
      const int m = m0 + pwm * (BM / PWM) + 16 * i + (lane & 15);
      if (m < p.M) {
        const int r = m / W, ow = m - r * W;
        const int oh = r % p.H;
        sbase[i] = (r - r_lo) * W2 + ow;
        vmask[i] = 2 | (oh > 0 ? 1 : 0) | (oh < p.H - 1 ? 4 : 0);
      } else {
        sbase[i] = 0;
        vmask[i] = 0;
      }
    }
    constexpr int SPT = MID / 32;   // K steps per tap
    constexpr int NKA = 9 * SPT;
    constexpr int PD = CHAIN_PD;  // weight K steps prefetched into registers
    const uint16_t* const wp = p.w2 + static_cast<long>(pwn * (MID / PWN) + (lane & 15)) * p.kpad2 + 8 * lg;
    bf16x8_t wr[PD][CF];
#pragma unroll
    for (int s = 0; s < PD; ++s)
#pragma unroll
      for (int j = 0; j < CF; ++j) wr[s][j] = *reinterpret_cast<const bf16x8_t*>(wp + j * 16L * p.kpad2 + s * 32);
    wait_vmcnt<0>();  // the patch landed (the weight loads above retire with it)
    lds_barrier();
    CHAIN_STAMP(4);  // patch DMA issue + wait (patch mode; its time is also inside segment 0 of ring mode)
    bf16x8_t fx[2][PFI];
    int soff[PFI], sws[PFI];
    auto tap_slots = [&](int t) __attribute__((always_inline)) {
      const int kh = t / 3, kw = t - 3 * (t / 3);
#pragma unroll
      for (int i = 0; i < PFI; ++i) {
        const int s0 = sbase[i] + kh * W2 + kw;
        const int slot = (vmask[i] >> kh) & 1 ? s0 : (NZ == 8 ? W + 1 + ((s0 - W - 1) & 7) : 0);
        soff[i] = slot * RB;
        sws[i] = psw<MID>(slot);
      }
    };
    auto read_px = [&](int s, bf16x8_t (&f)[PFI]) __attribute__((always_inline)) {
      const int q = (s % SPT) * 4 + lg;
#pragma unroll
      for (int i = 0; i < PFI; ++i) {
        f[i] = *reinterpret_cast<const bf16x8_t*>(smem + soff[i] + ((q ^ sws[i]) << 4));
      }
    };
    tap_slots(0);
    read_px(0, fx[0]);
#pragma unroll
    for (int s = 0; s < NKA; ++s) {
      if (s + 1 < NKA) {
        if ((s + 1) % SPT == 0) tap_slots((s + 1) / SPT);
        read_px(s + 1, fx[(s + 1) & 1]);
      }
#pragma unroll
      for (int i = 0; i < PFI; ++i)
#pragma unroll
        for (int j = 0; j < CF; ++j)
          pacc[i][j] = mfma_16x16x32<F16>(wr[s % PD][j], fx[s & 1][i], pacc[i][j]);
#if AI4E_CHAIN_WHATIF != 1  // what-if 1 (diagnostic, wrong numerics): no phase-A weight loads inside the K-loop
      if (s + PD < NKA) {
#pragma unroll
        for (int j = 0; j < CF; ++j)
          wr[s % PD][j] = *reinterpret_cast<const bf16x8_t*>(wp + j * 16L * p.kpad2 + (s + PD) * 32);
      }
#endif
    }
    lds_barrier();  // every wave finished reading the patch before phases B/C reuse the LDS
  } else {
    const int OHW = p.OH * p.OW;
    int ih0[CA], iw0[CA];
    const uint16_t* rowp[CA];
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int m = m0 + 16 * (wave + 4 * i) + rin;
      if (m < p.M) {
        const int img = m / OHW;
        const int rem = m - img * OHW;
        const int oh = rem / p.OW;
        const int ow = rem - oh * p.OW;
        ih0[i] = oh * p.stride - 1;
        iw0[i] = ow * p.stride - 1;
        rowp[i] = p.x + (static_cast<long>(img) * p.H * p.W + static_cast<long>(ih0[i]) * p.W + iw0[i]) * p.ldx +
                  8 * c;
      } else {
        ih0[i] = -(1 << 28);
        iw0[i] = 0;
        rowp[i] = nullptr;
      }
    }
    TapWalk tw;
    const int rowjump = (p.W - 3) * p.ldx;
    const uint16_t* const wsrc = p.w2 + static_cast<long>(16 * wave + rin) * p.kpad2 + 8 * c;
    const long wstep = 64L * p.kpad2;
    constexpr int NKA = 9 * MID / BK;  // even: MID % 64 == 0

    auto issue_a = [&](int kt) __attribute__((always_inline)) {
      const uint32_t xs = PX + (kt % STAGES) * BM * 64;
      const uint32_t ws = PX + Cfg::A_PX + (kt % STAGES) * MID * 64;
      const int toff = tw.off;
      const bool tap_ok = tw.kh < 3;
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const bool ok = tap_ok && static_cast<unsigned>(ih0[i] + tw.kh) < static_cast<unsigned>(p.H) &&
                        static_cast<unsigned>(iw0[i] + tw.kw) < static_cast<unsigned>(p.W);
        glds16(ok ? static_cast<const void*>(rowp[i] + toff) : zero, xs + 16 * (wave + 4 * i) * 64);
      }
      tw.next(BK, MID, 3, p.ldx, rowjump);
      const bool live = kt < NKA;
#pragma unroll
      for (int i = 0; i < CB; ++i)
        glds16(live ? static_cast<const void*>(wsrc + i * wstep + kt * BK) : zero, ws + 16 * (wave + 4 * i) * 64);
    };

    bf16x8_t fw0[4], fx0[FI], fw1[4], fx1[FI];
#define KC_READ(FW, FX, KT)                                                                             \
  {                                                                                                     \
    const uint8_t* x_ = smem + ((KT) % STAGES) * BM * 64 + (wm * WPX) * 64 + fofs;                      \
    const uint8_t* w_ = smem + Cfg::A_PX + ((KT) % STAGES) * MID * 64 + (wn * 64) * 64 + fofs;         \
    _Pragma("unroll") for (int j = 0; j < 4; ++j) FW[j] = *reinterpret_cast<const bf16x8_t*>(w_ + j * 1024); \
    _Pragma("unroll") for (int i = 0; i < FI; ++i) FX[i] = *reinterpret_cast<const bf16x8_t*>(x_ + i * 1024); \
  }
#define KC_STEP(KT, FWC, FXC, FWN, FXN)                                                                 \
  {                                                                                                     \
    const int kt_ = (KT);                                                                               \
    wait_vmcnt<(STAGES - 3) * (CA + CB)>();                                                             \
    lds_barrier();                                                                                      \
    KC_READ(FWN, FXN, kt_ + 1)                                                                          \
    _Pragma("unroll") for (int i = 0; i < FI; ++i)                                                      \
      _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                     \
        acc[i][j] = mfma_16x16x32<F16>(FWC[j], FXC[i], acc[i][j]);        \
    issue_a(kt_ + STAGES - 1);                                                                          \
  }
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s) issue_a(s);
    wait_vmcnt<(STAGES - 2) * (CA + CB)>();
    lds_barrier();
    KC_READ(fw0, fx0, 0)
    for (int kt = 0; kt < NKA; kt += 2) {
      KC_STEP(kt, fw0, fx0, fw1, fx1)
      KC_STEP(kt + 1, fw1, fx1, fw0, fx0)
    }
    wait_vmcnt<0>();
    lds_barrier();  // ring idle: every wave finished its reads, every DMA landed
#undef KC_STEP
#undef KC_READ
  }
  CHAIN_STAMP(0);  // phase A (3x3 main loop, patch or ring)
  float* const bias_lds = reinterpret_cast<float*>(smem + Cfg::LDS);  // [NBIAS] (BIAS_LDS); visible after pass 0's barrier
  if constexpr (Cfg::BIAS_LDS) {
#pragma unroll
    for (int e = 0; e < 2; ++e)
      if (tid + 256 * e < Cfg::NBIAS) bias_lds[tid + 256 * e] = bstage[e];
  }

  // ================= passes: B (c3 chunk), Y epilogue, C (c1' partial) =================
  // Weight stream step t: pass t / SP; NB steps of W3 rows [64 pp, +64) (B, k = 32 kb of MID), then
  // NC steps of W1' (all MIDN rows, k columns 64 pp + 32 kb) (C, NEXT only).
  constexpr int SPW = NEXT ? SP : NB;
  constexpr int NW = Cfg::NP * SPW;
  int ops = 0;        // vector-memory ops this wave issued since the phase-A drain
  int stage_end[NW];  // ops count right after stage t was issued (constants after unrolling)
  auto issue_w = [&](int t) __attribute__((always_inline)) {
    if (t >= NW) return;
    const int pp = t / SPW, r = t % SPW;
    const uint32_t ws = RING + (t % STAGES) * Cfg::SLOT * 64;
    if (r < NB) {  // 64 rows: one DMA per wave
      glds16(p.w3 + static_cast<long>(pp * 64 + 16 * wave + rin) * p.kpad3 + r * BK + 8 * c, ws + 16 * wave * 64);
      ops += 1;
      if (Cfg::BIAS_RING && r == 0) {  // bias chunk: wave w, lane l < 4 -> channels pp*64 + 16w + 4l .. +3
        glds16(lane < 4 ? static_cast<const void*>(p.b3 + pp * 64 + 16 * wave + 4 * lane) : zero,
               ws + 64 * 64 + wave * 1024);
        ops += 1;
      }
    } else {
      const uint16_t* src = p.w1n + static_cast<long>(16 * wave + rin) * p.kpad1n + pp * 64 + (r - NB) * BK + 8 * c;
#pragma unroll
      for (int i = 0; i < CBC; ++i) glds16(src + i * 64L * p.kpad1n, ws + 16 * (wave + 4 * i) * 64);
      ops += CBC;
    }
    stage_end[t] = ops;
  };
  if constexpr (DOWN) {
    // block input X0 -> K blocks MID/32.. of the B operand tile (before the weight prologue, so the first
    // stage wait also retires it); rows past M re-read row M-1 (never stored)
#pragma unroll
    for (int s = 0; s < BM / 32; ++s) {
      const int q = wave + 4 * s;
      const int kb = q / (BM / 16), rb = q % (BM / 16);
      const int row = rb * 16 + rin;
      glds16(p.x0 + static_cast<long>(min(m0 + row, p.M - 1)) * p.ldx0 + kb * BK + 8 * ct,
             sb + (MID / 32 + kb) * BM * 64 + rb * 16 * 64);
    }
    ops += BM / 32;
  }
#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t) issue_w(t);

  // T2 epilogue: + b2, ReLU, bf16 -> t2buf (phase A wave layout); the lane-group bias select once per j
  // (readfirstlane is convergent: hipcc does not CSE it across the i loop)
  if constexpr (PATCH && CF % 2 == 0) {
    // pairs of 16-channel blocks (j, j + 1) of one K block -> one 16-B write per lane and fragment
#pragma unroll
    for (int jp = 0; jp < CF / 2; ++jp) {
      const int nb = pwn * (MID / PWN) + 32 * jp;
      const f32x4_t b0 = bias4(p.b2 + nb, lg), b1 = bias4(p.b2 + nb + 16, lg);
#pragma unroll
      for (int i = 0; i < PFI; ++i) {
        const int r = pwm * (BM / PWM) + 16 * i + (lane & 15);
        f32x4_t a = pacc[i][2 * jp] + b0, b = pacc[i][2 * jp + 1] + b1;
        swap16(a, b);
        *reinterpret_cast<uint4*>(t2buf + tile_off16<BM>(r, nb / 8 + swap_chunk(lg))) = relu8<F16>(a, b);
      }
    }
  } else if constexpr (PATCH && PFI % 2 == 0) {
    // one 16-channel block per wave (MID 64): pairs of fragments 16 rows apart -> one 16-B write per lane
#pragma unroll
    for (int j = 0; j < CF; ++j) {
      const int nb = pwn * (MID / PWN) + 16 * j;
      const f32x4_t bj = bias4(p.b2 + nb, lg);
#pragma unroll
      for (int ip = 0; ip < PFI / 2; ++ip) {
        const int r = pwm * (BM / PWM) + 32 * ip + (lane & 15) + 16 * (lg & 1);
        f32x4_t a = pacc[2 * ip][j] + bj, b = pacc[2 * ip + 1][j] + bj;
        swap16(a, b);
        *reinterpret_cast<uint4*>(t2buf + tile_off16<BM>(r, nb / 8 + (lg >> 1))) = relu8<F16>(a, b);
      }
    }
  } else if constexpr (PATCH) {
    static_assert(!PATCH, "patch-mode T2 epilogue: CF or PFI even");
  }
  f32x4_t b2v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) b2v[j] = PATCH ? f32x4_t{0.f, 0.f, 0.f, 0.f} : bias4(p.b2 + wn * 64 + 16 * j, lg);
#pragma unroll
  for (int i = 0; i < (PATCH ? 0 : FI); ++i) {
    const int r = wm * WPX + 16 * i + (lane & 15);
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      f32x4_t a = acc[i][2 * jp] + b2v[2 * jp], b = acc[i][2 * jp + 1] + b2v[2 * jp + 1];
      swap16(a, b);
      *reinterpret_cast<uint4*>(t2buf + tile_off16<BM>(r, (wn * 64 + 32 * jp) / 8 + swap_chunk(lg))) = relu8<F16>(a, b);
    }
  }

  const int wmc = wave % Cfg::WMC, wnc = wave / Cfg::WMC;
  f32x4_t accn[FIC][4];  // T1' accumulators (NEXT), phase C wave layout, live across the passes
#pragma unroll
  for (int i = 0; i < FIC; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) accn[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // Per weight step: wait for the step's stage, barrier (which also orders the refill at the end of
  // the step: the DMA of step t goes into the slot of stage t-1, which every wave has finished reading),
  // fragments, MFMAs. Single-buffered fragments; the second workgroup on the CU covers the LDS latency.
  auto step_wait = [&](int t) __attribute__((always_inline)) {
    wait_vmcnt_n(ops - stage_end[t]);
    lds_barrier();
  };
  // B segment: this wave's BPW pixels x the 64 channels of chunk pp, K = MID from T2
  auto seg_b = [&](f32x4_t (&a)[BFI][4], int t0) {
#pragma unroll
    for (int kk = 0; kk < NB; ++kk) {
      const int t = t0 + kk;
      step_wait(t);
      bf16x8_t fw[4], fx[BFI];
      const uint8_t* w_ = smem + Cfg::RING + (t % STAGES) * Cfg::SLOT * 64 + fofs;
      const uint8_t* x_ = t2buf + kk * BM * 64 + (wave * Cfg::BPW) * 64 + tofs;
#pragma unroll
      for (int j = 0; j < 4; ++j) fw[j] = *reinterpret_cast<const bf16x8_t*>(w_ + j * 1024);
#pragma unroll
      for (int i = 0; i < BFI; ++i) fx[i] = *reinterpret_cast<const bf16x8_t*>(x_ + i * 1024);
      if (Cfg::BIAS_RING && kk == 0) {  // the first MFMA of each accumulator starts from the ring-borne bias
        const uint8_t* b_ = smem + Cfg::RING + (t % STAGES) * Cfg::SLOT * 64 + 64 * 64 + lg * 16;
        f32x4_t bj[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bj[j] = *reinterpret_cast<const f32x4_t*>(b_ + j * 1024);
#pragma unroll
        for (int i = 0; i < BFI; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) a[i][j] = mfma_16x16x32<F16>(fw[j], fx[i], bj[j]);
      } else {
#pragma unroll
        for (int i = 0; i < BFI; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            a[i][j] = mfma_16x16x32<F16>(fw[j], fx[i], a[i][j]);
      }
      issue_w(t + STAGES - 1);
    }
  };
  // C segment: accn += Y chunk [BM x 64] . W1'[:, chunk]^T (phase A wave layout)
  auto seg_c = [&](int t0) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < NC; ++kk) {
      const int t = t0 + kk;
      step_wait(t);
      bf16x8_t fw[4], fx[FIC];
      const uint8_t* w_ = smem + Cfg::RING + (t % STAGES) * Cfg::SLOT * 64 + (wnc * 64) * 64 + fofs;
      const uint8_t* x_ = ybuf + kk * BM * 64 + (wmc * WPXC) * 64 + tofs;
#pragma unroll
      for (int j = 0; j < 4; ++j) fw[j] = *reinterpret_cast<const bf16x8_t*>(w_ + j * 1024);
#pragma unroll
      for (int i = 0; i < FIC; ++i) fx[i] = *reinterpret_cast<const bf16x8_t*>(x_ + i * 1024);
#pragma unroll
      for (int i = 0; i < FIC; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          accn[i][j] = mfma_16x16x32<F16>(fw[j], fx[i], accn[i][j]);
      issue_w(t + STAGES - 1);
    }
  };

  // 16-B copy-out of a K-blocked [BM x W] tile (W = 64 or MID) to rows m0.. of a [M x ld] bf16 matrix.
  // Every store is unconditional (tail rows go to the sink) so the wave's vmcnt bookkeeping stays exact;
  // row bases are computed once per matrix and each pass adds its column offset as an immediate.
  auto row_bases = [&](auto wc, uint16_t* dst, int ld, uint16_t** base) __attribute__((always_inline)) {
    constexpr int CPR = decltype(wc)::value / 8;  // 16-B chunks per row
    constexpr int N = BM * CPR / 256;
#pragma unroll
    for (int e = 0; e < N; ++e) {
      const int g = tid + 256 * e;
      const int r = g / CPR, cq = g % CPR;
      base[e] = m0 + r < p.M ? dst + static_cast<long>(m0 + r) * ld + 8 * cq : p.sink;
    }
  };
  auto copy_out = [&](auto wc, const uint8_t* tile, uint16_t* const* base, int coff) __attribute__((always_inline)) {
    constexpr int CPR = decltype(wc)::value / 8;
    constexpr int N = BM * CPR / 256;
#pragma unroll
    for (int e = 0; e < N; ++e) {
      const int g = tid + 256 * e;
      const int r = g / CPR, cq = g % CPR;
      const uint4 v = *reinterpret_cast<const uint4*>(tile + (cq >> 2) * BM * 64 + r * 64 + (((cq & 3) ^ swt(r)) << 4));
      ai4e_conv::st16_stream(base[e] + coff, v);
    }
    ops += N;
  };
  using W64 = std::integral_constant<int, 64>;
  using WMIDN = std::integral_constant<int, NEXT ? MIDN : 64>;
  uint16_t* ybase[Cfg::NS];
  row_bases(W64{}, p.y, C4, ybase);


  auto pass = [&](auto ppc) __attribute__((always_inline)) {
    constexpr int pp = decltype(ppc)::value;
    if constexpr (pp > 0) copy_out(W64{}, ybuf, ybase, (pp - 1) * 64);
    lds_barrier();  // previous Y chunk fully consumed (and T2 visible at pass 0)
    // residual chunk R_pp -> ybuf (K-blocked swizzled [BM x 64], 16-B DMA rows; rows past M re-read
    // row M-1, never stored); none in DOWN mode (the projection is part of the B GEMM)
#pragma unroll
    for (int s = 0; s < (DOWN ? 0 : Cfg::NR); ++s) {
      const int q = wave + 4 * s;
      const int kb = q / (BM / 16), rb = q % (BM / 16);
      const int row = rb * 16 + rin;
      ai4e_conv::glds16_stream(p.res + static_cast<long>(min(m0 + row, p.M - 1)) * C4 + pp * 64 + kb * BK + 8 * ct,
             sb + Cfg::T2_BYTES + kb * BM * 64 + rb * 16 * 64);
    }
    ops += DOWN ? 0 : Cfg::NR;
    const int r_end = ops;

    f32x4_t accb[BFI][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4_t b0 = f32x4_t{0.f, 0.f, 0.f, 0.f};
      if constexpr (Cfg::BIAS_LDS) b0 = *reinterpret_cast<const f32x4_t*>(bias_lds + pp * 64 + 16 * j + 4 * lg);
#pragma unroll
      for (int i = 0; i < BFI; ++i) accb[i][j] = b0;  // B accumulators start at the c3 bias
    }
    seg_b(accb, pp * SPW);

    if constexpr (!DOWN) {
      wait_vmcnt_n(ops - r_end);
      lds_barrier();  // residual chunk visible
    }
#pragma unroll
    for (int i = 0; i < BFI; ++i) {
      const int r = wave * Cfg::BPW + 16 * i + (lane & 15);
      constexpr bool BSEED = Cfg::BIAS_LDS || Cfg::BIAS_RING;  // bias already in the accumulators
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        f32x4_t a = accb[i][2 * jp], b = accb[i][2 * jp + 1];
        if constexpr (!BSEED) {
          a += bias4(p.b3 + pp * 64 + 32 * jp, lg);
          b += bias4(p.b3 + pp * 64 + 32 * jp + 16, lg);
        }
        swap16(a, b);
        uint4* yp = reinterpret_cast<uint4*>(ybuf + tile_off16<BM>(r, 4 * jp + swap_chunk(lg)));
        const float f[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
        *yp = epilogue8<F16>(f, !DOWN, DOWN ? make_uint4(0u, 0u, 0u, 0u) : *yp, true);
      }
    }
    if constexpr (NEXT) {
      seg_c(pp * SPW + NB);  // its first barrier publishes the Y chunk
    } else {
      lds_barrier();
    }
  };
  static_assert(Cfg::NP == 4 || Cfg::NP == 8, "passes");
  CHAIN_STAMP(1);  // B/C weight prologue + T2 epilogue
  pass(std::integral_constant<int, 0>{});
  pass(std::integral_constant<int, 1>{});
  pass(std::integral_constant<int, 2>{});
  pass(std::integral_constant<int, 3>{});
  if constexpr (Cfg::NP == 8) {
    pass(std::integral_constant<int, 4>{});
    pass(std::integral_constant<int, 5>{});
    pass(std::integral_constant<int, 6>{});
    pass(std::integral_constant<int, 7>{});
  }
  CHAIN_STAMP(2);  // passes (B, Y epilogue + residual, C)
  copy_out(W64{}, ybuf, ybase, (Cfg::NP - 1) * 64);

  if constexpr (NEXT) {
    // T1' epilogue through the (idle) T2 (+ Y) buffer, then 16-B copy-out
    if constexpr (MIDN > MID) lds_barrier();  // the staging overlaps the Y chunk the copy-out just read
    f32x4_t b1v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      b1v[j] = Cfg::BIAS_LDS ? *reinterpret_cast<const f32x4_t*>(bias_lds + C4 + wnc * 64 + 16 * j + 4 * lg)
                             : bias4(p.b1n + wnc * 64 + 16 * j, lg);
#pragma unroll
    for (int i = 0; i < FIC; ++i) {
      const int r = wmc * WPXC + 16 * i + (lane & 15);
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        f32x4_t a = accn[i][2 * jp] + b1v[2 * jp], b = accn[i][2 * jp + 1] + b1v[2 * jp + 1];
        swap16(a, b);
        *reinterpret_cast<uint4*>(t2buf + tile_off16<BM>(r, (wnc * 64 + 32 * jp) / 8 + swap_chunk(lg))) = relu8<F16>(a, b);
      }
    }
    lds_barrier();
    uint16_t* tbase[BM * MIDN / 8 / 256];
    row_bases(WMIDN{}, p.t1n, MIDN, tbase);
    copy_out(WMIDN{}, t2buf, tbase, 0);
  }
#if AI4E_CHAIN_STAMPS
  wait_vmcnt<0>();
  CHAIN_STAMP(3);  // last Y chunk + T1' epilogue + copy-out (stores drained)
  if (lane == 0 && blockIdx.x * 4 + wave < CHAIN_MAXW) {
#pragma unroll
    for (int k = 0; k < CHAIN_NSEG; ++k) g_chain_stamps[(blockIdx.x * 4 + wave) * CHAIN_NSEG + k] = ch_sum[k];
  }
#endif
}

// Patch mode (phase A from an LDS patch of the input rows) applies to stride 1, an input row of whole 1-KB
// DMA pieces, a dense [N, H, W, MID] input, 128-pixel tiles and a patch that fits the config's LDS.
// Returns the patch row stride in slots (W + 8 where that fits, else W + 2), 0 = no patch mode.
template <int MID, int BM>
int patch_fits(const ChainParams& p, int lds_bytes) {
  if (BM != 128 || p.stride != 1 || p.ldx != MID || (p.W * MID * 2) % 1024) return 0;
  const long rows = (BM - 1 + p.W - 1) / p.W + 1 + 2;  // most rows BM consecutive pixels touch, + 2 halo rows
  const long rb = MID * 2;
  if (rows * (p.W + 8) * rb <= lds_bytes) return p.W + 8;
  return rows * (p.W + 2) * rb <= lds_bytes ? p.W + 2 : 0;
}

template <int MID, int MIDN, bool DOWN = false, bool F16 = false>
int launch_chain(ChainParams p, hipStream_t s, bool patch = false) {
  constexpr int BM = 128, ST = 4;
  constexpr bool BL = true;
  using Cfg = ChainCfg<MID, BM, MIDN, DOWN, ST, BL>;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(conv_chain_kernel<MID, BM, MIDN, DOWN, ST, BL, false, F16>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::LDS_ALL) != hipSuccess)
      return AI4E_ELAUNCH;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(conv_chain_kernel<MID, BM, MIDN, DOWN, ST, BL, true, F16>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::LDS_ALL) != hipSuccess)
      return AI4E_ELAUNCH;
    attr = true;
  }
  const int nb = ai4e_cdiv(p.M, Cfg::BM);
  if (patch && (p.pw2 = patch_fits<MID, BM>(p, Cfg::LDS)) > 0) {
    hipLaunchKernelGGL((conv_chain_kernel<MID, BM, MIDN, DOWN, ST, BL, true, F16>), dim3(nb), dim3(256), Cfg::LDS_ALL,
                       s, p);
    return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
  }
  hipLaunchKernelGGL((conv_chain_kernel<MID, BM, MIDN, DOWN, ST, BL, false, F16>), dim3(nb), dim3(256),
                     Cfg::LDS_ALL, s, p);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

template <typename T>
T* symbol_ptr(const void* sym) {
  void* a = nullptr;
  return hipGetSymbolAddress(&a, sym) == hipSuccess ? static_cast<T*>(a) : nullptr;
}

}  // namespace

namespace {
// fp16 (the ensemble's crop classifier, v_mfma_f32_16x16x32_f16): the default 128-pixel tiles with phase A from the
// LDS patch where the shape allows it, else the LDS-DMA ring; no A/B reference configs
int chain_f16(const ChainParams& p, bool down, bool next, int mid, int midn, hipStream_t stream) {
  if (down) return launch_chain<64, 64, true, true>(p, stream, true);
  if (mid == 64) {
    if (next && midn == 128) return launch_chain<64, 128, false, true>(p, stream, true);
    return next ? launch_chain<64, 64, false, true>(p, stream, true) : launch_chain<64, 0, false, true>(p, stream, true);
  }
  return next ? launch_chain<128, 128, false, true>(p, stream, true) : launch_chain<128, 0, false, true>(p, stream, true);
}

int chain_fwd(bool f16, const void* x, const void* w2, const void* b2, const void* w3, const void* b3,
              const void* res, void* y, const void* w1n, const void* b1n, void* t1n, int N, int H,
              int W, int ldx, int mid, int midn, int stride, int kpad2, int kpad3, int kpad1n,
              int tile_cfg, const void* x0, int ldx0, hipStream_t stream) {
  if (midn == 0) midn = mid;
  // DOWN mode (x0 given, res null): the residual is the 1x1 projection of x0 [M, ldx0] (64 channels), folded
  // into w3 = [W3 | Wd] (kpad3 >= mid + 64) and b3 = b3 + bd; MID 64, same-width chained c1', stride 1.
  const bool down = x0 != nullptr;
  if (down && (res || mid != 64 || midn != 64 || !w1n || stride != 1 || ldx0 % 8 || ldx0 < 64 || kpad3 < 128))
    return AI4E_EINVAL;
  if (down) res = x0;  // placeholder for the null checks below; never read
  if ((mid != 64 && mid != 128) || (midn != mid && !(mid == 64 && midn == 128)) || ldx % 8 || ldx < mid || kpad2 < 9 * mid || kpad2 % 64 ||
      kpad3 < mid || kpad3 % 8 || (stride != 1 && stride != 2) || !x || !w2 || !b2 || !w3 || !b3 || !res || !y ||
      (w1n && (!b1n || !t1n || kpad1n < 4 * mid || kpad1n % 8)))
    return AI4E_EINVAL;
  ChainParams p{};
  p.x = static_cast<const uint16_t*>(x);
  p.w2 = static_cast<const uint16_t*>(w2);
  p.b2 = static_cast<const float*>(b2);
  p.w3 = static_cast<const uint16_t*>(w3);
  p.b3 = static_cast<const float*>(b3);
  p.res = static_cast<const uint16_t*>(res);
  p.y = static_cast<uint16_t*>(y);
  p.w1n = static_cast<const uint16_t*>(w1n);
  p.b1n = static_cast<const float*>(b1n);
  p.t1n = static_cast<uint16_t*>(t1n);
  static const uint16_t* zero_p = symbol_ptr<const uint16_t>(HIP_SYMBOL(g_chain_zero));
  static uint16_t* sink_p = symbol_ptr<uint16_t>(HIP_SYMBOL(g_chain_sink));
  p.zero = zero_p;
  p.sink = sink_p;
  if (!p.zero || !p.sink) return AI4E_ELAUNCH;
  p.H = H; p.W = W; p.ldx = ldx; p.stride = stride;
  p.OH = (H + 2 - 3) / stride + 1;
  p.OW = (W + 2 - 3) / stride + 1;
  p.M = N * p.OH * p.OW;
  p.kpad2 = kpad2; p.kpad3 = kpad3; p.kpad1n = kpad1n;
  p.x0 = static_cast<const uint16_t*>(x0);
  p.ldx0 = ldx0;
  if (p.M <= 0) return AI4E_OK;
  const bool next = w1n != nullptr;
  if (f16) return chain_f16(p, down, next, mid, midn, stream);
  // tile_cfg: 3 = phase A from the LDS input patch where the shape allows it (stride 1, patch fits; the default),
  // else (and for any other value) the LDS-DMA ring; 128-pixel tiles either way
  const bool patch = (tile_cfg & 7) == 3;
  if (down) return launch_chain<64, 64, true>(p, stream, patch);
  if (mid == 64) {
    if (next && midn == 128) return launch_chain<64, 128>(p, stream, patch);
    return next ? launch_chain<64, 64>(p, stream, patch) : launch_chain<64, 0>(p, stream, patch);
  }
  return next ? launch_chain<128, 128>(p, stream, patch) : launch_chain<128, 0>(p, stream, patch);
}
}  // namespace

// Fused bottleneck chain (see header). x: T1 NHWC [N,H,W,ldx] bf16 (MID channels at offset 0);
// w2 [>=MID rows, kpad2 >= 9*MID] (k = (kh, kw, c)); w3 [>=4*MID rows, kpad3 >= MID];
// w1n [>=MIDN rows, kpad1n >= 4*MID] (nullptr: no next block, t1n unused); res, y [M, 4*MID];
// t1n [M, MIDN]. 3x3, pad 1, stride 1 or 2. (MID, MIDN) in {(64, 64), (64, 128), (128, 128)}; midn 0 = mid.
AI4E_API int ai4e_conv_chain_fwd(const void* x, const void* w2, const void* b2, const void* w3, const void* b3,
                                 const void* res, void* y, const void* w1n, const void* b1n, void* t1n, int N, int H,
                                 int W, int ldx, int mid, int midn, int stride, int kpad2, int kpad3, int kpad1n,
                                 int tile_cfg, const void* x0, int ldx0, hipStream_t stream) {
  return chain_fwd(false, x, w2, b2, w3, b3, res, y, w1n, b1n, t1n, N, H, W, ldx, mid, midn, stride, kpad2, kpad3,
                   kpad1n, tile_cfg, x0, ldx0, stream);
}

// The same chain on fp16 activations and weights (f16 MFMA, fp32 accumulation; tile_cfg ignored).
AI4E_API int ai4e_conv_chain_f16_fwd(const void* x, const void* w2, const void* b2, const void* w3, const void* b3,
                                     const void* res, void* y, const void* w1n, const void* b1n, void* t1n, int N, int H,
                                     int W, int ldx, int mid, int midn, int stride, int kpad2, int kpad3, int kpad1n,
                                     int tile_cfg, const void* x0, int ldx0, hipStream_t stream) {
  return chain_fwd(true, x, w2, b2, w3, b3, res, y, w1n, b1n, t1n, N, H, W, ldx, mid, midn, stride, kpad2, kpad3,
                   kpad1n, tile_cfg, x0, ldx0, stream);
}

#if AI4E_CHAIN_STAMPS
// Diagnostic build only: per-wave phase cycle sums of the last chain launch (65536 waves x 4).
AI4E_API int ai4e_chain_stamps_read(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_chain_stamps), sizeof(g_chain_stamps)) == hipSuccess ? AI4E_OK
                                                                                                      : AI4E_ELAUNCH;
}
#endif
