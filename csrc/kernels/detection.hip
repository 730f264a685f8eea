// K4 NMS (IoU bitmask + on-GPU greedy reduction), K5 RoIAlign (NHWC) and crop-and-resize
// (detector -> classifier hand-off, preprocess fused) — the irregular detection ops.
#include "common.h"

namespace {

constexpr int NMS_BLOCK = 64;  // one wave64 per 64x64 IoU tile; a 64-bit word per row

// boxes [B, N, 4] (x1,y1,x2,y2), sorted by descending score per image.
// mask [B, N, W] (W = ceil(N/64)): bit j of mask[b][i][jb] set <=> j = 64*jb+bit > i and IoU(i,j) > thr.
__global__ __launch_bounds__(NMS_BLOCK) void nms_mask_kernel(const float4* __restrict__ boxes, int N, float thr,
                                                            unsigned long long* __restrict__ mask) {
  const int b = blockIdx.z;
  const int ib = blockIdx.y, jb = blockIdx.x;
  const int W = (N + NMS_BLOCK - 1) / NMS_BLOCK;
  if (jb < ib) return;  // lower triangle never needed
  // VALU-bound (B * N^2 / 2 box pairs): the areas are computed once per box, and IoU > thr is tested as
  // inter > thr * union (union > 0) instead of a full-precision division per pair (~30 -> ~16 VALU per pair)
  __shared__ float4 sb[NMS_BLOCK];
  __shared__ float sarea[NMS_BLOCK];
  const int t = threadIdx.x;
  const int j = jb * NMS_BLOCK + t;
  if (j < N) {
    const float4 v = boxes[static_cast<long>(b) * N + j];
    sb[t] = v;
    sarea[t] = (v.z - v.x) * (v.w - v.y);
  }
  __syncthreads();
  const int i = ib * NMS_BLOCK + t;
  if (i >= N) return;
  const float4 bi = boxes[static_cast<long>(b) * N + i];
  const float ai = (bi.z - bi.x) * (bi.w - bi.y);
  unsigned long long bits = 0;
  const int jn = min(NMS_BLOCK, N - jb * NMS_BLOCK);
  auto pair = [&](int k) __attribute__((always_inline)) {
    const float4 bj = sb[k];
    const float iw = fmaxf(fminf(bi.z, bj.z) - fmaxf(bi.x, bj.x), 0.f);
    const float ih = fmaxf(fminf(bi.w, bj.w) - fmaxf(bi.y, bj.y), 0.f);
    const float inter = iw * ih;
    const float ua = ai + sarea[k] - inter;
    return ua > 0.f && inter > thr * ua;
  };
  if (jn == NMS_BLOCK) {
    // full column block: a uniform, fully unrolled walk (constant LDS offsets and bit positions); the diagonal
    // block's j <= i pairs are masked off afterwards instead of starting each lane's loop at its own t + 1
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int k = 0; k < 32; ++k) lo |= pair(k) ? (1u << k) : 0u;
#pragma unroll
    for (int k = 0; k < 32; ++k) hi |= pair(k + 32) ? (1u << k) : 0u;
    bits = (static_cast<unsigned long long>(hi) << 32) | lo;
    if (ib == jb) bits &= t == 63 ? 0ull : ~0ull << (t + 1);
  } else {
    for (int k = (ib == jb ? t + 1 : 0); k < jn; ++k)
      if (pair(k)) bits |= 1ull << k;
  }
  mask[(static_cast<long>(b) * N + i) * W + jb] = bits;
}

// 64-bit lane read (two v_readlane_b32) for the greedy scan below.
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), l);
  const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), l);
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}

// Greedy scan, one workgroup of NMS_MW_WAVES waves per image (round 5; the one-wave form it replaced, 210 vs
// 121 µs for the RPN call at batch 32, is in profiles/r5_pruned/). The scan is serial in the 64-box blocks; the
// one-wave form spent most of its time on the memory latency of OR-ing each block's kept rows into the bitmap (one
// round trip per 8 kept boxes) and of the next block's diagonal words, both on the critical path. Here:
//  * wave 0 resolves the blocks' diagonals; it prefetches each block's diagonal word AND the two words after it, two
//    blocks ahead, so the contribution of a block's kept boxes to the next two blocks' diagonals is an OR over lanes
//    of registers already loaded (no load on the critical path);
//  * waves 1..N-1 OR the kept rows' remaining words (> wb+2) into their partial bitmaps; their loads are issued
//    after a block is resolved and consumed two blocks later (with one block to land, the block period stretched
//    to the load latency: ~2.9 us per 64-box block);
//  * per block, two workgroup barriers: the row waves publish their partial word of the block, wave 0 publishes the
//    block's kept bits.
// Same greedy result as the sequential algorithm (same kept set, same order).
constexpr int NMS_MW_WAVES = 9;
constexpr int NMS_MW_ROWS = (64 + NMS_MW_WAVES - 2) / (NMS_MW_WAVES - 1);  // kept rows per row wave per block
static_assert(NMS_MW_ROWS * (NMS_MW_WAVES - 1) == 64, "row waves split a block's 64 bit positions evenly");

// a wave-uniform value read from LDS lands in VGPRs; moving it to SGPRs keeps the scalar loops scalar (a ctz of a
// VGPR value gives a VGPR lane index, and v_readlane with a VGPR index becomes a waterfall loop)
__device__ __forceinline__ unsigned long long uniform_u64(unsigned long long v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}

__device__ __forceinline__ unsigned long long wave_or_u64(unsigned long long v) {
  uint32_t lo = static_cast<uint32_t>(v), hi = static_cast<uint32_t>(v >> 32);
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    lo |= static_cast<uint32_t>(__shfl_xor(static_cast<int>(lo), m, 64));
    hi |= static_cast<uint32_t>(__shfl_xor(static_cast<int>(hi), m, 64));
  }
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}

__global__ __launch_bounds__(64 * NMS_MW_WAVES) void nms_reduce_mw_kernel(const unsigned long long* __restrict__ mask,
                                                                         const int* __restrict__ valid, int N,
                                                                         int max_out, int* __restrict__ keep,
                                                                         int* __restrict__ count) {
  __shared__ unsigned long long s_part[NMS_MW_WAVES];
  __shared__ unsigned long long s_keep;
  __shared__ int s_kept;
  const int b = blockIdx.x;
  const int W = (N + 63) / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = valid ? min(valid[b], N) : N;
  const unsigned long long* const mb = mask + static_cast<long>(b) * N * W;
  const int nblk = (n + 63) / 64;
  if (wave == 0) {
    int kept = 0;
    // words of block k's rows: the diagonal (col k) and the next two (cols k+1, k+2); prefetched two blocks ahead
    struct Diag {
      unsigned long long d, n1, n2;
    };
    auto diag_words = [&](int wb) __attribute__((always_inline)) {
      const int i_l = 64 * wb + lane;
      const bool in = wb < nblk && i_l < n;
      const long row = static_cast<long>(i_l) * W;
      Diag g;
      g.d = in ? mb[row + wb] : 0ull;
      g.n1 = in && wb + 1 < W ? mb[row + wb + 1] : 0ull;
      g.n2 = in && wb + 2 < W ? mb[row + wb + 2] : 0ull;
      return g;
    };
    // three register sets used round robin with STATIC roles (the loop body is unrolled by 3): rotating them with
    // copies made the compiler wait for every outstanding load (vmcnt(0)) at the first use, i.e. for the prefetch
    // issued two blocks ahead
    Diag dA = diag_words(0), dB = diag_words(1), dC;
    // kept boxes' contributions to a later block's diagonal word that the row waves have not OR-ed yet:
    // c1 = block wb-1 at word wb, c2a = block wb-2 at word wb, c2b = block wb-1 at word wb+1
    unsigned long long c1 = 0, c2a = 0, c2b = 0;
    // one block: prefetch block wb+2 into `into`, resolve block wb from `cur`; false when the scan is over
    auto step = [&](int wb, const Diag& cur, Diag& into) __attribute__((always_inline)) {
      into = diag_words(wb + 2);  // consumed two blocks later
      if (lane == 0) s_part[0] = 0ull;
      __syncthreads();  // B1: the row waves' partial words of block wb are published (blocks <= wb-3)
      unsigned long long remw = c1 | c2a;
#pragma unroll
      for (int w = 1; w < NMS_MW_WAVES; ++w) remw |= s_part[w];
      remw = uniform_u64(remw);
      const int inblk = min(64, n - 64 * wb);
      unsigned long long alive = ~remw & (inblk == 64 ? ~0ull : ((1ull << inblk) - 1));
      unsigned long long keepbits = 0, k1 = 0, k2 = 0;
      int kb = 0;
      while (alive && kept + kb < max_out) {
        const int i = __builtin_ctzll(alive);
        keepbits |= 1ull << i;
        ++kb;
        alive &= ~(1ull << i);
        alive &= ~readlane_u64(cur.d, i);
        // the kept box's words of the next two blocks, read in the same scalar loop (a 64-lane OR reduction by
        // shuffles cost ~12 dependent LDS round trips per word)
        k1 |= readlane_u64(cur.n1, i);
        k2 |= readlane_u64(cur.n2, i);
      }
      if ((keepbits >> lane) & 1ull)
        keep[static_cast<long>(b) * max_out + kept + __builtin_popcountll(keepbits & ((1ull << lane) - 1))] =
            64 * wb + lane;
      kept += kb;
      c1 = k1;   // block wb at word wb+1
      c2a = c2b; // block wb-1 at word wb+1
      c2b = k2;  // block wb at word wb+2
      if (lane == 0) {
        s_keep = keepbits;
        s_kept = kept;
      }
      __syncthreads();  // B2: block wb resolved
      return wb + 1 < nblk && kept < max_out;
    };
    for (int wb = 0; wb < nblk; wb += 3) {
      if (!step(wb, dA, dC)) break;
      if (!step(wb + 1, dB, dA)) break;
      if (!step(wb + 2, dC, dB)) break;
    }
    if (lane == 0) count[b] = min(kept, max_out);
    // the rows past the count are padding (-1): the caller needs no fill launch
    for (int i = min(kept, max_out) + lane; i < max_out; i += 64) keep[static_cast<long>(b) * max_out + i] = -1;
    return;
  }
  // row waves: partial bitmap words lane and lane + 64. A block's kept rows are loaded after its B2 and OR-ed two
  // blocks later (pA), so two block periods hide the load latency; words wb+1 and wb+2 come from wave 0's carries
  unsigned long long rem0 = 0, rem1 = 0;
  // two row buffers with static roles (the loop body is unrolled by 2; see wave 0's note on register rotation):
  // at block wb the buffer of parity wb holds block wb-2's rows, is OR-ed, then refilled with block wb's rows
  unsigned long long pa0[NMS_MW_ROWS], pa1[NMS_MW_ROWS], pb0[NMS_MW_ROWS], pb1[NMS_MW_ROWS];
#pragma unroll
  for (int u = 0; u < NMS_MW_ROWS; ++u) pa0[u] = pa1[u] = pb0[u] = pb1[u] = 0ull;
  const int w0 = lane, w1 = lane + 64;
  auto rstep = [&](int wb, unsigned long long (&q0)[NMS_MW_ROWS], unsigned long long (&q1)[NMS_MW_ROWS])
      __attribute__((always_inline)) {
    if (lane == (wb & 63)) s_part[wave] = wb < 64 ? rem0 : rem1;  // blocks <= wb-3
    __syncthreads();  // B1
    __syncthreads();  // B2
#pragma unroll
    for (int u = 0; u < NMS_MW_ROWS; ++u) {  // block wb-2's rows
      rem0 |= q0[u];
      rem1 |= q1[u];
    }
    unsigned long long kbits = uniform_u64(s_keep);
    const int kept = __builtin_amdgcn_readfirstlane(s_kept);
    // this wave's share of the block's kept rows: the kept boxes at bit positions [8 (wave-1), 8 wave)
    const bool ok0 = w0 > wb + 2 && w0 < W, ok1 = w1 > wb + 2 && w1 < W;
    const int base_bit = NMS_MW_ROWS * (wave - 1);
    long rows[NMS_MW_ROWS];
#pragma unroll
    for (int q = 0; q < NMS_MW_ROWS; ++q)  // (static indices: a compacted runtime-indexed array went to scratch)
      rows[q] = ((kbits >> (base_bit + q)) & 1ull) ? static_cast<long>(64 * wb + base_bit + q) * W : -1;
#pragma unroll
    for (int q = 0; q < NMS_MW_ROWS; ++q) {
      q0[q] = rows[q] >= 0 && ok0 ? mb[rows[q] + w0] : 0ull;
      q1[q] = rows[q] >= 0 && ok1 ? mb[rows[q] + w1] : 0ull;
    }
    return wb + 1 < nblk && kept < max_out;
  };
  for (int wb = 0; wb < nblk; wb += 2) {
    if (!rstep(wb, pa0, pa1)) break;
    if (!rstep(wb + 1, pb0, pb1)) break;
  }
}

// RPN proposals of one FPN level, decoded straight into the all-level buffers (replaces ~20 small PyTorch
// launches per level: gather of deltas and anchors, box decode, clip, sigmoid, min-size mask, concat).
// head: bf16 [B, HW, ldh] (A objectness logits, then 4A deltas per pixel); idx: int64 [B, k] top-k flat
// indices pos * A + a; anchors fp32 [HW * A, 4]; outputs at columns [off, off + k) of boxes [B, KT, 4],
// scores [B, KT] (sigmoid, -1 for boxes under min_size) and lvl [B, KT].
__global__ __launch_bounds__(256) void rpn_decode_kernel(const uint16_t* __restrict__ head, const long* __restrict__ idx,
                                                         const float4* __restrict__ anchors, float4* __restrict__ boxes,
                                                         float* __restrict__ scores, float* __restrict__ lvl, int B,
                                                         int HW, int ldh, int A, int k, int KT, int off, float level,
                                                         float img_h, float img_w, float min_size, float clip) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= B * k) return;
  const int b = t / k, j = t - b * k;
  const long flat = idx[static_cast<long>(b) * k + j];
  const int pos = static_cast<int>(flat / A), a = static_cast<int>(flat - static_cast<long>(pos) * A);
  const uint16_t* hp = head + (static_cast<long>(b) * HW + pos) * ldh;
  const float obj = bf16_to_f32(hp[a]);
  const float dx = bf16_to_f32(hp[A + 4 * a]), dy = bf16_to_f32(hp[A + 4 * a + 1]);
  const float dw = fminf(bf16_to_f32(hp[A + 4 * a + 2]), clip), dh = fminf(bf16_to_f32(hp[A + 4 * a + 3]), clip);
  const float4 an = anchors[flat];
  const float w = an.z - an.x, h = an.w - an.y;
  const float cx = an.x + 0.5f * w, cy = an.y + 0.5f * h;
  const float pcx = dx * w + cx, pcy = dy * h + cy, pw = expf(dw) * w, ph = expf(dh) * h;
  const float x1 = fminf(fmaxf(pcx - 0.5f * pw, 0.f), img_w), y1 = fminf(fmaxf(pcy - 0.5f * ph, 0.f), img_h);
  const float x2 = fminf(fmaxf(pcx + 0.5f * pw, 0.f), img_w), y2 = fminf(fmaxf(pcy + 0.5f * ph, 0.f), img_h);
  const long o = static_cast<long>(b) * KT + off + j;
  boxes[o] = make_float4(x1, y1, x2, y2);
  scores[o] = (x2 - x1 < min_size || y2 - y1 < min_size) ? -1.f : 1.f / (1.f + expf(-obj));
  lvl[o] = level;
}

// RPN top-k of one FPN level (replaces the logits copy + torch.topk, whose multi-block path is not safe to replay in a
// HIP graph once other allocations have come and gone between replays: bench/replay_repro.py, profiles/r4_replay/).
// One 1024-thread workgroup per image reads the A objectness logits per pixel straight from the RPN head (bf16
// [B, HW, ldh]) and selects the k largest by a two-pass 8-bit radix select on order-preserving 16-bit keys (LDS
// histograms; NaN above +inf, as torch.topk). Ties of the k-th largest key are taken lowest flat index first, so the
// selected SET is the k largest by (value desc, index asc), the same set as a stable descending sort's first k
// (ops/detection.py's CPU path). Output: the k flat indices pos * A + a (int64, [B, k]): every key above the k-th in
// index order, then the taken ties in index order — deterministic, no global atomics, every write inside [0, k) by
// construction (the host guarantees k <= HW * A).
// Histogram updates are run-length coalesced per thread (a thread adds its count for a bin once per run of equal bins
// instead of once per element): the RPN logits of a level crowd into a few high-byte bins, and one LDS atomic per
// element serialized those lanes (68.8 % bank conflicts, profiles/r4h_det/pmc_by_kernel.txt).
constexpr int TOPK_THREADS = 1024;

__device__ __forceinline__ uint32_t bf16_order_key(uint16_t v) {
  return (v & 0x8000u) ? (~static_cast<uint32_t>(v) & 0xffffu) : (static_cast<uint32_t>(v) | 0x8000u);
}

// Wave-aggregated LDS histogram update: the lanes of a wave that hold the same bin add their count with ONE atomic
// (a loop over the distinct bins present, usually 2-5 for the RPN logits' high bytes) instead of 64 atomics that
// serialize on the same bank. Called from wave-uniform control flow.
__device__ __forceinline__ void wave_hist_add(int* hist, int bin, bool valid) {
  const int lane = threadIdx.x & 63;
  unsigned long long active = __ballot(valid);
  while (active) {
    const int leader = __ffsll(static_cast<long long>(active)) - 1;
    const int lb = __shfl(bin, leader, 64);
    const unsigned long long same = __ballot(valid && bin == lb);
    if (lane == leader) atomicAdd(&hist[lb], static_cast<int>(__popcll(same)));
    active &= ~same;
    valid = valid && bin != lb;
  }
}

// The radix-select bin step, in parallel: the bin d holding the k-th largest key (counting down from 255; keys above
// it: cum0 + the bins above d) is the one whose exclusive suffix sum is < k and inclusive one >= k (bin 0 when fewer
// than k keys). Threads 0..255 (4 waves): wave-level inclusive scan + the waves' totals. Was one thread walking up to
// 256 bins with an LDS round trip each: ~11 us per pass, the fixed cost that made a 300-key level take 26 us.
__device__ __forceinline__ void topk_select_bin(const int* hist, int k, int cum0, int* sel_bin, int* sel_cum,
                                                int* wsum) {
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  int h = 0, v = 0;
  if (t < 256) {
    h = hist[255 - t];  // t-th bin from the top
    v = h;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(v, off, 64);
      if (lane >= off) v += y;
    }
    if (lane == 63) wsum[w] = v;
  }
  __syncthreads();
  if (t < 256) {
    int base = cum0;
    for (int q = 0; q < w; ++q) base += wsum[q];
    const int incl = base + v, above = incl - h, d = 255 - t;
    if (above < k && (incl >= k || d == 0)) {
      *sel_bin = d;
      *sel_cum = above;
    }
  }
  __syncthreads();
}

// Exclusive scans of two per-thread counts over the 1024 threads: wave shuffles, then the 16 wave totals.
__device__ __forceinline__ void topk_scan2(int a, int c, int& ea, int& ec, int* wa, int* wc) {
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  int va = a, vc = c;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int ya = __shfl_up(va, off, 64), yc = __shfl_up(vc, off, 64);
    if (lane >= off) {
      va += ya;
      vc += yc;
    }
  }
  if (lane == 63) {
    wa[w] = va;
    wc[w] = vc;
  }
  __syncthreads();
  int ba = 0, bc = 0;
  for (int q = 0; q < w; ++q) {
    ba += wa[q];
    bc += wc[q];
  }
  ea = ba + va - a;
  ec = bc + vc - c;
}

constexpr int TOPK_UNROLL = 8;       // keys a thread has in flight per histogram step
constexpr int TOPK_MASK_WORDS = 4;   // pass 3 keeps a chunk's > / == flags in registers for chunks <= 128 keys

__global__ __launch_bounds__(TOPK_THREADS) void rpn_topk_kernel(const uint16_t* __restrict__ head, int HW, int ldh,
                                                                int A, int k, long* __restrict__ idx) {
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int n = HW * A;
  const uint16_t* const hb = head + static_cast<long>(b) * HW * ldh;
  __shared__ int hist[256];
  __shared__ int sel[3];  // high byte of the k-th key, its low byte, keys above it
  __shared__ int wa[TOPK_THREADS / 64], wc[TOPK_THREADS / 64];
  auto key_at = [&](int e) __attribute__((always_inline)) {
    const int pos = e / A;
    return bf16_order_key(hb[static_cast<long>(pos) * ldh + (e - pos * A)]);
  };
  // passes 1 / 2: the histogram of the high byte, then of the low byte among keys with the selected high byte. Every
  // thread keeps TOPK_UNROLL keys in flight (the loop is latency-bound: one workgroup per image), and the updates
  // are wave-aggregated (the logits crowd into a few bins)
  // a pixel's A <= 4 logits as one 8-byte load (the head rows are 8-byte aligned: ldh % 4 == 0) instead of A loads
  const bool vec = A <= 4 && (ldh & 3) == 0 && (reinterpret_cast<uintptr_t>(head) & 7) == 0;
  auto pix4 = [&](int pos) __attribute__((always_inline)) {
    return *reinterpret_cast<const uint2*>(hb + static_cast<long>(pos) * ldh);
  };
  auto lane16 = [](const uint2& v, int a) __attribute__((always_inline)) {
    const uint32_t w = a < 2 ? v.x : v.y;
    return static_cast<uint16_t>((a & 1) ? (w >> 16) : (w & 0xffffu));
  };
  auto histogram = [&](int pass, uint32_t hi) __attribute__((always_inline)) {
    if (t < 256) hist[t] = 0;
    __syncthreads();
    if (vec) {
      for (int p0 = 0; p0 < HW; p0 += TOPK_THREADS * TOPK_UNROLL) {
        uint2 pv[TOPK_UNROLL];
#pragma unroll
        for (int u = 0; u < TOPK_UNROLL; ++u) {
          const int pos = p0 + u * TOPK_THREADS + t;
          pv[u] = pos < HW ? pix4(pos) : make_uint2(0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < TOPK_UNROLL; ++u) {
          const bool inp = p0 + u * TOPK_THREADS + t < HW;
          for (int a = 0; a < A; ++a) {  // (A is workgroup-uniform: the wave-aggregated update stays uniform)
            const uint32_t kk = bf16_order_key(lane16(pv[u], a));
            if (pass == 0) {
              wave_hist_add(hist, static_cast<int>(kk >> 8), inp);
            } else if (inp && (kk >> 8) == hi) {
              atomicAdd(&hist[kk & 255u], 1);
            }
          }
        }
      }
      __syncthreads();
      return;
    }
    for (int e0 = 0; e0 < n; e0 += TOPK_THREADS * TOPK_UNROLL) {
      uint32_t kk[TOPK_UNROLL];
#pragma unroll
      for (int u = 0; u < TOPK_UNROLL; ++u) {
        const int e = e0 + u * TOPK_THREADS + t;
        kk[u] = e < n ? key_at(e) : 0xffffffffu;
      }
#pragma unroll
      for (int u = 0; u < TOPK_UNROLL; ++u) {
        if (pass == 0) {  // high bytes: a few hot bins, one atomic per distinct bin per wave
          wave_hist_add(hist, static_cast<int>(kk[u] >> 8), kk[u] != 0xffffffffu);
        } else if (kk[u] != 0xffffffffu && (kk[u] >> 8) == hi) {  // low bytes of one high bin: spread, few keys
          atomicAdd(&hist[kk[u] & 255u], 1);
        }
      }
    }
    __syncthreads();
  };
  histogram(0, 0u);
  topk_select_bin(hist, k, 0, &sel[0], &sel[2], wa);
  const uint32_t hi = static_cast<uint32_t>(sel[0]);
  const int cum_hi = sel[2];
  histogram(1, hi);
  topk_select_bin(hist, k, cum_hi, &sel[1], &sel[2], wa);
  const uint32_t T = (hi << 8) | static_cast<uint32_t>(sel[1]);
  const int gt = sel[2], need = k - gt;  // keys above T; ties of T to take
  // pass 3: thread t owns the contiguous index range [e0, e1) (index order across threads), per-thread counts,
  // exclusive scans, then the writes; the counting loop remembers each key's > / == flags in registers so the write
  // loop does not read the keys again (chunks of <= 32 * TOPK_MASK_WORDS keys; longer ones re-read)
  const int chunk = (n + TOPK_THREADS - 1) / TOPK_THREADS;
  const int e0 = min(n, t * chunk), e1 = min(n, e0 + chunk);
  const bool masked = chunk <= 32 * TOPK_MASK_WORDS;
  uint32_t mg[TOPK_MASK_WORDS] = {0u, 0u, 0u, 0u}, me[TOPK_MASK_WORDS] = {0u, 0u, 0u, 0u};
  int cg = 0, ce = 0;
  int cur_pos = -1;
  uint2 cur_v = make_uint2(0u, 0u);
  auto key_seq = [&](int e) __attribute__((always_inline)) {  // keys in index order: one load per pixel
    if (!vec) return key_at(e);
    const int pos = e / A;
    if (pos != cur_pos) {
      cur_pos = pos;
      cur_v = pix4(pos);
    }
    return bf16_order_key(lane16(cur_v, e - pos * A));
  };
  for (int e = e0; e < e1; e += TOPK_UNROLL) {
    uint32_t kk[TOPK_UNROLL];
#pragma unroll
    for (int u = 0; u < TOPK_UNROLL; ++u) kk[u] = e + u < e1 ? key_seq(e + u) : 0u;
#pragma unroll
    for (int u = 0; u < TOPK_UNROLL; ++u) {
      if (e + u >= e1) break;
      const bool g = kk[u] > T, q = kk[u] == T;
      cg += g;
      ce += q;
      const int j = e + u - e0;
      if (masked) {
#pragma unroll
        for (int w = 0; w < TOPK_MASK_WORDS; ++w)  // (register-select: no runtime-indexed array)
          if ((j >> 5) == w) {
            mg[w] |= static_cast<uint32_t>(g) << (j & 31);
            me[w] |= static_cast<uint32_t>(q) << (j & 31);
          }
      }
    }
  }
  int og, oe;
  topk_scan2(cg, ce, og, oe, wa, wc);
  long* const out = idx + static_cast<long>(b) * k;
  if (masked) {
#pragma unroll
    for (int w = 0; w < TOPK_MASK_WORDS; ++w) {
      uint32_t m = mg[w] | me[w];
      while (m) {
        const int bit = __builtin_ctz(m);
        m &= m - 1;
        const int e = e0 + 32 * w + bit;
        if ((mg[w] >> bit) & 1u) {
          out[og++] = e;
        } else if (oe < need) {
          out[gt + oe++] = e;
        }
      }
    }
    return;
  }
  for (int e = e0; e < e1; ++e) {
    const uint32_t kk = key_at(e);
    if (kk > T) {
      out[og++] = e;
    } else if (kk == T && oe < need) {
      out[gt + oe++] = e;
    }
  }
}

// Descending sort of every row of fp32 scores [B, N] (N <= 8192) -> order [B, N] int64, ties by lower index first: one
// 1024-thread workgroup per row runs a bitonic network over next_pow2(N) 64-bit keys (order(score) << 32 | ~index) in LDS.
// Replaces torch.argsort for the RPN's all-level proposal sort (N = 4300 at 640^2, above the library's in-place small
// sort, so it went to a multi-kernel library sort with temporaries; kept out of captured graphs, profiles/r4_replay/).
constexpr int ROWSORT_THREADS = 1024, ROWSORT_MAX = 8192;

__device__ __forceinline__ uint32_t f32_order_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(ROWSORT_THREADS) void row_sort_desc_kernel(const float* __restrict__ scores, int N, int P,
                                                                       long* __restrict__ order) {
  __shared__ unsigned long long key[ROWSORT_MAX];
  const int t = threadIdx.x;
  const float* const sr = scores + static_cast<long>(blockIdx.x) * N;
  for (int i = t; i < P; i += ROWSORT_THREADS)  // padding keys are 0: below every real key (whose low word is ~i > 0)
    key[i] = i < N ? (static_cast<unsigned long long>(f32_order_key(sr[i])) << 32) | (0xffffffffu - static_cast<uint32_t>(i))
                   : 0ull;
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = t; i < P; i += ROWSORT_THREADS) {
        const int l = i ^ j;
        if (l > i) {
          const unsigned long long a = key[i], c = key[l];
          if (((i & k) == 0) ? (a < c) : (a > c)) {  // descending runs where bit k of i is clear
            key[i] = c;
            key[l] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  long* const o = order + static_cast<long>(blockIdx.x) * N;
  for (int i = t; i < N; i += ROWSORT_THREADS) o[i] = static_cast<long>(0xffffffffu - static_cast<uint32_t>(key[i]));
}

// Sort + select of one NMS stage (the proposals' all-level sort, the detections' per-class sort), one 1024-thread
// workgroup per row: the row's scores are sorted descending in LDS (the bitonic network of row_sort_desc_kernel, ties by
// lower index), then the same workgroup gathers the sorted scores and boxes, the boxes offset by their group
// (group * scale: batched NMS across FPN levels / classes by coordinate offsets), the sorted group values and the
// number of valid entries (score >= 0; invalid ones carry -1 and sort last). Groups come from `grp` (fp32, e.g. the
// FPN level) or, with grp null, from the index: group = index % grp_mod + 1 (the detections' class label, as laid out
// by det_decode_kernel). Replaces argsort (a library radix sort over 4 K+ keys, not graph-safe) + four gathers + a
// sum-reduction + the offset arithmetic: ~10 library launches per NMS stage.
// Register-resident bitonic network: thread t holds keys t * KPT .. t * KPT + KPT - 1 in registers. Steps with
// partner distance j < KPT are compare-exchanges inside a thread, KPT <= j < 64 KPT cross lanes of one wave by
// shuffles (no barrier), and only j >= 64 KPT (the last log2(total / 64 KPT) steps of each merge: 10 of the 91 steps
// at 8192 keys) go through LDS with barriers. The LDS steps use a transposed layout (key (t, r) at r * 1024 + t) so a
// wave's reads are consecutive. Same network, same comparisons: the same order as the all-LDS form.
template <int KPT, int J>
__device__ __forceinline__ void bitonic_regs(unsigned long long (&v)[KPT], int base, int k) {
#pragma unroll
  for (int r = 0; r < KPT; ++r) {
    if ((r & J) == 0) {
      const bool desc = ((base + r) & k) == 0;
      const unsigned long long a = v[r], c = v[r + J];
      const unsigned long long hi = a > c ? a : c, lo = a > c ? c : a;
      v[r] = desc ? hi : lo;
      v[r + J] = desc ? lo : hi;
    }
  }
}

template <int KPT>
__global__ __launch_bounds__(ROWSORT_THREADS) void sort_select_kernel(
    const float* __restrict__ scores, const float4* __restrict__ boxes, const float* __restrict__ grp, int grp_mod,
    float scale, int N, int P, float* __restrict__ s_out, float4* __restrict__ b_out, float4* __restrict__ boff_out,
    float* __restrict__ g_out, long* __restrict__ lab_out, int* __restrict__ valid) {
  __shared__ unsigned long long key[ROWSORT_MAX];
  __shared__ int nvalid;
  const int t = threadIdx.x;
  const long row = blockIdx.x;
  const float* const sr = scores + row * N;
  if (t == 0) nvalid = 0;
  constexpr int total = KPT * ROWSORT_THREADS;  // >= P (padding keys 0 sort last)
  const int base = t * KPT;
  unsigned long long v[KPT];
#pragma unroll
  for (int r = 0; r < KPT; ++r) {
    const int i = base + r;
    v[r] = i < N ? (static_cast<unsigned long long>(f32_order_key(sr[i])) << 32) | (0xffffffffu - static_cast<uint32_t>(i))
                 : 0ull;
  }
  (void)P;
  for (int k = 2; k <= total; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j < KPT) {
        if constexpr (KPT > 4) { if (j == 4) bitonic_regs<KPT, 4>(v, base, k); }
        if constexpr (KPT > 2) { if (j == 2) bitonic_regs<KPT, 2>(v, base, k); }
        if constexpr (KPT > 1) { if (j == 1) bitonic_regs<KPT, 1>(v, base, k); }
        continue;
      }
      const int m = j / KPT;  // partner thread t ^ m, same register r
      if (m < 64) {
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
          const unsigned long long x = v[r];
          const uint32_t ylo = static_cast<uint32_t>(__shfl_xor(static_cast<int>(static_cast<uint32_t>(x)), m, 64));
          const uint32_t yhi = static_cast<uint32_t>(__shfl_xor(static_cast<int>(static_cast<uint32_t>(x >> 32)), m, 64));
          const unsigned long long y = (static_cast<unsigned long long>(yhi) << 32) | ylo;
          const int i = base + r;
          const bool keep_hi = ((i & j) == 0) == ((i & k) == 0);
          v[r] = keep_hi ? (x > y ? x : y) : (x > y ? y : x);
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < KPT; ++r) key[r * ROWSORT_THREADS + t] = v[r];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < KPT; ++r) {
        const unsigned long long x = v[r], y = key[r * ROWSORT_THREADS + (t ^ m)];
        const int i = base + r;
        const bool keep_hi = ((i & j) == 0) == ((i & k) == 0);
        v[r] = keep_hi ? (x > y ? x : y) : (x > y ? y : x);
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int r = 0; r < KPT; ++r) key[base + r] = v[r];  // natural order for the gathers below
  __syncthreads();
  int mine = 0;
  for (int i = t; i < N; i += ROWSORT_THREADS) {
    const int src = static_cast<int>(0xffffffffu - static_cast<uint32_t>(key[i]));
    const float sc = sr[src];
    const float4 bx = boxes[row * N + src];
    const float g = grp ? grp[row * N + src] : static_cast<float>(src % grp_mod + 1);
    const float o = g * scale;
    s_out[row * N + i] = sc;
    b_out[row * N + i] = bx;
    boff_out[row * N + i] = make_float4(bx.x + o, bx.y + o, bx.z + o, bx.w + o);
    if (g_out) g_out[row * N + i] = g;
    if (lab_out) lab_out[row * N + i] = static_cast<long>(g);
    mine += sc >= 0.f;
  }
  if (mine) atomicAdd(&nvalid, mine);
  __syncthreads();
  if (t == 0) valid[row] = nvalid;
}

// Rows kept by NMS: out[b, j] = src[b, keep[b, j]] for boxes (float4), scores and labels (each optional), zero where
// keep is -1 (padding past the image's count). Replaces clamp + three gathers + masked_fill.
__global__ __launch_bounds__(256) void gather_keep_kernel(const int* __restrict__ keep, int K, int N,
                                                          const float4* __restrict__ bsrc, const float* __restrict__ ssrc,
                                                          const long* __restrict__ lsrc, float4* __restrict__ bout,
                                                          float* __restrict__ sout, long* __restrict__ lout,
                                                          float* __restrict__ rout, int total) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const long b = i / K;
  const int k = keep[i];
  const bool ok = k >= 0 && k < N;
  const long src = b * N + (ok ? k : 0);
  const float4 bx = ok && bsrc ? bsrc[src] : make_float4(0.f, 0.f, 0.f, 0.f);
  if (bout) bout[i] = bx;
  if (rout) {  // RoIAlign rows (image, x1, y1, x2, y2): no arange + cat launches
    float* r = rout + 5L * i;
    r[0] = static_cast<float>(b);
    r[1] = bx.x;
    r[2] = bx.y;
    r[3] = bx.z;
    r[4] = bx.w;
  }
  if (sout) sout[i] = ok ? ssrc[src] : 0.f;
  if (lout) lout[i] = ok ? lsrc[src] : 0;
}

// Box-head postprocess (one thread per (image, RoI, foreground class)): softmax over the RoI's nc logits,
// the class's box decoded from its proposal with the regression weights, clipped; score -1 unless the RoI
// is real (r < count[b]), the score clears thresh and the box is at least 1e-2 wide and high.
// pred: fp32 [B, R, ldp] (nc logits, then 4 nc deltas); props fp32 [B, R, 4]; outputs [B, R * (nc - 1)].
// pred element as fp32 (T = float, or uint16_t = the predictor's bf16 output read without a conversion launch)
__device__ __forceinline__ float pred_at(const float* p, int i) { return p[i]; }
__device__ __forceinline__ float pred_at(const uint16_t* p, int i) {
  return __uint_as_float(static_cast<uint32_t>(p[i]) << 16);
}

template <typename T>
__global__ __launch_bounds__(256) void det_decode_kernel(const T* __restrict__ pred, const float4* __restrict__ props,
                                                         const int* __restrict__ count, float4* __restrict__ boxes,
                                                         float* __restrict__ scores, long* __restrict__ labels, int B,
                                                         int R, int ldp, int nc, float4 wts, float img_h, float img_w,
                                                         float thresh, float clip) {
  const int ncf = nc - 1;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= B * R * ncf) return;
  const int b = t / (R * ncf);
  const int rc = t - b * R * ncf;
  const int r = rc / ncf, c = rc - r * ncf + 1;
  const T* lp = pred + (static_cast<long>(b) * R + r) * ldp;
  float mx = pred_at(lp, 0);
  for (int q = 1; q < nc; ++q) mx = fmaxf(mx, pred_at(lp, q));
  float den = 0.f;
  for (int q = 0; q < nc; ++q) den += expf(pred_at(lp, q) - mx);
  const float sc = expf(pred_at(lp, c) - mx) / den;
  const float4 pr = props[static_cast<long>(b) * R + r];
  const T* dp = lp + nc + 4 * c;
  const float w = pr.z - pr.x, h = pr.w - pr.y;
  const float cx = pr.x + 0.5f * w, cy = pr.y + 0.5f * h;
  const float dx = pred_at(dp, 0) / wts.x, dy = pred_at(dp, 1) / wts.y;
  const float dw = fminf(pred_at(dp, 2) / wts.z, clip), dh = fminf(pred_at(dp, 3) / wts.w, clip);
  const float pcx = dx * w + cx, pcy = dy * h + cy, pw = expf(dw) * w, ph = expf(dh) * h;
  const float x1 = fminf(fmaxf(pcx - 0.5f * pw, 0.f), img_w), y1 = fminf(fmaxf(pcy - 0.5f * ph, 0.f), img_h);
  const float x2 = fminf(fmaxf(pcx + 0.5f * pw, 0.f), img_w), y2 = fminf(fmaxf(pcy + 0.5f * ph, 0.f), img_h);
  const bool ok = r < count[b] && sc > thresh && x2 - x1 >= 1e-2f && y2 - y1 >= 1e-2f;
  boxes[t] = make_float4(x1, y1, x2, y2);
  scores[t] = ok ? sc : -1.f;
  labels[t] = c;
}

__device__ __forceinline__ void bilinear_acc8(const uint16_t* __restrict__ feat, int H, int W, int C, float y, float x,
                                              int c8, float w, float* acc) {
  if (y < -1.f || y > H || x < -1.f || x > W) return;
  y = fmaxf(y, 0.f);
  x = fmaxf(x, 0.f);
  int y0 = static_cast<int>(y), x0 = static_cast<int>(x), y1, x1;
  if (y0 >= H - 1) { y1 = y0 = H - 1; y = static_cast<float>(y0); } else { y1 = y0 + 1; }
  if (x0 >= W - 1) { x1 = x0 = W - 1; x = static_cast<float>(x0); } else { x1 = x0 + 1; }
  const float ly = y - y0, lx = x - x0, hy = 1.f - ly, hx = 1.f - lx;
  const float ws[4] = {hy * hx * w, hy * lx * w, ly * hx * w, ly * lx * w};
  const long offs[4] = {(static_cast<long>(y0) * W + x0) * C, (static_cast<long>(y0) * W + x1) * C,
                        (static_cast<long>(y1) * W + x0) * C, (static_cast<long>(y1) * W + x1) * C};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint4 v = *reinterpret_cast<const uint4*>(feat + offs[k] + 8 * c8);
    float a, b;
    unpack_bf16x2(v.x, a, b); acc[0] += ws[k] * a; acc[1] += ws[k] * b;
    unpack_bf16x2(v.y, a, b); acc[2] += ws[k] * a; acc[3] += ws[k] * b;
    unpack_bf16x2(v.z, a, b); acc[4] += ws[k] * a; acc[5] += ws[k] * b;
    unpack_bf16x2(v.w, a, b); acc[6] += ws[k] * a; acc[7] += ws[k] * b;
  }
}

// RoIAlign (torchvision semantics) on an NHWC bf16 feature map; rois [R, 5] = (img, x1, y1, x2, y2).
__global__ __launch_bounds__(256) void roi_align_kernel(const uint16_t* __restrict__ feat, const float* __restrict__ rois,
                                                        uint16_t* __restrict__ out, int H, int W, int C, int R, int PH,
                                                        int PW, int sampling, float scale, int aligned) {
  const int C8 = C >> 3;
  const long total = static_cast<long>(R) * PH * PW * C8;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += static_cast<long>(gridDim.x) * 256) {
    const int c8 = static_cast<int>(idx % C8);
    long t = idx / C8;
    const int pw = static_cast<int>(t % PW);
    t /= PW;
    const int ph = static_cast<int>(t % PH);
    const int r = static_cast<int>(t / PH);
    const float* roi = rois + 5L * r;
    const int img = static_cast<int>(roi[0]);
    const float off = aligned ? 0.5f : 0.f;
    const float x1 = roi[1] * scale - off, y1 = roi[2] * scale - off;
    float rw = roi[3] * scale - off - x1, rh = roi[4] * scale - off - y1;
    if (!aligned) {
      rw = fmaxf(rw, 1.f);
      rh = fmaxf(rh, 1.f);
    }
    const float bh = rh / PH, bw = rw / PW;
    const int gh = sampling > 0 ? sampling : static_cast<int>(ceilf(rh / PH));
    const int gw = sampling > 0 ? sampling : static_cast<int>(ceilf(rw / PW));
    const float inv = 1.f / fmaxf(gh * gw, 1);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint16_t* f = feat + static_cast<long>(img) * H * W * C;
    for (int iy = 0; iy < gh; ++iy) {
      const float y = y1 + ph * bh + (iy + 0.5f) * bh / gh;
      for (int ix = 0; ix < gw; ++ix) {
        const float x = x1 + pw * bw + (ix + 0.5f) * bw / gw;
        bilinear_acc8(f, H, W, C, y, x, c8, inv, acc);
      }
    }
    *reinterpret_cast<uint4*>(out + (((static_cast<long>(r) * PH + ph) * PW + pw) * C) + 8 * c8) =
        make_uint4(pack_bf16x2(acc[0], acc[1]), pack_bf16x2(acc[2], acc[3]), pack_bf16x2(acc[4], acc[5]),
                   pack_bf16x2(acc[6], acc[7]));
  }
}

// Multi-level (FPN P2..P5) RoIAlign: the level of each RoI is picked in-kernel (Lin et al. eq. 1,
// canonical size 224 at level 4, clamped to [2, 5]) so the whole box head has static shapes and is
// HIP-graph capturable (no per-level nonzero/gather on the host).
struct FpnLevels {
  const uint16_t* f[4];
  int h[4], w[4];
  float scale[4];
};

// One workgroup per (RoI, output row): the RoI's level, scale and bin geometry are workgroup-uniform
// (scalar loads, computed once per lane instead of once per 8-channel output), and lanes walk (pw, c8)
// with 32-bit index math — the flat grid-stride form spent ~6 64-bit div/mods per output.
__global__ __launch_bounds__(256) void roi_align_fpn_kernel(FpnLevels lv, const float* __restrict__ rois,
                                                            uint16_t* __restrict__ out, int C, int R, int PH, int PW,
                                                            int sampling, int aligned) {
  const int C8 = C >> 3;
  const int r = blockIdx.x / PH;
  const int ph = blockIdx.x - r * PH;
  const float* roi = rois + 5L * r;
  const float area = fmaxf(roi[3] - roi[1], 0.f) * fmaxf(roi[4] - roi[2], 0.f);
  int l = static_cast<int>(floorf(4.f + log2f(sqrtf(area) / 224.f + 1e-6f)));
  l = min(max(l, 2), 5) - 2;
  const int H = lv.h[l], W = lv.w[l];
  const float scale = lv.scale[l];
  const int img = static_cast<int>(roi[0]);
  const float off = aligned ? 0.5f : 0.f;
  const float x1 = roi[1] * scale - off, y1 = roi[2] * scale - off;
  float rw = roi[3] * scale - off - x1, rh = roi[4] * scale - off - y1;
  if (!aligned) {
    rw = fmaxf(rw, 1.f);
    rh = fmaxf(rh, 1.f);
  }
  const float bh = rh / PH, bw = rw / PW;
  const int gh = sampling > 0 ? sampling : static_cast<int>(ceilf(rh / PH));
  const int gw = sampling > 0 ? sampling : static_cast<int>(ceilf(rw / PW));
  const float inv = 1.f / fmaxf(gh * gw, 1);
  const uint16_t* f = lv.f[l] + static_cast<long>(img) * H * W * C;
  uint16_t* o = out + (static_cast<long>(r) * PH + ph) * PW * C;
  for (int e = threadIdx.x; e < PW * C8; e += 256) {
    const int pw = e / C8, c8 = e - pw * C8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int iy = 0; iy < gh; ++iy) {
      const float y = y1 + ph * bh + (iy + 0.5f) * bh / gh;
      for (int ix = 0; ix < gw; ++ix) {
        const float x = x1 + pw * bw + (ix + 0.5f) * bw / gw;
        bilinear_acc8(f, H, W, C, y, x, c8, inv, acc);
      }
    }
    *reinterpret_cast<uint4*>(o + static_cast<long>(pw) * C + 8 * c8) =
        make_uint4(pack_bf16x2(acc[0], acc[1]), pack_bf16x2(acc[2], acc[3]), pack_bf16x2(acc[4], acc[5]),
                   pack_bf16x2(acc[6], acc[7]));
  }
}

// Same op, one workgroup per RoI (PW * C/8 <= 256 lanes, one (pw, 8-channel chunk) each) walking the output
// rows in order: the sample rows of bin row ph and ph+1 share feature rows, and with the whole RoI on one CU
// those re-reads hit its L1 instead of going to L2 from 7 different CUs (the per-row grid's pattern).
// Each XCD takes a contiguous range of RoIs (one image's proposals at a time) instead of every 8th: 620 vs 645 µs
// per call at batch 32; taking the RoIs y-sorted per image as well was neutral (profiles/r5_roi_order/).
__global__ __launch_bounds__(256) void roi_align_fpn_roi_kernel(FpnLevels lv, const float* __restrict__ rois,
                                                                uint16_t* __restrict__ out, int C, int R, int PH,
                                                                int PW, int sampling, int aligned) {
  const int C8 = C >> 3;
  const int r = xcd_remap(blockIdx.x, gridDim.x);
  const float* roi = rois + 5L * r;
  const float area = fmaxf(roi[3] - roi[1], 0.f) * fmaxf(roi[4] - roi[2], 0.f);
  int l = static_cast<int>(floorf(4.f + log2f(sqrtf(area) / 224.f + 1e-6f)));
  l = min(max(l, 2), 5) - 2;
  const int H = lv.h[l], W = lv.w[l];
  const float scale = lv.scale[l];
  const int img = static_cast<int>(roi[0]);
  const float off = aligned ? 0.5f : 0.f;
  const float x1 = roi[1] * scale - off, y1 = roi[2] * scale - off;
  float rw = roi[3] * scale - off - x1, rh = roi[4] * scale - off - y1;
  if (!aligned) {
    rw = fmaxf(rw, 1.f);
    rh = fmaxf(rh, 1.f);
  }
  const float bh = rh / PH, bw = rw / PW;
  const int gh = sampling > 0 ? sampling : static_cast<int>(ceilf(rh / PH));
  const int gw = sampling > 0 ? sampling : static_cast<int>(ceilf(rw / PW));
  const float inv = 1.f / fmaxf(gh * gw, 1);
  const uint16_t* f = lv.f[l] + static_cast<long>(img) * H * W * C;
  const int t = threadIdx.x;
  if (t >= PW * C8) return;
  const int pw = t / C8, c8 = t - pw * C8;
  uint16_t* o = out + static_cast<long>(r) * PH * PW * C + static_cast<long>(pw) * C + 8 * c8;
  if (gh == 2 && gw == 2) {
    // sampling 2 (the box head's setting): per output row, the 4 samples' 16 corner offsets and weights first
    // (out-of-range samples get weight 0 instead of a branch), then all 16 loads in flight, then the FMAs
    int xo[2][2];
    float xw[2][2];
    bool xok[2];
#pragma unroll
    for (int ix = 0; ix < 2; ++ix) {
      float x = x1 + pw * bw + (ix + 0.5f) * bw * 0.5f;
      xok[ix] = !(x < -1.f || x > W);
      x = fmaxf(x, 0.f);
      int x0 = static_cast<int>(x), x1i;
      if (x0 >= W - 1) { x1i = x0 = W - 1; x = static_cast<float>(x0); } else { x1i = x0 + 1; }
      const float lx = x - x0;
      xo[ix][0] = x0 * C + 8 * c8;
      xo[ix][1] = x1i * C + 8 * c8;
      xw[ix][0] = 1.f - lx;
      xw[ix][1] = lx;
    }
    for (int ph = 0; ph < PH; ++ph) {
      long ro[2][2];
      float yw[2][2];
#pragma unroll
      for (int iy = 0; iy < 2; ++iy) {
        float y = y1 + ph * bh + (iy + 0.5f) * bh * 0.5f;
        const bool yok = !(y < -1.f || y > H);
        y = fmaxf(y, 0.f);
        int y0 = static_cast<int>(y), y1i;
        if (y0 >= H - 1) { y1i = y0 = H - 1; y = static_cast<float>(y0); } else { y1i = y0 + 1; }
        const float ly = y - y0;
        ro[iy][0] = static_cast<long>(y0) * W * C;
        ro[iy][1] = static_cast<long>(y1i) * W * C;
        yw[iy][0] = yok ? (1.f - ly) * inv : 0.f;
        yw[iy][1] = yok ? ly * inv : 0.f;
      }
      uint4 v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q)  // q = ((iy * 2 + ix) * 2 + cy) * 2 + cx
        v[q] = *reinterpret_cast<const uint4*>(f + ro[q >> 3][(q >> 1) & 1] + xo[(q >> 2) & 1][q & 1]);
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int iy = q >> 3, ix = (q >> 2) & 1, cy = (q >> 1) & 1, cx = q & 1;
        const float w = xok[ix] ? yw[iy][cy] * xw[ix][cx] : 0.f;
        float a, b;
        unpack_bf16x2(v[q].x, a, b); acc[0] += w * a; acc[1] += w * b;
        unpack_bf16x2(v[q].y, a, b); acc[2] += w * a; acc[3] += w * b;
        unpack_bf16x2(v[q].z, a, b); acc[4] += w * a; acc[5] += w * b;
        unpack_bf16x2(v[q].w, a, b); acc[6] += w * a; acc[7] += w * b;
      }
      *reinterpret_cast<uint4*>(o + static_cast<long>(ph) * PW * C) =
          make_uint4(pack_bf16x2(acc[0], acc[1]), pack_bf16x2(acc[2], acc[3]), pack_bf16x2(acc[4], acc[5]),
                     pack_bf16x2(acc[6], acc[7]));
    }
    return;
  }
  for (int ph = 0; ph < PH; ++ph) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int iy = 0; iy < gh; ++iy) {
      const float y = y1 + ph * bh + (iy + 0.5f) * bh / gh;
      for (int ix = 0; ix < gw; ++ix) {
        const float x = x1 + pw * bw + (ix + 0.5f) * bw / gw;
        bilinear_acc8(f, H, W, C, y, x, c8, inv, acc);
      }
    }
    *reinterpret_cast<uint4*>(o + static_cast<long>(ph) * PW * C) =
        make_uint4(pack_bf16x2(acc[0], acc[1]), pack_bf16x2(acc[2], acc[3]), pack_bf16x2(acc[4], acc[5]),
                   pack_bf16x2(acc[6], acc[7]));
  }
}

// Crop + bilinear resize + normalize: uint8 image [N, H, W, C<=8], boxes [R, 5] = (img, x1, y1, x2, y2)
// in pixels -> bf16 [R, OH, OW, 8] normalized (classifier stem input). norm = mean[8] ++ std[8].
__global__ __launch_bounds__(256) void crop_resize_kernel(const uint8_t* __restrict__ img, const float* __restrict__ boxes,
                                                          uint16_t* __restrict__ out, const float* __restrict__ norm, int H,
                                                          int W, int C, int R, int OH, int OW) {
  const long total = static_cast<long>(R) * OH * OW;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += static_cast<long>(gridDim.x) * 256) {
    const int ox = static_cast<int>(idx % OW);
    long t = idx / OW;
    const int oy = static_cast<int>(t % OH);
    const int r = static_cast<int>(t / OH);
    const float* bx = boxes + 5L * r;
    const int n = static_cast<int>(bx[0]);
    const float sx = bx[1] + (ox + 0.5f) * (bx[3] - bx[1]) / OW - 0.5f;
    const float sy = bx[2] + (oy + 0.5f) * (bx[4] - bx[2]) / OH - 0.5f;
    const float cy = fminf(fmaxf(sy, 0.f), H - 1.f), cx = fminf(fmaxf(sx, 0.f), W - 1.f);
    const int y0 = static_cast<int>(cy), x0 = static_cast<int>(cx);
    const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
    const float ly = cy - y0, lx = cx - x0;
    const uint8_t* base = img + static_cast<long>(n) * H * W * C;
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      if (c < C) {
        const float a = base[(static_cast<long>(y0) * W + x0) * C + c], b = base[(static_cast<long>(y0) * W + x1) * C + c];
        const float d = base[(static_cast<long>(y1) * W + x0) * C + c], e = base[(static_cast<long>(y1) * W + x1) * C + c];
        const float pix = (1 - ly) * ((1 - lx) * a + lx * b) + ly * ((1 - lx) * d + lx * e);
        v[c] = (pix * (1.f / 255.f) - norm[c]) / norm[8 + c];
      } else {
        v[c] = 0.f;
      }
    }
    reinterpret_cast<uint4*>(out)[idx] =
        make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
  }
}

// Crop + bilinear resize to uint8 [R, OH, OW, C] (no normalization): the detector -> classifier
// wire format of the ensemble (3 bytes per pixel instead of 16 for bf16x8; the classifier stem
// normalizes on its side) and the GPU resize of K7 (a whole-image box).
__global__ __launch_bounds__(256) void crop_resize_u8_kernel(const uint8_t* __restrict__ img,
                                                             const float* __restrict__ boxes, uint8_t* __restrict__ out,
                                                             int H, int W, int C, int R, int OH, int OW) {
  const long total = static_cast<long>(R) * OH * OW;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += static_cast<long>(gridDim.x) * 256) {
    const int ox = static_cast<int>(idx % OW);
    long t = idx / OW;
    const int oy = static_cast<int>(t % OH);
    const int r = static_cast<int>(t / OH);
    const float* bx = boxes + 5L * r;
    const int n = static_cast<int>(bx[0]);
    const float sx = bx[1] + (ox + 0.5f) * (bx[3] - bx[1]) / OW - 0.5f;
    const float sy = bx[2] + (oy + 0.5f) * (bx[4] - bx[2]) / OH - 0.5f;
    const float cy = fminf(fmaxf(sy, 0.f), H - 1.f), cx = fminf(fmaxf(sx, 0.f), W - 1.f);
    const int y0 = static_cast<int>(cy), x0 = static_cast<int>(cx);
    const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
    const float ly = cy - y0, lx = cx - x0;
    const uint8_t* base = img + static_cast<long>(n) * H * W * C;
    uint8_t* o = out + idx * C;
    for (int c = 0; c < C; ++c) {
      const float a = base[(static_cast<long>(y0) * W + x0) * C + c], b = base[(static_cast<long>(y0) * W + x1) * C + c];
      const float d = base[(static_cast<long>(y1) * W + x0) * C + c], e = base[(static_cast<long>(y1) * W + x1) * C + c];
      const float pix = (1 - ly) * ((1 - lx) * a + lx * b) + ly * ((1 - lx) * d + lx * e);
      o[c] = static_cast<uint8_t>(fminf(fmaxf(pix + 0.5f, 0.f), 255.f));
    }
  }
}

inline int grid_for(long work) {
  long g = (work + 255) / 256;
  return static_cast<int>(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace

AI4E_API int ai4e_nms_mask(const void* boxes, int B, int N, float thr, void* mask, hipStream_t s) {
  if (N <= 0) return AI4E_OK;
  const int nb = (N + NMS_BLOCK - 1) / NMS_BLOCK;
  hipLaunchKernelGGL(nms_mask_kernel, dim3(nb, nb, B), dim3(NMS_BLOCK), 0, s, static_cast<const float4*>(boxes), N, thr,
                     static_cast<unsigned long long*>(mask));
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

AI4E_API int ai4e_nms_reduce(const void* mask, const void* valid, int B, int N, int max_out, void* keep, void* count,
                             hipStream_t s) {
  if (N > 8192) return AI4E_EINVAL;
  hipLaunchKernelGGL(nms_reduce_mw_kernel, dim3(B), dim3(64 * NMS_MW_WAVES), 0, s,
                     static_cast<const unsigned long long*>(mask), static_cast<const int*>(valid), N, max_out,
                     static_cast<int*>(keep), static_cast<int*>(count));
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

AI4E_API int ai4e_rpn_decode(const void* head, const void* idx, const void* anchors, void* boxes, void* scores,
                             void* lvl, int B, int HW, int ldh, int A, int k, int KT, int off, float level, float img_h,
                             float img_w, float min_size, float clip, hipStream_t s) {
  if (B <= 0 || k <= 0) return AI4E_OK;
  if (!head || !idx || !anchors || !boxes || !scores || !lvl || A <= 0 || ldh < 5 * A || off + k > KT) return AI4E_EINVAL;
  hipLaunchKernelGGL(rpn_decode_kernel, dim3((B * k + 255) / 256), dim3(256), 0, s, static_cast<const uint16_t*>(head),
                     static_cast<const long*>(idx), static_cast<const float4*>(anchors), static_cast<float4*>(boxes),
                     static_cast<float*>(scores), static_cast<float*>(lvl), B, HW, ldh, A, k, KT, off, level, img_h,
                     img_w, min_size, clip);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

AI4E_API int ai4e_row_sort_desc(const void* scores, int B, int N, void* order, hipStream_t s) {
  if (B <= 0 || N <= 0) return AI4E_OK;
  if (!scores || !order || N > ROWSORT_MAX) return AI4E_EINVAL;
  int P = 1;
  while (P < N) P <<= 1;
  hipLaunchKernelGGL(row_sort_desc_kernel, dim3(B), dim3(ROWSORT_THREADS), 0, s, static_cast<const float*>(scores), N, P,
                     static_cast<long*>(order));
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

AI4E_API int ai4e_sort_select(const void* scores, const void* boxes, const void* grp, int grp_mod, float scale, int B,
                              int N, void* s_out, void* b_out, void* boff_out, void* g_out, void* lab_out, void* valid,
                              hipStream_t s) {
  if (B <= 0 || N <= 0) return AI4E_OK;
  if (!scores || !boxes || !s_out || !b_out || !boff_out || !valid || N > ROWSORT_MAX || (!grp && grp_mod < 1))
    return AI4E_EINVAL;
  int P = 1;
  while (P < N) P <<= 1;
#define AI4E_SORT_SELECT(KPT)                                                                                      \
  hipLaunchKernelGGL((sort_select_kernel<KPT>), dim3(B), dim3(ROWSORT_THREADS), 0, s,                                \
                     static_cast<const float*>(scores), static_cast<const float4*>(boxes),                           \
                     static_cast<const float*>(grp), grp_mod, scale, N, P, static_cast<float*>(s_out),              \
                     static_cast<float4*>(b_out), static_cast<float4*>(boff_out), static_cast<float*>(g_out),      \
                     static_cast<long*>(lab_out), static_cast<int*>(valid))
  if (P > 4 * ROWSORT_THREADS)
    AI4E_SORT_SELECT(8);
  else if (P > 2 * ROWSORT_THREADS)
    AI4E_SORT_SELECT(4);
  else if (P > ROWSORT_THREADS)
    AI4E_SORT_SELECT(2);
  else
    AI4E_SORT_SELECT(1);
#undef AI4E_SORT_SELECT
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

AI4E_API int ai4e_gather_keep(const void* keep, int B, int K, int N, const void* bsrc, const void* ssrc, const void* lsrc,
                              void* bout, void* sout, void* lout, void* rout, hipStream_t s) {
  if (B <= 0 || K <= 0) return AI4E_OK;
  if (!keep || N <= 0 || (bout && !bsrc) || (sout && !ssrc) || (lout && !lsrc) || (rout && !bsrc)) return AI4E_EINVAL;
  const int total = B * K;
  hipLaunchKernelGGL(gather_keep_kernel, dim3((total + 255) / 256), dim3(256), 0, s, static_cast<const int*>(keep), K, N,
                     static_cast<const float4*>(bsrc), static_cast<const float*>(ssrc), static_cast<const long*>(lsrc),
                     static_cast<float4*>(bout), static_cast<float*>(sout), static_cast<long*>(lout),
                     static_cast<float*>(rout), total);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

AI4E_API int ai4e_rpn_topk(const void* head, int B, int HW, int ldh, int A, int k, void* idx, hipStream_t s) {
  if (B <= 0 || k <= 0) return AI4E_OK;
  if (!head || !idx || A < 1 || ldh < A || k > HW * A || static_cast<long>(HW) * A >= (1L << 31)) return AI4E_EINVAL;
  hipLaunchKernelGGL(rpn_topk_kernel, dim3(B), dim3(TOPK_THREADS), 0, s, static_cast<const uint16_t*>(head), HW, ldh, A,
                     k, static_cast<long*>(idx));
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

AI4E_API int ai4e_det_decode(const void* pred, const void* props, const void* count, void* boxes, void* scores,
                             void* labels, int B, int R, int ldp, int nc, const float* wts4, float img_h, float img_w,
                             float thresh, float clip, int pred_bf16, hipStream_t s) {
  if (B <= 0 || R <= 0) return AI4E_OK;
  if (!pred || !props || !count || !boxes || !scores || !labels || !wts4 || nc < 2 || ldp < 5 * nc) return AI4E_EINVAL;
  const long n = static_cast<long>(B) * R * (nc - 1);
  const dim3 g(static_cast<unsigned>((n + 255) / 256));
  const float4 w = make_float4(wts4[0], wts4[1], wts4[2], wts4[3]);
  if (pred_bf16)
    hipLaunchKernelGGL(det_decode_kernel<uint16_t>, g, dim3(256), 0, s, static_cast<const uint16_t*>(pred),
                       static_cast<const float4*>(props), static_cast<const int*>(count), static_cast<float4*>(boxes),
                       static_cast<float*>(scores), static_cast<long*>(labels), B, R, ldp, nc, w, img_h, img_w, thresh,
                       clip);
  else
    hipLaunchKernelGGL(det_decode_kernel<float>, g, dim3(256), 0, s, static_cast<const float*>(pred),
                       static_cast<const float4*>(props), static_cast<const int*>(count), static_cast<float4*>(boxes),
                       static_cast<float*>(scores), static_cast<long*>(labels), B, R, ldp, nc, w, img_h, img_w, thresh,
                       clip);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

AI4E_API int ai4e_roi_align_nhwc(const void* feat, const void* rois, void* out, int H, int W, int C, int R, int PH,
                                 int PW, int sampling, float scale, int aligned, int unused, hipStream_t s) {
  (void)unused;
  if (C % 8) return AI4E_EINVAL;
  if (R <= 0) return AI4E_OK;
  hipLaunchKernelGGL(roi_align_kernel, dim3(grid_for(static_cast<long>(R) * PH * PW * (C / 8))), dim3(256), 0, s,
                     static_cast<const uint16_t*>(feat), static_cast<const float*>(rois), static_cast<uint16_t*>(out), H,
                     W, C, R, PH, PW, sampling, scale, aligned);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

// feats: 4 NHWC bf16 maps (P2..P5) of one batch; hw = {h0, w0, h1, w1, ...}; scales = 1/stride per level.
AI4E_API int ai4e_roi_align_fpn_nhwc(const void* f0, const void* f1, const void* f2, const void* f3, const int* hw,
                                     const float* scales, const void* rois, void* out, int C, int R, int PH, int PW,
                                     int sampling, int aligned, hipStream_t s) {
  if (C % 8) return AI4E_EINVAL;
  if (R <= 0) return AI4E_OK;
  FpnLevels lv;
  const void* fs[4] = {f0, f1, f2, f3};
  for (int i = 0; i < 4; ++i) {
    lv.f[i] = static_cast<const uint16_t*>(fs[i]);
    lv.h[i] = hw[2 * i];
    lv.w[i] = hw[2 * i + 1];
    lv.scale[i] = scales[i];
  }
  if (static_cast<long>(R) * PH >= (1L << 31)) return AI4E_EINVAL;
  // one workgroup per RoI; per (RoI, output row) only when a row's (column, 8-channel chunk) lanes exceed 256
  if (PW * (C / 8) <= 256)
    hipLaunchKernelGGL(roi_align_fpn_roi_kernel, dim3(static_cast<unsigned>(R)), dim3(256), 0, s, lv,
                       static_cast<const float*>(rois), static_cast<uint16_t*>(out), C, R, PH, PW, sampling, aligned);
  else
    hipLaunchKernelGGL(roi_align_fpn_kernel, dim3(static_cast<unsigned>(R * PH)), dim3(256), 0, s,
                       lv, static_cast<const float*>(rois), static_cast<uint16_t*>(out), C, R, PH, PW, sampling, aligned);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

// mode 0: normalized bf16 [R, OH, OW, 8]; mode 1: uint8 [R, OH, OW, C] (norm unused).
AI4E_API int ai4e_crop_resize_nhwc(const void* img, const void* boxes, void* out, const void* norm, int H, int W, int C,
                                   int R, int OH, int OW, int mode, hipStream_t s) {
  if (C > 8 || C < 1) return AI4E_EINVAL;
  if (R <= 0) return AI4E_OK;
  if (mode == 1) {
    hipLaunchKernelGGL(crop_resize_u8_kernel, dim3(grid_for(static_cast<long>(R) * OH * OW)), dim3(256), 0, s,
                       static_cast<const uint8_t*>(img), static_cast<const float*>(boxes), static_cast<uint8_t*>(out), H,
                       W, C, R, OH, OW);
    return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
  }
  hipLaunchKernelGGL(crop_resize_kernel, dim3(grid_for(static_cast<long>(R) * OH * OW)), dim3(256), 0, s,
                     static_cast<const uint8_t*>(img), static_cast<const float*>(boxes), static_cast<uint16_t*>(out),
                     static_cast<const float*>(norm), H, W, C, R, OH, OW);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}
