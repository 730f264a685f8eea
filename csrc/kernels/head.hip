// K8 tail — classifier head epilogue: softmax over the logits row + top-k, one wave64 per image.
//
// Replaces the 5-launch PyTorch tail (bf16->fp32 cast, softmax, radix top-k, sort, index cast) that the
// serving engine ran after the graph's classifier GEMM. Each lane holds ceil(C/64) logits in registers;
// max and sum-of-exp are wave reductions (DPP/permute through __shfl_xor), then k rounds of a wave
// argmax (value, lowest index on ties) remove one winner at a time. Probabilities are exp(x - max) / sum,
// the same fp32 math as torch.softmax.
#include "common.h"

namespace {

constexpr int HEAD_MAXC = 64 * 32;  // up to 2048 classes per row (32 per lane)

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int PER_LANE>
__global__ __launch_bounds__(256) void softmax_topk_kernel(const uint16_t* __restrict__ logits, int ld, int N, int C,
                                                           int k, int* __restrict__ top_idx,
                                                           float* __restrict__ top_prob) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const uint16_t* x = logits + static_cast<long>(row) * ld;
  float v[PER_LANE];
#pragma unroll
  for (int j = 0; j < PER_LANE; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < C ? bf16_to_f32(x[c]) : -INFINITY;
  }
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < PER_LANE; ++j) m = fmaxf(m, v[j]);
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < PER_LANE; ++j) s += (lane + 64 * j < C) ? __expf(v[j] - m) : 0.f;
  const float inv = 1.f / wave_sum(s);
  for (int r = 0; r < k; ++r) {
    // lane-local best (lowest index wins ties), then a wave argmax on (value, index)
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < PER_LANE; ++j) {
      const int c = lane + 64 * j;
      if (v[j] > bv || (v[j] == bv && c < bi)) {
        bv = v[j];
        bi = c;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      top_idx[static_cast<long>(row) * k + r] = bi < C ? bi : 0;
      top_prob[static_cast<long>(row) * k + r] = bi < C ? __expf(bv - m) * inv : 0.f;
    }
    // the owner lane retires the winner
    if ((bi & 63) == lane) {
#pragma unroll
      for (int j = 0; j < PER_LANE; ++j)
        if (lane + 64 * j == bi) v[j] = -INFINITY;
    }
  }
}

}  // namespace

// logits: [N, ld] bf16 (C valid columns); top_idx [N, k] int32, top_prob [N, k] fp32. C <= 2048, k <= C.
AI4E_API int ai4e_softmax_topk(const void* logits, int ld, int N, int C, int k, void* top_idx, void* top_prob,
                               hipStream_t s) {
  if (!logits || !top_idx || !top_prob || C <= 0 || C > HEAD_MAXC || ld < C || k <= 0 || k > C) return AI4E_EINVAL;
  if (N <= 0) return AI4E_OK;
  const dim3 grid(ai4e_cdiv(N, 4)), block(256);
  auto* x = static_cast<const uint16_t*>(logits);
  auto* ti = static_cast<int*>(top_idx);
  auto* tp = static_cast<float*>(top_prob);
  if (C <= 64 * 16)
    hipLaunchKernelGGL(softmax_topk_kernel<16>, grid, block, 0, s, x, ld, N, C, k, ti, tp);
  else
    hipLaunchKernelGGL(softmax_topk_kernel<32>, grid, block, 0, s, x, ld, N, C, k, ti, tp);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}
