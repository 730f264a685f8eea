// K6 tile-stitch for tiled land-cover segmentation: blend overlapping tile logits into the mosaic
// and take the per-pixel argmax (+ optional softmax probabilities).
//
// Gather form (no atomics): tiles lie on a regular grid (origin ty*stride, tx*stride, size ts), so each
// output pixel finds the <= ceil(ts/stride)^2 tiles that cover it, weights each by a separable
// trapezoid window (ramp over `ov` pixels at tile edges, flat centre) and normalises by the weight
// sum. Deterministic, one HBM pass over the tiles, and shardable by rows: a GPU that owns mosaic
// rows [row0, row0+H) passes only its local tile rows [ty0, ty0 + nty) (the halo tiles it computed
// redundantly) — the spatial-parallel plan of runtime/spatial.py.
#include "common.h"

namespace {

__device__ __forceinline__ float ramp(int i, int ts, int ov) {
  if (ov <= 0) return 1.f;
  const float a = (i + 0.5f) / ov, b = (ts - i - 0.5f) / ov;
  return fminf(1.f, fminf(a, b));
}

// tiles [nty, ntx, ts, ts, C] bf16 logits (local tile rows); cls [H, W] uint8; prob [H, W, C] bf16 or null.
__global__ __launch_bounds__(256) void stitch_kernel(const uint16_t* __restrict__ tiles, uint8_t* __restrict__ cls,
                                                     uint16_t* __restrict__ prob, int H, int W, int C, int ts, int stride,
                                                     int ntx, int ty0, int nty, int ov, int row0) {
  const long total = static_cast<long>(H) * W;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += static_cast<long>(gridDim.x) * 256) {
    const int x = static_cast<int>(idx % W);
    const int yl = static_cast<int>(idx / W);
    const int y = yl + row0;  // global mosaic row
    float acc[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) acc[c] = 0.f;
    float wsum = 0.f;
    const int tyl = max(ty0, (y - ts + stride) / stride), tyh = min(ty0 + nty - 1, y / stride);
    const int txl = max(0, (x - ts + stride) / stride), txh = min(ntx - 1, x / stride);
    for (int ty = tyl; ty <= tyh; ++ty) {
      const int iy = y - ty * stride;
      if (iy < 0 || iy >= ts) continue;
      const float wy = ramp(iy, ts, ov);
      for (int tx = txl; tx <= txh; ++tx) {
        const int ix = x - tx * stride;
        if (ix < 0 || ix >= ts) continue;
        const float w = wy * ramp(ix, ts, ov);
        const uint16_t* p = tiles + ((((static_cast<long>(ty - ty0) * ntx + tx) * ts + iy) * ts + ix) * C);
        for (int c = 0; c < C; ++c) acc[c] += w * bf16_to_f32(p[c]);
        wsum += w;
      }
    }
    const float inv = wsum > 0.f ? 1.f / wsum : 0.f;
    int best = 0;
    float bv = -INFINITY;
    for (int c = 0; c < C; ++c) {
      acc[c] *= inv;
      if (acc[c] > bv) {
        bv = acc[c];
        best = c;
      }
    }
    cls[idx] = static_cast<uint8_t>(best);
    if (prob) {
      float s = 0.f;
      for (int c = 0; c < C; ++c) s += __expf(acc[c] - bv);
      const float is = 1.f / s;
      for (int c = 0; c < C; ++c) prob[idx * C + c] = f32_to_bf16(__expf(acc[c] - bv) * is);
    }
  }
}

inline int grid_for(long work) {
  long g = (work + 255) / 256;
  return static_cast<int>(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

}  // namespace

// geom = {ts, stride, ntx, ty0, nty, ov, row0} packed as ints after H, W, C.
AI4E_API int ai4e_tile_stitch(const void* tiles, void* cls, void* prob, int H, int W, int C, int ts, int stride, int ntx,
                              int ty0, int nty, int ov, int row0, hipStream_t s) {
  if (C > 16 || C < 1 || stride <= 0 || stride > ts) return AI4E_EINVAL;
  hipLaunchKernelGGL(stitch_kernel, dim3(grid_for(static_cast<long>(H) * W)), dim3(256), 0, s,
                     static_cast<const uint16_t*>(tiles), static_cast<uint8_t*>(cls), static_cast<uint16_t*>(prob), H, W,
                     C, ts, stride, ntx, ty0, nty, ov, row0);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}
