// CU partitioning for the serving engine: HIP streams restricted to a subset of the chip's 256 CUs
// (hipExtStreamCreateWithCUMask), so two stages of a batch pipeline can own disjoint CU sets instead of
// time-slicing every CU between two full-chip kernel streams (runtime/engine.py, AI4E_ENGINE_CU_SPLIT).
//
// Why: the ResNet-50 front (stem, layer1/2 chains) is HBM-bound and the back (layer3/4) is MFMA/latency-bound,
// but every kernel fills all 256 CUs with workgroups whose LDS footprint leaves no room for the other stream's,
// so two concurrent batches mostly take turns per CU. A CU mask gives each stage a fixed share of every XCD.
//
// A census kernel reports where the workgroups of a launch actually ran (XCC id from HW_REG_XCC_ID, and the
// SE / CU ids from HW_REG_HW_ID), which is how the host learns the mask-bit -> XCD numbering on this part.
#include "common.h"

namespace {

__global__ __launch_bounds__(64) void cu_census_kernel(int* __restrict__ out, int spin) {
  unsigned xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  // keep the workgroup resident for a while so later workgroups spread over the allowed CUs
  long t0 = clock64();
  while (clock64() - t0 < spin) {
  }
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = static_cast<int>(xcc & 0xf);
    out[2 * blockIdx.x + 1] = static_cast<int>(hw);
  }
}

}  // namespace

// Stream whose kernels may only run on the CUs whose bits are set in mask[0 .. nwords) (bit i of word w = CU
// 32 w + i in the runtime's numbering). Returns the hipStream_t through *out.
AI4E_API int ai4e_stream_create_cu_mask(const uint32_t* mask, int nwords, void** out) {
  if (!mask || nwords <= 0 || !out) return AI4E_EINVAL;
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(nwords), mask) != hipSuccess) return AI4E_ELAUNCH;
  *out = s;
  return AI4E_OK;
}

AI4E_API int ai4e_stream_destroy(void* s) {
  return hipStreamDestroy(static_cast<hipStream_t>(s)) == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}

// The CU mask the runtime applied to stream s (nwords words; the device's CU count rounded up to 32).
AI4E_API int ai4e_stream_get_cu_mask(void* s, uint32_t* mask, int nwords) {
  if (!mask || nwords <= 0) return AI4E_EINVAL;
  return hipExtStreamGetCUMask(static_cast<hipStream_t>(s), static_cast<uint32_t>(nwords), mask) == hipSuccess
             ? AI4E_OK
             : AI4E_ELAUNCH;
}

// nblocks one-wave workgroups on stream s; out[2 b] = XCC id, out[2 b + 1] = HW_ID register of workgroup b.
AI4E_API int ai4e_cu_census(int* out, int nblocks, int spin_cycles, hipStream_t s) {
  if (!out || nblocks <= 0) return AI4E_EINVAL;
  hipLaunchKernelGGL(cu_census_kernel, dim3(nblocks), dim3(64), 0, s, out, spin_cycles);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}
