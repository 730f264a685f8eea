// Breadcrumbs: progress counters a captured HIP graph bumps at named points, in host-mapped coherent memory that the
// host reads while the GPU runs (no sync, no copy). A replay that stops (fault or hang) leaves every counter before
// the stopping point one ahead of the counters after it, which names the stage that never finished.
// Diagnostic only (AI4E_BREADCRUMBS=1, ops/debug.py); one single-lane kernel per mark, plain vector stores.
#include <hip/hip_runtime.h>

#include <cstring>

#include "common.h"

namespace {

__global__ __launch_bounds__(64) void crumb_kernel(int* p, int idx) {
  if (threadIdx.x == 0) {
    volatile int* q = p + idx;
    *q = *q + 1;
    __threadfence_system();
  }
}

}  // namespace

AI4E_API int ai4e_crumbs_alloc(int n, void* host_out, void* dev_out) {
  void* h = nullptr;
  void* d = nullptr;
  if (n <= 0 || hipHostMalloc(&h, static_cast<size_t>(n) * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) !=
                    hipSuccess)
    return AI4E_EINVAL;
  std::memset(h, 0, static_cast<size_t>(n) * sizeof(int));
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) return AI4E_ELAUNCH;
  *static_cast<void**>(host_out) = h;
  *static_cast<void**>(dev_out) = d;
  return AI4E_OK;
}

AI4E_API int ai4e_crumb(void* dev, int idx, hipStream_t s) {
  hipLaunchKernelGGL(crumb_kernel, dim3(1), dim3(64), 0, s, static_cast<int*>(dev), idx);
  return hipGetLastError() == hipSuccess ? AI4E_OK : AI4E_ELAUNCH;
}
