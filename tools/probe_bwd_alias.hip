// Probe (tooling, not product): does the packed backward speed up when the grad_out rows it
// gathers stay in L2? Rewrites a plan's backward records so that row r reads grad_out row
// r % mod (the per-instruction line pattern is unchanged; the working set shrinks to mod
// rows). The results are wrong afterwards: time only, then discard the plan.
#include <hip/hip_runtime.h>

#include "../spgemm-gnn_amd/csrc/common.h"

__global__ void alias_rows_kernel(uint32_t* rec, int64_t E, uint32_t row_bytes, uint32_t mod) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t r = rec[3 * e] / row_bytes;
    rec[3 * e] = (r % mod) * row_bytes;
  }
}

extern "C" int probe_alias_rows(maxk_plan* p, int mod, void* stream) {
  if (!p || !p->bwd_rec || mod <= 0) return -1;
  hipLaunchKernelGGL(alias_rows_kernel, dim3(4096), dim3(256), 0, (hipStream_t)stream,
                     p->bwd_rec, (int64_t)p->num_edges, (uint32_t)p->dim_origin * 4u,
                     (uint32_t)mod);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
