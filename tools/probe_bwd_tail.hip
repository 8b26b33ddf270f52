// Per-work-group timing of the column-block backward (tooling, round 5): how long each of a
// launch's work-groups runs, to see how much of the kernel is the tail of its single round of
// tasks. Includes the product sources with the kernel's probe hooks defined: thread
// 0 of every work-group stores s_memrealtime (100 MHz) at its start and after its stores.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -shared -fPIC -munsafe-fp-atomics -Iinclude \
//         -Ispgemm-gnn_amd/csrc tools/probe_bwd_tail.hip spgemm-gnn_amd/csrc/plan.hip \
//         spgemm-gnn_amd/csrc/maxk_topk.hip spgemm-gnn_amd/csrc/capi.cpp \
//         -o tools/libprobe_bwd_tail.so
//   MAXK_HIP_LIB=tools/libprobe_bwd_tail.so python tools/probe_bwd_tail.py
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ unsigned long long g_wg_clock[2][1 << 16];

#define MAXK_BWD_PROBE_BEGIN()                                                     \
  do {                                                                             \
    if (threadIdx.x == 0 && blockIdx.x < (1u << 16))                               \
      g_wg_clock[0][blockIdx.x] = __builtin_amdgcn_s_memrealtime();                \
  } while (0)
#define MAXK_BWD_PROBE_END()                                                       \
  do {                                                                             \
    __syncthreads();                                                               \
    if (threadIdx.x == 0 && blockIdx.x < (1u << 16))                               \
      g_wg_clock[1][blockIdx.x] = __builtin_amdgcn_s_memrealtime();                \
  } while (0)

#include "../spgemm-gnn_amd/csrc/spgemm.hip"

extern "C" int probe_bwd_clocks(unsigned long long* host, int n) {
  if (n > (1 << 16)) n = 1 << 16;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wg_clock), sizeof(unsigned long long) * n, 0,
                          hipMemcpyDeviceToHost) != hipSuccess) return -2;
  if (hipMemcpyFromSymbol(host + n, HIP_SYMBOL(g_wg_clock), sizeof(unsigned long long) * n,
                          sizeof(unsigned long long) * (1 << 16), hipMemcpyDeviceToHost) != hipSuccess)
    return -3;
  return n;
}
