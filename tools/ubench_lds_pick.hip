// LDS cost of the backward candidate "stage each (block, row) pair's grad_out row in LDS once,
// then pick the selected features from LDS" (tooling, round 5). One work-group of
// 512 threads (8 waves, as sspmm_bwd4_kernel) per CU; each wave loops over `iters` steps of
// one pattern; device time / wave-steps per CU = cycles per wave-step (all 8 waves of the CU
// share its LDS). The lane layout is the kernel's: L lanes per edge (F = 4 slots per lane,
// lane q owns slots q + L * j), 64 / L edges per step; selector words staged in LDS.
//
//   mode 0  candidate picks: per lane one selector word (ds_read_b32) + 4 ds_read_b32 picks
//           from the edge's staged 1 KB row (ring of 8 rows per wave, edges 4 per row)
//   mode 1  current update: per lane one selector word + ds_read_b128 + 2 ds_cmpst_rtn_b64 on
//           the accumulators of a random column of a C-column block (KS = 4 L floats)
//   mode 2  staging only: global_load_lds_dwordx4 (LDS-DMA, 1 KB per wave instruction) of random
//           1 KB rows of an L2-resident buffer into the ring, one per step
//   mode 3  modes 0 + 1 + one staging DMA every `dma_every` steps (the candidate's whole LDS
//           stream: edges per (block, row) pair x ... per pair)
//   mode 4  staging through registers: global_load_dwordx4 of the 1 KB row + ds_write_b128
//   mode 5  modes 0 + 1 + one register-staged row every `dma_every` steps
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -shared -fPIC tools/ubench_lds_pick.hip \
//         -o tools/libubench_lds_pick.so && python tools/ubench_lds_pick.py
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kRing = 8;      // staged rows per wave: 8 KB per wave, 64 KB per work-group
constexpr int kSelCols = 1024;  // columns of the staged selector table

template <int MODE>
__global__ __launch_bounds__(512) void lds_pick_kernel(const uint32_t* __restrict__ selw_g,
                                                       int L, int C, int dma_every,
                                                       const float* __restrict__ gsrc,
                                                       int gsrc_rows, int iters,
                                                       float* __restrict__ sink) {
  extern __shared__ __align__(16) float lds[];
  // [0, 64 KB): rings; then the selector words [kSelCols][L]; then (mode 1/3) accumulators
  float* ring = lds + (threadIdx.x >> 6) * kRing * 256;
  uint32_t* selw = reinterpret_cast<uint32_t*>(lds + 8 * kRing * 256);
  float* accs = lds + 8 * kRing * 256 + kSelCols * L;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int eps = 64 / L;
  const int slot = lane / L, q = lane - slot * L;
  const int KS = 4 * L;
  for (int i = threadIdx.x; i < 8 * kRing * 256; i += 512) lds[i] = (float)(i & 255);
  for (int i = threadIdx.x; i < kSelCols * L; i += 512) selw[i] = selw_g[i];
  if (MODE == 1 || MODE == 3 || MODE == 5)
    for (int i = threadIdx.x; i < C * KS; i += 512) accs[i] = 0.f;
  __syncthreads();
  float acc = 0.f;
  uint32_t seed = blockIdx.x * 7919u + (uint32_t)w * 104729u;  // wave-uniform: one row per wave instruction
  for (int it = 0; it < iters; ++it) {
    const int e = it * eps + slot + w * 131;
    if (MODE == 4 || (MODE == 5 && it % dma_every == 0)) {
      seed = seed * 1664525u + 1013904223u;
      const int gr = (int)((seed >> 8) % (uint32_t)gsrc_rows);
      const float4 v = *reinterpret_cast<const float4*>(gsrc + (size_t)gr * 256 + 4 * lane);
      *reinterpret_cast<float4*>(ring + (it % kRing) * 256 + 4 * lane) = v;
    }
    if (MODE == 2 || (MODE == 3 && it % dma_every == 0)) {
      seed = seed * 1664525u + 1013904223u;
      const int gr = (int)((seed >> 8) % (uint32_t)gsrc_rows);
      __builtin_amdgcn_global_load_lds(gsrc + (size_t)gr * 256 + 4 * lane,
                                       ring + (it % kRing) * 256, 16, 0, 0);
    }
    if (MODE == 0 || MODE == 1 || MODE == 3 || MODE == 5) {
      const uint32_t sw = selw[(e & (kSelCols - 1)) * L + q];
      if (MODE == 0 || MODE == 3 || MODE == 5) {
        const float* rw = ring + ((e >> 2) & (kRing - 1)) * 256;
        acc += rw[sw & 255u] + rw[(sw >> 8) & 255u] + rw[(sw >> 16) & 255u] + rw[sw >> 24];
      }
      if (MODE == 1 || MODE == 3 || MODE == 5) {
        const int c = (int)(((uint32_t)e * 2654435761u) >> 8) % C;
        float* ap = accs + c * KS + 4 * q;
        const uint4 o = *reinterpret_cast<const uint4*>(ap);
        unsigned long long* a = reinterpret_cast<unsigned long long*>(ap);
        unsigned long long e0 = (unsigned long long)o.x | ((unsigned long long)o.y << 32);
        unsigned long long e1 = (unsigned long long)o.z | ((unsigned long long)o.w << 32);
        __hip_atomic_compare_exchange_strong(a, &e0, e0 + (sw & 1u), __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_compare_exchange_strong(a + 1, &e1, e1 + (sw & 2u), __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        acc += (float)(e0 & 1) + (float)(e1 & 1);
      }
    }
    if ((MODE == 2 || MODE == 4) && (it & 7) == 7) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      acc += ring[(it % kRing) * 256 + lane];
    }
  }
  sink[blockIdx.x * 512 + threadIdx.x] = acc;
}

extern "C" float ubench_lds_pick(int mode, const uint32_t* selw, int L, int C, int dma_every,
                                 const float* gsrc, int gsrc_rows, int iters, int grid,
                                 float* sink, int reps) {
  const size_t lds = (size_t)(8 * kRing * 256 + kSelCols * L + ((mode == 1 || mode == 3 || mode == 5) ? C * 4 * L : 0)) * 4;
  if (lds > 160 * 1024) return -2.f;
  const void* fns[6] = {(const void*)lds_pick_kernel<0>, (const void*)lds_pick_kernel<1>,
                        (const void*)lds_pick_kernel<2>, (const void*)lds_pick_kernel<3>,
                        (const void*)lds_pick_kernel<4>, (const void*)lds_pick_kernel<5>};
  for (int m = 0; m < 6; ++m)
    (void)hipFuncSetAttribute(fns[m], hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  auto launch = [&]() {
    switch (mode) {
      case 0: hipLaunchKernelGGL(lds_pick_kernel<0>, dim3(grid), dim3(512), lds, 0, selw, L, C, dma_every, gsrc, gsrc_rows, iters, sink); break;
      case 1: hipLaunchKernelGGL(lds_pick_kernel<1>, dim3(grid), dim3(512), lds, 0, selw, L, C, dma_every, gsrc, gsrc_rows, iters, sink); break;
      case 2: hipLaunchKernelGGL(lds_pick_kernel<2>, dim3(grid), dim3(512), lds, 0, selw, L, C, dma_every, gsrc, gsrc_rows, iters, sink); break;
      case 4: hipLaunchKernelGGL(lds_pick_kernel<4>, dim3(grid), dim3(512), lds, 0, selw, L, C, dma_every, gsrc, gsrc_rows, iters, sink); break;
      case 5: hipLaunchKernelGGL(lds_pick_kernel<5>, dim3(grid), dim3(512), lds, 0, selw, L, C, dma_every, gsrc, gsrc_rows, iters, sink); break;
      default: hipLaunchKernelGGL(lds_pick_kernel<3>, dim3(grid), dim3(512), lds, 0, selw, L, C, dma_every, gsrc, gsrc_rows, iters, sink); break;
    }
  };
  launch();
  if (hipDeviceSynchronize() != hipSuccess) return -1.f;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r) launch();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  if (hipGetLastError() != hipSuccess) return -1.f;
  return ms / reps;
}
