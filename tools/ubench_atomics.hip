// Micro-benchmark (tooling, not product): accumulation primitives on gfx950, same traffic
// shape as the SpGEMM/SSpMM inner loops (64 lanes x 4 features, random targets in a
// 256-float LDS row or in a 15 MB global table).
//   0 ds_add_f32          1 ds_add_u32        2 ds_add_u64         3 ds_add_f64
//   4 ds_read/ds_write RMW (racy)             5 global f32 atomic, agent scope, 15 MB table
//   6 global f32 atomic, workgroup scope      7 plain global store, 15 MB table
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int ITERS = 256;

// f32 add on LDS through the integer CAS path (ds_read_b32 + ds_cmpst_rtn_b32 loop).
__device__ __forceinline__ void lds_add_cas(float* p, float v) {
  unsigned* u = reinterpret_cast<unsigned*>(p);
  unsigned old = *u;
  while (true) {
    const unsigned assumed = old;
    old = atomicCAS(u, assumed, __float_as_uint(__uint_as_float(assumed) + v));
    if (old == assumed) break;
  }
}

template <int V>
__global__ __launch_bounds__(256) void kern(float* __restrict__ table, int table_words,
                                            float* __restrict__ out) {
  __shared__ double acc[16 * 256];
  float* accf = reinterpret_cast<float*>(acc);
  for (int i = threadIdx.x; i < 16 * 256; i += 256) acc[i] = 0.0;
  __syncthreads();
  uint32_t h = (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
  const int row = (threadIdx.x >> 6) * 4;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      h = h * 1664525u + 1013904223u;
      const uint32_t s = h >> 24;
      const float x = (float)(h & 0xffff) * 1e-5f;
      if (V == 0) {
        __hip_atomic_fetch_add(accf + row * 256 + s, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else if (V == 1) {
        __hip_atomic_fetch_add(reinterpret_cast<uint32_t*>(accf) + row * 256 + s, (uint32_t)h,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else if (V == 2) {
        __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(acc) + row * 256 + s,
                               (unsigned long long)h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else if (V == 3) {
        __hip_atomic_fetch_add(acc + row * 256 + s, (double)x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else if (V == 4) {
        accf[row * 256 + s] += x;
      } else if (V == 8) {
        lds_add_cas(accf + row * 256 + s, x);
      } else {
        // global: 64-B segments like an SSpMM edge (16 lanes x 4 B contiguous per column)
        const uint32_t col = (h >> 8) % (uint32_t)(table_words / 16);
        float* p = table + (size_t)col * 16 + (threadIdx.x & 15);
        if (V == 5) __hip_atomic_fetch_add(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (V == 6) __hip_atomic_fetch_add(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else *p = x;
      }
    }
  }
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = accf[threadIdx.x] + (float)acc[threadIdx.x + 256];
}

extern "C" float ubench_atomics(int variant, float* table, int table_words, float* out, int nwg,
                                int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto launch = [&]() {
    switch (variant) {
#define CASE(n) case n: hipLaunchKernelGGL(kern<n>, nwg, 256, 0, 0, table, table_words, out); break;
      CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
#undef CASE
    }
  };
  launch();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

// Backward inner loop (block-major, row-sorted edges; k=16; 512 threads; LDS block
// accumulator) with the LDS update swapped: 0 ds_add_f32, 1 racy RMW, 2 none.
template <int V>
__global__ __launch_bounds__(512) void bwd_kern(const int4* __restrict__ tasks,
                                                const int* __restrict__ erow,
                                                const int* __restrict__ ecol,
                                                const float* __restrict__ ev,
                                                const float* __restrict__ G,
                                                const uint8_t* __restrict__ sp_index,
                                                float* __restrict__ grad, int D) {
  constexpr int K = 16, L = 4, EPS = 16, U = 8, KS = 16;
  extern __shared__ double accd[];
  float* acc = reinterpret_cast<float*>(accd);
  const int4 t = tasks[blockIdx.x];  // col0, ncols, e0, e1
  for (int i = threadIdx.x; i < t.y * KS * (V == 4 ? 2 : 1); i += 512) acc[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = lane >> 2, q = lane & 3;
  float reg = 0.f;
  for (int base = t.z + wave * EPS * U; base < t.w; base += 8 * EPS * U) {
    int r[U], c[U];
    float v[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * EPS + slot;
      ok[u] = e < t.w;
      const int ec = ok[u] ? e : t.w - 1;
      r[u] = erow[ec];
      c[u] = ecol[ec];
      v[u] = ev[ec];
    }
    uint32_t s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) s[u] = *reinterpret_cast<const uint32_t*>(sp_index + (size_t)c[u] * K + q * 4);
    float g[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float* gr = G + (size_t)(V == 5 ? (r[u] & 255) : r[u]) * D;
#pragma unroll
      for (int j = 0; j < 4; ++j) g[u][j] = (V == 6) ? v[u] * (float)j : gr[(s[u] >> (8 * j)) & 0xff];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (ok[u]) {
        float* a = acc + (c[u] - t.x) * KS + q;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (V == 0) __hip_atomic_fetch_add(a + j * L, v[u] * g[u][j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          else if (V == 1) a[j * L] += v[u] * g[u][j];
          else if (V == 3 || V == 5 || V == 6) lds_add_cas(a + j * L, v[u] * g[u][j]);
          else if (V == 4) __hip_atomic_fetch_add(accd + (c[u] - t.x) * KS + q + j * L, (double)(v[u] * g[u][j]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          else reg += v[u] * g[u][j];
        }
      }
    }
  }
  __syncthreads();
  if (V == 2) acc[threadIdx.x] += reg;
  __syncthreads();
  for (int i = threadIdx.x; i < t.y * K; i += 512) grad[(size_t)t.x * K + i] = acc[(i / K) * KS + (i % K)];
}

extern "C" float ubench_bwd(int variant, const int4* tasks, int ntasks, const int* erow,
                            const int* ecol, const float* ev, const float* G,
                            const uint8_t* sp_index, float* grad, int D, int lds, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipFuncSetAttribute((const void*)bwd_kern<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)bwd_kern<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)bwd_kern<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)bwd_kern<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)bwd_kern<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)bwd_kern<5>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipFuncSetAttribute((const void*)bwd_kern<6>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  auto launch = [&]() {
    if (variant == 0) hipLaunchKernelGGL(bwd_kern<0>, ntasks, 512, lds, 0, tasks, erow, ecol, ev, G, sp_index, grad, D);
    if (variant == 1) hipLaunchKernelGGL(bwd_kern<1>, ntasks, 512, lds, 0, tasks, erow, ecol, ev, G, sp_index, grad, D);
    if (variant == 2) hipLaunchKernelGGL(bwd_kern<2>, ntasks, 512, lds, 0, tasks, erow, ecol, ev, G, sp_index, grad, D);
    if (variant == 3) hipLaunchKernelGGL(bwd_kern<3>, ntasks, 512, lds, 0, tasks, erow, ecol, ev, G, sp_index, grad, D);
    if (variant == 4) hipLaunchKernelGGL(bwd_kern<4>, ntasks, 512, lds, 0, tasks, erow, ecol, ev, G, sp_index, grad, D);
    if (variant == 5) hipLaunchKernelGGL(bwd_kern<5>, ntasks, 512, lds, 0, tasks, erow, ecol, ev, G, sp_index, grad, D);
    if (variant == 6) hipLaunchKernelGGL(bwd_kern<6>, ntasks, 512, lds, 0, tasks, erow, ecol, ev, G, sp_index, grad, D);
  };
  launch();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}
