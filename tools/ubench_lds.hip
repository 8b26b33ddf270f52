// Micro-benchmark (tooling, not product): what bounds the SpGEMM forward's inner loop on
// gfx950? Same structure as spgemm_fwd_kernel<4> (16 rows x 256 f32 LDS accumulator per
// 256-thread work-group, k=16: 4 lanes per edge, a dwordx4 value + a dword selector
// gather per lane), with the LDS update swapped per variant:
//   0: ds_add_f32 (product)          1: ds_read + v_add + ds_write (racy, timing only)
//   2: no LDS update (register sum)  3: ds_add_f32, no global gathers (LDS atomics only)
//   4: ds_add_u32 (integer atomics)  5: ds_add_f32 with a conflict-free address pattern
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int R = 16, D = 256, K = 16, EPS = 16, U = 8;

template <int V>
__global__ __launch_bounds__(256) void kern(const int* __restrict__ idx,
                                            const float* __restrict__ sp_data,
                                            const uint8_t* __restrict__ sp_index,
                                            float* __restrict__ out, int edges_per_wg) {
  __shared__ float acc[R * D];
  for (int i = threadIdx.x; i < R * D; i += 256) acc[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = lane >> 2, l0 = (lane & 3) * 4;
  const int e0 = blockIdx.x * edges_per_wg;
  float reg = 0.f;
  for (int base = wave * EPS * U; base < edges_per_wg; base += 4 * EPS * U) {
    int c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = (V == 3) ? (lane * 977 + u * 131 + base) & 0x3ffff
                                                : idx[e0 + base + u * EPS + slot];
    float4 x[U];
    uint32_t s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (V == 3 || V == 5) {
        x[u] = make_float4(c[u] * 1e-9f, 1.f, 2.f, 3.f);
        s[u] = (V == 5) ? ((uint32_t)(lane * 4) & 0xff) * 0x01010101u + 0x03020100u
                        : (uint32_t)(c[u] * 2654435761u);
      } else {
        const size_t off = (size_t)c[u] * K + l0;
        x[u] = *reinterpret_cast<const float4*>(sp_data + off);
        s[u] = *reinterpret_cast<const uint32_t*>(sp_index + off);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = (base / 64 + u) & (R - 1);
      float* a = acc + row * D;
      const float vals[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t sj = (s[u] >> (8 * j)) & 0xff;
        if (V == 0 || V == 3 || V == 5) {
          __hip_atomic_fetch_add(a + sj, vals[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (V == 1) {
          a[sj] += vals[j];
        } else if (V == 2) {
          reg += vals[j] * (float)sj;
        } else if (V == 4) {
          __hip_atomic_fetch_add(reinterpret_cast<unsigned*>(a) + sj, (unsigned)vals[j],
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
  }
  if (V == 2) acc[threadIdx.x] = reg;
  __syncthreads();
  float* dst = out + (size_t)blockIdx.x * R * D;
  for (int i = threadIdx.x; i < R * D; i += 256) dst[i] = acc[i];
}

extern "C" float ubench_run(int variant, const int* idx, const float* sp_data,
                            const uint8_t* sp_index, float* out, int nwg, int edges_per_wg,
                            int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto launch = [&]() {
    switch (variant) {
      case 0: hipLaunchKernelGGL(kern<0>, nwg, 256, 0, 0, idx, sp_data, sp_index, out, edges_per_wg); break;
      case 1: hipLaunchKernelGGL(kern<1>, nwg, 256, 0, 0, idx, sp_data, sp_index, out, edges_per_wg); break;
      case 2: hipLaunchKernelGGL(kern<2>, nwg, 256, 0, 0, idx, sp_data, sp_index, out, edges_per_wg); break;
      case 3: hipLaunchKernelGGL(kern<3>, nwg, 256, 0, 0, idx, sp_data, sp_index, out, edges_per_wg); break;
      case 4: hipLaunchKernelGGL(kern<4>, nwg, 256, 0, 0, idx, sp_data, sp_index, out, edges_per_wg); break;
      case 5: hipLaunchKernelGGL(kern<5>, nwg, 256, 0, 0, idx, sp_data, sp_index, out, edges_per_wg); break;
    }
  };
  launch();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / reps;
}
