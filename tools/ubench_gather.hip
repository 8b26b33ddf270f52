// Micro-benchmark (tooling, not product): CBSR gather throughput on gfx950 for the
// SpGEMM forward's access shape (k=16: 4 lanes per edge, 16 edges per wave instruction,
// 8 independent sub-steps per wave), by table layout and column locality.
//   0 separate tables: 64-B value row + 16-B selector row (the API layout)
//   1 packed 128-B records {values, selectors, pad}
//   2 packed 80-B records {values, selectors}
//   3 separate tables, columns confined to a window of `window` nodes (L2-resident)
//   4 packed 128-B records, same window
//   5 values only (no selector gather)
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int K = 16, EPS = 16, U = 8;

template <int V>
__global__ __launch_bounds__(256) void gkern(const int* __restrict__ idx,
                                             const float* __restrict__ data,
                                             const uint8_t* __restrict__ sel,
                                             const uint8_t* __restrict__ packed,
                                             float* __restrict__ out, int edges_per_wg,
                                             int window) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = lane >> 2, q = lane & 3;
  const int e0 = blockIdx.x * edges_per_wg;
  float accv = 0.f;
  uint32_t accs = 0;
  // window > 0: per-WG window at a WG-specific offset; window < 0: one global window
  // [0, -window) shared by every work-group (L2-resident for all of them)
  const int wabs = window < 0 ? -window : window;
  const int wbase = (V == 3 || V == 4) && window > 0 ? (blockIdx.x * 7919) % (232965 - wabs) : 0;
  for (int base = wave * EPS * U; base < edges_per_wg; base += 4 * EPS * U) {
    int c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c[u] = idx[e0 + base + u * EPS + slot];
      if (V == 3 || V == 4) c[u] = wbase + c[u] % wabs;
    }
    float4 x[U];
    uint32_t s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (V == 0 || V == 3 || V == 5) {
        x[u] = *reinterpret_cast<const float4*>(data + (size_t)c[u] * K + q * 4);
        s[u] = V == 5 ? 0u : *reinterpret_cast<const uint32_t*>(sel + (size_t)c[u] * K + q * 4);
      } else {
        const size_t rec = (V == 2) ? 80 : 128;
        const uint8_t* p = packed + (size_t)c[u] * rec;
        x[u] = *reinterpret_cast<const float4*>(p + q * 16);
        s[u] = *reinterpret_cast<const uint32_t*>(p + 64 + q * 4);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      accv += x[u].x + x[u].y + x[u].z + x[u].w;
      accs ^= s[u];
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = accv + (float)accs;
}

extern "C" float ubench_gather(int variant, const int* idx, const float* data, const uint8_t* sel,
                               const uint8_t* packed, float* out, int nwg, int edges_per_wg,
                               int window, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto launch = [&]() {
    switch (variant) {
#define CASE(n) case n: hipLaunchKernelGGL(gkern<n>, nwg, 256, 0, 0, idx, data, sel, packed, out, edges_per_wg, window); break;
      CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5)
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
