// Micro-benchmark (tooling, not product): the atomic-free interleaved SpGEMM forward at
// k = 4L (L lanes per edge, one float4 of values + one dword of 4 selectors per lane, gathered
// straight from sp_data / sp_index), SLOTS = 64 / L accumulator rows per wave (f64,
// wave-private LDS). Each wave instruction takes one edge of each of its rows, so no two
// lanes update the same LDS word and a read-add-write replaces ds_add_f64.
//   cv[base_g + t * SLOTS + j] = {col, val bits} of step t of slot j (col = ~0u: padding)
//   grp[g] = {base, steps, rows[SLOTS] (row | split << 31, -1 = empty)}
// ROT: each wave starts its sweep at step floor(frac(clock / (tps * steps)) * steps) and
// wraps, so waves running together gather from the same column window (rows are
// column-sorted and a slot's edges are spread evenly over the steps).
// MODE 0: f64 read-add-write; 1: ds_add_f64.
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int D = 256, DS = D + 1;

template <int L, int MODE, int U, int ROT>
__global__ __launch_bounds__(256) void fwd_ilk(const int* __restrict__ grp, int ngrp,
                                               const uint2* __restrict__ cv,
                                               const float* __restrict__ sp_data,
                                               const uint8_t* __restrict__ sp_index,
                                               float* __restrict__ out, int tps) {
  constexpr int SLOTS = 64 / L, K = 4 * L;
  extern __shared__ __align__(16) double sm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = blockIdx.x * 4 + wave;
  if (g >= ngrp) return;
  double* acc = sm + (size_t)wave * SLOTS * DS;
  for (int i = lane; i < SLOTS * DS; i += 64) acc[i] = 0.0;
  const int slot = lane / L, q = lane % L;
  const int* gp = grp + (size_t)g * (2 + SLOTS);
  const int base = gp[0], steps = gp[1];
  double* arow = acc + slot * DS;
  const uint2* c0 = cv + base + slot;
  int t0 = 0;
  if (ROT && steps > 0) {
    const uint64_t turn = (uint64_t)tps * (uint64_t)steps;
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    t0 = (int)((now % turn) / (uint64_t)tps);
    t0 = __builtin_amdgcn_readfirstlane(t0);
  }
  for (int s = 0; s < steps; s += U) {
    uint2 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int t = t0 + min(s + u, steps - 1);
      if (t >= steps) t -= steps;
      w[u] = c0[(size_t)t * SLOTS];
    }
    float4 x[U];
    uint32_t sel[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t c = (w[u].x == ~0u) ? 0 : w[u].x;
      x[u] = *reinterpret_cast<const float4*>(sp_data + c * K + q * 4);
      sel[u] = *reinterpret_cast<const uint32_t*>(sp_index + c * K + q * 4);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = s + u < steps && w[u].x != ~0u;
      const float v = ok ? __uint_as_float(w[u].y) : 0.f;
      const double p0 = ok ? (double)(v * x[u].x) : 0.0, p1 = ok ? (double)(v * x[u].y) : 0.0;
      const double p2 = ok ? (double)(v * x[u].z) : 0.0, p3 = ok ? (double)(v * x[u].w) : 0.0;
      const uint32_t sv = sel[u];
      double* a0 = arow + (sv & 0xffu);
      double* a1 = arow + ((sv >> 8) & 0xffu);
      double* a2 = arow + ((sv >> 16) & 0xffu);
      double* a3 = arow + (sv >> 24);
      if (MODE == 0) {
        const double o0 = *a0, o1 = *a1, o2 = *a2, o3 = *a3;
        *a0 = o0 + p0;
        *a1 = o1 + p1;
        *a2 = o2 + p2;
        *a3 = o3 + p3;
        __builtin_amdgcn_sched_barrier(0);
      } else {
        atomicAdd(a0, p0);
        atomicAdd(a1, p1);
        atomicAdd(a2, p2);
        atomicAdd(a3, p3);
      }
    }
  }
  for (int j = 0; j < SLOTS; ++j) {
    const int r = gp[2 + j];
    if (r == -1) continue;
    const int row = r & 0x7fffffff;
    const double* a = acc + j * DS + lane * 4;
    const float4 o = make_float4((float)a[0], (float)a[1], (float)a[2], (float)a[3]);
    float* dst = out + (size_t)row * D + lane * 4;
    if (r < 0) {
      atomicAdd(dst, o.x);
      atomicAdd(dst + 1, o.y);
      atomicAdd(dst + 2, o.z);
      atomicAdd(dst + 3, o.w);
    } else {
      *reinterpret_cast<float4*>(dst) = o;
    }
  }
}

extern "C" float ubench_fwd_ilk(int k, int mode, int rot, int u16, int tps, const void* grp,
                                int ngrp, const void* cv, const void* sd, const void* si,
                                float* out, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int L = k / 4, SLOTS = 64 / L;
  const size_t lds = (size_t)4 * SLOTS * DS * sizeof(double);
  auto launch = [&]() {
    const int grid = (ngrp + 3) / 4;
#define K1(LL, M, UU, R)                                                                     \
  do {                                                                                       \
    (void)hipFuncSetAttribute((const void*)fwd_ilk<LL, M, UU, R>,                            \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);         \
    hipLaunchKernelGGL((fwd_ilk<LL, M, UU, R>), grid, 256, lds, 0, (const int*)grp, ngrp,    \
                       (const uint2*)cv, (const float*)sd, (const uint8_t*)si, out, tps);    \
  } while (0)
#define K2(LL, M, UU)             \
  do {                            \
    if (rot) K1(LL, M, UU, 1);    \
    else K1(LL, M, UU, 0);        \
  } while (0)
#define K3(LL, M)                 \
  do {                            \
    if (u16) K2(LL, M, 16);       \
    else K2(LL, M, 8);            \
  } while (0)
    if (L == 4) {
      if (mode == 0) K3(4, 0); else K3(4, 1);
    } else if (L == 8) {
      if (mode == 0) K3(8, 0); else K3(8, 1);
    } else {
      if (mode == 0) K3(16, 0); else K3(16, 1);
    }
#undef K3
#undef K2
#undef K1
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
