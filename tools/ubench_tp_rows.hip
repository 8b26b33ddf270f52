// Micro-benchmark (tooling, not product): the two-pass backward's row pass
// (spgemm.hip sspmm_bwd_rows_kernel) on an ogbn-products-shaped problem, in variants that
// separate its costs. Every variant writes the same products (checked by the driver), except
// the ones marked "probe" (time only).
//
//   VAR 0  product organisation: U = 4 sub-steps, each a quad-batched record load, a selector
//          dword gather and a buffer_store_b128 (nt) per lane
//   VAR 1  the same with plain stores
//   VAR 2  software-pipelined: the next step's records and selectors are loaded before this
//          step's stores are issued (vmcnt counts stores with loads in issue order, so a
//          step that loads after the previous step's stores waits for those stores too)
//   VAR 3  VAR 2 with plain stores
//   VAR 4  probe: no stores (the products are kept live through an xor)
//   VAR 5  VAR 2 with sc1 (write-through, L2-dropping) stores
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kWave = 64;
constexpr int kMaxDim = 256;
constexpr int kColBits = 26;
constexpr uint32_t kColMask = (1u << kColBits) - 1;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int W>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, W * 0x55, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t quad_pick(uint32_t v, int u) {
  switch (u & 3) {
    case 0: return quad_bcast<0>(v);
    case 1: return quad_bcast<1>(v);
    case 2: return quad_bcast<2>(v);
    default: return quad_bcast<3>(v);
  }
}

template <int VAR, int U, int R>
__global__ __launch_bounds__(256) void rows_kernel(const int32_t* __restrict__ ptr,
                                                   const uint32_t* __restrict__ erec,
                                                   const float* __restrict__ G,
                                                   const uint8_t* __restrict__ sp_index,
                                                   float* __restrict__ T, int N, int D, int k,
                                                   uint32_t* __restrict__ sink) {
  __shared__ float grow[256 / kWave][R * kMaxDim];
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int r0 = (blockIdx.x * (256 / kWave) + w) * R;
  if (r0 >= N) return;
  const int r1 = min(N, r0 + R);
  const int e0 = __builtin_amdgcn_readfirstlane(ptr[r0]);
  const int e1 = __builtin_amdgcn_readfirstlane(ptr[r1]);
  if (e0 >= e1) return;
  {
    float x[R][kMaxDim / kWave];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const float* g = G + (size_t)min(r0 + j, N - 1) * D;
#pragma unroll
      for (int i = 0; i < kMaxDim / kWave; ++i) x[j][i] = g[lane + i * kWave];
    }
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
      for (int i = 0; i < kMaxDim / kWave; ++i) grow[w][j * kMaxDim + lane + i * kWave] = x[j][i];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int L = k >> 2;
  const int EPS = kWave / L;
  const int slot = lane / L;
  const int q = lane - slot * L;
  const int qq = lane & 3;
  const float* row = grow[w];
  const __amdgpu_buffer_rsrc_t tr = __builtin_amdgcn_make_buffer_rsrc(
      T + (size_t)e0 * k, (short)0, (int)((uint32_t)(e1 - e0) * (uint32_t)k * 4u), 0x00020000);
  constexpr int AUX = (VAR == 1 || VAR == 3) ? 0 : (VAR == 5 ? 16 : 2);
  constexpr bool PIPE = VAR == 2 || VAR == 3 || VAR == 5;
  uint32_t live = 0;
  auto load_step = [&](int base, uint32_t (&c)[U], float (&v)[U], uint32_t (&sw)[U]) {
#pragma unroll
    for (int j = 0; j < U / 4; ++j) {
      const uint2 w2 = *reinterpret_cast<const uint2*>(
          erec + 2 * (size_t)min(base + (4 * j + qq) * EPS + slot, e1 - 1));
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        c[4 * j + i] = quad_pick(w2.x, i);
        v[4 * j + i] = __uint_as_float(quad_pick(w2.y, i));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      sw[u] = *reinterpret_cast<const uint32_t*>(sp_index + (size_t)(c[u] & kColMask) * k + 4 * q);
  };
  auto compute_store = [&](int base, const uint32_t (&c)[U], const float (&v)[U],
                           const uint32_t (&sw)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * EPS + slot;
      const float* rw = row + (R > 1 ? (c[u] >> kColBits) * kMaxDim : 0);
      const uint32_t off = e < e1 ? ((uint32_t)(e - e0) * (uint32_t)k + 4u * q) * 4u : 0xfffffff0u;
      u32x4 o;
      o.x = __float_as_uint(v[u] * rw[sw[u] & 0xffu]);
      o.y = __float_as_uint(v[u] * rw[(sw[u] >> 8) & 0xffu]);
      o.z = __float_as_uint(v[u] * rw[(sw[u] >> 16) & 0xffu]);
      o.w = __float_as_uint(v[u] * rw[sw[u] >> 24]);
      if constexpr (VAR == 4) live ^= o.x ^ o.y ^ o.z ^ o.w;
      else __builtin_amdgcn_raw_buffer_store_b128(o, tr, off, 0, AUX);
    }
  };
  uint32_t c[U], sw[U];
  float v[U];
  if constexpr (PIPE) {
    // issue order per step i: selectors of step i+1, records of step i+2, then step i's LDS
    // reads and stores. The wait for a load then never covers an older store: the records
    // of i+1 were issued before the stores of i-1, the selectors of i before the records of
    // i+1 and the stores of i-1 (all loads clamped to valid edges, no branches)
    const int S = EPS * U;
    auto load_raw = [&](int base, uint2 (&raw)[U / 4]) {
#pragma unroll
      for (int j = 0; j < U / 4; ++j)
        raw[j] = *reinterpret_cast<const uint2*>(
            erec + 2 * (size_t)min(base + (4 * j + qq) * EPS + slot, e1 - 1));
    };
    auto decode = [&](const uint2 (&raw)[U / 4], uint32_t (&cc)[U], float (&vv)[U]) {
#pragma unroll
      for (int j = 0; j < U / 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          cc[4 * j + i] = quad_pick(raw[j].x, i);
          vv[4 * j + i] = __uint_as_float(quad_pick(raw[j].y, i));
        }
    };
    auto load_sel = [&](const uint32_t (&cc)[U], uint32_t (&ss)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u)
        ss[u] = *reinterpret_cast<const uint32_t*>(sp_index + (size_t)(cc[u] & kColMask) * k + 4 * q);
    };
    uint2 raw0[U / 4], raw1[U / 4];
    load_raw(e0, raw0);
    load_raw(e0 + S, raw1);
    decode(raw0, c, v);
    load_sel(c, sw);
    for (int base = e0; base < e1; base += S) {
      uint32_t cn[U], swn[U];
      float vn[U];
      decode(raw1, cn, vn);
      load_sel(cn, swn);
      load_raw(base + 2 * S, raw1);
      compute_store(base, c, v, sw);
#pragma unroll
      for (int u = 0; u < U; ++u) { c[u] = cn[u]; v[u] = vn[u]; sw[u] = swn[u]; }
    }
  } else {
    for (int base = e0; base < e1; base += EPS * U) {
      load_step(base, c, v, sw);
      compute_store(base, c, v, sw);
    }
  }
  if constexpr (VAR == 4)
    if (live == 0x12345678u) sink[0] = live;
}

template <int VAR>
static float run(const int32_t* ptr, const uint32_t* erec, const float* G, const uint8_t* sel,
                 float* T, int N, int D, int k, uint32_t* sink, int reps) {
  constexpr int R = 4;
  const dim3 grid((N + 4 * R - 1) / (4 * R));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((rows_kernel<VAR, 4, R>), grid, dim3(256), 0, 0, ptr, erec, G, sel, T, N, D,
                     k, sink);
  hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((rows_kernel<VAR, 4, R>), grid, dim3(256), 0, 0, ptr, erec, G, sel, T, N,
                       D, k, sink);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms / reps;
}

extern "C" float ubench_tp_rows(int var, const int32_t* ptr, const uint32_t* erec, const float* G,
                                const uint8_t* sel, float* T, int N, int D, int k,
                                uint32_t* sink, int reps) {
  switch (var) {
    case 0: return run<0>(ptr, erec, G, sel, T, N, D, k, sink, reps);
    case 1: return run<1>(ptr, erec, G, sel, T, N, D, k, sink, reps);
    case 2: return run<2>(ptr, erec, G, sel, T, N, D, k, sink, reps);
    case 3: return run<3>(ptr, erec, G, sel, T, N, D, k, sink, reps);
    case 4: return run<4>(ptr, erec, G, sel, T, N, D, k, sink, reps);
    default: return run<5>(ptr, erec, G, sel, T, N, D, k, sink, reps);
  }
}
