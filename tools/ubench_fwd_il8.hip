// Micro-benchmark (tooling, not product): atomic-free SpGEMM forward prototype, k = 16,
// 8 lanes per edge. Record of column c (128-B stride): lane q's 12 bytes at q*12 =
// {x[2q], x[2q+1], sel[2q] | sel[2q+1] << 8}, so ONE dwordx3 gather per lane gives both values
// and their selectors (one cache line per edge, no second selector gather). A wave owns 8
// accumulator rows (f64, wave-private LDS, 16 KB) and each instruction processes one edge of
// each of its 8 rows, so no two lanes of an instruction update the same LDS word.
//   cv[base_g + t * 8 + j] = {col, val bits} of step t of slot j of group g (val 0 = padding)
//   grp[g] = {base, steps, pad, pad, rows[8] (row | split << 31, -1 = empty)}
// MODE 0: f64 read-add-write; 1: ds_add_f64; 2: no LDS update. CVW: 1 = one wide cv load per
// U steps + ds_swizzle broadcast.
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int D = 256, SLOTS = 8, DS = D + 1;

struct Grp8 {
  int base, steps, pad0, pad1;
  int rows[SLOTS];
};

template <int MODE, int U, int NW, int CVW, int R16 = 0>
__global__ __launch_bounds__(NW * 64) void fwd_il8(const Grp8* __restrict__ grp, int ngrp,
                                                   const uint2* __restrict__ cv,
                                                   const uint8_t* __restrict__ rec,
                                                   float* __restrict__ out) {
  extern __shared__ __align__(16) double sm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = blockIdx.x * NW + wave;
  if (g >= ngrp) return;
  double* acc = sm + (size_t)wave * SLOTS * DS;
  if (MODE != 2)
    for (int i = lane; i < SLOTS * DS; i += 64) acc[i] = 0.0;
  const int slot = lane >> 3, q = lane & 7;
  const Grp8* gp = grp + g;
  const int base = gp->base, steps = gp->steps;
  double* arow = acc + slot * DS;
  float sink = 0.f;
  const uint2* c0 = cv + base + slot;
  for (int t = 0; t < steps; t += U) {
    uint32_t col[U], vb[U];
    if (CVW) {
      // lane (j, q) loads step t + q of slot j; step u is then broadcast from lane (j, u)
      static_assert(U == 8, "wide cv load: one step per lane of the slot");
      const uint2 w = c0[(size_t)min(t + q, steps - 1) * SLOTS];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        col[u] = (uint32_t)__shfl((int)w.x, (slot << 3) | u, 64);
        vb[u] = (uint32_t)__shfl((int)w.y, (slot << 3) | u, 64);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint2 w = c0[(size_t)min(t + u, steps - 1) * SLOTS];
        col[u] = w.x;
        vb[u] = w.y;
      }
    }
    uint3 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (R16) {  // 16-B lane chunks: one full 128-B line per edge, dwordx4
        const uint4 y = *reinterpret_cast<const uint4*>(rec + (size_t)col[u] * 128 + q * 16);
        x[u] = make_uint3(y.x, y.y, y.z);
      } else {
        x[u] = *reinterpret_cast<const uint3*>(rec + (size_t)col[u] * 128 + q * 12);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float v = (t + u < steps) ? __uint_as_float(vb[u]) : 0.f;
      const float p0 = v * __uint_as_float(x[u].x), p1 = v * __uint_as_float(x[u].y);
      const uint32_t sv = x[u].z;
      if (MODE == 0) {
        double* a0 = arow + (sv & 0xffu);
        double* a1 = arow + ((sv >> 8) & 0xffu);
        const double o0 = *a0, o1 = *a1;
        *a0 = o0 + p0;
        *a1 = o1 + p1;
        __builtin_amdgcn_sched_barrier(0);
      } else if (MODE == 1) {
        atomicAdd(arow + (sv & 0xffu), (double)p0);
        atomicAdd(arow + ((sv >> 8) & 0xffu), (double)p1);
      } else {
        sink += p0 + p1 + (float)(sv & 1);
      }
    }
  }
  for (int j = 0; j < SLOTS; ++j) {
    const int r = gp->rows[j];
    if (r == -1) continue;
    const int row = r & 0x7fffffff;
    const double* a = acc + j * DS + lane * 4;
    float4 o = MODE == 2 ? make_float4(sink, 0.f, 0.f, 0.f)
                         : make_float4((float)a[0], (float)a[1], (float)a[2], (float)a[3]);
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

extern "C" float ubench_fwd_il8(int mode, int nw, int cvw, int r16, const void* grp, int ngrp,
                                const void* cv, const void* rec, float* out, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const size_t lds = mode == 2 ? 0 : (size_t)nw * SLOTS * DS * sizeof(double);
  auto launch = [&]() {
    const int grid = (ngrp + nw - 1) / nw;
#define L1(M, NWW, CW, RR)                                                                   \
  do {                                                                                       \
    (void)hipFuncSetAttribute((const void*)fwd_il8<M, 8, NWW, CW, RR>,                       \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);         \
    hipLaunchKernelGGL((fwd_il8<M, 8, NWW, CW, RR>), grid, NWW * 64, lds, 0,                 \
                       (const Grp8*)grp, ngrp, (const uint2*)cv, (const uint8_t*)rec, out);  \
  } while (0)
#define L(M, NWW, CW)              \
  do {                             \
    if (r16) L1(M, NWW, CW, 1);    \
    else L1(M, NWW, CW, 0);        \
  } while (0)
#define LM(NWW, CW)                 \
  do {                              \
    if (mode == 0) L(0, NWW, CW);   \
    else if (mode == 1) L(1, NWW, CW); \
    else L(2, NWW, CW);             \
  } while (0)
    if (nw == 4) {
      if (cvw) LM(4, 1);
      else LM(4, 0);
    } else {
      if (cvw) LM(1, 1);
      else LM(1, 0);
    }
#undef LM
#undef L
#undef L1
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
