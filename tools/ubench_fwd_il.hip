// Micro-benchmark (tooling, not product): an atomic-free SpGEMM forward prototype.
// Each wave owns 16 accumulator rows (f64, wave-private LDS) and every wave instruction
// processes one edge of each of its 16 rows (k = 16: 4 lanes per edge), so no two lanes of an
// instruction update the same LDS word and a plain read-add-write replaces ds_add_f64. LDS
// operations of one wave execute in issue order, so the RMW of sub-step u+1 sees the writes of
// sub-step u. The edge schedule is built by tools/ubench_fwd_il.py:
//   cv[base_g + t * 16 + j] = {col, val bits} of step t of slot j of group g (val 0 = padding)
//   grp[g] = {base, steps, rows[16] (row | split << 31, -1 = empty)}
// MODE 0: f64 read-add-write; 1: ds_add_f64 atomics; 2: no LDS update (sum in a register).
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int K = 16, D = 256, SLOTS = 16, DS = D + 1;

struct Grp {
  int base, steps, pad0, pad1;
  int rows[SLOTS];
};

template <int MODE, int U, int NW>
__global__ __launch_bounds__(NW * 64) void fwd_il(const Grp* __restrict__ grp, int ngrp,
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
  const int slot = lane >> 2, q = lane & 3;
  const Grp* gp = grp + g;
  const int base = gp->base, steps = gp->steps;
  double* arow = acc + slot * DS;
  float sink = 0.f;
  const uint2* c0 = cv + base + slot;
  for (int t = 0; t < steps; t += U) {
    uint2 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = c0[(size_t)min(t + u, steps - 1) * SLOTS];
    float4 x[U];
    uint32_t s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint8_t* rp = rec + (size_t)w[u].x * 128;
      x[u] = *reinterpret_cast<const float4*>(rp + q * 16);
      s[u] = *reinterpret_cast<const uint32_t*>(rp + 64 + q * 4);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float v = (t + u < steps) ? __uint_as_float(w[u].y) : 0.f;
      const float p0 = v * x[u].x, p1 = v * x[u].y, p2 = v * x[u].z, p3 = v * x[u].w;
      const uint32_t sv = s[u];
      if (MODE == 0) {
        double* a0 = arow + (sv & 0xffu);
        double* a1 = arow + ((sv >> 8) & 0xffu);
        double* a2 = arow + ((sv >> 16) & 0xffu);
        double* a3 = arow + (sv >> 24);
        const double o0 = *a0, o1 = *a1, o2 = *a2, o3 = *a3;
        *a0 = o0 + p0;
        *a1 = o1 + p1;
        *a2 = o2 + p2;
        *a3 = o3 + p3;
        // keep the next sub-step's reads behind these writes (same wave, in-order LDS)
        __builtin_amdgcn_sched_barrier(0);
      } else if (MODE == 1) {
        atomicAdd(arow + (sv & 0xffu), (double)p0);
        atomicAdd(arow + ((sv >> 8) & 0xffu), (double)p1);
        atomicAdd(arow + ((sv >> 16) & 0xffu), (double)p2);
        atomicAdd(arow + (sv >> 24), (double)p3);
      } else {
        sink += p0 + p1 + p2 + p3 + (float)(sv & 1);
      }
    }
  }
  // write back the 16 rows: lane owns 4 consecutive features of each row
  for (int j = 0; j < SLOTS; ++j) {
    const int r = gp->rows[j];
    if (r == -1) continue;
    const int row = r & 0x7fffffff;
    const double* a = acc + j * DS + lane * 4;
    float4 o = MODE == 2 ? make_float4(0.f, 0.f, 0.f, 0.f)
                         : make_float4((float)a[0], (float)a[1], (float)a[2], (float)a[3]);
    if (MODE == 2) o.x += sink;
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

extern "C" float ubench_fwd_il(int mode, int nw, const void* grp, int ngrp, const void* cv,
                               const void* rec, float* out, int reps, int u16) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  // mode 3: no LDS update and no LDS allocation (occupancy bound by registers only)
  const size_t lds = mode == 3 ? 0 : (size_t)nw * SLOTS * DS * sizeof(double);
  auto launch = [&]() {
    const int grid = (ngrp + nw - 1) / nw;
#define L(M, UU, NWW)                                                                        \
  do {                                                                                       \
    (void)hipFuncSetAttribute((const void*)fwd_il<M, UU, NWW>,                               \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);         \
    hipLaunchKernelGGL((fwd_il<M, UU, NWW>), grid, NWW * 64, lds, 0, (const Grp*)grp, ngrp,  \
                       (const uint2*)cv, (const uint8_t*)rec, out);                          \
  } while (0)
    if (mode == 3) {
      if (u16) L(2, 16, 4);
      else L(2, 8, 4);
    } else if (u16) {
      if (mode == 0) L(0, 16, 4);
      else if (mode == 1) L(1, 16, 4);
      else L(2, 16, 4);
    } else if (nw == 4) {
      if (mode == 0) L(0, 8, 4);
      else if (mode == 1) L(1, 8, 4);
      else L(2, 8, 4);
    } else if (nw == 2) {
      if (mode == 0) L(0, 8, 2);
      else if (mode == 1) L(1, 8, 2);
      else L(2, 8, 2);
    } else {
      if (mode == 0) L(0, 8, 1);
      else if (mode == 1) L(1, 8, 1);
      else L(2, 8, 1);
    }
#undef L
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
