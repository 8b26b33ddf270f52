// SpGEMM forward (row-wise product over CBSR features) and SSpMM backward (outer product
// sampled at the selector) for gfx950.
//
// Reference kernels: spmm_kernel_opt2_sparse_v3 and
// spmm_kernel_opt2_sparse_backward_v3 give every 32-lane warp one <=64-nz chunk of a CSR
// row (".warp4" metadata), accumulate into a per-warp LDS row and write it back with one
// global float atomic per feature per chunk (forward), or scatter every product with a
// global float atomic into grad_sp (backward). On MI355X global float atomics execute at
// the memory side at ~1.3 TB/s, so both are restructured here:
//
//   forward : a 256-thread work-group owns <= 16 whole destination rows (LDS accumulator
//             16 x D f32); its edges are processed flat (64/(k/4) edges per wave
//             instruction, 4 features per lane: one dwordx4 value load + one dword
//             selector load), scattered into LDS with ds_add_f32, and the rows are written
//             back once with coalesced dwordx4 stores. Only rows longer than the task cap
//             are split, and only those use global atomics.
//   backward: a 512-thread work-group owns a block of source columns whose k-wide
//             gradients live in LDS; it sweeps the block's edges in destination-row
//             order (plan-built block-major edge list), gathering grad_out[r, sel] and
//             accumulating into LDS; the block is stored (or atomically flushed when a
//             block is shared by several work-groups) once at the end.
#include "common.h"

namespace maxk {

// --------------------------------------------------------------------------------------
// forward
// --------------------------------------------------------------------------------------
template <int VEC>
__global__ __launch_bounds__(kFwdThreads) void spgemm_fwd_kernel(
    const FwdTask* __restrict__ tasks, const int32_t* __restrict__ ptr,
    const int32_t* __restrict__ idx, const float* __restrict__ val,
    const float* __restrict__ sp_data, const uint8_t* __restrict__ sp_index,
    float* __restrict__ out, int D, int k) {
  // f64 LDS accumulators: on gfx950 ds_add_f64 sustains ~9x the rate of ds_add_f32
  // (tools/ubench_atomics: 1.85e12 vs 2.0e11 adds/s chip-wide), and f64 sums make the
  // f32 result independent of the atomic arrival order in all but pathological cases.
  extern __shared__ __align__(16) double smem_d[];
  const FwdTask t = tasks[blockIdx.x];
  const bool split = t.nrows < 0;
  const int nrows = split ? 1 : t.nrows;
  double* acc = smem_d;
  int* sptr = reinterpret_cast<int*>(smem_d + kFwdTileRows * D);
  const int n = nrows * D;
  for (int i = threadIdx.x * 2; i < n; i += kFwdThreads * 2)
    *reinterpret_cast<double2*>(acc + i) = make_double2(0.0, 0.0);
  for (int i = threadIdx.x; i <= nrows; i += kFwdThreads)
    sptr[i] = split ? (i == 0 ? t.e0 : t.e1) : ptr[t.row0 + i];
  __syncthreads();

  // lanes per edge: VEC==4 => k % 4 == 0 and k/4 <= 64; VEC==1 => min(k, 64) lanes that
  // loop over the row's k entries.
  const int L = (VEC == 4) ? k / 4 : (k < kWave ? k : kWave);
  const int EPS = kWave / L;      // edges per wave instruction
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int slot = lane / L;
  const int l0 = (lane - slot * L) * VEC;
  const bool lane_on = slot < EPS;
  constexpr int kWaves = kFwdThreads / kWave;

  if constexpr (VEC == 4) {
    // U sub-steps per iteration with every load issued before the first LDS update: the
    // chain idx/val -> CBSR row -> LDS has two dependent global round trips, so memory-
    // level parallelism comes from U independent sub-steps per wave. Out-of-range lanes
    // load a clamped (valid) edge and skip the update.
    constexpr int U = kFwdUnroll;
    const int last = t.e1 - 1;
    for (int base = t.e0 + wave * EPS * U; base < t.e1; base += kWaves * EPS * U) {
      int c[U], rl[U];
      float v[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + u * EPS + slot;
        ok[u] = lane_on && e < t.e1;
        const int ec = ok[u] ? e : last;
        c[u] = idx[ec];
        v[u] = val[ec];
        int lo = 0, hi = nrows - 1;  // row of ec: last j with sptr[j] <= ec
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (sptr[mid] <= ec) lo = mid; else hi = mid - 1;
        }
        rl[u] = lo;
      }
      float4 x[U];
      uint32_t sel[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t off = (size_t)c[u] * k + l0;
        x[u] = *reinterpret_cast<const float4*>(sp_data + off);
        sel[u] = *reinterpret_cast<const uint32_t*>(sp_index + off);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (ok[u]) {
          double* arow = acc + rl[u] * D;
          const uint32_t sv = sel[u];
          lds_add(arow + (sv & 0xffu), (double)(v[u] * x[u].x));
          lds_add(arow + ((sv >> 8) & 0xffu), (double)(v[u] * x[u].y));
          lds_add(arow + ((sv >> 16) & 0xffu), (double)(v[u] * x[u].z));
          lds_add(arow + (sv >> 24), (double)(v[u] * x[u].w));
        }
      }
    }
  } else {
    for (int base = t.e0 + wave * EPS; base < t.e1; base += kWaves * EPS) {
      const int e = base + slot;
      if (lane_on && e < t.e1) {
        int lo = 0, hi = nrows - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (sptr[mid] <= e) lo = mid; else hi = mid - 1;
        }
        const int c = idx[e];
        const float v = val[e];
        double* arow = acc + lo * D;
        const size_t rb = (size_t)c * k;
        for (int l = l0; l < k; l += L)
          lds_add(arow + sp_index[rb + l], (double)(v * sp_data[rb + l]));
      }
    }
  }
  __syncthreads();

  float* dst = out + (size_t)t.row0 * D;
  if (!split) {
    if ((D & 3) == 0) {
      for (int i = threadIdx.x * 4; i < n; i += kFwdThreads * 4) {
        const double2 a = *reinterpret_cast<const double2*>(acc + i);
        const double2 b = *reinterpret_cast<const double2*>(acc + i + 2);
        *reinterpret_cast<float4*>(dst + i) =
            make_float4((float)a.x, (float)a.y, (float)b.x, (float)b.y);
      }
    } else {
      for (int i = threadIdx.x; i < n; i += kFwdThreads) dst[i] = (float)acc[i];
    }
  } else {
    for (int i = threadIdx.x; i < D; i += kFwdThreads) global_add(dst + i, (float)acc[i]);
  }
}

__global__ void zero_rows_kernel(const int32_t* __restrict__ rows, int nrows, float* out,
                                 int D) {
  const int r = blockIdx.x;
  if (r >= nrows) return;
  float* dst = out + (size_t)rows[r] * D;
  for (int i = threadIdx.x; i < D; i += blockDim.x) dst[i] = 0.f;
}

// --------------------------------------------------------------------------------------
// backward
// --------------------------------------------------------------------------------------
// Flat edge processing in (column block, destination row) order: the edges one wave
// instruction covers share few rows of grad_out, so its gathers stay in the CU's L1.
// Accumulation: f64 LDS atomics (ds_add_f64 ~9x the ds_add_f32 rate on gfx950; any wave
// may update any column of the block, which is what keeps the row locality).
template <int F>
__global__ __launch_bounds__(kBwdThreads) void sspmm_bwd_kernel(
    const BwdTask* __restrict__ tasks, const int32_t* __restrict__ erow,
    const int32_t* __restrict__ ecol, const float* __restrict__ evals,
    const float* __restrict__ G, const uint8_t* __restrict__ sp_index,
    float* __restrict__ grad_sp, int D, int k) {
  extern __shared__ __align__(16) double bacc[];  // [ncols][k]
  const BwdTask t = tasks[blockIdx.x];
  const int n = t.ncols * k;
  for (int i = threadIdx.x; i < n; i += kBwdThreads) bacc[i] = 0.0;
  __syncthreads();

  const int L = bwd_lanes(k);
  const int EPS = kWave / L;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int slot = lane / L;
  const int q = lane - slot * L;
  const bool lane_on = slot < EPS;
  constexpr int kWaves = kBwdThreads / kWave;
  constexpr int U = kBwdUnroll;
  const int last = t.e1 - 1;

  for (int base = t.e0 + wave * EPS * U; base < t.e1; base += kWaves * EPS * U) {
    int r[U], c[U];
    float v[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * EPS + slot;
      ok[u] = lane_on && e < t.e1;
      const int ec = ok[u] ? e : last;
      r[u] = erow[ec];
      c[u] = ecol[ec];
      v[u] = evals[ec];
    }
    if constexpr (F == 4) {
      uint32_t sel[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        sel[u] = *reinterpret_cast<const uint32_t*>(sp_index + (size_t)c[u] * k + q * 4);
      float g[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float* grow = G + (size_t)r[u] * D;
        g[u][0] = grow[sel[u] & 0xffu];
        g[u][1] = grow[(sel[u] >> 8) & 0xffu];
        g[u][2] = grow[(sel[u] >> 16) & 0xffu];
        g[u][3] = grow[sel[u] >> 24];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (ok[u]) {
          double* a = bacc + (c[u] - t.col0) * k + q * 4;
          lds_add(a, (double)(v[u] * g[u][0]));
          lds_add(a + 1, (double)(v[u] * g[u][1]));
          lds_add(a + 2, (double)(v[u] * g[u][2]));
          lds_add(a + 3, (double)(v[u] * g[u][3]));
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (ok[u]) {
          const float* grow = G + (size_t)r[u] * D;
          const uint8_t* srow = sp_index + (size_t)c[u] * k;
          double* a = bacc + (c[u] - t.col0) * k;
          for (int l = q; l < k; l += L) lds_add(a + l, (double)(v[u] * grow[srow[l]]));
        }
      }
    }
  }
  __syncthreads();

  float* dst = grad_sp + (size_t)t.col0 * k;
  if (t.shared) {
    for (int i = threadIdx.x; i < n; i += kBwdThreads) global_add(dst + i, (float)bacc[i]);
  } else {
    for (int i = threadIdx.x; i < n; i += kBwdThreads) dst[i] = (float)bacc[i];
  }
}

// --------------------------------------------------------------------------------------
// dense CSR SpMM comparator: one wavefront per destination row, 4 features per lane.
// --------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dense_spmm_kernel(
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
    const float* __restrict__ val, const float* __restrict__ X, float* __restrict__ Y,
    int N, int D) {
  const int lane = threadIdx.x & (kWave - 1);
  const int row = blockIdx.x * (256 / kWave) + threadIdx.x / kWave;
  if (row >= N) return;
  const int e0 = ptr[row], e1 = ptr[row + 1];
  for (int d0 = lane * 4; d0 < D; d0 += kWave * 4) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int e = e0; e < e1; ++e) {
      const float v = val[e];
      const float4 x = *reinterpret_cast<const float4*>(X + (size_t)idx[e] * D + d0);
      a.x = fmaf(v, x.x, a.x);
      a.y = fmaf(v, x.y, a.y);
      a.z = fmaf(v, x.z, a.z);
      a.w = fmaf(v, x.w, a.w);
    }
    *reinterpret_cast<float4*>(Y + (size_t)row * D + d0) = a;
  }
}

static size_t fwd_lds_bytes(int D) {
  return (size_t)kFwdTileRows * D * sizeof(double) + (kFwdTileRows + 1) * sizeof(int);
}

size_t bwd_lds_bytes(int block_cols, int k) { return (size_t)block_cols * k * sizeof(double); }

}  // namespace maxk

using namespace maxk;

static int check_plan(const maxk_plan* plan, const int32_t* ptr, const int32_t* idx,
                      int32_t N, int64_t E, int32_t k, int32_t D, const char* who) {
  MAXK_CHECK_ARG(plan != nullptr, std::string(who) + ": plan is null");
  if (plan->num_nodes != N || plan->num_edges != E || plan->dim_k != k ||
      plan->dim_origin != D || plan->src_ptr != ptr || plan->src_idx != idx) {
    set_error(std::string(who) + ": plan was built for a different graph / k / D");
    return MAXK_ERR_PLAN_MISMATCH;
  }
  return MAXK_OK;
}

extern "C" int maxk_spgemm_forward(const maxk_plan* plan, const int32_t* ptr,
                                   const int32_t* idx, const float* val,
                                   const float* sp_data, const uint8_t* sp_index, float* out,
                                   int32_t N, int64_t E, int32_t k, int32_t D, void* stream) {
  MAXK_CHECK_ARG(N >= 0 && E >= 0, "maxk_spgemm_forward: negative size");
  MAXK_CHECK_ARG(D >= 1 && D <= kMaxDim, "maxk_spgemm_forward: dim_origin must be in [1, 256]");
  MAXK_CHECK_ARG(k >= 1 && k <= D, "k must be between 1 and input dimension");
  int rc = check_plan(plan, ptr, idx, N, E, k, D, "maxk_spgemm_forward");
  if (rc) return rc;
  if (N == 0) return MAXK_OK;
  MAXK_CHECK_ARG(out && sp_data && sp_index && (E == 0 || (idx && val)) && ptr,
                 "maxk_spgemm_forward: null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (plan->n_zero_rows > 0) {
    hipLaunchKernelGGL(zero_rows_kernel, dim3(plan->n_zero_rows), dim3(256), 0, s,
                       plan->zero_rows, plan->n_zero_rows, out, D);
    MAXK_LAUNCH_CHECK("zero_rows launch");
  }
  const size_t lds = fwd_lds_bytes(D);
  if (k % 4 == 0)
    hipLaunchKernelGGL(spgemm_fwd_kernel<4>, dim3(plan->n_fwd_tasks), dim3(kFwdThreads), lds,
                       s, plan->fwd_tasks, ptr, idx, val, sp_data, sp_index, out, D, k);
  else
    hipLaunchKernelGGL(spgemm_fwd_kernel<1>, dim3(plan->n_fwd_tasks), dim3(kFwdThreads), lds,
                       s, plan->fwd_tasks, ptr, idx, val, sp_data, sp_index, out, D, k);
  MAXK_LAUNCH_CHECK("spgemm_fwd launch");
  return MAXK_OK;
}

extern "C" int maxk_sspmm_backward(const maxk_plan* plan, const int32_t* ptr,
                                   const int32_t* idx, const float* val,
                                   const float* grad_out, const uint8_t* sp_index,
                                   float* grad_sp, int32_t N, int64_t E, int32_t k, int32_t D,
                                   void* stream) {
  (void)val;  // the plan holds the block-major snapshot of val
  MAXK_CHECK_ARG(N >= 0 && E >= 0, "maxk_sspmm_backward: negative size");
  MAXK_CHECK_ARG(D >= 1 && D <= kMaxDim, "maxk_sspmm_backward: dim_origin must be in [1, 256]");
  MAXK_CHECK_ARG(k >= 1 && k <= D, "k must be between 1 and input dimension");
  int rc = check_plan(plan, ptr, idx, N, E, k, D, "maxk_sspmm_backward");
  if (rc) return rc;
  if (N == 0) return MAXK_OK;
  MAXK_CHECK_ARG(grad_out && sp_index && grad_sp, "maxk_sspmm_backward: null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (plan->n_bwd_shared > 0)
    MAXK_HIP_TRY(hipMemsetAsync(grad_sp, 0, (size_t)plan->num_cols * k * sizeof(float), s));
  const size_t lds = bwd_lds_bytes(plan->bwd_block_cols, k);
  if (plan->n_bwd_tasks == 0) return MAXK_OK;
  static bool attr_set = false;  // allow > 64 KiB of dynamic LDS (gfx950 has 160 KiB/CU)
  if (!attr_set) {
    MAXK_HIP_TRY(hipFuncSetAttribute((const void*)sspmm_bwd_kernel<4>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, kBwdLdsBudget));
    MAXK_HIP_TRY(hipFuncSetAttribute((const void*)sspmm_bwd_kernel<1>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, kBwdLdsBudget));
    attr_set = true;
  }
  if (bwd_feats(k) == 4)
    hipLaunchKernelGGL(sspmm_bwd_kernel<4>, dim3(plan->n_bwd_tasks), dim3(kBwdThreads), lds, s,
                       plan->bwd_tasks, plan->bwd_row, plan->bwd_col, plan->bwd_val, grad_out,
                       sp_index, grad_sp, D, k);
  else
    hipLaunchKernelGGL(sspmm_bwd_kernel<1>, dim3(plan->n_bwd_tasks), dim3(kBwdThreads), lds, s,
                       plan->bwd_tasks, plan->bwd_row, plan->bwd_col, plan->bwd_val, grad_out,
                       sp_index, grad_sp, D, k);
  MAXK_LAUNCH_CHECK("sspmm_bwd launch");
  return MAXK_OK;
}

extern "C" int maxk_dense_spmm_csr(const int32_t* ptr, const int32_t* idx, const float* val,
                                   const float* X, float* Y, int32_t N, int32_t D,
                                   void* stream) {
  MAXK_CHECK_ARG(N >= 0 && D >= 1, "maxk_dense_spmm_csr: bad size");
  MAXK_CHECK_ARG(D % 4 == 0, "maxk_dense_spmm_csr: dim must be a multiple of 4");
  if (N == 0) return MAXK_OK;
  MAXK_CHECK_ARG(ptr && X && Y, "maxk_dense_spmm_csr: null pointer");
  hipLaunchKernelGGL(dense_spmm_kernel, dim3((N + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     ptr, idx, val, X, Y, N, D);
  MAXK_LAUNCH_CHECK("dense_spmm launch");
  return MAXK_OK;
}
