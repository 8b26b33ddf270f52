// Graph plan: the partition metadata the two SpGEMM kernels run on.
//
// The reference reads a precomputed ".warp4" file from disk on every call
// (SPMM_MAXK::do_test SO@0x24bf0 -> cuda_read_array<int> SO@0x252c0; chunk rule SURVEY
// §8 a4; generator generate_meta.py absent) and never uses the `ptr` it is given. Here the
// metadata is derived once from the CSR row pointer and the column indices and cached by
// the caller:
//
//   forward : tasks of <= 32 whole rows with <= cap edges (heavy first); rows longer
//             than cap are split into segments whose outputs are pre-zeroed and summed
//             with float atomics (the only atomics left in the forward). Each task's edges
//             are sorted by column (8-B words {column | row-in-task, val}) with window
//             offsets for the clock-rotated sweep.
//   backward: a stable radix sort of the edges by source-column block
//             (hipcub::DeviceRadixSort, keys = block of the column's position) gives the
//             block-major, row-sorted edge list, packed as 12-B records {row * D * 4, column
//             in block, val}; each block's stream is cut into equal-edge chunk tasks emitted
//             in order of their first row (XCD-aware). Low-reuse graphs get the two-pass
//             metadata instead (CSR-order edge records, column pointers).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstring>
#include <vector>

#include <cstdlib>

#include "common.h"

namespace maxk {


__global__ void expand_rows_kernel(const int32_t* __restrict__ ptr, int N,
                                   int32_t* __restrict__ row_of) {
  const int lane = threadIdx.x & (kWave - 1);
  const int row = blockIdx.x * (256 / kWave) + threadIdx.x / kWave;
  if (row >= N) return;
  const int e1 = ptr[row + 1];
  for (int e = ptr[row] + lane; e < e1; e += kWave) row_of[e] = row;
}

// Forward edge order: every forward task's edges contiguous (tasks in launch order) and
// sorted by source column inside the task, so the work-groups running at the same time -
// similar-sized tasks, heavy first - sweep the CBSR table in step and its recently used
// records stay in L2. starts/ranks/row0s: the tasks sorted by their first CSR edge.
__global__ void fwd_key_kernel(const int32_t* __restrict__ idx, const int32_t* __restrict__ row_of,
                               int64_t E, const int32_t* __restrict__ starts,
                               const int32_t* __restrict__ ranks,
                               const int32_t* __restrict__ row0s, int ntasks, int cbits,
                               uint64_t* __restrict__ keys, int32_t* __restrict__ ids,
                               int32_t* __restrict__ rl_of) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    int lo = 0, hi = ntasks - 1;  // last task whose first edge <= e
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (starts[mid] <= e) lo = mid; else hi = mid - 1;
    }
    keys[e] = ((uint64_t)ranks[lo] << cbits) | (uint64_t)(uint32_t)idx[e];
    ids[e] = (int32_t)e;
    rl_of[e] = row_of[e] - row0s[lo];
  }
}

// off[t * (B + 1) + b] = first edge of task t whose column is >= b * NC / B (the task's
// edges are column-sorted).
__global__ void fwd_phase_kernel(const FwdTask* __restrict__ tasks, int ntasks,
                                 const uint2* __restrict__ cv, int NC, int B,
                                 int32_t* __restrict__ off) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ntasks * (B + 1)) return;
  const int t = i / (B + 1), b = i - t * (B + 1);
  const FwdTask tk = tasks[t];
  const uint32_t bound = (uint32_t)((int64_t)NC * b / B);
  int lo = tk.e0, hi = tk.e1;
  if (b == B) { off[i] = hi; return; }
  if (b == 0) { off[i] = lo; return; }
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((cv[mid].x & kFwdColMask) < bound) lo = mid + 1; else hi = mid;
  }
  off[i] = lo;
}

__global__ void gather_fwd_kernel(const int32_t* __restrict__ perm,
                                  const int32_t* __restrict__ idx,
                                  const int32_t* __restrict__ rl_of,
                                  const float* __restrict__ val, int64_t E,
                                  uint2* __restrict__ cv, bool with_cr) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < E;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int32_t e = perm[j];
    // one 8-B edge word {column | row-in-tile << kFwdColBits, val}: a single load per edge
    if (with_cr) cv[j].x = (uint32_t)idx[e] | ((uint32_t)rl_of[e] << kFwdColBits);
    cv[j].y = __float_as_uint(val ? val[e] : 1.0f);
  }
}

// Fixed-point forward bounds per task (spgemm.hip, fwd_fix_scale), from the CSR values in a
// fixed reduction order (so every plan of the same graph gets the same bounds and the
// integer sums make the forward bitwise reproducible). fwd_row_sums_kernel: one wavefront
// per row, rs[r] = {sum |val|, min nonzero |val|, 1 if a value is not finite}.
__global__ __launch_bounds__(256) void fwd_row_sums_kernel(const int32_t* __restrict__ ptr,
                                                           const float* __restrict__ val, int N,
                                                           float4* __restrict__ rs) {
  const int lane = threadIdx.x & (kWave - 1);
  const int r = blockIdx.x * (256 / kWave) + threadIdx.x / kWave;
  if (r >= N) return;
  float sum = 0.f, mn = 3.0e38f, bad = 0.f;
  for (int e = ptr[r] + lane; e < ptr[r + 1]; e += kWave) {
    const float a = fabsf(val ? val[e] : 1.0f);
    if (!(a <= 3.0e38f)) bad = 1.f;
    sum += a;
    if (a > 0.f) mn = fminf(mn, a);
  }
  for (int o = kWave / 2; o > 0; o >>= 1) {
    sum += __shfl_xor(sum, o);
    mn = fminf(mn, __shfl_xor(mn, o));
    bad = fmaxf(bad, __shfl_xor(bad, o));
  }
  if (lane == 0) rs[r] = make_float4(sum, mn, bad, 0.f);
}

// Per task: sexp with every row's sum |val| <= 2^sexp (2^-10 of headroom for the f32 sums;
// a split task takes its whole row's sum, an upper bound), gexp = sexp - vexp with every
// nonzero |val| >= 2^vexp. Non-finite values force the f64 path (gexp = 1000).
__global__ void fwd_fix_stats_kernel(const FwdTask* __restrict__ tasks, int ntasks,
                                     const float4* __restrict__ rs, int2* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntasks) return;
  const FwdTask task = tasks[t];
  const int nr = task.nrows < 0 ? 1 : task.nrows;
  float smax = 0.f, vmin = 3.0e38f;
  bool bad = false;
  for (int i = 0; i < nr; ++i) {
    const float4 q = rs[task.row0 + i];
    smax = fmaxf(smax, q.x);
    vmin = fminf(vmin, q.y);
    bad = bad || q.z != 0.f;
  }
  int2 r = make_int2(0, 0);
  if (bad || !(smax < 3.0e38f)) {
    r.y = 1000;
  } else if (smax > 0.f && vmin < 3.0e38f) {
    int es = 0, ev = 0;
    (void)frexpf(smax * (1.0f + 0x1p-10f), &es);  // smax * (1 + 2^-10) < 2^es
    (void)frexpf(vmin, &ev);                       // vmin >= 2^(ev - 1)
    r.x = es;
    r.y = es - (ev - 1);
  }
  out[t] = r;
}

// Row sums, then per-task bounds (plan create and maxk_plan_refresh_values).
static hipError_t fwd_fix_stats(const maxk_plan* p, const int32_t* ptr, const float* val,
                                hipStream_t s) {
  float4* rs = nullptr;
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&rs), sizeof(float4) * std::max(p->num_nodes, 1), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fwd_row_sums_kernel, dim3((p->num_nodes + 3) / 4), dim3(256), 0, s, ptr,
                     val, p->num_nodes, rs);
  hipLaunchKernelGGL(fwd_fix_stats_kernel, dim3((p->n_fwd_tasks + 255) / 256), dim3(256), 0, s,
                     p->fwd_tasks, p->n_fwd_tasks, rs, p->fwd_fix);
  e = hipGetLastError();
  const hipError_t f = hipFreeAsync(rs, s);
  return e != hipSuccess ? e : f;
}

// Sort key of each edge for the backward: its source-column block c / C (a stable radix
// sort then yields the block-major, destination-row-sorted edge list). Also validates the
// column ids: any idx outside [0, NC) sets *bad (the compute kernels index the CBSR tables
// with idx and must never read outside them).
__global__ void bwd_key_kernel(const int32_t* __restrict__ idx, int64_t E, int C, int NC,
                               uint32_t* __restrict__ keys, int32_t* __restrict__ ids,
                               int* __restrict__ bad, const int32_t* __restrict__ colpos) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int c = idx[e];
    if (c < 0 || c >= NC) atomicOr(bad, 1);
    const int cc = c < 0 ? 0 : (c >= NC ? NC - 1 : c);
    keys[e] = (uint32_t)((colpos ? colpos[cc] : cc) / C);  // block of the column's position
    ids[e] = (int32_t)e;
  }
}

// The same with the destination row's position in the block stream as the low key bits:
// key = block << rbits | (ra * row + rb) mod N (bwd_row_order 2, a bijection of the rows:
// gcd(ra, N) = 1), so a stable sort gives block-major streams whose (block, row) runs come in
// scattered row order (the edges of a run stay together, in CSR order).
__global__ void bwd_key64_kernel(const int32_t* __restrict__ idx, const int32_t* __restrict__ row_of,
                                 int64_t E, int C, int NC, uint64_t* __restrict__ keys,
                                 int32_t* __restrict__ ids, int* __restrict__ bad,
                                 const int32_t* __restrict__ colpos, int64_t ra, int64_t rb, int N,
                                 int rbits) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int c = idx[e];
    if (c < 0 || c >= NC) atomicOr(bad, 1);
    const int cc = c < 0 ? 0 : (c >= NC ? NC - 1 : c);
    const uint64_t blk = (uint64_t)((colpos ? colpos[cc] : cc) / C);
    const uint64_t rp = (uint64_t)((ra * (int64_t)row_of[e] + rb) % N);
    keys[e] = (blk << rbits) | rp;
    ids[e] = (int32_t)e;
  }
}

// Dense runs of the ascending-row block streams: window w = sorted edges [w Wn, (w+1) Wn) is
// dense when it holds fewer than Wn / 16 (block, row) runs, i.e. > 16 edges per run on average
// (consecutive rows each with many edges into one block).
__global__ void dense_window_kernel(const uint32_t* __restrict__ bkey, const int32_t* __restrict__ perm,
                                    const int32_t* __restrict__ row_of, int64_t E, int Wn,
                                    int* __restrict__ ndense) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e0 = w * Wn;
  if (e0 + Wn > E) return;
  int runs = 1;
  int32_t pr = row_of[perm[e0]];
  uint32_t pk = bkey[e0];
  for (int64_t e = e0 + 1; e < e0 + Wn; ++e) {
    const int32_t r = row_of[perm[e]];
    const uint32_t kk = bkey[e];
    runs += (r != pr || kk != pk) ? 1 : 0;
    pr = r;
    pk = kk;
  }
  if (runs * 16 < Wn) atomicAdd(ndense, 1);
}

__global__ void key_block_kernel(const uint64_t* __restrict__ k64, int64_t E, int rbits,
                                 uint32_t* __restrict__ blk) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x)
    blk[e] = (uint32_t)(k64[e] >> rbits);
}

// Column of each reordered edge's block position and its destination row (plan-time
// temporaries for the records and the chunk bounds).
__global__ void gather_bwd_kernel(const int32_t* __restrict__ perm,
                                  const int32_t* __restrict__ row_of,
                                  const int32_t* __restrict__ idx, int64_t E,
                                  int32_t* __restrict__ brow, int32_t* __restrict__ bcol,
                                  const int32_t* __restrict__ colpos) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < E;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int32_t e = perm[j];
    brow[j] = row_of[e];
    bcol[j] = colpos ? colpos[idx[e]] : idx[e];  // the column's block position
  }
}

// Backward records {row * D * 4 (byte offset of the grad_out row; big: the row index),
// column within the block, val}; with row == nullptr only the val field is refreshed from
// the CSR order through perm.
__global__ void build_bwd_rec_kernel(const int32_t* __restrict__ perm,
                                     const int32_t* __restrict__ row,
                                     const int32_t* __restrict__ col,
                                     const float* __restrict__ val, int64_t E, int C, int D,
                                     int big, uint32_t* __restrict__ rec) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid_for caps the grid
    rec[3 * e + 2] = __float_as_uint(val ? val[perm[e]] : 1.0f);
    if (!row) continue;
    rec[3 * e] = big ? (uint32_t)row[e] : (uint32_t)row[e] * (uint32_t)D * 4u;
    rec[3 * e + 1] = (uint32_t)(col[e] % C);
  }
}

// offs[b] = first position j with skeys[j] >= b, b in [0, nkeys].
__global__ void key_offsets_kernel(const uint32_t* __restrict__ skeys, int64_t E, int nkeys,
                                   int32_t* __restrict__ offs) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > nkeys) return;
  int64_t lo = 0, hi = E;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (skeys[mid] < (uint32_t)b) lo = mid + 1; else hi = mid;
  }
  offs[b] = (int32_t)lo;
}

// Two-pass backward edge records in CSR order: {column | (row % R) << kFwdColBits, val}
// (idx == nullptr: only the val field is refreshed).
__global__ void build_erec_kernel(const int32_t* __restrict__ idx,
                                  const int32_t* __restrict__ row_of, int R,
                                  const float* __restrict__ val, int64_t E,
                                  uint32_t* __restrict__ erec) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    if (idx) erec[2 * e] = (uint32_t)idx[e] | ((uint32_t)(row_of[e] % R) << kFwdColBits);
    erec[2 * e + 1] = __float_as_uint(val ? val[e] : 1.0f);
  }
}

__global__ void gather_i32_kernel(const int32_t* __restrict__ src, const int32_t* __restrict__ at,
                                  int n, int32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = src[at[i]];
}

// Two-pass row chunks: out[p * NC + c] = first column-sorted position of column c whose row
// is >= rows[p] (positions [colptr[c], colptr[c+1]) hold CSR edges perm[.] in row order).
__global__ void tp_colptr_kernel(const int32_t* __restrict__ colptr, const int32_t* __restrict__ perm,
                                 const int32_t* __restrict__ row_of, int NC,
                                 const int32_t* __restrict__ rows, int P, int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)(P + 1) * NC) return;
  const int p = (int)(i / NC), c = (int)(i - (int64_t)p * NC);
  int a = colptr[c], b = colptr[c + 1];
  if (p == P) { out[i] = b; return; }
  const int32_t r = rows[p];
  while (a < b) {
    const int m = (a + b) >> 1;
    if (row_of[perm[m]] < r) a = m + 1; else b = m;
  }
  out[i] = a;
}

// ---------------------------------------------------------------------------------------
// Column orders of the column blocks (maxk_plan_options.col_order).
//
// Scattered (2): p -> column (a p + b) mod NC with gcd(a, NC) = 1, a ~ 0.618 NC: every
// contiguous range of positions (a block) takes columns spread evenly over the ID range, so a
// community of consecutive IDs is shared by all blocks instead of filling a few of its own.
// The caller's order (4) is range- and permutation-checked on the host before any device
// scatter uses it.
__global__ void affine_order_kernel(int NC, int64_t a, int64_t b, int32_t* __restrict__ order) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= NC) return;
  order[p] = (int32_t)((a * (int64_t)p + b) % NC);
}

__global__ void invert_order_kernel(const int32_t* __restrict__ order, int NC,
                                    int32_t* __restrict__ pos) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < NC) pos[order[p]] = p;  // order is a checked permutation of [0, NC)
}

__global__ void iota_kernel(int n, int32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = i;
}

static void dfree(void* q) { if (q) (void)hipFree(q); }

// The large streamed plan arrays (forward edge words, backward records). MAXK_PLAN_MALLOC=
// contiguous asks the runtime for physically contiguous memory (hipDeviceMallocContiguous),
// falling back to hipMalloc when it cannot (round 6 experiment on allocation-dependent kernel
// times).
static hipError_t plan_malloc(void** q, size_t bytes) {
  static const int mode = [] {
    const char* e = std::getenv("MAXK_PLAN_MALLOC");
    return (e && std::string(e) == "contiguous") ? 1 : 0;
  }();
  if (mode == 1 && hipExtMallocWithFlags(q, bytes, hipDeviceMallocContiguous) == hipSuccess)
    return hipSuccess;
  (void)hipGetLastError();
  return hipMalloc(q, bytes);
}
template <class T>
static hipError_t plan_malloc(T** q, size_t bytes) {
  return plan_malloc(reinterpret_cast<void**>(q), bytes);
}

static int grid_for(int64_t n, int threads) {
  int64_t g = (n + threads - 1) / threads;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 65536));
}

static void free_plan(maxk_plan* p) {
  if (!p) return;
  dfree(p->fwd_tasks);
  dfree(p->fwd_rec);
  dfree(p->fwd_perm);
  dfree(p->fwd_cv);
  dfree(p->fwd_fix);
  dfree(p->fwd_rowptr);
  dfree(p->fwd_phase_off);
  dfree(p->zero_rows);
  dfree(p->bwd_tasks);
  dfree(p->bwd_perm);
  dfree(p->bwd_rec);
  dfree(p->bwd_sel);
  dfree(p->bwd_colptr);
  dfree(p->bwd_erec);
  dfree(p->bwd_tbuf);
  dfree(p->bwd_combine);
  dfree(p->bwd_colptr2);
  dfree(p->bwd_corder);
  delete p;
}

// Column order of the column blocks (col_order 2 scattered, 4 the caller's): *order = device
// int32 [NC], order[p] = column at position p. The caller's order must be a permutation of
// [0, NC): *bad is set otherwise, and nothing is scattered with it.
static hipError_t build_col_order(int mode, int NC, const int32_t* user, hipStream_t s,
                                  int32_t** order, bool* bad) {
  *bad = false;
  hipError_t e = hipMalloc(order, sizeof(int32_t) * (size_t)NC);
  if (e != hipSuccess) return e;
  if (mode == 4) {
    std::vector<int32_t> ho(NC);
    e = hipMemcpyAsync(ho.data(), user, sizeof(int32_t) * NC, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    std::vector<uint8_t> seen(NC, 0);
    for (int i = 0; i < NC && !*bad; ++i) {
      const int32_t c = ho[i];
      *bad = c < 0 || c >= NC || seen[c];
      if (!*bad) seen[c] = 1;
    }
    if (*bad) return hipSuccess;
    return hipMemcpyAsync(*order, ho.data(), sizeof(int32_t) * NC, hipMemcpyHostToDevice, s);
  }
  // a ~ 0.618 NC, coprime with NC (b: a fixed offset)
  int64_t a = std::max<int64_t>(1, (int64_t)(0.6180339887 * NC));
  auto gcd = [](int64_t x, int64_t y) { while (y) { const int64_t t = x % y; x = y; y = t; } return x; };
  while (gcd(a, NC) != 1) ++a;
  hipLaunchKernelGGL(affine_order_kernel, dim3((NC + 255) / 256), dim3(256), 0, s, NC, a % NC,
                     (int64_t)(NC / 3), *order);
  return hipGetLastError();
}

// Forward task list from a host copy of ptr.
static void build_fwd_tasks(const std::vector<int32_t>& hp, int N, int R, int64_t cap_opt,
                            std::vector<FwdTask>& tasks, std::vector<int32_t>& zero_rows) {
  const int64_t E = hp[N];
  const int ntiles = (N + R - 1) / R;
  const int64_t avg = ntiles ? (E + ntiles - 1) / ntiles : 0;
  // 1.5 x the average tile (round 3: 2 x, before that 4 x): heavy tiles split into a few more
  // tasks balance the tail and keep the tiles running together closer to the rotation clock
  // (Reddit k = 16 / 32 / 64: 1.096 / 1.689 / 3.131 -> 1.083 / 1.680 / 3.079 ms, k = 8 equal;
  // 1.25 x is slower, profiles/r04/fwd_task_cap_ab.jsonl)
  const int64_t cap = cap_opt > 0 ? cap_opt : std::max<int64_t>(4096, avg + avg / 2);
  auto push_rows = [&](int r0, int r1) {
    if (r1 > r0) tasks.push_back(FwdTask{r0, r1 - r0, hp[r0], hp[r1]});
  };
  for (int r0 = 0; r0 < N; r0 += R) {
    const int r1 = std::min(N, r0 + R);
    if ((int64_t)hp[r1] - hp[r0] <= cap) {
      push_rows(r0, r1);
      continue;
    }
    int g0 = r0;
    for (int r = r0; r < r1; ++r) {
      const int64_t deg = (int64_t)hp[r + 1] - hp[r];
      if (deg > cap) {
        push_rows(g0, r);
        for (int64_t s = hp[r]; s < hp[r + 1]; s += cap)
          tasks.push_back(FwdTask{r, -1, (int32_t)s, (int32_t)std::min<int64_t>(s + cap, hp[r + 1])});
        zero_rows.push_back(r);
        g0 = r + 1;
      } else if ((int64_t)hp[r + 1] - hp[g0] > cap) {
        push_rows(g0, r);
        g0 = r;
      }
    }
    push_rows(g0, r1);
  }
  std::stable_sort(tasks.begin(), tasks.end(), [](const FwdTask& a, const FwdTask& b) {
    return (a.e1 - a.e0) > (b.e1 - b.e0);
  });
}

}  // namespace maxk

using namespace maxk;

extern "C" int maxk_plan_create(const int32_t* ptr, const int32_t* idx, const float* val,
                                int32_t N, int64_t E, int32_t D, int32_t k, void* stream,
                                maxk_plan** out_plan) {
  return maxk_plan_create_rect(ptr, idx, val, N, N, E, D, k, stream, out_plan);
}

extern "C" int maxk_plan_create_rect(const int32_t* ptr, const int32_t* idx, const float* val,
                                     int32_t N, int32_t NC, int64_t E, int32_t D, int32_t k,
                                     void* stream, maxk_plan** out_plan) {
  return maxk_plan_create_ex(ptr, idx, val, N, NC, E, D, k, nullptr, stream, out_plan);
}

static int plan_create_impl(const int32_t* ptr, const int32_t* idx, const float* val, int32_t N,
                            int32_t NC, int64_t E, int32_t D, int32_t k,
                            const maxk_plan_options& o, const int32_t* user_order, void* stream,
                            maxk_plan** out_plan);

extern "C" int maxk_plan_create_ex(const int32_t* ptr, const int32_t* idx, const float* val,
                                   int32_t N, int32_t NC, int64_t E, int32_t D, int32_t k,
                                   const maxk_plan_options* opts, void* stream,
                                   maxk_plan** out_plan) {
  // the round-1 layout create_ex shipped with (through fwd_rot_rate, 120 bytes): reading the
  // later 144-byte ABI-1 layout here would read 24 bytes past a round-1 caller's struct.
  // Fields from offset 120 on are set through maxk_plan_create_sized
  return maxk_plan_create_sized(ptr, idx, val, N, NC, E, D, k, opts,
                                opts ? MAXK_PLAN_OPTIONS_V1_BYTES : 0, nullptr, stream, out_plan);
}

extern "C" int maxk_plan_create_sized(const int32_t* ptr, const int32_t* idx, const float* val,
                                      int32_t N, int32_t NC, int64_t E, int32_t D, int32_t k,
                                      const maxk_plan_options* opts, int64_t opts_bytes,
                                      const int32_t* col_order, void* stream,
                                      maxk_plan** out_plan) {
  MAXK_CHECK_ARG(out_plan != nullptr, "maxk_plan_create: out_plan is null");
  *out_plan = nullptr;
  MAXK_CHECK_ARG(opts_bytes >= 0 && opts_bytes % 4 == 0 && (opts || opts_bytes == 0),
                 "maxk_plan_create_sized: opts_bytes must be a multiple of 4 (0 with no opts)");
  maxk_plan_options o{};
  const int64_t mine = (int64_t)sizeof(maxk_plan_options);
  if (opts) {
    std::memcpy(&o, opts, (size_t)std::min(opts_bytes, mine));
    // a newer caller's fields this library does not know must be 0 (their default)
    const uint8_t* extra = reinterpret_cast<const uint8_t*>(opts);
    for (int64_t b = mine; b < opts_bytes; ++b)
      MAXK_CHECK_ARG(extra[b] == 0, "maxk_plan_create_sized: unknown option fields are set "
                                    "(the caller's maxk_plan_options is newer than this library)");
  }
  return plan_create_impl(ptr, idx, val, N, NC, E, D, k, o, col_order, stream, out_plan);
}

// Options whose other values selected kernel organisations that ABI 3 removed (slower on every
// measured configuration and never chosen automatically): only 0 and the
// behaviour that remains are accepted.
#define MAXK_CHECK_REMOVED(cond, msg)                                                      \
  do {                                                                                     \
    if (!(cond)) {                                                                         \
      ::maxk::set_error(std::string("maxk_plan_create: ") + msg + " (removed in ABI 3)");  \
      return MAXK_ERR_UNSUPPORTED;                                                         \
    }                                                                                      \
  } while (0)

static int check_options(const maxk_plan_options& o) {
  MAXK_CHECK_ARG(o.fwd_tile_rows >= 0 && o.fwd_tile_rows <= kFwdMaxTileRows,
                 "maxk_plan_create: fwd_tile_rows must be in [0, 64]");
  MAXK_CHECK_ARG(o.fwd_accumulator >= 0 && o.fwd_accumulator <= MAXK_ACC_F32_CAS &&
                     o.bwd_accumulator >= 0 && o.bwd_accumulator <= MAXK_ACC_F32_CAS,
                 "maxk_plan_create: unknown accumulator kind");
  MAXK_CHECK_REMOVED(o.fwd_accumulator != MAXK_ACC_F32_CAS, "fwd_accumulator = f32 CAS");
  MAXK_CHECK_REMOVED(o.bwd_accumulator != MAXK_ACC_F64, "bwd_accumulator = f64");
  MAXK_CHECK_ARG(o.bwd_lds_bytes >= 0 && o.bwd_lds_bytes <= kBwdLdsBudget && o.bwd_tasks_per_cu >= 0 &&
                     o.fwd_task_cap >= 0 && o.bwd_min_task_edges >= 0 && o.bwd_piece_edges >= 0 &&
                     o.bwd_tp_chunks >= 0 && o.fwd_rot_windows >= 0 && o.fwd_rot_rate >= 0,
                 "maxk_plan_create: bad option value (negative, or bwd_lds_bytes > 160 KiB)");
  MAXK_CHECK_ARG(o.bwd_features_per_lane >= 0 && o.bwd_features_per_lane <= 4 &&
                     o.bwd_features_per_lane != 3,
                 "maxk_plan_create: bwd_features_per_lane must be 0, 2 or 4");
  MAXK_CHECK_REMOVED(o.bwd_features_per_lane != 1, "bwd_features_per_lane = 1");
  MAXK_CHECK_REMOVED(o.fwd_phases <= 1, "fwd_phases > 1");
  MAXK_CHECK_REMOVED(o.fwd_persistent == 0, "fwd_persistent");
  MAXK_CHECK_REMOVED(o.fwd_unroll == 0 || o.fwd_unroll == 8 || o.fwd_unroll == 4,
                     "fwd_unroll other than 4 or 8");
  MAXK_CHECK_ARG(o.fwd_unroll != 4 || o.fwd_waves != 4,
                 "maxk_plan_create: fwd_unroll 4 needs 8 forward waves");
  MAXK_CHECK_ARG(o.bwd_unroll == 0 || o.bwd_unroll == 8 || o.bwd_unroll == 12 ||
                     o.bwd_unroll == 16,
                 "maxk_plan_create: bwd_unroll must be 0, 8, 12 or 16");
  // the backward shapes that exist (spgemm.hip BWD_SHAPES): 16 waves x 8 sub-steps, 12 x 8 or
  // 12, 8 x 8, 12 or 16 (an unroll with no kernel is refused, not replaced)
  MAXK_CHECK_ARG(o.bwd_waves != 16 || o.bwd_unroll == 0 || o.bwd_unroll == 8,
                 "maxk_plan_create: bwd_waves 16 runs bwd_unroll 8 only");
  MAXK_CHECK_ARG(o.bwd_waves != 12 || o.bwd_unroll != 16,
                 "maxk_plan_create: bwd_waves 12 runs bwd_unroll 8 or 12");
  MAXK_CHECK_REMOVED(o.bwd_order != 1, "bwd_order = 1 (heavy-first tasks)");
  MAXK_CHECK_ARG(o.bwd_order >= 0 && o.bwd_order <= 3, "maxk_plan_create: bwd_order must be 0, 2 or 3");
  MAXK_CHECK_ARG(o.bwd_slot_groups >= 0 && o.bwd_slot_groups <= 64 &&
                     (o.bwd_slot_groups & (o.bwd_slot_groups - 1)) == 0,
                 "maxk_plan_create: bwd_slot_groups must be 0 or a power of two <= 64");
  MAXK_CHECK_REMOVED(o.bwd_acc_pad == 0 || o.bwd_acc_pad == 2, "bwd_acc_pad = 1");
  MAXK_CHECK_REMOVED(o.bwd_sel_lds == 0 || o.bwd_sel_lds == 1, "bwd_sel_lds = 2");
  MAXK_CHECK_ARG(o.fwd_rotate >= 0 && o.fwd_rotate <= 2,
                 "maxk_plan_create: fwd_rotate must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.bwd_algo >= 0 && o.bwd_algo <= 3,
                 "maxk_plan_create: bwd_algo must be 0 (auto), 1 (column blocks) or 3 (two-pass)");
  MAXK_CHECK_REMOVED(o.bwd_algo != 2, "bwd_algo = 2 (column-major)");
  MAXK_CHECK_ARG(o.fwd_waves == 0 || o.fwd_waves == 4 || o.fwd_waves == 8,
                 "maxk_plan_create: fwd_waves must be 0, 4 or 8");
  MAXK_CHECK_ARG(o.bwd_waves == 0 || o.bwd_waves == 8 || o.bwd_waves == 12 || o.bwd_waves == 16,
                 "maxk_plan_create: bwd_waves must be 0, 8, 12 or 16");
  MAXK_CHECK_ARG(o.fwd_handout >= 0 && o.fwd_handout <= 2 && o.bwd_handout >= 0 && o.bwd_handout <= 2,
                 "maxk_plan_create: fwd_handout / bwd_handout must be 0, 1 or 2");
  MAXK_CHECK_REMOVED((o.fwd_prefetch == 0 || o.fwd_prefetch == 2) &&
                         (o.bwd_prefetch == 0 || o.bwd_prefetch == 2),
                     "fwd_prefetch / bwd_prefetch = 1");
  MAXK_CHECK_REMOVED(o.fwd_record_bytes == 0, "fwd_record_bytes");
  MAXK_CHECK_REMOVED(o.fwd_branchless == 0 || o.fwd_branchless == 1, "fwd_branchless = 2");
  MAXK_CHECK_ARG(o.fwd_chunk3 >= 0 && o.fwd_chunk3 <= 3,
                 "maxk_plan_create: fwd_chunk3 must be 0, 1, 2 or 3");
  MAXK_CHECK_REMOVED(o.bwd_cas64 == 0 || o.bwd_cas64 == 1, "bwd_cas64 = 2");
  MAXK_CHECK_REMOVED(o.quad_loads == 0, "quad_loads");
  MAXK_CHECK_ARG(o.fwd_two_tables >= 0 && o.fwd_two_tables <= 2,
                 "maxk_plan_create: fwd_two_tables must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.external_workspace == 0 || o.external_workspace == 1,
                 "maxk_plan_create: external_workspace must be 0 or 1");
  MAXK_CHECK_ARG(o.bwd_flush >= 0 && o.bwd_flush <= 2,
                 "maxk_plan_create: bwd_flush must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.bwd_chunk_bounds >= 0 && o.bwd_chunk_bounds <= 3,
                 "maxk_plan_create: bwd_chunk_bounds must be 0 or 2");
  MAXK_CHECK_REMOVED(o.bwd_chunk_bounds == 0 || o.bwd_chunk_bounds == 2,
                     "bwd_chunk_bounds 1 (shared rows) / 3 (equal cost)");
  MAXK_CHECK_ARG(o.fwd_fixed >= 0 && o.fwd_fixed <= 2,
                 "maxk_plan_create: fwd_fixed must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.bwd_tp_store >= 0 && o.bwd_tp_store <= 2,
                 "maxk_plan_create: bwd_tp_store must be 0 or 1");
  MAXK_CHECK_REMOVED(o.bwd_tp_store != 2, "bwd_tp_store = 2 (column-order products)");
  MAXK_CHECK_REMOVED(o.bwd_row_cost == 0, "bwd_row_cost");
  MAXK_CHECK_ARG(o.col_order >= 0 && o.col_order <= 4,
                 "maxk_plan_create: col_order must be 0, 1, 2 or 4");
  MAXK_CHECK_REMOVED(o.col_order != 3, "col_order = 3 (clustered)");
  MAXK_CHECK_ARG(o.bwd_row_order >= 0 && o.bwd_row_order <= 2,
                 "maxk_plan_create: bwd_row_order must be 0, 1 or 2");
  return MAXK_OK;
}

static int device_cus() {
  int dev = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
      prop.multiProcessorCount > 0)
    return prop.multiProcessorCount;
  return 256;
}

static int plan_create_impl(const int32_t* ptr, const int32_t* idx, const float* val, int32_t N,
                            int32_t NC, int64_t E, int32_t D, int32_t k,
                            const maxk_plan_options& o, const int32_t* user_order, void* stream,
                            maxk_plan** out_plan) {
  *out_plan = nullptr;
  if (const int rc = check_options(o)) return rc;
  MAXK_CHECK_ARG(o.col_order != 4 || user_order != nullptr || NC == 0,
                 "maxk_plan_create: col_order 4 needs the col_order argument");
  MAXK_CHECK_ARG(NC >= 0 && (E == 0 || NC > 0), "maxk_plan_create: num_cols out of range");
  if ((uint32_t)NC > kFwdColMask + 1u) {
    set_error("maxk_plan_create: more than 2^26 source columns is not supported");
    return MAXK_ERR_UNSUPPORTED;
  }
  MAXK_CHECK_ARG(N >= 0 && E >= 0 && E < (int64_t)INT32_MAX,
                 "maxk_plan_create: sizes out of range (E must fit int32)");
  MAXK_CHECK_ARG(D >= 1 && D <= kMaxDim, "maxk_plan_create: dim_origin must be in [1, 256]");
  MAXK_CHECK_ARG(k >= 1 && k <= D, "k must be between 1 and input dimension");
  MAXK_CHECK_ARG(ptr != nullptr && (E == 0 || idx != nullptr), "maxk_plan_create: null pointer");
  hipStream_t s = (hipStream_t)stream;

  maxk_plan* p = new maxk_plan();
  p->external_ws = o.external_workspace;
  p->num_nodes = N;
  p->num_cols = NC;
  p->num_edges = E;
  p->dim_origin = D;
  p->dim_k = k;
  p->src_ptr = ptr;
  p->src_idx = idx;
  p->cus = device_cus();
  const int cus = p->cus;
  // Forward tile rows: 32, or, where a CU's LDS holds only two 32-row accumulators anyway
  // (D >= 213), as many rows as still fit two work-groups (39 at D = 256): more rows share
  // each gathered record while the work-groups per CU stay at two. Reddit D = 256, forward
  // ms 32 / 38 / 39 rows (tools/fwd_opts_sweep.py, profiles/r06/fwd_tile_rows.jsonl): k = 16
  // 1.022 / 0.996 / 0.989, k = 64 2.844 / 2.824 / 2.818, k = 8 0.891 / 0.876 (38), k = 32
  // 1.572 / 1.549 (38); ogbn-proteins k = 16 0.666 / 0.659 (38); yelp 0.468 / 0.461 / 0.464;
  // flickr 0.0666 / 0.0683 / 0.0680. 40 rows leave one work-group per CU: +43 %. Only with
  // enough tiles for >= 5 rounds of two per CU: fewer, larger tiles lengthen the last round
  // (flickr, 89 K rows, +2 %; an 8-GPU Reddit shard, 29 K rows: forward 0.146-0.151 ->
  // 0.155-0.163 ms per rank, profiles/r06/shard_w8_all_ranks_39rows.jsonl).
  const int fwd_row_bytes = (D + kFwdRowPad) * 8;
  const int fwd_two_wg_rows = std::min(kFwdMaxTileRows, (kBwdLdsBudget / 2 - 256) / fwd_row_bytes);
  const bool fwd_lds_two_wg = 3 * kFwdTileRows * fwd_row_bytes > kBwdLdsBudget &&
                              (int64_t)N >= (int64_t)fwd_two_wg_rows * 10 * cus;
  p->fwd_tile_rows = o.fwd_tile_rows ? o.fwd_tile_rows
                     : fwd_lds_two_wg ? fwd_two_wg_rows : kFwdTileRows;
  // 8 waves per forward work-group, their windows from an LDS counter (below): more gathers
  // in flight per CU (Reddit k = 8 / 32 / 64 -4 / -7 / -9 %, k = 20..60 -4..-24 %), except
  // where the 4-wave sweep's column span is what keeps the records in L2: k = 16 (8 waves
  // +36 %, L2 hit 62 -> 37 %) and k = 48 (+28 %; 4 sub-steps per wave instead, -4 %).
  // profiles/r05/fwd_waves_sweep.jsonl
  const int waves_rec = o.fwd_waves ? o.fwd_waves : (k == 16 && o.fwd_unroll != 4 ? 4 : 8);
  // pair chunks {2 values, 2 selector bytes} per lane (round 6): one gather gives a lane its
  // values and selectors, k / 2 lanes per edge (quad-shared edge words when k / 2 % 4 == 0).
  // Half the edges per instruction of the records kernel, so 8 waves keep as many in flight
  // (Reddit k = 16: 4 waves 1.419 ms, 8 waves 1.029 against 1.078 for the records kernel).
  // Default at k = 16, pack fused into the statistics pass (profiles/r06/fwd_pair_chunks.jsonl,
  // forward with its pass: Reddit 1.077 -> 1.008 ms, ogbn-proteins 0.712 -> 0.666, ogbn-products
  // 3.02 -> 2.92, yelp 0.521 -> 0.468, flickr 0.080 -> 0.067); not at k = 8 (4 lanes: 0.896
  // vs 0.891 lane chunks), 12 / 20 / 24 (6 / 10 / 12 lanes, no quads: +13..+92 %) or 32 (+19 %)
  p->fwd_chunk2 = (o.fwd_chunk3 == 3 || (o.fwd_chunk3 == 0 && k == 16)) && k % 2 == 0 &&
                  k / 2 <= kWave;
  p->fwd_waves = p->fwd_chunk2 && !o.fwd_waves ? 8 : waves_rec;
  p->fwd_unroll = o.fwd_unroll ? o.fwd_unroll : (p->fwd_waves == 8 && k == 48 ? 4 : 8);
  // lane-chunk records by default where the 4-values-per-lane layout fits k badly (Reddit:
  // k = 8 0.95 vs 1.02 ms, k = 24 1.93 vs 2.09 ms; k = 16 / 32 / 64 are slower with chunks),
  // and for every k % 4 != 0 up to 192 (beyond: one lane per feature, f64)
  p->fwd_chunk3 = (o.fwd_chunk3 == 1 ||
                   ((o.fwd_chunk3 == 0 || (o.fwd_chunk3 == 3 && !p->fwd_chunk2)) && k % 16 != 0)) &&
                  (k + 2) / 3 <= kWave;
  // Fixed-point forward (LdsFix; the packed 4-values-per-lane and lane-chunk kernels).
  // Measured (tools/fwd_fixed_sweep.py, fixed vs f64 ms): Reddit k = 16 1.22 / 1.34,
  // k = 24 1.57 / 1.95, k = 32 1.80 / 2.46, k = 64 3.45 / 4.81; ogbn-proteins k = 16 0.80 / 0.93,
  // k = 64 2.22 / 3.37. Not by default at k < 16 (Reddit k = 8 0.93 / 0.91, the stats pass
  // included) or on tables past the packed-record thresholds, whose gathers are HBM-bound
  // (ogbn-products k = 16 3.14 / 3.02, k = 32 4.86 / 4.78).
  const bool big_table = (double)std::max(NC, 1) * 5.0 * k >
                         (k >= 32 ? kFwdPackedTableBytes : kFwdPackedTableBytes16);
  p->fwd_fixed = (o.fwd_fixed == 1 || (o.fwd_fixed == 0 && k >= 16 && !big_table)) &&
                 (k % 4 == 0 || p->fwd_chunk3 || p->fwd_chunk2);
  // forward quad-shared edge-word loads with the fixed-point kernel (k = 16 1.19 -> 1.16 ms,
  // k = 32 1.81 -> 1.78); neutral-to-slower on the f64 kernel
  p->fwd_quad = p->fwd_fixed;

  // ---- backward kernel shape (column blocks)
  const int lds_budget = o.bwd_lds_bytes ? o.bwd_lds_bytes : kBwdLdsBudget;
  // k = 8: two slots per lane, so a gather instruction covers 16 edges (4 lanes per edge)
  // instead of 32, when a column block sees few edges per grad_out row (32 edges then span
  // ~4 rows: Reddit, 7.7 edges per (block, row), 1.151 -> 1.125 ms with unroll 12); with
  // more (ogbn-proteins, 15) the 32 edges share ~2 rows and 4 slots per lane stay faster
  // (0.831 vs 0.877 ms). Edges per (block, row) estimated from the LDS budget. k = 2 mod 4:
  // two slots per lane need no padding slot.
  bool two_slots = false;
  if (k == 8 && N > 0 && NC > 0) {
    const double c0 = std::min<double>(NC, (lds_budget - 16) / (5.0 * k));
    two_slots = (double)E / N * c0 / NC < 10.0;
  }
  int F = o.bwd_features_per_lane ? o.bwd_features_per_lane
                                  : (two_slots || (k % 4 == 2 && k <= 2 * kWave) ? 2 : 4);
  if (F == 2 && (k + 1) / 2 > kWave) F = 4;  // L = k / 2 lanes must fit a wave
  p->bwd_feats = F;
  // Slot groups: the k selector slots are split into S groups of k/S consecutive (sorted,
  // hence clustered) slots, one work-group per (block, group). An edge then touches the few
  // grad_out lines its group's features fall in, and a block spans S times more columns.
  // Auto at k >= 32 with few edges per (block, row): two groups (Reddit, ~1.9 edges per
  // block row at k = 32: 2.88 -> 2.66 ms; k = 64, ~1.0: 4.88 -> 4.71; ogbn-proteins k = 64,
  // ~1.9: 3.32 -> 3.25); with more reuse one group stays faster (ogbn-proteins k = 32, ~3.1:
  // 1.82 vs 1.86).
  const int kF = (k + F - 1) / F * F;  // k padded to whole lanes
  // Round 5 (16 counter-fed waves, one round of tasks): two groups from k = 16 and below 4.5
  // edges per (block, row) (Reddit, 3.9 at k = 16: 1.468 -> 1.436 ms; k = 24, 2.6: 2.373 ->
  // 2.110; ogbn-proteins k = 16 / 24 at 8.2 / 5.5 stay at one group, +8 % with two;
  // profiles/r05/bwd_slot_groups_sweep.jsonl)
  int S = o.bwd_slot_groups ? o.bwd_slot_groups : 1;
  if (o.bwd_slot_groups == 0 && F == 4 && k >= 16 && k % 8 == 0 && N > 0 && NC > 0) {
    const double c1 = std::min<double>(NC, (lds_budget - 16) / (5.0 * k));
    if ((double)E / N * c1 / NC < 4.5) S = 2;
  }
  while (S > 1 && kF % (F * S) != 0) S >>= 1;
  // Two groups of 8 slots (k = 16): two slots per lane, so an edge keeps 4 lanes and an
  // instruction 16 edges (quad record loads) over the doubled runs; the CAS pairs then carry
  // half the slots each (Reddit k = 16 1.420 -> 1.375 ms, an 8-GPU shard 0.371 -> 0.365;
  // at k = 24, 6 lanes per edge, +17 %: profiles/r05/bwd_two_slots_groups.jsonl)
  if (o.bwd_features_per_lane == 0 && F == 4 && S == 2 && kF / S == 8) {
    F = 2;
    p->bwd_feats = F;
  }
  p->bwd_slot_groups = S;
  p->bwd_kp = kF;
  p->bwd_ks = kF / S;  // accumulators per column and group (64-bit CAS pairs: unpadded)
  p->bwd_unroll = o.bwd_unroll ? o.bwd_unroll : (F == 2 ? 12 : 8);
  p->bwd_waves = o.bwd_waves ? o.bwd_waves : (k >= 32 ? 12 : 8);
  p->bwd_big = (uint64_t)N * (uint64_t)D * 4u > 0xffffffffull;  // 32-bit buffer offsets
  // bytes of LDS per column: ks f32 accumulators + ks staged selector bytes
  int C = std::max(1, (lds_budget - 16) / (5 * p->bwd_ks));
  C = std::min(C, std::max(NC, 1));

  int32_t* row_of = nullptr;
  uint32_t* keys_in = nullptr;
  uint32_t* keys_out = nullptr;
  int32_t* ids_in = nullptr;
  int32_t* brow = nullptr;   // destination row / block position of each reordered edge
  int32_t* bcol = nullptr;
  void* temp = nullptr;
  int32_t* d_offs = nullptr;
  int* d_bad = nullptr;
  int32_t* order = nullptr;   // column order: position -> column (col_order 2, 4)
  int32_t* colpos = nullptr;  // column -> position
  auto fail = [&](int rc) {
    dfree(order); dfree(colpos); dfree(row_of); dfree(keys_in); dfree(keys_out); dfree(ids_in);
    dfree(brow); dfree(bcol); dfree(temp); dfree(d_offs); dfree(d_bad);
    free_plan(p);
    return rc;
  };
#define PLAN_TRY(expr)                                                            \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      set_error(std::string("maxk_plan_create: ") + #expr + ": " + hipGetErrorString(_e)); \
      return fail((int)_e);                                                       \
    }                                                                             \
  } while (0)
  auto need_row_of = [&]() -> hipError_t {
    if (row_of || E == 0) return hipSuccess;
    hipError_t e = hipMalloc(&row_of, sizeof(int32_t) * E);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(expand_rows_kernel, dim3((N + 3) / 4), dim3(256), 0, s, ptr, N, row_of);
    return hipGetLastError();
  };

  // ---------------- forward
  std::vector<int32_t> hp(N + 1);
  PLAN_TRY(hipMemcpyAsync(hp.data(), ptr, sizeof(int32_t) * (N + 1), hipMemcpyDeviceToHost, s));
  PLAN_TRY(hipStreamSynchronize(s));
  if (hp[0] != 0 || (int64_t)hp[N] != E) {
    set_error("maxk_plan_create: ptr[0] must be 0 and ptr[N] must equal num_edges");
    return fail(MAXK_ERR_INVALID_ARG);
  }
  for (int r = 0; r < N; ++r) {
    if (hp[r + 1] < hp[r]) {
      set_error("maxk_plan_create: ptr must be non-decreasing");
      return fail(MAXK_ERR_INVALID_ARG);
    }
  }
  // ---------------- column order (col_order 2 scattered, 4 the caller's): the column blocks
  // take position ranges of it. The forward keeps its column-sorted sweep (sweeping in a
  // clustered order measured much slower: k = 16 1.07 -> 1.36 ms, k = 32 1.61 -> 2.75)
  const int order_mode = o.col_order == 0 ? 1 : o.col_order;
  if (order_mode >= 2 && NC > 0) {
    bool bad_order = false;
    PLAN_TRY(build_col_order(order_mode, NC, user_order, s, &order, &bad_order));
    if (bad_order) {
      set_error("maxk_plan_create: col_order is not a permutation of [0, num_cols)");
      return fail(MAXK_ERR_INVALID_ARG);
    }
    PLAN_TRY(hipMalloc(&colpos, sizeof(int32_t) * NC));
    hipLaunchKernelGGL(invert_order_kernel, dim3((NC + 255) / 256), dim3(256), 0, s, order, NC, colpos);
    PLAN_TRY(hipGetLastError());
  }

  std::vector<FwdTask> ftasks;
  std::vector<int32_t> zrows;
  build_fwd_tasks(hp, N, p->fwd_tile_rows, o.fwd_task_cap, ftasks, zrows);
  p->n_fwd_tasks = (int32_t)ftasks.size();
  p->n_zero_rows = (int32_t)zrows.size();
  if (!ftasks.empty()) {
    // permuted edge order (see fwd_key_kernel): tasks keep their CSR edge sets
    const int nt = (int)ftasks.size();
    std::vector<int32_t> torder(nt);
    for (int i = 0; i < nt; ++i) torder[i] = i;
    // by first edge, and among equal first edges the empty tasks (an edgeless tile shares its
    // e0 with the next tile) before the one task that owns edges there: fwd_key_kernel takes
    // the LAST task whose first edge is <= e (an edgeless tile ordered last took the next
    // tile's edges, whose rows then stayed zero: tests/test_gpu_fuzz.py)
    std::sort(torder.begin(), torder.end(), [&](int a, int b) {
      if (ftasks[a].e0 != ftasks[b].e0) return ftasks[a].e0 < ftasks[b].e0;
      return ftasks[a].e1 < ftasks[b].e1;
    });
    std::vector<int32_t> starts(nt), ranks(nt), row0s(nt);
    for (int i = 0; i < nt; ++i) {
      starts[i] = ftasks[torder[i]].e0;
      ranks[i] = torder[i];
      row0s[i] = ftasks[torder[i]].row0;
    }
    int32_t pos = 0;
    for (int i = 0; i < nt; ++i) {  // new contiguous ranges, launch order
      const int32_t len = ftasks[i].e1 - ftasks[i].e0;
      ftasks[i].e0 = pos;
      ftasks[i].e1 = pos + len;
      pos += len;
    }
    if (E > 0) {
      int cbits = 1;
      while ((1ll << cbits) < (long long)NC) ++cbits;
      int tbits = 1;
      while ((1ll << tbits) < (long long)nt) ++tbits;
      int32_t *d_starts = nullptr, *d_ranks = nullptr, *d_row0s = nullptr, *d_rl = nullptr,
              *d_ids = nullptr;
      uint64_t *d_kin = nullptr, *d_kout = nullptr;
      void* d_tmp = nullptr;
      const hipError_t fe = [&]() -> hipError_t {
        hipError_t e = need_row_of();
        if (e == hipSuccess) e = hipMalloc(&d_starts, sizeof(int32_t) * nt);
        if (e == hipSuccess) e = hipMalloc(&d_ranks, sizeof(int32_t) * nt);
        if (e == hipSuccess) e = hipMalloc(&d_row0s, sizeof(int32_t) * nt);
        if (e == hipSuccess) e = hipMemcpyAsync(d_starts, starts.data(), sizeof(int32_t) * nt, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(d_ranks, ranks.data(), sizeof(int32_t) * nt, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(d_row0s, row0s.data(), sizeof(int32_t) * nt, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMalloc(&d_rl, sizeof(int32_t) * E);
        if (e == hipSuccess) e = hipMalloc(&d_ids, sizeof(int32_t) * E);
        if (e == hipSuccess) e = hipMalloc(&d_kin, sizeof(uint64_t) * E);
        if (e == hipSuccess) e = hipMalloc(&d_kout, sizeof(uint64_t) * E);
        if (e == hipSuccess) e = hipMalloc(&p->fwd_perm, sizeof(int32_t) * E);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(fwd_key_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s, idx, row_of, E,
                           d_starts, d_ranks, d_row0s, nt, cbits, d_kin, d_ids, d_rl);
        e = hipGetLastError();
        size_t tb = 0;
        if (e == hipSuccess)
          e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, d_kin, d_kout, d_ids, p->fwd_perm,
                                                 (int)E, 0, cbits + tbits, s);
        if (e == hipSuccess) e = hipMalloc(&d_tmp, tb);
        if (e == hipSuccess)
          e = hipcub::DeviceRadixSort::SortPairs(d_tmp, tb, d_kin, d_kout, d_ids, p->fwd_perm,
                                                 (int)E, 0, cbits + tbits, s);
        // one word past the end, zero (column 0, row 0, value 0): the forward's 16-B edge-word
        // loads read edges in pairs from an even index, and a masked lane still gathers the
        // record of the column it read
        if (e == hipSuccess) e = plan_malloc(&p->fwd_cv, sizeof(uint2) * (E + 1));
        if (e == hipSuccess) e = hipMemsetAsync(p->fwd_cv + E, 0, sizeof(uint2), s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(gather_fwd_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s, p->fwd_perm,
                           idx, d_rl, val, E, p->fwd_cv, true);
        e = hipGetLastError();
        return e == hipSuccess ? hipStreamSynchronize(s) : e;
      }();
      dfree(d_starts); dfree(d_ranks); dfree(d_row0s); dfree(d_rl); dfree(d_ids);
      dfree(d_kin); dfree(d_kout); dfree(d_tmp);
      PLAN_TRY(fe);
      p->device_bytes += (int64_t)E * 12 + 8;
    }
    PLAN_TRY(hipMalloc(&p->fwd_tasks, sizeof(FwdTask) * ftasks.size()));
    PLAN_TRY(hipMemcpyAsync(p->fwd_tasks, ftasks.data(), sizeof(FwdTask) * ftasks.size(),
                            hipMemcpyHostToDevice, s));
    p->device_bytes += sizeof(FwdTask) * ftasks.size();
    if (p->fwd_fixed) {
      PLAN_TRY(hipMalloc(&p->fwd_fix, sizeof(int2) * ftasks.size()));
      p->device_bytes += sizeof(int2) * ftasks.size();
      // a copy of ptr: maxk_plan_refresh_values recomputes the bounds without the caller's
      PLAN_TRY(hipMalloc(&p->fwd_rowptr, sizeof(int32_t) * ((size_t)N + 1)));
      PLAN_TRY(hipMemcpyAsync(p->fwd_rowptr, ptr, sizeof(int32_t) * ((size_t)N + 1),
                              hipMemcpyDeviceToDevice, s));
      p->device_bytes += sizeof(int32_t) * ((int64_t)N + 1);
      PLAN_TRY(fwd_fix_stats(p, p->fwd_rowptr, val, s));
    }
    // Column windows: one launch whose tiles start their column-sorted sweep at the window a
    // shared clock points to (fwd_rot_ticks per window, about one tile's duration per full
    // turn), so the tiles running together on an XCD gather from nearby columns (L2 reuse).
    int B = 1;
    p->fwd_rot_ticks = 0;
    // Not on graphs whose columns see few edges: each record is then used ~E / NC times over
    // the whole pass and the aligned sweep finds little to share (ogbn-products, 50 edges per
    // column, k = 32: 4.79 -> 4.71 ms without it; Reddit, 493: k = 16 1.11 -> 1.08 with it)
    const bool low_reuse = o.fwd_rotate == 0 && NC > 0 && (double)E / NC < 64.0;
    if (o.fwd_rotate != 2 && !low_reuse && (k % 4 == 0 || p->fwd_chunk3 || p->fwd_chunk2)) {
      // the fixed-point kernel sweeps faster: more windows at large k, a higher slot rate
      // (tools/fwd_opts_sweep.py, Reddit: k = 16 1.23 -> 1.19 ms with 260 M edges/s per slot,
      // k = 32 1.81 -> 1.77 with 140 M and 32 windows, k = 64 3.44 -> 3.23 with 64 windows)
      const int Bd = p->fwd_fixed ? (k >= 64 ? 64 : k >= 32 ? 32 : kFwdRotWindows) : kFwdRotWindows;
      B = o.fwd_rot_windows > 0 ? std::min(o.fwd_rot_windows, 64) : Bd;
      // one turn of the clock per tile: the measured per-slot rate scales as ~1/k (Reddit:
      // 2.4e8, 1.65e8, 0.9e8 edges/s per slot at k = 8, 16, 32)
      const double rate = o.fwd_rot_rate > 0 ? o.fwd_rot_rate * 1e6
                                             : std::min(5e8, std::max(2e7, (p->fwd_fixed ? kFwdSlotEdgeRateFixed : kFwdSlotEdgeRate) * 16.0 / k));
      const double tile_ticks = (double)E / nt / rate * 1e8;  // s_memrealtime: 100 MHz
      p->fwd_rot_ticks = (int)std::max(1.0, tile_ticks / B);
    }
    B = std::max(1, std::min(B, std::max(NC, 1)));
    p->fwd_phases = B;
    PLAN_TRY(hipMalloc(&p->fwd_phase_off, sizeof(int32_t) * nt * (B + 1)));
    p->device_bytes += sizeof(int32_t) * nt * (B + 1);
    hipLaunchKernelGGL(fwd_phase_kernel, dim3((nt * (B + 1) + 255) / 256), dim3(256), 0, s,
                       p->fwd_tasks, nt, p->fwd_cv, NC, B, p->fwd_phase_off);
    PLAN_TRY(hipGetLastError());
  }
  if (!zrows.empty()) {
    PLAN_TRY(hipMalloc(&p->zero_rows, sizeof(int32_t) * zrows.size()));
    PLAN_TRY(hipMemcpyAsync(p->zero_rows, zrows.data(), sizeof(int32_t) * zrows.size(),
                            hipMemcpyHostToDevice, s));
    p->device_bytes += sizeof(int32_t) * zrows.size();
  }

  // Two tables (no record pack): Reddit k = 32 2.65 -> 2.53 ms, k = 64 4.98 -> 4.92 (k = 16:
  // 1.35 vs 1.39 packed); and where the per-call pack of all NC records costs more than it
  // saves: below kFwdPackMinEdgesPerCol edges per column, or below kFwdPackMinEdgesPerColL2
  // with an L2-resident selector table (per-rank forward on row shards at k = 16: Reddit
  // W = 8, 62 edges per column and a 3.7 MB selector table, 0.172 ms packed vs 0.183 two
  // tables, W = 4 (123) 0.757 vs 0.805 ms for the rank's whole step; ogbn-proteins W = 8, 75
  // edges per column and 2.1 MB of selectors, 0.144 packed vs 0.138 two tables). But on a
  // large table, whose gathers mostly miss L2, the record's one line beats the two tables'
  // two (values + selectors): at k = 16 from tens of MB (yelp, 57 MB: 0.645 -> 0.54 ms packed;
  // ogbn-products, 196 MB: 4.84 -> 2.95; flickr, 7 MB at 11 edges per column, stays faster
  // with two tables), at k = 32 only from HBM-sized tables (ogbn-products 392 MB: 4.95 ->
  // 4.77; yelp 115 MB: 0.67 two tables vs 0.73); never at k = 64 (ogbn-products 7.08 two
  // tables vs 7.44)
  const bool sel_l2 = (double)std::max(NC, 1) * k <= kFwdSelL2Bytes;
  const bool few_edges = E < kFwdPackMinEdgesPerCol * std::max(NC, 1) ||
                         (sel_l2 && E < kFwdPackMinEdgesPerColL2 * std::max(NC, 1));
  p->fwd_two_tables = !p->fwd_chunk3 && !p->fwd_chunk2 && k % 4 == 0 &&
                      (o.fwd_two_tables == 1 ||
                       (o.fwd_two_tables == 0 &&
                        (k >= 64 || (!big_table && (k >= 32 || few_edges)))));
  if (p->fwd_two_tables) {
    // no workspace: the kernel gathers from sp_data / sp_index
  } else if ((p->fwd_chunk3 || p->fwd_chunk2) && NC > 0) {
    const int b = (p->fwd_chunk3 ? (k + 2) / 3 : k / 2) * 16;
    p->fwd_rec_bytes = b <= 64 ? 64 : b <= 128 ? 128 : b;
    p->fwd_ws_bytes = (int64_t)NC * p->fwd_rec_bytes;
  } else if (k % 4 == 0 && NC > 0) {
    p->fwd_rec_bytes = cbsr_record_bytes(k);
    p->fwd_ws_bytes = (int64_t)NC * p->fwd_rec_bytes;
  }
  if (p->fwd_fix) {  // the call's {max |x|, min |x|} words after the records
    p->fwd_xstat_off = (p->fwd_ws_bytes + 255) / 256 * 256;
    p->fwd_ws_bytes = p->fwd_xstat_off + 256;
  }
  if (p->fwd_ws_bytes > 0 && !p->external_ws) {  // plan-owned per-call pack buffer
    PLAN_TRY(hipMalloc(&p->fwd_rec, (size_t)p->fwd_ws_bytes));
    p->device_bytes += p->fwd_ws_bytes;
  }

  // ---------------- backward
  // Two-pass backward (bwd_algo = 3; auto when a column block would see each grad_out row it
  // fetches about once): a row pass stages grad_out[r] in LDS once per row and writes each
  // edge's k products into its slot of an E x k workspace (CSR order), then a column pass
  // gathers the slots of each column's in-edges and sums them. Trades 8k bytes of workspace
  // traffic per edge for gathers that stop missing (ogbn-products k = 32: a block of 1023
  // columns gets 0.02 edges per row it touches).
  // Rows per wavefront of the row pass: enough that a wavefront has ~256 edges, at most
  // kBwdRowsPerWave, so low-degree rows do not leave most of the 64/L edge slots idle
  // (ogbn-products, 50 edges per row, k = 32: R = 1 8.65 ms, 4 8.67, 8 9.07 for both passes)
  const int Lt = k / 4;
  int R = 1;
  while (R < kBwdRowsPerWave && (double)R * E / std::max(N, 1) < 256.0) R *= 2;
  bool tp_fits = true;  // each wavefront's slots are addressed with 32-bit byte offsets
  for (int r0 = 0; r0 < N && tp_fits; r0 += R)
    tp_fits = (uint64_t)(hp[std::min(N, r0 + R)] - hp[r0]) * (uint64_t)k * 4u < 0x80000000ull;
  const bool tp_ok = E > 0 && k % 4 == 0 && (Lt & (Lt - 1)) == 0 && Lt <= kWave && NC > 0 &&
                     tp_fits;
  bool twopass = tp_ok && o.bwd_algo == 3;
  if (tp_ok && o.bwd_algo == 0) {
    const double reuse = (double)E / std::max(N, 1) * (double)std::min(C, NC) / NC;
    size_t free_b = 0, total_b = 0;
    const bool fits = hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
                      (double)E * k * 4.0 < 0.5 * (double)free_b;
    twopass = reuse < kBwdTwoPassReuse && fits;
  }
  p->bwd_twopass = twopass;
  p->bwd_tp_rows = R;
  if (twopass) C = 1;
  // the column order applies to the column blocks (the two-pass sorts by the column itself)
  const int32_t* bcolpos = twopass ? nullptr : colpos;
  // row order inside the blocks' streams: scattered by an affine bijection ra * row + rb mod N
  const bool row_hash_ok = !twopass && E > 0 && N > 1;
  bool row_hash = row_hash_ok && o.bwd_row_order == 2;
  int64_t ra = 1, rb = 0;
  int rbits = 1;
  if (row_hash_ok) {
    auto gcd = [](int64_t x, int64_t y) { while (y) { const int64_t t = x % y; x = y; y = t; } return x; };
    ra = std::max<int64_t>(1, (int64_t)(0.6180339887 * N));
    while (gcd(ra, N) != 1) ++ra;
    ra %= N;
    rb = N / 7;
    while ((1ll << rbits) < (long long)N) ++rbits;
  }
  auto row_pos = [&](int32_t r) -> int64_t { return row_hash ? (ra * (int64_t)r + rb) % N : r; };
  int nblocks = NC > 0 ? (NC + C - 1) / C : 0;
  if (!twopass && nblocks >= kXcds) {
    // a multiple of the XCD count, so every XCD owns the same number of column blocks; and
    // of 8 per XCD when that many blocks are needed anyway (measured: 64 / 128 / 256 blocks
    // for k = 8 / 16 / 32 on Reddit ran 10-25 % faster than 72 / 120 / 240)
    const int q = nblocks >= kXcds * 8 ? kXcds * 8 : kXcds;
    nblocks = (nblocks + q - 1) / q * q;
    C = (NC + nblocks - 1) / nblocks;
    nblocks = (NC + C - 1) / C;
  }
  p->bwd_block_cols = C;
  p->n_bwd_blocks = nblocks;
  std::vector<int64_t> offs(twopass ? 1 : nblocks + 1, 0);
  p->bwd_row_order = twopass ? 0 : 1;
  if (E > 0) {
    PLAN_TRY(need_row_of());
    PLAN_TRY(hipMalloc(&keys_in, sizeof(uint32_t) * E));
    PLAN_TRY(hipMalloc(&keys_out, sizeof(uint32_t) * E));
    PLAN_TRY(hipMalloc(&ids_in, sizeof(int32_t) * E));
    PLAN_TRY(hipMalloc(&p->bwd_perm, sizeof(int32_t) * E));
    PLAN_TRY(hipMalloc(&d_bad, sizeof(int)));
    PLAN_TRY(hipMemsetAsync(d_bad, 0, sizeof(int), s));
    int end_bit = 1;
    while ((1ll << end_bit) < (long long)nblocks) ++end_bit;
    // the block-major sort: keys_out = block id of each sorted edge, bwd_perm = its CSR id
    auto sort_blocks = [&](bool hash) -> hipError_t {
      size_t temp_bytes = 0;
      dfree(temp);
      temp = nullptr;
      if (!hash) {
        hipLaunchKernelGGL(bwd_key_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s, idx, E, C, NC,
                           keys_in, ids_in, d_bad, bcolpos);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess)
          e = hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, keys_in, keys_out, ids_in,
                                                 p->bwd_perm, (int)E, 0, end_bit, s);
        if (e == hipSuccess) e = hipMalloc(&temp, temp_bytes);
        if (e != hipSuccess) return e;
        return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, ids_in,
                                                  p->bwd_perm, (int)E, 0, end_bit, s);
      }
      // 64-bit keys {block, row position}; their block ids then go to keys_out
      uint64_t *k64_in = nullptr, *k64_out = nullptr;
      const hipError_t ke = [&]() -> hipError_t {
        hipError_t e = hipMalloc(&k64_in, sizeof(uint64_t) * E);
        if (e == hipSuccess) e = hipMalloc(&k64_out, sizeof(uint64_t) * E);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(bwd_key64_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s, idx, row_of,
                           E, C, NC, k64_in, ids_in, d_bad, bcolpos, ra, rb, N, rbits);
        e = hipGetLastError();
        if (e == hipSuccess)
          e = hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, k64_in, k64_out, ids_in,
                                                 p->bwd_perm, (int)E, 0, end_bit + rbits, s);
        if (e == hipSuccess) e = hipMalloc(&temp, temp_bytes);
        if (e == hipSuccess)
          e = hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k64_in, k64_out, ids_in,
                                                 p->bwd_perm, (int)E, 0, end_bit + rbits, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(key_block_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s, k64_out, E,
                           rbits, keys_out);
        e = hipGetLastError();
        return e == hipSuccess ? hipStreamSynchronize(s) : e;
      }();
      dfree(k64_in);
      dfree(k64_out);
      return ke;
    };
    PLAN_TRY(sort_blocks(row_hash));
    if (row_hash_ok && o.bwd_row_order == 0) {
      // auto: scatter the rows when the ascending-row streams are mostly dense runs, i.e. many
      // consecutive rows with many edges into the same block (an ID-ordered community: Reddit
      // size, 41 communities, k = 16: 2.31 -> 1.59 ms; k = 32: 3.62 -> 2.45); with rows that
      // are unrelated to their neighbours the ascending order is 2-3 % faster (uniform
      // Reddit: 1.686 vs 1.715 ms at k = 16, 2.61 vs 2.69 at k = 32)
      constexpr int Wn = 2048;
      const int64_t nw = E / Wn;
      if (nw > 0) {
        int* d_nd = nullptr;
        int nd = 0;
        const hipError_t de = [&]() -> hipError_t {
          hipError_t e = hipMalloc(&d_nd, sizeof(int));
          if (e == hipSuccess) e = hipMemsetAsync(d_nd, 0, sizeof(int), s);
          if (e != hipSuccess) return e;
          hipLaunchKernelGGL(dense_window_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s,
                             keys_out, p->bwd_perm, row_of, E, Wn, d_nd);
          e = hipGetLastError();
          if (e == hipSuccess) e = hipMemcpyAsync(&nd, d_nd, sizeof(int), hipMemcpyDeviceToHost, s);
          return e == hipSuccess ? hipStreamSynchronize(s) : e;
        }();
        dfree(d_nd);
        PLAN_TRY(de);
        if (nd > nw / 4) {
          row_hash = true;
          PLAN_TRY(sort_blocks(true));
        }
      }
    }
    if (!twopass) p->bwd_row_order = row_hash ? 2 : 1;
    if (twopass) {
      PLAN_TRY(plan_malloc(&p->bwd_erec, sizeof(uint32_t) * 2 * (size_t)E));
      // row chunks: the workspace holds one chunk's products
      int P = o.bwd_tp_chunks > 0
                  ? o.bwd_tp_chunks
                  : (int)std::max<int64_t>(1, (int64_t)std::ceil((double)E * k * 4.0 /
                                                                  kBwdTwoPassWorkspaceCap));
      P = std::max(1, std::min(P, std::max(N, 1)));
      p->bwd_tp_chunks = P;
      p->tp_rows.assign(P + 1, 0);
      p->tp_edges.assign(P + 1, 0);
      int64_t max_chunk = 0;
      for (int q = 1; q <= P; ++q) {
        int32_t r = N;
        if (q < P) {
          // a multiple of R: the row pass's wavefronts stage rows r0 .. r0 + R - 1 with
          // r0 % R == 0 (the edge records carry row % R)
          const int64_t target = E * q / P;
          r = (int32_t)(std::lower_bound(hp.begin(), hp.end(), (int32_t)target) - hp.begin());
          r = std::max(p->tp_rows[q - 1], std::min(r / R * R, N));
        }
        p->tp_rows[q] = r;
        p->tp_edges[q] = hp[r];
        max_chunk = std::max<int64_t>(max_chunk, p->tp_edges[q] - p->tp_edges[q - 1]);
      }
      p->bwd_ws_bytes = max_chunk * k * 4;  // one row chunk of the E x k product workspace
      if (!p->external_ws) {
        PLAN_TRY(hipMalloc(&p->bwd_tbuf, (size_t)p->bwd_ws_bytes));
        p->device_bytes += p->bwd_ws_bytes;
      }
      p->device_bytes += (int64_t)E * 12;  // erec + bwd_perm
      hipLaunchKernelGGL(build_erec_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s, idx,
                         row_of, R, val, E, p->bwd_erec);
    } else {
      PLAN_TRY(hipMalloc(&brow, sizeof(int32_t) * E));
      PLAN_TRY(hipMalloc(&bcol, sizeof(int32_t) * E));
      hipLaunchKernelGGL(gather_bwd_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s,
                         p->bwd_perm, row_of, idx, E, brow, bcol, bcolpos);
    }
    PLAN_TRY(hipMalloc(&d_offs, sizeof(int32_t) * (nblocks + 1)));
    hipLaunchKernelGGL(key_offsets_kernel, dim3(nblocks / 256 + 1), dim3(256), 0, s, keys_out,
                       E, nblocks, d_offs);
    PLAN_TRY(hipGetLastError());
    int bad = 0;
    PLAN_TRY(hipMemcpyAsync(&bad, d_bad, sizeof(int), hipMemcpyDeviceToHost, s));
    if (twopass) {
      // column pointers of the column-sorted edge list stay on the device
      p->bwd_colptr = d_offs;
      d_offs = nullptr;
      p->device_bytes += sizeof(int32_t) * (nblocks + 1);
      if (p->bwd_tp_chunks > 1) {
        // per-chunk column pointers (rows ascend within a column of the stable sort)
        const int P = p->bwd_tp_chunks;
        int32_t* d_rows = nullptr;
        const hipError_t ce = [&]() -> hipError_t {
          hipError_t e = hipMalloc(&d_rows, sizeof(int32_t) * (P + 1));
          if (e == hipSuccess) e = hipMemcpyAsync(d_rows, p->tp_rows.data(), sizeof(int32_t) * (P + 1),
                                                  hipMemcpyHostToDevice, s);
          if (e == hipSuccess) e = hipMalloc(&p->bwd_colptr2, sizeof(int32_t) * (size_t)(P + 1) * NC);
          if (e != hipSuccess) return e;
          const int64_t n = (int64_t)(P + 1) * NC;
          hipLaunchKernelGGL(tp_colptr_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                             p->bwd_colptr, p->bwd_perm, row_of, NC, d_rows, P, p->bwd_colptr2);
          e = hipGetLastError();
          return e == hipSuccess ? hipStreamSynchronize(s) : e;
        }();
        dfree(d_rows);
        PLAN_TRY(ce);
        p->device_bytes += sizeof(int32_t) * (int64_t)(P + 1) * NC;
      }
      PLAN_TRY(hipStreamSynchronize(s));
    } else {
      std::vector<int32_t> offs32(nblocks + 1);
      PLAN_TRY(hipMemcpyAsync(offs32.data(), d_offs, sizeof(int32_t) * (nblocks + 1),
                              hipMemcpyDeviceToHost, s));
      PLAN_TRY(hipStreamSynchronize(s));
      for (int b = 0; b <= nblocks; ++b) offs[b] = offs32[b];
    }
    if (bad) {
      set_error("maxk_plan_create: idx contains column ids outside [0, num_cols)");
      return fail(MAXK_ERR_INVALID_ARG);
    }
  }
  std::vector<BwdTask> btasks;
  int nshared = 0;
  if (!twopass && E > 0 && nblocks > 0) {
    // Task count: about kBwdTasksPerCu work-groups per CU, each of its block's chunks with
    // >= kBwdMinTaskEdges edges (every chunk clears and stores its whole block, C * k
    // floats), but not fewer tasks than CUs while those keep >= 4k edges (a row shard of an
    // 8-GPU partition: 256 tasks of ~56k edges ran 0.24 ms, 512 of ~28k 0.27, 128 0.40)
    const int64_t target_tasks = (int64_t)(o.bwd_tasks_per_cu ? o.bwd_tasks_per_cu : kBwdTasksPerCu) * cus;
    const int64_t bS = (int64_t)nblocks * S;
    const int64_t chunks = std::max<int64_t>(1, (target_tasks + bS - 1) / bS);
    const int64_t min_task_edges = o.bwd_min_task_edges > 0 ? o.bwd_min_task_edges : kBwdMinTaskEdges;
    int64_t nch64 = std::min<int64_t>(chunks, E / ((int64_t)nblocks * min_task_edges));
    const int64_t fl = ((int64_t)cus + bS - 1) / bS;
    if (o.bwd_min_task_edges == 0 && nch64 < fl && E / ((int64_t)nblocks * fl) >= 4096)
      nch64 = std::min<int64_t>(chunks, fl);
    nch64 = std::max<int64_t>(1, nch64);
    // One work-group per CU: a task count just past a multiple of the CUs leaves the last
    // round mostly idle (ogbn-proteins k = 32: 192 blocks x 3 chunks = 2.25 rounds, 2.37 ms;
    // x 4 = 3 rounds, 1.82 ms). With the default knobs take, among the chunk counts from one
    // round of tasks (fl) up to nch + 2 (keeping >= 0.6 x the minimum task above nch), the
    // FEWEST whose tasks fill their rounds within 0.05 of the best: every task zeroes and
    // stores its block and stages its selectors, so with the counter-fed 16-wave work-groups
    // one full round beats two (Reddit k = 8 / 16 / 32: 512 -> 256 tasks -2.8 / -2.0 / -1.8 %,
    // ogbn-proteins k = 16 -1.4 %; profiles/r05/bwd_task_rounds.jsonl)
    if (o.bwd_tasks_per_cu == 0 && o.bwd_min_task_edges == 0) {
      auto fill = [&](int64_t c) {
        const int64_t t = bS * c;
        return (double)t / ((double)((t + cus - 1) / cus) * cus);
      };
      // the fill counts tasks, not edges: go below nch only while the blocks hold similar edge
      // counts (largest <= 2x the mean), so a skewed block cannot become a one-round tail
      // 
      int64_t max_nnz = 0;
      for (int b = 0; b < nblocks; ++b) max_nnz = std::max<int64_t>(max_nnz, offs[b + 1] - offs[b]);
      const bool even_blocks = max_nnz * (int64_t)nblocks <= 2 * E;
      const int64_t lo = even_blocks ? std::max<int64_t>(1, std::min(nch64, fl)) : nch64;
      int64_t hi = nch64;
      for (int64_t c = nch64 + 1; c <= nch64 + 2; ++c) {
        if ((double)E / ((double)nblocks * c) < 0.6 * kBwdMinTaskEdges) break;
        hi = c;
      }
      double bestf = 0.0;
      for (int64_t c = lo; c <= hi; ++c) bestf = std::max(bestf, fill(c));
      int64_t best = hi;
      for (int64_t c = lo; c <= hi; ++c)
        if (fill(c) >= bestf - 0.05) { best = c; break; }
      nch64 = best;
    }
    const int nch = (int)nch64;
    // Chunk j of block b holds edges [j, j+1) * nnz_b / nch of the block's row-sorted stream.
    // On a graph without column locality these are about the same row bounds in every block
    // (the work-groups that run together sweep the same rows of G); with locality (a
    // community linking mostly into its own blocks) every task keeps an equal share instead
    // of a few tasks carrying most of a chunk (41-community Reddit-size graph, k = 16: 3.38
    // -> 2.18 ms; the scattered row order then takes it to 1.60).
    std::vector<std::vector<int32_t>> cbd((size_t)nblocks);
    for (int b = 0; b < nblocks; ++b) {
      const int64_t o0 = offs[b], nnz = offs[b + 1] - offs[b];
      cbd[b].resize(nch + 1);
      for (int j = 0; j <= nch; ++j) cbd[b][j] = (int32_t)(o0 + nnz * j / nch);
    }
    // Pieces: a (block, chunk) task holding more than twice the average task's edges is cut
    // into pieces of equal edge counts (work-groups of their own).
    const int64_t avg_task = std::max<int64_t>(1, E / ((int64_t)nblocks * nch));
    const int64_t piece_cap = o.bwd_piece_edges > 0 ? (int64_t)o.bwd_piece_edges
                                                    : std::max<int64_t>(2 * avg_task, 16384);
    const bool slab_flush = o.bwd_flush != 1;
    auto npieces = [&](int64_t e) {
      return (int32_t)std::max<int64_t>(1, (e + piece_cap - 1) / piece_cap);
    };
    std::vector<int32_t> pieces_of((size_t)nblocks, 0);
    for (int b = 0; b < nblocks; ++b)
      for (int j = 0; j < nch; ++j) pieces_of[b] += npieces((int64_t)cbd[b][j + 1] - cbd[b][j]);
    // compact slab regions: block b's pieces 1 .. P_b - 1 own C x k floats each
    std::vector<int64_t> slab_base((size_t)nblocks, -1);
    std::vector<int4> comb;
    int64_t slab_floats = 0;
    for (int b = 0; b < nblocks; ++b) {
      if (pieces_of[b] > 1) ++nshared;
      if (slab_flush && pieces_of[b] > 1) {
        slab_base[b] = slab_floats;
        const int ncols_b = std::min(C, NC - b * C);
        comb.push_back(make_int4((int)slab_floats, pieces_of[b] - 1, b * C, ncols_b));
        slab_floats += (int64_t)(pieces_of[b] - 1) * C * k;
      }
    }
    if (slab_floats >= (int64_t)INT32_MAX) {  // task offsets are int32: flush atomically
      comb.clear();
      slab_floats = 0;
      std::fill(slab_base.begin(), slab_base.end(), -1);
    }
    // Row-major emission: chunks ordered by the first destination row they sweep (then by
    // block), so the work-groups that run together sweep about the same rows of G and share
    // its lines in L2; work-group i runs on XCD i % 8 (dealt round-robin; speed only), so
    // consecutive tasks spread over the XCDs and every XCD gets the same share.
    std::vector<int32_t> first_row((size_t)nblocks * nch);
    {
      std::vector<int32_t> starts;
      for (int b = 0; b < nblocks; ++b)
        for (int j = 0; j < nch; ++j)
          starts.push_back(std::min<int32_t>(cbd[b][j], (int32_t)std::max<int64_t>(E - 1, 0)));
      int32_t *d_st = nullptr, *d_fr = nullptr;
      const hipError_t fe = [&]() -> hipError_t {
        hipError_t e = hipMalloc(&d_st, sizeof(int32_t) * starts.size());
        if (e == hipSuccess) e = hipMalloc(&d_fr, sizeof(int32_t) * starts.size());
        if (e == hipSuccess) e = hipMemcpyAsync(d_st, starts.data(), sizeof(int32_t) * starts.size(),
                                                hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(gather_i32_kernel, dim3((unsigned)((starts.size() + 255) / 256)),
                           dim3(256), 0, s, brow, d_st, (int)starts.size(), d_fr);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(first_row.data(), d_fr, sizeof(int32_t) * starts.size(),
                                                hipMemcpyDeviceToHost, s);
        return e == hipSuccess ? hipStreamSynchronize(s) : e;
      }();
      dfree(d_st);
      dfree(d_fr);
      PLAN_TRY(fe);
    }
    struct ChunkRef { int64_t row; int b, j; };
    std::vector<ChunkRef> order_c;
    for (int b = 0; b < nblocks; ++b)
      for (int j = 0; j < nch; ++j) order_c.push_back(ChunkRef{row_pos(first_row[(size_t)b * nch + j]), b, j});
    std::stable_sort(order_c.begin(), order_c.end(),
                     [](const ChunkRef& a, const ChunkRef& b) { return a.row < b.row; });
    // a block's chunks must come in chunk order (piece numbering, slab regions)
    std::vector<int32_t> next_chunk((size_t)nblocks, 0);
    for (ChunkRef& cr : order_c) cr.j = next_chunk[cr.b]++;
    std::vector<int32_t> next_piece((size_t)nblocks, 0);
    for (const ChunkRef& cr : order_c) {
      const int b = cr.b;
      const int32_t e0 = cbd[b][cr.j], e1 = cbd[b][cr.j + 1];
      const int np = npieces((int64_t)e1 - e0);
      for (int q = 0; q < np; ++q) {
        const int piece = next_piece[b]++;
        for (int g = 0; g < S; ++g) {  // the groups of a block share its edge stream
          BwdTask t{};
          t.col0 = b * C;
          t.ncols = std::min(C, NC - t.col0);
          t.e0 = (int32_t)(e0 + ((int64_t)e1 - e0) * q / np);
          t.e1 = (int32_t)(e0 + ((int64_t)e1 - e0) * (q + 1) / np);
          t.shared = pieces_of[b] > 1;
          t.group = g;
          t.chunk = piece;
          t.slab = (slab_base[b] >= 0 && piece > 0)
                       ? (int32_t)(slab_base[b] + (int64_t)(piece - 1) * C * k) : -1;
          btasks.push_back(t);
        }
      }
    }
    if (!comb.empty()) {
      p->bwd_slab_floats = slab_floats;
      p->n_bwd_combine = (int32_t)comb.size();
      PLAN_TRY(hipMalloc(&p->bwd_combine, sizeof(int4) * comb.size()));
      PLAN_TRY(hipMemcpyAsync(p->bwd_combine, comb.data(), sizeof(int4) * comb.size(),
                              hipMemcpyHostToDevice, s));
      PLAN_TRY(hipStreamSynchronize(s));
      p->device_bytes += sizeof(int4) * comb.size();
    }
  }
  // default on (Reddit k = 16: 1.665 -> 1.626 ms, an 8-GPU row shard 0.241 -> 0.226). Round 4
  // measured them +0.7-1.5 % with two slot groups (profiles/r04/bwd_order_ab.jsonl); with the
  // round-5 kernel (counter-fed 16 waves, one round) they gain there too: k = 16 / 24 / 32 / 64
  // -1.5 / -0.7 / -0.4 / -0.3 % (profiles/r05/bwd_order_ab.jsonl)
  const bool windows = o.bwd_order == 2 || o.bwd_order == 0;
  if (windows && btasks.size() >= 2 * (size_t)kXcds) {
    // XCD row windows: work-group i runs on XCD i % 8, one task per CU at a time. Within each
    // round of `cus` consecutive (row-sorted) tasks, XCD x gets the x-th contiguous run of
    // them, so the work-groups sharing an XCD's L2 sweep one row window of G instead of every
    // window the round spans
    const size_t R = (size_t)cus;
    std::vector<BwdTask> dealt(btasks.size());
    for (size_t r0 = 0; r0 < btasks.size(); r0 += R) {
      const size_t n = std::min(R, btasks.size() - r0);
      const size_t per = n / kXcds;
      for (size_t q = 0; q < n; ++q)
        dealt[r0 + q] = (n % kXcds == 0) ? btasks[r0 + (q % kXcds) * per + q / kXcds] : btasks[r0 + q];
    }
    btasks.swap(dealt);
  }
  p->n_bwd_tasks = (int32_t)btasks.size();
  p->n_bwd_shared = nshared;
  // window hand-out (profiles/r05/handout_ab.jsonl): the backward always takes
  // its windows from an LDS counter (k = 8..64 -2..-6 %, W = 8 shards -2 %); the forward with
  // 8 waves and at k <= 16 (-0.3 %, W = 8 shards -1..-5 %); 4 waves above k = 16 keep the
  // static interleave (+2..3 % with the counter)
  p->bwd_handout = o.bwd_handout ? o.bwd_handout : 2;
  p->fwd_handout = o.fwd_handout ? o.fwd_handout : (k <= 16 || p->fwd_waves == 8 ? 2 : 1);
  if (o.bwd_waves == 0 && (o.bwd_unroll == 12 || o.bwd_unroll == 16)) {
    // an explicit unroll picks the waves that run it: 12 x 12, 8 x 16
    p->bwd_waves = o.bwd_unroll == 12 ? 12 : 8;
  } else if (o.bwd_waves == 0) {
    if (p->bwd_handout == 2 && !p->bwd_big) {
      // handed-out windows leave no wave a longer share than its neighbours, so more waves
      // only add latency hiding: 16 per work-group (Reddit k = 16 1.646 -> 1.504 ms, k = 64
      // 4.257 -> 4.035, ogbn-proteins k = 16 1.191 -> 0.972; k = 10 / 12 within 0.4 % of
      // 12 waves; an 8-GPU shard 0.365 -> 0.363; profiles/r05/bwd_waves_handout.jsonl)
      p->bwd_waves = 16;
    } else if (p->n_bwd_tasks > 0 && p->n_bwd_tasks <= cus) {
      // static interleave, one round of tasks (at most one work-group per CU, e.g. an 8-GPU
      // row shard: 256 tasks): the CU has only that work-group's waves to hide its gathers
      // (k = 16: 0.227 -> 0.206 ms with 12; profiles/r05/w8_bwd_waves.jsonl)
      p->bwd_waves = 12;
    }
  }
  // the shape that actually launches: the 16-wave shape runs U = 8, 12 waves U
  // = 8 or 12, and grad_out > 4 GiB (64-bit gathers) one shape, 8 waves x 8
  if (p->bwd_waves != 8 && !(p->bwd_waves == 12 && p->bwd_unroll == 12)) p->bwd_unroll = 8;
  if (p->bwd_big) {
    p->bwd_waves = 8;
    p->bwd_unroll = 8;
  }
  if (!btasks.empty()) {
    PLAN_TRY(hipMalloc(&p->bwd_tasks, sizeof(BwdTask) * btasks.size()));
    PLAN_TRY(hipMemcpyAsync(p->bwd_tasks, btasks.data(), sizeof(BwdTask) * btasks.size(),
                            hipMemcpyHostToDevice, s));
    p->device_bytes += sizeof(BwdTask) * btasks.size();
  }
  if (!twopass && E > 0) {
    // the column blocks' records (padded: a wave may read past the last task's end)
    PLAN_TRY(plan_malloc(&p->bwd_rec, sizeof(uint32_t) * 3 * (size_t)(E + kBwdRecPad)));
    PLAN_TRY(hipMemsetAsync(p->bwd_rec + 3 * E, 0, sizeof(uint32_t) * 3 * kBwdRecPad, s));
    hipLaunchKernelGGL(build_bwd_rec_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s, p->bwd_perm,
                       brow, bcol, val, E, C, D, p->bwd_big, p->bwd_rec);
    PLAN_TRY(hipGetLastError());
    // per-call workspace: the slab regions of split blocks (the kernel stages the selectors
    // from sp_index itself; no selector words since round 5)
    p->bwd_slab_off = 0;
    p->bwd_ws_bytes = p->bwd_slab_floats * 4;
    if (!p->external_ws && p->bwd_ws_bytes > 0)
      PLAN_TRY(hipMalloc(&p->bwd_sel, (size_t)p->bwd_ws_bytes));
    p->device_bytes += (int64_t)E * 16 + 12ll * kBwdRecPad + (!p->external_ws ? p->bwd_ws_bytes : 0);
  }
  PLAN_TRY(hipStreamSynchronize(s));
  // the column order stays with the plan when the column blocks use it
  p->col_order = 1;
  if (order && bcolpos) {
    p->col_order = order_mode;
    p->bwd_corder = order;
    p->device_bytes += sizeof(int32_t) * (int64_t)NC;
    order = nullptr;
  }
  dfree(order); dfree(colpos); dfree(row_of); dfree(keys_in); dfree(keys_out); dfree(ids_in);
  dfree(brow); dfree(bcol); dfree(temp); dfree(d_offs); dfree(d_bad);
#undef PLAN_TRY
  *out_plan = p;
  return MAXK_OK;
}

extern "C" int maxk_plan_refresh_values(maxk_plan* p, const float* val, void* stream) {
  MAXK_CHECK_ARG(p != nullptr, "maxk_plan_refresh_values: plan is null");
  if (p->num_edges == 0) return MAXK_OK;
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_for(p->num_edges, 256);
  if (p->bwd_erec)
    hipLaunchKernelGGL(build_erec_kernel, dim3(g), dim3(256), 0, s, nullptr, nullptr, 1, val,
                       p->num_edges, p->bwd_erec);
  else if (p->bwd_rec)
    hipLaunchKernelGGL(build_bwd_rec_kernel, dim3(g), dim3(256), 0, s, p->bwd_perm, nullptr,
                       nullptr, val, p->num_edges, p->bwd_block_cols, p->dim_origin, p->bwd_big,
                       p->bwd_rec);
  if (p->fwd_perm)
    hipLaunchKernelGGL(gather_fwd_kernel, dim3(g), dim3(256), 0, s, p->fwd_perm, nullptr, nullptr,
                       val, p->num_edges, p->fwd_cv, false);
  if (p->fwd_fix && p->n_fwd_tasks > 0) {
    const hipError_t e = fwd_fix_stats(p, p->fwd_rowptr, val, s);
    if (e != hipSuccess) {
      set_error(std::string("maxk_plan_refresh_values: ") + hipGetErrorString(e));
      return (int)e;
    }
  }
  MAXK_LAUNCH_CHECK("maxk_plan_refresh_values launch");
  return MAXK_OK;
}

extern "C" int maxk_plan_get_info(const maxk_plan* p, maxk_plan_info* info) {
  // the version-1 fields only (a binding of ABI 1 passes a struct that ends at bwd_algo)
  return maxk_plan_get_info_sized(p, info, (int64_t)offsetof(maxk_plan_info, col_order));
}

extern "C" int maxk_plan_get_info_sized(const maxk_plan* p, maxk_plan_info* out,
                                        int64_t info_bytes) {
  MAXK_CHECK_ARG(p != nullptr && out != nullptr && info_bytes >= 0,
                 "maxk_plan_get_info: null pointer");
  maxk_plan_info info{};
  info.num_nodes = p->num_nodes;
  info.num_cols = p->num_cols;
  info.num_edges = p->num_edges;
  info.dim_origin = p->dim_origin;
  info.dim_k = p->dim_k;
  info.fwd_tasks = p->n_fwd_tasks;
  info.fwd_split_rows = p->n_zero_rows;
  info.bwd_block_cols = p->bwd_block_cols;
  info.bwd_blocks = p->n_bwd_blocks;
  info.bwd_tasks = p->n_bwd_tasks;
  info.bwd_shared_blocks = p->n_bwd_shared;
  info.device_bytes = p->device_bytes;
  info.bwd_algo = p->bwd_twopass ? MAXK_BWD_TWO_PASS : MAXK_BWD_COLUMN_BLOCKS;
  info.col_order = p->col_order;
  info.bwd_chunk_bounds = p->bwd_twopass ? 0 : 2;
  info.bwd_tp_chunks = p->bwd_twopass ? p->bwd_tp_chunks : 1;
  info.bwd_row_order = p->bwd_row_order;
  info.bwd_workspace_peak = p->bwd_ws_bytes;
  info.fwd_handout = p->fwd_handout;
  info.bwd_handout = p->bwd_handout;
  info.fwd_waves = p->fwd_waves;
  info.fwd_unroll = p->fwd_unroll;
  info.bwd_waves = p->bwd_twopass ? 0 : p->bwd_waves;  // the two-pass kernels have one shape
  info.bwd_unroll = p->bwd_twopass ? 0 : p->bwd_unroll;
  if (p->fwd_chunk2) {
    info.fwd_layout = 4;
    info.fwd_record_bytes = p->fwd_rec_bytes;
  } else if (p->fwd_chunk3) {
    info.fwd_layout = 2;
    info.fwd_record_bytes = p->fwd_rec_bytes;
  } else if (p->dim_k % 4 != 0) {
    info.fwd_layout = 3;
  } else if (!p->fwd_two_tables) {
    info.fwd_layout = 1;
    info.fwd_record_bytes = p->fwd_rec_bytes;
  }
  std::memcpy(out, &info, (size_t)std::min<int64_t>(info_bytes, (int64_t)sizeof(maxk_plan_info)));
  return MAXK_OK;
}

extern "C" int maxk_plan_get_col_order(const maxk_plan* p, int32_t* order, void* stream) {
  MAXK_CHECK_ARG(p != nullptr && (order != nullptr || p->num_cols == 0),
                 "maxk_plan_get_col_order: null pointer");
  if (p->num_cols == 0) return MAXK_OK;
  hipStream_t s = (hipStream_t)stream;
  if (p->bwd_corder) {
    MAXK_HIP_TRY(hipMemcpyAsync(order, p->bwd_corder, sizeof(int32_t) * (size_t)p->num_cols,
                                hipMemcpyDeviceToDevice, s));
  } else {
    hipLaunchKernelGGL(iota_kernel, dim3((p->num_cols + 255) / 256), dim3(256), 0, s,
                       p->num_cols, order);
    MAXK_LAUNCH_CHECK("maxk_plan_get_col_order launch");
  }
  return MAXK_OK;
}

extern "C" int maxk_plan_workspace_bytes(const maxk_plan* p, int64_t* fwd_bytes,
                                         int64_t* bwd_bytes) {
  MAXK_CHECK_ARG(p != nullptr, "maxk_plan_workspace_bytes: plan is null");
  if (fwd_bytes) *fwd_bytes = p->fwd_ws_bytes;
  if (bwd_bytes) *bwd_bytes = p->bwd_ws_bytes;
  return MAXK_OK;
}

extern "C" int maxk_plan_destroy(maxk_plan* p) {
  free_plan(p);
  return MAXK_OK;
}
