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
//             (hipcub::DeviceRadixSort, keys = idx / block_cols) gives the block-major,
//             row-sorted edge list, packed as 12-B records {row * D * 4, column in block,
//             val}; each block's range is cut into row-chunk tasks (same row bounds in every
//             block, XCD-aware order).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstring>
#include <vector>

#include "common.h"

namespace maxk {

size_t acc_bytes(int acc);


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

__global__ void invert_perm_kernel(const int32_t* __restrict__ perm, int64_t E,
                                   int32_t* __restrict__ inv) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < E;
       j += (int64_t)gridDim.x * blockDim.x)
    inv[perm[j]] = (int32_t)j;
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

__global__ void gather_bwd_kernel(const int32_t* __restrict__ perm,
                                  const int32_t* __restrict__ row_of,
                                  const int32_t* __restrict__ idx,
                                  const float* __restrict__ val, int64_t E,
                                  int32_t* __restrict__ brow, int32_t* __restrict__ bcol,
                                  float* __restrict__ bval, const int32_t* __restrict__ colpos) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < E;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int32_t e = perm[j];
    if (brow) brow[j] = row_of[e];
    if (bcol) bcol[j] = colpos ? colpos[idx[e]] : idx[e];  // the column's block position
    bval[j] = val ? val[e] : 1.0f;
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

// Backward chunk boundaries: for block b (edges [boffs[b], boffs[b+1]) sorted by row) and row
// bound j, the first edge of the block whose row is >= rows[j].
__global__ void chunk_offsets_kernel(const int32_t* __restrict__ erow,
                                     const int32_t* __restrict__ boffs, int nblocks,
                                     const int32_t* __restrict__ rows, int nb,
                                     int32_t* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nblocks * nb) return;
  const int b = t / nb, j = t - b * nb;
  int64_t lo = boffs[b], hi = boffs[b + 1];
  const int32_t r = rows[j];
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (erow[mid] < r) lo = mid + 1; else hi = mid;
  }
  out[t] = (int32_t)lo;
}

// Packed backward records {row * D * 4 (byte offset of the grad_out row), column within the
// block, val}; with perm != nullptr only the val field is refreshed from the CSR order.
__global__ void build_bwd_rec_kernel(const int32_t* __restrict__ perm,
                                     const int32_t* __restrict__ row,
                                     const int32_t* __restrict__ col,
                                     const float* __restrict__ val, int64_t E, int C, int D,
                                     uint32_t* __restrict__ rec) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {  // grid_for caps the grid
    if (perm) {
      rec[3 * e + 2] = __float_as_uint(val[perm[e]]);
      continue;
    }
    rec[3 * e] = (uint32_t)row[e] * (uint32_t)D * 4u;
    rec[3 * e + 1] = (uint32_t)(col[e] % C);
    rec[3 * e + 2] = __float_as_uint(val[e]);
  }
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

// ---------------------------------------------------------------------------------------
// Cost-balanced backward chunks (bwd_chunk_bounds 3). An edge costs 4 quarter-units; the first
// edge of every (column block, destination row) run costs rc4 more: the block's gathers fetch
// that row's grad_out lines once per pair, so a task's time follows its edges plus its pairs
// (a row with 110 edges into a block - an ID-ordered community - costs about as much as 4
// rows with one edge each). cost[e] is written in place and prefix-summed (hipcub).
__global__ void bwd_cost_kernel(const uint32_t* __restrict__ bkey, const int32_t* __restrict__ row,
                                int64_t E, int rc4, int64_t* __restrict__ cost) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    const bool first = e == 0 || bkey[e] != bkey[e - 1] || row[e] != row[e - 1];
    cost[e] = 4 + (first ? rc4 : 0);
  }
}

__global__ void gather_i32_kernel(const int32_t* __restrict__ src, const int32_t* __restrict__ at,
                                  int n, int32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = src[at[i]];
}

// out[i] = first e in [lo[i], hi[i]) with cum[e] > target[i] (hi[i] if none); cum ascends.
__global__ void upper_bound_kernel(const int64_t* __restrict__ cum, const int64_t* __restrict__ target,
                                   const int64_t* __restrict__ lo, const int64_t* __restrict__ hi,
                                   int n, int32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t a = lo[i], b = hi[i];
  const int64_t t = target[i];
  while (a < b) {
    const int64_t m = (a + b) >> 1;
    if (cum[m] > t) b = m; else a = m + 1;
  }
  out[i] = (int32_t)a;
}

// cum[offs[b] - 1] (0 for offs[b] == 0): the cost of all blocks before b.
__global__ void block_cost_kernel(const int64_t* __restrict__ cum, const int32_t* __restrict__ offs,
                                  int nb, int64_t* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > nb) return;
  out[b] = offs[b] > 0 ? cum[offs[b] - 1] : 0;
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
// Column orders of the backward blocks (maxk_plan_options.col_order).
//
// Scattered (2): p -> column (a p + b) mod NC with gcd(a, NC) = 1, a ~ 0.618 NC: every
// contiguous range of positions (a block) takes columns spread evenly over the ID range, so a
// community of consecutive IDs is shared by all blocks instead of filling a few of its own.
__global__ void affine_order_kernel(int NC, int64_t a, int64_t b, int32_t* __restrict__ order) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= NC) return;
  order[p] = (int32_t)((a * (int64_t)p + b) % NC);
}

__global__ void invert_order_kernel(const int32_t* __restrict__ order, int NC,
                                    int32_t* __restrict__ pos) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < NC) pos[order[p]] = p;
}

// Clustered (3): a spectral embedding of the columns by subspace iteration on M^T M, M the
// row-normalised adjacency: X <- centre(normalise(M^T (M X))), kEmbedDims random +-1 starting
// vectors, kEmbedIters rounds. After a few rounds X lies in the span of the leading
// eigenvectors, where columns that appear in the same rows (a community) sit close together;
// a Morton sort of the quantised coordinates then puts them at neighbouring positions, i.e.
// in the same blocks. On graphs without such structure the order is as good as random.
constexpr int kEmbedDims = 8;
constexpr int kEmbedIters = 3;

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__global__ void embed_init_kernel(int NC, float* __restrict__ X) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)NC * kEmbedDims) return;
  X[i] = (mix32((uint32_t)i * 2654435761u + 97u) & 1u) ? 1.f : -1.f;
}

// out[r] = mean over the edges (r, c) of in[c] (one wavefront per row; lanes stride over the
// row's edges, each holding kEmbedDims partial sums, then a shuffle reduction).
__global__ __launch_bounds__(256) void embed_spmm_kernel(const int32_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ nbr, int N,
                                                         const float* __restrict__ in,
                                                         float* __restrict__ out) {
  const int lane = threadIdx.x & (kWave - 1);
  const int r = blockIdx.x * (256 / kWave) + threadIdx.x / kWave;
  if (r >= N) return;
  const int e0 = ptr[r], e1 = ptr[r + 1];
  float a[kEmbedDims];
#pragma unroll
  for (int j = 0; j < kEmbedDims; ++j) a[j] = 0.f;
  for (int e = e0 + lane; e < e1; e += kWave) {
    const float4* x = reinterpret_cast<const float4*>(in + (size_t)nbr[e] * kEmbedDims);
    const float4 u = x[0], v = x[1];
    a[0] += u.x; a[1] += u.y; a[2] += u.z; a[3] += u.w;
    a[4] += v.x; a[5] += v.y; a[6] += v.z; a[7] += v.w;
  }
#pragma unroll
  for (int j = 0; j < kEmbedDims; ++j)
    for (int o = kWave / 2; o > 0; o >>= 1) a[j] += __shfl_xor(a[j], o);
  if (lane < kEmbedDims) {
    float s = a[0];
#pragma unroll
    for (int j = 1; j < kEmbedDims; ++j) s = lane == j ? a[j] : s;
    out[(size_t)r * kEmbedDims + lane] = e1 > e0 ? s / (float)(e1 - e0) : 0.f;
  }
}

// Per-dimension sums and sums of squares (atomics per work-group) for centring/normalising.
__global__ __launch_bounds__(256) void embed_moments_kernel(const float* __restrict__ X, int NC,
                                                            float* __restrict__ mom) {
  __shared__ float sh[2 * kEmbedDims];
  if (threadIdx.x < 2 * kEmbedDims) sh[threadIdx.x] = 0.f;
  __syncthreads();
  const int j = threadIdx.x & (kEmbedDims - 1);
  float s = 0.f, q = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)NC * kEmbedDims;
       i += (int64_t)gridDim.x * blockDim.x) {  // blockDim % kEmbedDims == 0: i % 8 == j
    const float x = X[i];
    s += x;
    q += x * x;
  }
  atomicAdd(&sh[j], s);
  atomicAdd(&sh[kEmbedDims + j], q);
  __syncthreads();
  if (threadIdx.x < 2 * kEmbedDims) atomicAdd(&mom[threadIdx.x], sh[threadIdx.x]);
}

__global__ void embed_normalise_kernel(float* __restrict__ X, int NC, const float* __restrict__ mom) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)NC * kEmbedDims) return;
  const int j = (int)(i & (kEmbedDims - 1));
  const float mu = mom[j] / NC;
  const float var = fmaxf(mom[kEmbedDims + j] / NC - mu * mu, 0.f);
  X[i] = (X[i] - mu) * (var > 0.f ? rsqrtf(var) : 0.f);
}

// 64-bit Morton key of the 8 coordinates quantised to 8 bits (+-4 standard deviations).
__global__ void embed_morton_kernel(const float* __restrict__ X, int NC, uint64_t* __restrict__ key,
                                    int32_t* __restrict__ ids) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= NC) return;
  uint64_t k = 0;
  uint32_t q[kEmbedDims];
#pragma unroll
  for (int j = 0; j < kEmbedDims; ++j) {
    const float v = X[(size_t)c * kEmbedDims + j] * 32.f + 128.f;
    q[j] = (uint32_t)fminf(fmaxf(v, 0.f), 255.f);
  }
#pragma unroll
  for (int b = 7; b >= 0; --b)
#pragma unroll
    for (int j = 0; j < kEmbedDims; ++j) k = (k << 1) | ((q[j] >> b) & 1u);
  key[c] = k;
  ids[c] = c;
}

static void dfree(void* q) { if (q) (void)hipFree(q); }

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
  dfree(p->bwd_row);
  dfree(p->bwd_col);
  dfree(p->bwd_val);
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

// Column order of the backward blocks (col_order 2 scattered, 3 clustered, 4 the caller's):
// *order = device int32 [NC], order[p] = column at position p. row_of: row of each CSR edge.
static hipError_t build_col_order(int mode, const int32_t* ptr, const int32_t* idx,
                                  const int32_t* row_of, int N, int NC, int64_t E,
                                  const int32_t* user, hipStream_t s, int32_t** order) {
  hipError_t e = hipMalloc(order, sizeof(int32_t) * (size_t)NC);
  if (e != hipSuccess) return e;
  const int g = (NC + 255) / 256;
  if (mode == 4) return hipMemcpyAsync(*order, user, sizeof(int32_t) * (size_t)NC,
                                       hipMemcpyDeviceToDevice, s);
  if (mode == 2 || E == 0) {
    // a ~ 0.618 NC, coprime with NC (b: a fixed offset)
    int64_t a = std::max<int64_t>(1, (int64_t)(0.6180339887 * NC));
    auto gcd = [](int64_t x, int64_t y) { while (y) { const int64_t t = x % y; x = y; y = t; } return x; };
    while (gcd(a, NC) != 1) ++a;
    hipLaunchKernelGGL(affine_order_kernel, dim3(g), dim3(256), 0, s, NC, a % NC,
                       (int64_t)(NC / 3), *order);
    return hipGetLastError();
  }
  // clustered: column CSR (rows sorted by column), subspace iteration, Morton sort
  uint32_t *kin = nullptr, *kout = nullptr;
  int32_t *crow = nullptr, *cptr = nullptr, *ids = nullptr;
  float *X = nullptr, *Y = nullptr, *mom = nullptr;
  uint64_t *mk = nullptr, *mk2 = nullptr;
  void* tmp = nullptr;
  auto cleanup = [&]() {
    dfree(kin); dfree(kout); dfree(crow); dfree(cptr); dfree(ids); dfree(X); dfree(Y);
    dfree(mom); dfree(mk); dfree(mk2); dfree(tmp);
  };
#define ORD_TRY(x)                      \
  do {                                  \
    const hipError_t e_ = (x);          \
    if (e_ != hipSuccess) {             \
      cleanup();                        \
      return e_;                        \
    }                                   \
  } while (0)
  int cbits = 1;
  while ((1ll << cbits) < (long long)NC) ++cbits;
  ORD_TRY(hipMalloc(&kin, sizeof(uint32_t) * E));
  ORD_TRY(hipMalloc(&kout, sizeof(uint32_t) * E));
  ORD_TRY(hipMalloc(&crow, sizeof(int32_t) * E));
  ORD_TRY(hipMemcpyAsync(kin, idx, sizeof(int32_t) * E, hipMemcpyDeviceToDevice, s));
  size_t tb = 0;
  ORD_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kout, row_of, crow, (int)E, 0, cbits, s));
  ORD_TRY(hipMalloc(&tmp, std::max<size_t>(tb, 16)));
  ORD_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, kin, kout, row_of, crow, (int)E, 0, cbits, s));
  ORD_TRY(hipMalloc(&cptr, sizeof(int32_t) * ((size_t)NC + 1)));
  hipLaunchKernelGGL(key_offsets_kernel, dim3(NC / 256 + 1), dim3(256), 0, s, kout, E, NC, cptr);
  ORD_TRY(hipGetLastError());
  dfree(kin); kin = nullptr;
  ORD_TRY(hipMalloc(&X, sizeof(float) * kEmbedDims * (size_t)NC));
  ORD_TRY(hipMalloc(&Y, sizeof(float) * kEmbedDims * (size_t)std::max(N, 1)));
  ORD_TRY(hipMalloc(&mom, sizeof(float) * 2 * kEmbedDims));
  const int gx = (int)(((int64_t)NC * kEmbedDims + 255) / 256);
  hipLaunchKernelGGL(embed_init_kernel, dim3(gx), dim3(256), 0, s, NC, X);
  for (int it = 0; it < kEmbedIters; ++it) {
    hipLaunchKernelGGL(embed_spmm_kernel, dim3((N + 3) / 4), dim3(256), 0, s, ptr, idx, N, X, Y);
    hipLaunchKernelGGL(embed_spmm_kernel, dim3((NC + 3) / 4), dim3(256), 0, s, cptr, crow, NC, Y, X);
    ORD_TRY(hipMemsetAsync(mom, 0, sizeof(float) * 2 * kEmbedDims, s));
    hipLaunchKernelGGL(embed_moments_kernel, dim3(std::min(gx, 1024)), dim3(256), 0, s, X, NC, mom);
    hipLaunchKernelGGL(embed_normalise_kernel, dim3(gx), dim3(256), 0, s, X, NC, mom);
    ORD_TRY(hipGetLastError());
  }
  ORD_TRY(hipMalloc(&mk, sizeof(uint64_t) * NC));
  ORD_TRY(hipMalloc(&mk2, sizeof(uint64_t) * NC));
  ORD_TRY(hipMalloc(&ids, sizeof(int32_t) * NC));
  hipLaunchKernelGGL(embed_morton_kernel, dim3(g), dim3(256), 0, s, X, NC, mk, ids);
  ORD_TRY(hipGetLastError());
  size_t tb2 = 0;
  ORD_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, mk, mk2, ids, *order, NC, 0, 64, s));
  if (tb2 > tb) {
    dfree(tmp);
    tmp = nullptr;
    ORD_TRY(hipMalloc(&tmp, tb2));
  }
  ORD_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb2, mk, mk2, ids, *order, NC, 0, 64, s));
  ORD_TRY(hipStreamSynchronize(s));
  cleanup();
#undef ORD_TRY
  return hipSuccess;
}

// Forward task list from a host copy of ptr.
static void build_fwd_tasks(const std::vector<int32_t>& hp, int N, int R, int64_t cap_opt,
                            std::vector<FwdTask>& tasks, std::vector<int32_t>& zero_rows) {
  const int64_t E = hp[N];
  const int ntiles = (N + R - 1) / R;
  const int64_t avg = ntiles ? (E + ntiles - 1) / ntiles : 0;
  // 2 x the average tile (was 4 x): heavy tiles split into a few more tasks balance the tail
  // (an 8-GPU row shard of Reddit 0.203 -> 0.195 ms; Reddit k = 8 0.925 -> 0.911, k = 16,
  // ogbn-products and ogbn-proteins within noise)
  const int64_t cap = cap_opt > 0 ? cap_opt : std::max<int64_t>(4096, 2 * avg);
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
  // the version-1 layout: a binding of ABI 1 passes a struct of exactly these bytes
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

static int plan_create_impl(const int32_t* ptr, const int32_t* idx, const float* val, int32_t N,
                            int32_t NC, int64_t E, int32_t D, int32_t k,
                            const maxk_plan_options& o, const int32_t* user_order, void* stream,
                            maxk_plan** out_plan) {
  MAXK_CHECK_ARG(o.fwd_tile_rows >= 0 && o.fwd_tile_rows <= kFwdMaxTileRows,
                 "maxk_plan_create: fwd_tile_rows must be in [0, 32]");
  MAXK_CHECK_ARG(o.fwd_accumulator >= 0 && o.fwd_accumulator <= MAXK_ACC_F32_CAS &&
                     o.bwd_accumulator >= 0 && o.bwd_accumulator <= MAXK_ACC_F32_CAS,
                 "maxk_plan_create: unknown accumulator kind");
  MAXK_CHECK_ARG(o.fwd_fixed >= 0 && o.fwd_fixed <= 2,
                 "maxk_plan_create: fwd_fixed must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.bwd_row_cost >= 0 && o.bwd_row_cost <= 4096,
                 "maxk_plan_create: bwd_row_cost must be in [0, 4096]");
  MAXK_CHECK_ARG(o.col_order >= 0 && o.col_order <= 4,
                 "maxk_plan_create: col_order must be 0 .. 4");
  MAXK_CHECK_ARG(o.col_order != 4 || user_order != nullptr || NC == 0,
                 "maxk_plan_create: col_order 4 needs the col_order argument");
  MAXK_CHECK_ARG(o.bwd_tp_chunks >= 0, "maxk_plan_create: bwd_tp_chunks must be >= 0");
  MAXK_CHECK_ARG(o.bwd_row_order >= 0 && o.bwd_row_order <= 2,
                 "maxk_plan_create: bwd_row_order must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.bwd_tp_store >= 0 && o.bwd_tp_store <= 2,
                 "maxk_plan_create: bwd_tp_store must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.bwd_lds_bytes >= 0 && o.bwd_lds_bytes <= 160 * 1024 &&
                     o.bwd_tasks_per_cu >= 0 && o.fwd_task_cap >= 0 && o.fwd_phases >= 0 &&
                     o.bwd_min_task_edges >= 0 &&
                     o.fwd_phases <= 64,
                 "maxk_plan_create: bad option value");
  *out_plan = nullptr;
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

  MAXK_CHECK_ARG((o.fwd_unroll == 0 || o.fwd_unroll == 8 || o.fwd_unroll == 16) &&
                     (o.bwd_unroll == 0 || o.bwd_unroll == 4 || o.bwd_unroll == 8 ||
                      o.bwd_unroll == 12 || o.bwd_unroll == 16),
                 "maxk_plan_create: unroll must be 0, 8 or 16 (backward also 4 or 12)");
  MAXK_CHECK_ARG(o.bwd_algo >= 0 && o.bwd_algo <= 3,
                 "maxk_plan_create: bwd_algo must be 0 (auto), 1 (column blocks), 2 (CSC) or 3 "
                 "(two-pass)");
  MAXK_CHECK_ARG(o.fwd_rotate >= 0 && o.fwd_rotate <= 2,
                 "maxk_plan_create: fwd_rotate must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.bwd_sel_lds >= 0 && o.bwd_sel_lds <= 2,
                 "maxk_plan_create: bwd_sel_lds must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.quad_loads >= 0 && o.quad_loads <= 2,
                 "maxk_plan_create: quad_loads must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.bwd_cas64 >= 0 && o.bwd_cas64 <= 2,
                 "maxk_plan_create: bwd_cas64 must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.bwd_acc_pad >= 0 && o.bwd_acc_pad <= 2,
                 "maxk_plan_create: bwd_acc_pad must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.bwd_order == 0 || o.bwd_order == 1,
                 "maxk_plan_create: bwd_order must be 0 or 1");
  MAXK_CHECK_ARG(o.bwd_slot_groups >= 0 && o.bwd_slot_groups <= 64 &&
                     (o.bwd_slot_groups & (o.bwd_slot_groups - 1)) == 0,
                 "maxk_plan_create: bwd_slot_groups must be 0 or a power of two <= 64");
  MAXK_CHECK_ARG((o.fwd_waves == 0 || o.fwd_waves == 4 || o.fwd_waves == 6 || o.fwd_waves == 8) &&
                     (o.bwd_waves == 0 || o.bwd_waves == 8 || o.bwd_waves == 12 ||
                      o.bwd_waves == 16),
                 "maxk_plan_create: fwd_waves must be 0, 4, 6 or 8 and bwd_waves 0, 8, 12 or 16");
  MAXK_CHECK_ARG(o.fwd_prefetch >= 0 && o.fwd_prefetch <= 2 && o.bwd_prefetch >= 0 &&
                     o.bwd_prefetch <= 2 && o.fwd_branchless >= 0 && o.fwd_branchless <= 2,
                 "maxk_plan_create: fwd_prefetch / bwd_prefetch / fwd_branchless must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.fwd_record_bytes == 0 ||
                     (o.fwd_record_bytes % 16 == 0 &&
                      (o.fwd_chunk3 == 1 || (o.fwd_record_bytes >= 5 * k && k % 4 == 0))),
                 "maxk_plan_create: fwd_record_bytes must be 0 or a multiple of 16 >= 5k");
  MAXK_CHECK_ARG(o.fwd_chunk3 >= 0 && o.fwd_chunk3 <= 2, "maxk_plan_create: fwd_chunk3 must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.bwd_features_per_lane == 0 || o.bwd_features_per_lane == 1 ||
                     (o.bwd_features_per_lane == 2 && k % 2 == 0) ||
                     (o.bwd_features_per_lane == 4 && k % 4 == 0),
                 "maxk_plan_create: bwd_features_per_lane must be 0, 1, 2 (k % 2 == 0) or 4 (k % 4 == 0)");
  MAXK_CHECK_ARG(o.fwd_two_tables >= 0 && o.fwd_two_tables <= 2,
                 "maxk_plan_create: fwd_two_tables must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.external_workspace == 0 || o.external_workspace == 1,
                 "maxk_plan_create: external_workspace must be 0 or 1");
  MAXK_CHECK_ARG(o.bwd_flush >= 0 && o.bwd_flush <= 2,
                 "maxk_plan_create: bwd_flush must be 0, 1 or 2");
  MAXK_CHECK_ARG(o.bwd_piece_edges >= 0, "maxk_plan_create: bwd_piece_edges must be >= 0");
  MAXK_CHECK_ARG(o.bwd_chunk_bounds >= 0 && o.bwd_chunk_bounds <= 3,
                 "maxk_plan_create: bwd_chunk_bounds must be 0, 1, 2 or 3");
  maxk_plan* p = new maxk_plan();
  p->external_ws = o.external_workspace;
  p->num_nodes = N;
  p->num_cols = NC;
  p->num_edges = E;
  p->dim_origin = D;
  p->dim_k = k;
  p->src_ptr = ptr;
  p->src_idx = idx;
  p->fwd_tile_rows = o.fwd_tile_rows ? o.fwd_tile_rows : kFwdTileRows;
  p->fwd_unroll = o.fwd_unroll ? o.fwd_unroll : kFwdUnroll;
  p->bwd_unroll = o.bwd_unroll ? o.bwd_unroll : kBwdUnroll;
  // defaults measured on the Reddit-shaped graph (tools/sweep.py, profiles/r01)
  p->fwd_waves = o.fwd_waves ? o.fwd_waves : kFwdWaves;
  p->bwd_waves = o.bwd_waves ? o.bwd_waves : (k >= 32 ? 12 : kBwdWaves);
  p->fwd_prefetch = o.fwd_prefetch == 1;
  p->bwd_prefetch = o.bwd_prefetch == 1;
  // lane-chunk records by default where the 4-values-per-lane layout fits k badly (Reddit:
  // k = 8 0.95 vs 1.02 ms, k = 24 1.93 vs 2.09 ms; k = 16 / 32 / 64 are slower with chunks),
  // and for every k % 4 != 0 (the alternative is the 1-feature-per-lane kernel)
  p->fwd_chunk3 = (o.fwd_chunk3 == 1 || (o.fwd_chunk3 == 0 && k % 16 != 0)) && (k + 2) / 3 <= kWave;
  p->fwd_branchless = o.fwd_branchless == 0 ? (k >= 16 || p->fwd_chunk3) : (o.fwd_branchless == 1);
  {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
        prop.multiProcessorCount > 0)
      p->cus = prop.multiProcessorCount;
  }
  p->fwd_acc = o.fwd_accumulator ? o.fwd_accumulator : MAXK_ACC_F64;
  // Fixed-point forward (LdsFix; the packed 4-values-per-lane and lane-chunk kernels with the
  // f64 kind). Measured (tools/fwd_fixed_sweep.py, fixed vs f64 ms): Reddit k = 16 1.22 / 1.34,
  // k = 24 1.57 / 1.95, k = 32 1.80 / 2.46, k = 64 3.45 / 4.81; ogbn-proteins k = 16 0.80 / 0.93,
  // k = 64 2.22 / 3.37. Not by default at k < 16 (Reddit k = 8 0.93 / 0.91, the stats pass
  // included) or on tables past the packed-record thresholds, whose gathers are HBM-bound
  // (ogbn-products k = 16 3.14 / 3.02, k = 32 4.86 / 4.78).
  {
    const bool big = (double)std::max(NC, 1) * 5.0 * k >
                     (k >= 32 ? kFwdPackedTableBytes : kFwdPackedTableBytes16);
    p->fwd_fixed = (o.fwd_fixed == 1 || (o.fwd_fixed == 0 && k >= 16 && !big)) &&
                   p->fwd_acc == MAXK_ACC_F64 && (k % 4 == 0 || p->fwd_chunk3);
  }
  p->bwd_acc = o.bwd_accumulator ? o.bwd_accumulator : MAXK_ACC_F32_CAS;
  // k = 8: two slots per lane, so a gather instruction covers 16 edges (4 lanes per edge)
  // instead of 32, when a column block sees few edges per grad_out row (32 edges then span
  // ~4 rows: Reddit, 7.7 edges per (block, row), 1.151 -> 1.125 ms with unroll 12); with
  // more (ogbn-proteins, 15) the 32 edges share ~2 rows and 4 slots per lane stay faster
  // (0.831 vs 0.877 ms). Edges per (block, row) estimated from the LDS budget.
  bool two_slots = false;
  if (k == 8 && N > 0 && NC > 0) {
    const int lds0 = o.bwd_lds_bytes ? o.bwd_lds_bytes : kBwdLdsBudget;
    const double c0 = std::min<double>(NC, (lds0 - 16) / (5.0 * k));
    two_slots = (double)E / N * c0 / NC < 10.0;
  }
  p->bwd_feats = o.bwd_features_per_lane ? o.bwd_features_per_lane
                                         : (two_slots ? 2 : (k % 4 == 0 ? 4 : 1));
  if (p->bwd_feats == 2 && o.bwd_unroll == 0) p->bwd_unroll = 12;

  int32_t* row_of = nullptr;
  uint32_t* keys_in = nullptr;
  uint32_t* keys_out = nullptr;
  int32_t* ids_in = nullptr;
  void* temp = nullptr;
  int64_t* d_offs = nullptr;
  int* d_bad = nullptr;
  int32_t* order = nullptr;   // column order: position -> column (col_order 2..4)
  int32_t* colpos = nullptr;  // column -> position
  auto fail = [&](int rc) {
    dfree(order);
    dfree(colpos);
    dfree(row_of);
    dfree(keys_in);
    dfree(keys_out);
    dfree(ids_in);
    dfree(temp);
    dfree(d_offs);
    dfree(d_bad);
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
  // ---------------- column order (col_order 2 scattered, 3 clustered, 4 the caller's): the
  // backward's packed kernels take their column blocks as position ranges of it. The forward
  // keeps its column-sorted sweep: sweeping in the clustered order measured much slower
  // (shuffled 41-community Reddit-size graph: k = 16 1.07 -> 1.36 ms, k = 32 1.61 -> 2.75)
  const int order_mode = o.col_order == 0 ? 1 : o.col_order;
  if (order_mode >= 2 && NC > 0) {
    if (E > 0) {
      PLAN_TRY(hipMalloc(&row_of, sizeof(int32_t) * E));
      hipLaunchKernelGGL(expand_rows_kernel, dim3((N + 3) / 4), dim3(256), 0, s, ptr, N, row_of);
      PLAN_TRY(hipGetLastError());
    }
    PLAN_TRY(build_col_order(order_mode, ptr, idx, row_of, N, NC, E, user_order, s, &order));
    PLAN_TRY(hipMalloc(&colpos, sizeof(int32_t) * NC));
    PLAN_TRY(hipMemsetAsync(colpos, 0xff, sizeof(int32_t) * NC, s));
    hipLaunchKernelGGL(invert_order_kernel, dim3((NC + 255) / 256), dim3(256), 0, s, order, NC, colpos);
    PLAN_TRY(hipGetLastError());
    if (order_mode == 4) {  // the caller's order must be a permutation of [0, NC)
      std::vector<int32_t> ho(NC), hc(NC);
      PLAN_TRY(hipMemcpyAsync(ho.data(), order, sizeof(int32_t) * NC, hipMemcpyDeviceToHost, s));
      PLAN_TRY(hipStreamSynchronize(s));
      bool ok = true;
      for (int i = 0; i < NC && ok; ++i) ok = ho[i] >= 0 && ho[i] < NC;
      if (ok) {
        PLAN_TRY(hipMemcpyAsync(hc.data(), colpos, sizeof(int32_t) * NC, hipMemcpyDeviceToHost, s));
        PLAN_TRY(hipStreamSynchronize(s));
        for (int i = 0; i < NC && ok; ++i) ok = hc[i] >= 0 && ho[hc[i]] == i;
      }
      if (!ok) {
        set_error("maxk_plan_create: col_order is not a permutation of [0, num_cols)");
        return fail(MAXK_ERR_INVALID_ARG);
      }
    }
  }
  auto drop_order = [&]() {
    dfree(order);
    dfree(colpos);
    order = colpos = nullptr;
  };

  std::vector<FwdTask> ftasks;
  std::vector<int32_t> zrows;
  build_fwd_tasks(hp, N, p->fwd_tile_rows, o.fwd_task_cap, ftasks, zrows);
  p->n_fwd_tasks = (int32_t)ftasks.size();
  p->n_zero_rows = (int32_t)zrows.size();
  if (!ftasks.empty()) {
    // permuted edge order (see fwd_key_kernel): tasks keep their CSR edge sets
    const int nt = (int)ftasks.size();
    std::vector<int32_t> order(nt);
    for (int i = 0; i < nt; ++i) order[i] = i;
    // by first edge, and among equal first edges the empty tasks (an edgeless tile shares its
    // e0 with the next tile) before the one task that owns edges there: fwd_key_kernel takes
    // the LAST task whose first edge is <= e (an edgeless tile ordered last took the next
    // tile's edges, whose rows then stayed zero: tests/test_gpu_fuzz.py)
    std::sort(order.begin(), order.end(), [&](int a, int b) {
      if (ftasks[a].e0 != ftasks[b].e0) return ftasks[a].e0 < ftasks[b].e0;
      return ftasks[a].e1 < ftasks[b].e1;
    });
    std::vector<int32_t> starts(nt), ranks(nt), row0s(nt);
    for (int i = 0; i < nt; ++i) {
      starts[i] = ftasks[order[i]].e0;
      ranks[i] = order[i];
      row0s[i] = ftasks[order[i]].row0;
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
      auto fwd_cleanup = [&]() {
        dfree(d_starts); dfree(d_ranks); dfree(d_row0s); dfree(d_rl); dfree(d_ids);
        dfree(d_kin); dfree(d_kout); dfree(d_tmp);
      };
#define FWD_TRY(expr)                         \
  do {                                        \
    hipError_t _e2 = (expr);                  \
    if (_e2 != hipSuccess) {                  \
      fwd_cleanup();                          \
      PLAN_TRY(_e2);                          \
    }                                         \
  } while (0)
      if (!row_of) {
        FWD_TRY(hipMalloc(&row_of, sizeof(int32_t) * E));
        hipLaunchKernelGGL(expand_rows_kernel, dim3((N + 3) / 4), dim3(256), 0, s, ptr, N, row_of);
      }
      FWD_TRY(hipMalloc(&d_starts, sizeof(int32_t) * nt));
      FWD_TRY(hipMalloc(&d_ranks, sizeof(int32_t) * nt));
      FWD_TRY(hipMalloc(&d_row0s, sizeof(int32_t) * nt));
      FWD_TRY(hipMemcpyAsync(d_starts, starts.data(), sizeof(int32_t) * nt, hipMemcpyHostToDevice, s));
      FWD_TRY(hipMemcpyAsync(d_ranks, ranks.data(), sizeof(int32_t) * nt, hipMemcpyHostToDevice, s));
      FWD_TRY(hipMemcpyAsync(d_row0s, row0s.data(), sizeof(int32_t) * nt, hipMemcpyHostToDevice, s));
      FWD_TRY(hipMalloc(&d_rl, sizeof(int32_t) * E));
      FWD_TRY(hipMalloc(&d_ids, sizeof(int32_t) * E));
      FWD_TRY(hipMalloc(&d_kin, sizeof(uint64_t) * E));
      FWD_TRY(hipMalloc(&d_kout, sizeof(uint64_t) * E));
      FWD_TRY(hipMalloc(&p->fwd_perm, sizeof(int32_t) * E));
      hipLaunchKernelGGL(fwd_key_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s, idx, row_of, E,
                         d_starts, d_ranks, d_row0s, nt, cbits, d_kin, d_ids, d_rl);
      FWD_TRY(hipGetLastError());
      size_t tb = 0;
      FWD_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, d_kin, d_kout, d_ids, p->fwd_perm,
                                                 (int)E, 0, cbits + tbits, s));
      FWD_TRY(hipMalloc(&d_tmp, tb));
      FWD_TRY(hipcub::DeviceRadixSort::SortPairs(d_tmp, tb, d_kin, d_kout, d_ids, p->fwd_perm,
                                                 (int)E, 0, cbits + tbits, s));
      FWD_TRY(hipMalloc(&p->fwd_cv, sizeof(uint2) * E));
      hipLaunchKernelGGL(gather_fwd_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s, p->fwd_perm,
                         idx, d_rl, val, E, p->fwd_cv, true);
      FWD_TRY(hipGetLastError());
      FWD_TRY(hipStreamSynchronize(s));
      fwd_cleanup();
#undef FWD_TRY
      p->device_bytes += (int64_t)E * 12;
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
    // Column windows. Default: one launch whose tiles start their column-sorted sweep at the
    // window a shared clock points to (fwd_rot_ticks per window, about one tile's duration
    // per full turn), so the tiles running together on an XCD gather from nearby columns
    // (L2 reuse). fwd_phases > 1 instead runs the windows as separate launches.
    int B = o.fwd_phases;
    p->fwd_persistent = o.fwd_persistent ? 1 : 0;
    p->fwd_rot_ticks = 0;
    if (B <= 1 && o.fwd_rotate != 2 && (k % 4 == 0 || p->fwd_chunk3) && nt > 0) {
      // the fixed-point kernel sweeps faster: more windows at large k, a higher slot rate
      // (tools/fwd_opts_sweep.py, Reddit: k = 16 1.23 -> 1.19 ms with 260 M edges/s per slot,
      // k = 32 1.81 -> 1.77 with 140 M and 32 windows, k = 64 3.44 -> 3.23 with 64 windows)
      const int Bd = p->fwd_fixed ? (k >= 64 ? 64 : k >= 32 ? 32 : kFwdRotWindows) : kFwdRotWindows;
      B = o.fwd_rot_windows > 0 ? std::min(o.fwd_rot_windows, 64) : Bd;
      // one turn of the clock per tile: the measured per-slot rate scales as ~1/k (Reddit:
      // 2.4e8, 1.65e8, 0.9e8 edges/s per slot at k = 8, 16, 32; best sweep rates 300, 150-200,
      // 100 M)
      const double rate = o.fwd_rot_rate > 0 ? o.fwd_rot_rate * 1e6
                                             : std::min(5e8, std::max(2e7, (p->fwd_fixed ? kFwdSlotEdgeRateFixed : kFwdSlotEdgeRate) * 16.0 / k));
      const double tile_edges = (double)E / nt;
      const double tile_ticks = tile_edges / rate * 1e8;  // s_memrealtime: 100 MHz
      p->fwd_rot_ticks = (int)std::max(1.0, tile_ticks / B);
    }
    if (B == 0) B = 1;
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
  // with an L2-resident selector table (round 3, the pack fused into the statistics pass;
  // per-rank forward on row shards at k = 16: Reddit W = 8, 62 edges per column and a 3.7 MB
  // selector table, 0.172 ms packed vs 0.183 two tables, W = 4 (123) 0.757 vs 0.805 ms for
  // the rank's whole step; ogbn-proteins W = 8, 75 edges per column and 2.1 MB of selectors,
  // 0.144 packed vs 0.138 two tables; round 2 with a separate pack: Reddit W = 8 0.221
  // packed vs 0.207). But on a large table, whose gathers mostly miss L2, the record's one line
  // beats the two tables' two (values + selectors): at k = 16 from tens of MB (yelp, 57 MB:
  // 0.645 -> 0.54 ms packed; ogbn-products, 196 MB: 4.84 -> 2.95; flickr, 7 MB at 11 edges
  // per column, stays faster with two tables), at k = 32 only from HBM-sized tables
  // (ogbn-products 392 MB: 4.95 -> 4.77; yelp 115 MB: 0.67 two tables vs 0.73); never at
  // k = 64 (ogbn-products 7.08 two tables vs 7.44)
  const bool big_table = (double)std::max(NC, 1) * 5.0 * k >
                         (k >= 32 ? kFwdPackedTableBytes : kFwdPackedTableBytes16);
  const bool sel_l2 = (double)std::max(NC, 1) * k <= kFwdSelL2Bytes;
  const bool few_edges = E < kFwdPackMinEdgesPerCol * std::max(NC, 1) ||
                         (sel_l2 && E < kFwdPackMinEdgesPerColL2 * std::max(NC, 1));
  p->fwd_two_tables = !p->fwd_chunk3 && k % 4 == 0 &&
                      (o.fwd_two_tables == 1 ||
                       (o.fwd_two_tables == 0 &&
                        (k >= 64 || (!big_table && (k >= 32 || few_edges)))));
  if (p->fwd_two_tables) {
    // no workspace: the kernel gathers from sp_data / sp_index
  } else if (p->fwd_chunk3 && NC > 0) {
    const int b = (k + 2) / 3 * 16;
    if (o.fwd_record_bytes != 0 && o.fwd_record_bytes < b) {
      set_error("maxk_plan_create: fwd_record_bytes too small for the lane-chunk records");
      return fail(MAXK_ERR_INVALID_ARG);
    }
    p->fwd_rec_bytes = o.fwd_record_bytes ? o.fwd_record_bytes
                                          : (b <= 64 ? 64 : b <= 128 ? 128 : b);
    p->fwd_ws_bytes = (int64_t)NC * p->fwd_rec_bytes;
  } else if (k % 4 == 0 && NC > 0) {
    p->fwd_rec_bytes = o.fwd_record_bytes ? o.fwd_record_bytes : cbsr_record_bytes(k);
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
  // Column blocks of C columns (k f64 accumulators each, <= kBwdLdsBudget of LDS: one
  // 512-thread work-group per CU); each block's edge range is cut into chunks so that about
  // 2 x CUs work-groups exist; blocks with several chunks flush with float atomics.
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) {
      hipDeviceProp_t prop;
      if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
        cus = prop.multiProcessorCount;
    }
  }
  const int lds_budget = o.bwd_lds_bytes ? o.bwd_lds_bytes : kBwdLdsBudget;
  // packed path (sspmm_bwd4_kernel): f32 accumulators, 4 selector slots per lane, grad_out
  // addressable with 32-bit byte offsets
  // (or sspmm_bwd1_kernel: one slot per lane, k <= 64 lanes per edge)
  const bool packed = E > 0 &&
                      ((k % 4 == 0 && p->bwd_feats == 4) || (k % 2 == 0 && p->bwd_feats == 2 && k / 2 <= kWave) ||
                       (p->bwd_feats == 1 && k <= kWave)) &&
                      p->bwd_acc == MAXK_ACC_F32_CAS &&
                      (uint64_t)N * (uint64_t)D * 4u <= 0xffffffffull;
  // Slot groups: the k selector slots are split into S groups of k/S consecutive (sorted,
  // hence clustered) slots, one work-group per (block, group). An edge then touches the
  // few grad_out lines its group's features fall in, and a block spans S times more
  // columns, so more edges share each fetched row (SSpMM is bound by L1-miss requests).
  int S = 1;
  if (packed && (p->bwd_feats == 4 || p->bwd_feats == 2)) {
    S = o.bwd_slot_groups ? o.bwd_slot_groups : kBwdSlotGroups;
    if (o.bwd_slot_groups == 0 && p->bwd_feats == 4 && k >= 32 && k % 8 == 0 && N > 0 && NC > 0) {
      // k >= 32 with few edges per (block, row): two slot groups, i.e. k/8 lanes per edge and
      // blocks of twice the columns (Reddit, ~1.9 edges per block row at k = 32: 2.88 ->
      // 2.66 ms; k = 64, ~1.0: 4.88 -> 4.71; ogbn-proteins k = 64, ~1.9: 3.32 -> 3.25). With
      // more reuse one group stays faster (ogbn-proteins k = 32, ~3.1: 1.82 vs 1.86).
      const double c1 = std::min<double>(NC, (lds_budget - 16) / (5.0 * k));
      if ((double)E / N * c1 / NC < 2.5) S = 2;
    }
    while (S > 1 && (k % (p->bwd_feats * S)) != 0) S >>= 1;
  }
  p->bwd_slot_groups = S;
  const int nslots = k / S;
  // accumulator row stride: nslots + 1 (odd: columns start on different banks) or nslots
  // 64-bit CAS pairs (sspmm_bwd4_kernel<.., V>): KS even, unpadded by default
  // (Reddit k = 16: 2.06 -> 1.78 ms; k = 8 1.24 -> 1.16; k = 32 3.21 -> 3.09)
  p->bwd_cas64 = packed && (p->bwd_feats == 4 || p->bwd_feats == 2) && o.bwd_cas64 != 2;
  // (Reddit bwd k = 16 1.76 -> 1.70 ms, k = 32 3.08 -> 2.93, k = 64 5.43 -> 4.86; the forward's
  // 8-B edge words gain nothing: forward only on request)
  p->bwd_quad = o.quad_loads != 2;
  // forward quad-shared edge-word loads: with the fixed-point kernel (k = 16 1.19 -> 1.16 ms,
  // k = 32 1.81 -> 1.78); measured neutral-to-slower on the f64 kernel
  p->fwd_quad = o.quad_loads == 1 || (o.quad_loads == 0 && p->fwd_fixed);
  if (p->bwd_cas64) p->bwd_ks = nslots + (o.bwd_acc_pad == 1 ? 4 : 0);
  else p->bwd_ks = nslots + ((packed && o.bwd_acc_pad == 2) ? 0 : 1);
  p->bwd_sel_lds = packed && o.bwd_sel_lds != 2 ? 1 : 0;
  // bytes of LDS per column: accumulators (+ staged selector bytes, nslots per column)
  const int col_bytes = p->bwd_ks * (int)acc_bytes(p->bwd_acc) + (p->bwd_sel_lds ? nslots : 0);
  int C = std::max(1, (lds_budget - 16) / col_bytes);
  C = std::min(C, std::max(NC, 1));
  // Column-major (CSC) backward, option bwd_algo = 2: one wave per column sums its in-edges
  // in registers (C = 1: the block sort becomes a column sort). Measured slower than the
  // column blocks on every graph tried, sparse ones included (ogbn-products k = 32: 17.0 vs
  // 15.0 ms): a block sweeps its edges in row order, so the work-groups resident together
  // walk the rows of G in near lock-step and share its lines in L2 and the MALL (PMC: L2 hit
  // 10-43 % vs 2 % for CSC, 7.0 vs 8.0 L2 misses per edge); a column's in-edges come from
  // anywhere. Kept as an option for that comparison.
  const int Lc = k / p->bwd_feats;  // lanes per edge of the column-major kernel
  const bool csc_ok = E > 0 && p->bwd_feats != 2 && k % p->bwd_feats == 0 && (Lc & (Lc - 1)) == 0 &&
                      Lc <= kWave &&
                      (uint64_t)N * (uint64_t)D * 4u <= 0xffffffffull;
  p->bwd_csc = csc_ok && o.bwd_algo == 2;
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
  if (p->bwd_csc || p->bwd_twopass) {
    C = 1;
    p->bwd_sel_lds = 0;
  }
  const bool colsort = p->bwd_csc || p->bwd_twopass;
  const bool xcd_order = o.bwd_order == 0 && !colsort;
  // the column order applies to the packed column-block kernels (their tasks own position
  // ranges; the column-major kernels sort by the column itself)
  const int32_t* bcolpos = (colpos && packed && !colsort) ? colpos : nullptr;
  // row order inside the blocks' streams (column-block kernels; the shared row chunk bounds
  // need ascending rows): scattered by an affine bijection ra * row + rb mod N
  const bool row_hash_ok = !colsort && E > 0 && N > 1 && o.bwd_chunk_bounds != 1;
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
  if (xcd_order && nblocks >= kXcds) {
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
  std::vector<int64_t> offs(colsort ? 1 : nblocks + 1, 0);
  p->bwd_row_order = colsort ? 0 : 1;
  if (E > 0) {
    if (!row_of) {
      PLAN_TRY(hipMalloc(&row_of, sizeof(int32_t) * E));
      hipLaunchKernelGGL(expand_rows_kernel, dim3((N + 3) / 4), dim3(256), 0, s, ptr, N, row_of);
    }
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
        if (e != hipSuccess) return e;
        e = hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, keys_in, keys_out, ids_in,
                                               p->bwd_perm, (int)E, 0, end_bit, s);
        if (e != hipSuccess) return e;
        e = hipMalloc(&temp, temp_bytes);
        if (e != hipSuccess) return e;
        return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, ids_in,
                                                  p->bwd_perm, (int)E, 0, end_bit, s);
      }
      // 64-bit keys {block, row position}; their block ids then go to keys_out
      uint64_t *k64_in = nullptr, *k64_out = nullptr;
      const hipError_t ke = [&]() -> hipError_t {
        hipError_t e = hipMalloc(&k64_in, sizeof(uint64_t) * E);
        if (e != hipSuccess) return e;
        e = hipMalloc(&k64_out, sizeof(uint64_t) * E);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(bwd_key64_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s, idx, row_of,
                           E, C, NC, k64_in, ids_in, d_bad, bcolpos, ra, rb, N, rbits);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        e = hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, k64_in, k64_out, ids_in,
                                               p->bwd_perm, (int)E, 0, end_bit + rbits, s);
        if (e != hipSuccess) return e;
        e = hipMalloc(&temp, temp_bytes);
        if (e != hipSuccess) return e;
        e = hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k64_in, k64_out, ids_in,
                                               p->bwd_perm, (int)E, 0, end_bit + rbits, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(key_block_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s, k64_out, E,
                           rbits, keys_out);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        return hipStreamSynchronize(s);
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
          if (e != hipSuccess) return e;
          e = hipMemsetAsync(d_nd, 0, sizeof(int), s);
          if (e != hipSuccess) return e;
          hipLaunchKernelGGL(dense_window_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s,
                             keys_out, p->bwd_perm, row_of, E, Wn, d_nd);
          e = hipGetLastError();
          if (e != hipSuccess) return e;
          e = hipMemcpyAsync(&nd, d_nd, sizeof(int), hipMemcpyDeviceToHost, s);
          if (e != hipSuccess) return e;
          return hipStreamSynchronize(s);
        }();
        dfree(d_nd);
        PLAN_TRY(de);
        if (nd > nw / 4) {
          row_hash = true;
          PLAN_TRY(sort_blocks(true));
        }
      }
    }
    if (!colsort) p->bwd_row_order = row_hash ? 2 : 1;
    if (p->bwd_twopass) {
      PLAN_TRY(hipMalloc(&p->bwd_erec, sizeof(uint32_t) * 2 * (size_t)E));
      p->bwd_tp_csc = o.bwd_tp_store == 2;
      // row chunks: the workspace holds one chunk's products (column order: one chunk)
      int P = o.bwd_tp_chunks > 0
                  ? o.bwd_tp_chunks
                  : (int)std::max<int64_t>(1, (int64_t)std::ceil((double)E * k * 4.0 /
                                                                  kBwdTwoPassWorkspaceCap));
      P = std::max(1, std::min(P, std::max(N, 1)));
      if (p->bwd_tp_csc) P = 1;
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
      if (p->bwd_tp_csc) {  // bwd_perm becomes CSR edge -> column-order slot
        hipLaunchKernelGGL(invert_perm_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s,
                           p->bwd_perm, E, ids_in);
        PLAN_TRY(hipMemcpyAsync(p->bwd_perm, ids_in, sizeof(int32_t) * E,
                                hipMemcpyDeviceToDevice, s));
      }
    } else {
      PLAN_TRY(hipMalloc(&p->bwd_row, sizeof(int32_t) * E));
      PLAN_TRY(hipMalloc(&p->bwd_col, sizeof(int32_t) * E));
      PLAN_TRY(hipMalloc(&p->bwd_val, sizeof(float) * E));
      p->device_bytes += (int64_t)E * 16;
      hipLaunchKernelGGL(gather_bwd_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s,
                         p->bwd_perm, row_of, idx, val, E, p->bwd_row, p->bwd_col, p->bwd_val,
                         bcolpos);
    }
    PLAN_TRY(hipMalloc(&d_offs, sizeof(int32_t) * (nblocks + 1)));
    hipLaunchKernelGGL(key_offsets_kernel, dim3(nblocks / 256 + 1), dim3(256), 0, s, keys_out,
                       E, nblocks, reinterpret_cast<int32_t*>(d_offs));
    PLAN_TRY(hipGetLastError());
    int bad = 0;
    PLAN_TRY(hipMemcpyAsync(&bad, d_bad, sizeof(int), hipMemcpyDeviceToHost, s));
    if (colsort) {
      // column pointers of the column-sorted edge list stay on the device
      p->bwd_colptr = reinterpret_cast<int32_t*>(d_offs);
      d_offs = nullptr;
      p->device_bytes += sizeof(int32_t) * (nblocks + 1);
      if (p->bwd_twopass && p->bwd_tp_chunks > 1) {
        // per-chunk column pointers (rows ascend within a column of the stable sort)
        const int P = p->bwd_tp_chunks;
        int32_t* d_rows = nullptr;
        PLAN_TRY(hipMalloc(&d_rows, sizeof(int32_t) * (P + 1)));
        const hipError_t ce = [&]() -> hipError_t {
          hipError_t e = hipMemcpyAsync(d_rows, p->tp_rows.data(), sizeof(int32_t) * (P + 1),
                                        hipMemcpyHostToDevice, s);
          if (e != hipSuccess) return e;
          e = hipMalloc(&p->bwd_colptr2, sizeof(int32_t) * (size_t)(P + 1) * NC);
          if (e != hipSuccess) return e;
          const int64_t n = (int64_t)(P + 1) * NC;
          hipLaunchKernelGGL(tp_colptr_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                             p->bwd_colptr, p->bwd_perm, row_of, NC, d_rows, P, p->bwd_colptr2);
          e = hipGetLastError();
          if (e != hipSuccess) return e;
          return hipStreamSynchronize(s);
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
  const int64_t target_tasks = (int64_t)(o.bwd_tasks_per_cu ? o.bwd_tasks_per_cu : kBwdTasksPerCu) * cus;
  const int chunks = (int)std::max<int64_t>(
      1, (target_tasks + (int64_t)nblocks * S - 1) / std::max<int64_t>((int64_t)nblocks * S, 1));
  const int64_t min_task_edges = o.bwd_min_task_edges > 0 ? o.bwd_min_task_edges : kBwdMinTaskEdges;
  std::vector<BwdTask> btasks;
  int nshared = 0;
  if (colsort) {
    // no tasks: the column-major kernels run one wave per column
  } else if (xcd_order && E > 0 && nblocks > 0) {
    // Row-chunk-major, XCD-aware order. Chunk j of a block is the j-th equal share of its
    // row-sorted edge stream (below), so on graphs without column locality chunk j of every
    // block covers about the same rows and the work-groups that run together sweep the same
    // rows of G, sharing its lines in their XCD's L2. Work-groups are dealt round-robin over
    // the 8 XCDs (blockIdx % 8 labels the work-groups sharing an XCD; speed only, correctness
    // never depends on it): XCD x owns blocks b = x (mod 8) and walks (chunk, block) in
    // chunk-major order.
    // every chunk task clears and flushes its whole block (C * k floats) however few edges
    // it has: keep >= kBwdMinTaskEdges edges per task (a row shard of a multi-GPU partition
    // has 1/W of the edges over the same blocks)
    // ... but not fewer tasks than CUs while those keep >= 4k edges (a row shard of an
    // 8-GPU partition: 256 tasks of ~56k edges ran 0.24 ms, 512 of ~28k 0.27, 128 0.40; the
    // own-column part of such a shard, 1.8 M edges over 16 blocks: 16 tasks ran 0.35 ms)
    int64_t nch64 = std::min<int64_t>(chunks, E / ((int64_t)nblocks * min_task_edges));
    const int64_t fl = ((int64_t)cus + (int64_t)nblocks * S - 1) / ((int64_t)nblocks * S);
    if (o.bwd_min_task_edges == 0 && nch64 < fl && E / ((int64_t)nblocks * fl) >= 4096)
      nch64 = std::min<int64_t>(chunks, fl);
    nch64 = std::max<int64_t>(1, nch64);
    // One 512-thread work-group per CU: a task count just past a multiple of the CUs leaves
    // the last round mostly idle (ogbn-proteins k = 32: 192 blocks x 3 chunks = 2.25 rounds,
    // 2.37 ms; x 4 = 3 rounds, 1.82 ms). With the default knobs take the chunk count in
    // [nch, nch + 2] whose tasks fill their rounds best, keeping >= 0.6 x the minimum task.
    if (o.bwd_tasks_per_cu == 0 && o.bwd_min_task_edges == 0) {
      auto fill = [&](int64_t c) {
        const int64_t t = (int64_t)nblocks * S * c;
        return (double)t / ((double)((t + cus - 1) / cus) * cus);
      };
      int64_t best = nch64;
      for (int64_t c = nch64 + 1; c <= nch64 + 2; ++c) {
        if ((double)E / ((double)nblocks * c) < 0.6 * kBwdMinTaskEdges) break;
        if (fill(c) > fill(best) + 0.05) best = c;
      }
      nch64 = best;
    }
    const int nch = (int)nch64;
    // chunk bounds per block: cbd[b] = {offs[b], ..., offs[b+1]} (nch_b + 1 entries)
    // default: equal edges (an 8-GPU row shard of Reddit, ~2 chunks per block: 0.227 ms vs
    // 0.268 with cost bounds, whose per-block chunk counts leave rounds partly idle; the
    // ID-ordered community graphs that cost bounds were built for are handled by the
    // scattered row order, with which both run the same: 1.60 / 1.61 ms at k = 16)
    const int mode = o.bwd_chunk_bounds == 0 ? 2 : o.bwd_chunk_bounds;
    p->bwd_chunk_mode = mode;
    std::vector<std::vector<int32_t>> cbd((size_t)nblocks);
    int32_t *d_rb = nullptr, *d_co = nullptr;
    int64_t *d_cum = nullptr, *d_bc = nullptr, *d_tg = nullptr, *d_lo = nullptr, *d_hi = nullptr;
    void* d_scan = nullptr;
    auto chunk_cleanup = [&]() {
      dfree(d_rb); dfree(d_co); dfree(d_cum); dfree(d_bc); dfree(d_tg); dfree(d_lo); dfree(d_hi);
      dfree(d_scan);
      d_rb = d_co = nullptr;
      d_cum = d_bc = d_tg = d_lo = d_hi = nullptr;
      d_scan = nullptr;
    };
#define CH_TRY(x)                                          \
    do {                                                   \
      hipError_t e_ = (x);                                 \
      if (e_ != hipSuccess) {                              \
        chunk_cleanup();                                   \
        PLAN_TRY(e_);                                      \
      }                                                    \
    } while (0)
    if (mode == 1) {
      // shared row bounds: chunk j of every block covers the same rows [R_j, R_j+1) (equal
      // edge counts over the whole graph)
      std::vector<int32_t> co((size_t)nblocks * (nch + 1));
      std::vector<int32_t> rb(nch + 1);
      for (int j = 0; j <= nch; ++j) {
        const int64_t target = E * j / nch;
        rb[j] = (int32_t)(std::lower_bound(hp.begin(), hp.end(), (int32_t)target) - hp.begin());
      }
      rb[0] = 0;
      rb[nch] = N;
      CH_TRY(hipMalloc(&d_rb, sizeof(int32_t) * (nch + 1)));
      CH_TRY(hipMalloc(&d_co, sizeof(int32_t) * co.size()));
      CH_TRY(hipMemcpyAsync(d_rb, rb.data(), sizeof(int32_t) * (nch + 1), hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(chunk_offsets_kernel, dim3((int)((co.size() + 255) / 256)), dim3(256), 0, s,
                         p->bwd_row, reinterpret_cast<const int32_t*>(d_offs), nblocks, d_rb,
                         nch + 1, d_co);
      CH_TRY(hipGetLastError());
      CH_TRY(hipMemcpyAsync(co.data(), d_co, sizeof(int32_t) * co.size(), hipMemcpyDeviceToHost, s));
      CH_TRY(hipStreamSynchronize(s));
      for (int b = 0; b < nblocks; ++b)
        cbd[b].assign(co.begin() + (size_t)b * (nch + 1), co.begin() + (size_t)(b + 1) * (nch + 1));
    } else if (mode == 2) {
      // per-block bounds: chunk j of block b holds edges [j, j+1) * nnz_b / nch of the block's
      // row-sorted stream. On a graph without column locality these are the shared row
      // bounds to within a few rows (the work-groups that run together still sweep the same
      // rows of G); with locality (a community linking mostly into its own blocks) every
      // task keeps an equal share instead of a few tasks carrying most of a chunk
      // (41-community Reddit-size graph, k = 16: 3.38 -> 2.18 ms)
      for (int b = 0; b < nblocks; ++b) {
        const int64_t o0 = offs[b], nnz = offs[b + 1] - offs[b];
        cbd[b].resize(nch + 1);
        for (int j = 0; j <= nch; ++j) cbd[b][j] = (int32_t)(o0 + nnz * j / nch);
      }
    } else {
      // equal cost (bwd_cost_kernel: edges + rc4/4 per (block, row) pair). A task's time
      // follows the grad_out lines it fetches, once per pair, as much as its edges: with
      // column locality (an ID-ordered community) a block's stream is a dense run of
      // community rows (~100 edges per pair) between long sparse stretches (~1 edge per pair),
      // and equal-edge chunks of it differ several-fold in time. Each block gets chunks in
      // proportion to its cost (at least nch on average), each chunk an equal share of it.
      const int rc4 = o.bwd_row_cost ? o.bwd_row_cost : kBwdRowCost4;
      CH_TRY(hipMalloc(&d_cum, sizeof(int64_t) * E));
      hipLaunchKernelGGL(bwd_cost_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s, keys_out,
                         p->bwd_row, E, rc4, d_cum);
      CH_TRY(hipGetLastError());
      size_t sb = 0;
      CH_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, sb, d_cum, d_cum, (int)E, s));
      CH_TRY(hipMalloc(&d_scan, std::max<size_t>(sb, 16)));
      CH_TRY(hipcub::DeviceScan::InclusiveSum(d_scan, sb, d_cum, d_cum, (int)E, s));
      CH_TRY(hipMalloc(&d_bc, sizeof(int64_t) * (nblocks + 1)));
      hipLaunchKernelGGL(block_cost_kernel, dim3(nblocks / 256 + 1), dim3(256), 0, s, d_cum,
                         reinterpret_cast<const int32_t*>(d_offs), nblocks, d_bc);
      CH_TRY(hipGetLastError());
      std::vector<int64_t> bc(nblocks + 1);
      CH_TRY(hipMemcpyAsync(bc.data(), d_bc, sizeof(int64_t) * (nblocks + 1), hipMemcpyDeviceToHost, s));
      CH_TRY(hipStreamSynchronize(s));
      const double tau = std::max(1.0, (double)bc[nblocks] / ((double)nblocks * nch));
      std::vector<int64_t> tg, lo, hi;
      std::vector<int32_t> nchb(nblocks);
      for (int b = 0; b < nblocks; ++b) {
        const int64_t T = bc[b + 1] - bc[b], nnz = offs[b + 1] - offs[b];
        // rounded, but no task above 1.25 tau: one work-group per CU runs the tasks in rounds,
        // so a task count past a multiple of the CUs costs a round (ceil everywhere: Reddit
        // k = 16 tasks 512 -> ~560), and a block of ~1.5 tau in one chunk stretches one
        // (rounding alone: an 8-GPU row shard, ~2 chunks per block, 0.244 -> 0.303 ms)
        int64_t c = std::max<int64_t>({(int64_t)1, (int64_t)std::llround((double)T / tau),
                                       (int64_t)std::ceil((double)T / (1.25 * tau) - 1e-9)});
        c = std::min<int64_t>(c, std::max<int64_t>(1, std::min<int64_t>(nnz, 64ll * nch)));
        nchb[b] = (int32_t)c;
        for (int64_t j = 1; j < c; ++j) {
          tg.push_back(bc[b] + (int64_t)((double)T * j / c));
          lo.push_back(offs[b]);
          hi.push_back(offs[b + 1]);
        }
      }
      std::vector<int32_t> cut(tg.size());
      if (!tg.empty()) {
        const size_t m = tg.size();
        CH_TRY(hipMalloc(&d_tg, sizeof(int64_t) * m));
        CH_TRY(hipMalloc(&d_lo, sizeof(int64_t) * m));
        CH_TRY(hipMalloc(&d_hi, sizeof(int64_t) * m));
        CH_TRY(hipMalloc(&d_co, sizeof(int32_t) * m));
        CH_TRY(hipMemcpyAsync(d_tg, tg.data(), sizeof(int64_t) * m, hipMemcpyHostToDevice, s));
        CH_TRY(hipMemcpyAsync(d_lo, lo.data(), sizeof(int64_t) * m, hipMemcpyHostToDevice, s));
        CH_TRY(hipMemcpyAsync(d_hi, hi.data(), sizeof(int64_t) * m, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(upper_bound_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s,
                           d_cum, d_tg, d_lo, d_hi, (int)m, d_co);
        CH_TRY(hipGetLastError());
        CH_TRY(hipMemcpyAsync(cut.data(), d_co, sizeof(int32_t) * m, hipMemcpyDeviceToHost, s));
        CH_TRY(hipStreamSynchronize(s));
      }
      size_t ci = 0;
      for (int b = 0; b < nblocks; ++b) {
        cbd[b].push_back((int32_t)offs[b]);
        for (int j = 1; j < nchb[b]; ++j) cbd[b].push_back(std::max(cbd[b].back(), cut[ci++]));
        cbd[b].push_back((int32_t)offs[b + 1]);
      }
    }
    chunk_cleanup();
#undef CH_TRY
    // Pieces: a (block, chunk) task holding more than twice the average task's edges is cut
    // into pieces of equal edge counts (work-groups of their own, in the same chunk-major
    // slot). The shared row bounds assume edges spread evenly over the blocks; with column
    // locality (a community of rows linking mostly into its own blocks) a few
    // tasks would otherwise carry most of a chunk's edges. Cost-balanced chunks need none
    // (unless bwd_piece_edges asks for them).
    const int64_t avg_task = std::max<int64_t>(1, E / ((int64_t)nblocks * nch));
    const int64_t piece_cap = o.bwd_piece_edges > 0 ? (int64_t)o.bwd_piece_edges
                              : mode == 3 ? (int64_t)INT32_MAX
                                          : std::max<int64_t>(2 * avg_task, 16384);
    const bool slab_flush = packed && o.bwd_flush != 1;
    auto npieces = [&](int64_t e) {
      return (int32_t)std::max<int64_t>(1, (e + piece_cap - 1) / piece_cap);
    };
    std::vector<int32_t> pieces_of((size_t)nblocks, 0);
    for (int b = 0; b < nblocks; ++b)
      for (size_t j = 0; j + 1 < cbd[b].size(); ++j)
        pieces_of[b] += npieces((int64_t)cbd[b][j + 1] - cbd[b][j]);
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
    // its lines in L2. With nch equal-edge chunks per block on a graph without column
    // locality this is the chunk-major order (chunk j of every block starts near the same
    // row); with locality it keeps the sparse stretches of different blocks together.
    std::vector<int32_t> first_row;
    {
      std::vector<int32_t> starts;
      for (int b = 0; b < nblocks; ++b)
        for (size_t j = 0; j + 1 < cbd[b].size(); ++j)
          starts.push_back(std::min<int32_t>(cbd[b][j], (int32_t)std::max<int64_t>(E - 1, 0)));
      first_row.resize(starts.size());
      int32_t *d_st = nullptr, *d_fr = nullptr;
      auto fr_cleanup = [&]() { dfree(d_st); dfree(d_fr); };
      const hipError_t fe = [&]() -> hipError_t {
        hipError_t e = hipMalloc(&d_st, sizeof(int32_t) * starts.size());
        if (e != hipSuccess) return e;
        e = hipMalloc(&d_fr, sizeof(int32_t) * starts.size());
        if (e != hipSuccess) return e;
        e = hipMemcpyAsync(d_st, starts.data(), sizeof(int32_t) * starts.size(),
                           hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(gather_i32_kernel, dim3((unsigned)((starts.size() + 255) / 256)),
                           dim3(256), 0, s, p->bwd_row, d_st, (int)starts.size(), d_fr);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        e = hipMemcpyAsync(first_row.data(), d_fr, sizeof(int32_t) * starts.size(),
                           hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) return e;
        return hipStreamSynchronize(s);
      }();
      fr_cleanup();
      PLAN_TRY(fe);
    }
    struct ChunkRef { int64_t row; int b, j; };
    std::vector<ChunkRef> order_c;
    {
      size_t i = 0;
      for (int b = 0; b < nblocks; ++b)
        for (int j = 0; j + 1 < (int)cbd[b].size(); ++j)
          order_c.push_back(ChunkRef{row_pos(first_row[i++]), b, j});
    }
    std::stable_sort(order_c.begin(), order_c.end(),
                     [](const ChunkRef& a, const ChunkRef& b) { return a.row < b.row; });
    // a block's chunks must come in chunk order (piece numbering, slab regions)
    std::vector<int32_t> next_chunk((size_t)nblocks, 0);
    for (ChunkRef& cr : order_c) cr.j = next_chunk[cr.b]++;
    std::vector<int32_t> next_piece((size_t)nblocks, 0);
    std::vector<BwdTask> emitted;
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
          emitted.push_back(t);
        }
      }
    }
    if (slab_flush && !comb.empty()) {
      p->bwd_slab_floats = slab_floats;
      p->n_bwd_combine = (int32_t)comb.size();
      PLAN_TRY(hipMalloc(&p->bwd_combine, sizeof(int4) * comb.size()));
      PLAN_TRY(hipMemcpyAsync(p->bwd_combine, comb.data(), sizeof(int4) * comb.size(),
                              hipMemcpyHostToDevice, s));
      PLAN_TRY(hipStreamSynchronize(s));
      p->device_bytes += sizeof(int4) * comb.size();
    }
    // work-group i runs on XCD i % 8 (dealt round-robin; speed only): consecutive tasks of
    // the emission order spread over the XCDs, and every XCD gets the same share of them
    btasks = std::move(emitted);
  } else {
    for (int b = 0; b < nblocks; ++b) {
      const int64_t o0 = offs[b], o1 = offs[b + 1];
      const int64_t nnz = o1 - o0;
      const int nch = (int)std::max<int64_t>(1, std::min<int64_t>(chunks, nnz / min_task_edges));
      if (nch > 1) ++nshared;
      for (int i = 0; i < nch; ++i) {
        for (int g = 0; g < S; ++g) {
          BwdTask t{};
          t.col0 = b * C;
          t.ncols = std::min(C, NC - t.col0);
          t.e0 = (int32_t)(o0 + nnz * i / nch);
          t.e1 = (int32_t)(o0 + nnz * (i + 1) / nch);
          t.shared = nch > 1;
          t.group = g;
          btasks.push_back(t);
        }
      }
    }
    std::stable_sort(btasks.begin(), btasks.end(), [](const BwdTask& a, const BwdTask& b) {
      return (a.e1 - a.e0) > (b.e1 - b.e0);
    });
  }
  p->n_bwd_tasks = (int32_t)btasks.size();
  p->n_bwd_shared = nshared;
  if (!btasks.empty()) {
    PLAN_TRY(hipMalloc(&p->bwd_tasks, sizeof(BwdTask) * btasks.size()));
    PLAN_TRY(hipMemcpyAsync(p->bwd_tasks, btasks.data(), sizeof(BwdTask) * btasks.size(),
                            hipMemcpyHostToDevice, s));
    p->device_bytes += sizeof(BwdTask) * btasks.size();
  }
  // packed backward path: records instead of the three parallel arrays
  if (p->bwd_twopass) {
    // CSR-order records; bwd_perm (column order -> CSR edge) stays for the column pass
  } else if (packed || p->bwd_csc) {
    PLAN_TRY(hipMalloc(&p->bwd_rec, sizeof(uint32_t) * 3 * (size_t)(E + kBwdRecPad)));
    PLAN_TRY(hipMemsetAsync(p->bwd_rec + 3 * E, 0, sizeof(uint32_t) * 3 * kBwdRecPad, s));
    hipLaunchKernelGGL(build_bwd_rec_kernel, dim3(grid_for(E, 256)), dim3(256), 0, s, nullptr,
                       p->bwd_row, p->bwd_col, p->bwd_val, E, C, D, p->bwd_rec);
    PLAN_TRY(hipGetLastError());
    // per-call workspace: lane-ordered selector words (pack_sel_kernel, bwd_feats 4), then
    // the flush slabs
    const int64_t sel_bytes = (p->bwd_feats == 4 || p->bwd_feats == 2) ? (int64_t)std::max(NC, 1) * k : 0;
    p->bwd_slab_off = (sel_bytes + 255) / 256 * 256;
    // flush slabs (bwd_flush 0/2): global float atomics run at ~1.3 TB/s of added bytes and
    // need a memset grad_sp (an 8-GPU Reddit shard spent ~10 % of its backward there)
    p->bwd_ws_bytes = p->bwd_slab_floats > 0 ? p->bwd_slab_off + p->bwd_slab_floats * 4
                                             : sel_bytes;
    if (p->bwd_ws_bytes > 0 && !p->external_ws)
      PLAN_TRY(hipMalloc(&p->bwd_sel, (size_t)p->bwd_ws_bytes));
    PLAN_TRY(hipStreamSynchronize(s));
    dfree(p->bwd_row);
    dfree(p->bwd_col);
    dfree(p->bwd_val);
    p->bwd_row = p->bwd_col = nullptr;
    p->bwd_val = nullptr;
    p->device_bytes += (!p->external_ws ? p->bwd_ws_bytes : 0) +
                       12ll * kBwdRecPad;
  }
  PLAN_TRY(hipStreamSynchronize(s));
  // the column order stays with the plan when the backward blocks use it
  p->col_order = 1;
  if (order && bcolpos) p->col_order = order_mode;
  if (order && bcolpos) {
    p->bwd_corder = order;
    p->device_bytes += sizeof(int32_t) * (int64_t)NC;
    order = nullptr;
  }
  drop_order();
  dfree(row_of);
  dfree(keys_in);
  dfree(keys_out);
  dfree(ids_in);
  dfree(temp);
  dfree(d_offs);
  dfree(d_bad);
#undef PLAN_TRY
  *out_plan = p;
  return MAXK_OK;
}

extern "C" int maxk_plan_refresh_values(maxk_plan* p, const float* val, void* stream) {
  MAXK_CHECK_ARG(p != nullptr, "maxk_plan_refresh_values: plan is null");
  if (p->num_edges == 0) return MAXK_OK;
  if (p->bwd_erec)
    hipLaunchKernelGGL(build_erec_kernel, dim3(grid_for(p->num_edges, 256)), dim3(256), 0,
                       (hipStream_t)stream, nullptr, nullptr, 1, val, p->num_edges, p->bwd_erec);
  else if (p->bwd_rec)
    hipLaunchKernelGGL(build_bwd_rec_kernel, dim3(grid_for(p->num_edges, 256)), dim3(256), 0,
                       (hipStream_t)stream, p->bwd_perm, nullptr, nullptr, val, p->num_edges,
                       p->bwd_block_cols, p->dim_origin, p->bwd_rec);
  else
    hipLaunchKernelGGL(gather_bwd_kernel, dim3(grid_for(p->num_edges, 256)), dim3(256), 0,
                       (hipStream_t)stream, p->bwd_perm, nullptr, nullptr, val, p->num_edges,
                       nullptr, nullptr, p->bwd_val, nullptr);
  if (p->fwd_perm)
    hipLaunchKernelGGL(gather_fwd_kernel, dim3(grid_for(p->num_edges, 256)), dim3(256), 0,
                       (hipStream_t)stream, p->fwd_perm, nullptr, nullptr, val, p->num_edges,
                       p->fwd_cv, false);
  if (p->fwd_fix && p->n_fwd_tasks > 0) {
    const hipError_t e = fwd_fix_stats(p, p->fwd_rowptr, val, (hipStream_t)stream);
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
  maxk_plan_info full{};
  maxk_plan_info* info = &full;
  info->num_nodes = p->num_nodes;
  info->num_cols = p->num_cols;
  info->num_edges = p->num_edges;
  info->dim_origin = p->dim_origin;
  info->dim_k = p->dim_k;
  info->fwd_tasks = p->n_fwd_tasks;
  info->fwd_split_rows = p->n_zero_rows;
  info->bwd_block_cols = p->bwd_block_cols;
  info->bwd_blocks = p->n_bwd_blocks;
  info->bwd_tasks = p->n_bwd_tasks;
  info->bwd_shared_blocks = p->n_bwd_shared;
  info->device_bytes = p->device_bytes;
  info->bwd_algo = p->bwd_twopass ? 3 : p->bwd_csc ? 2 : 1;
  info->col_order = p->col_order;
  info->bwd_chunk_bounds = (p->bwd_twopass || p->bwd_csc) ? 0 : p->bwd_chunk_mode;
  info->bwd_tp_chunks = p->bwd_twopass ? p->bwd_tp_chunks : 1;
  info->bwd_row_order = p->bwd_row_order;
  info->bwd_workspace_peak = p->bwd_ws_bytes;
  std::memcpy(out, info, (size_t)std::min<int64_t>(info_bytes, (int64_t)sizeof(maxk_plan_info)));
  return MAXK_OK;
}

__global__ void iota_kernel(int n, int32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = i;
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
