// SpGEMM forward (row-wise product over CBSR features) and SSpMM backward (outer product
// sampled at the selector) for gfx950.
//
// Reference kernels: spmm_kernel_opt2_sparse_v3 and
// spmm_kernel_opt2_sparse_backward_v3 give every 32-lane warp one <=64-nz chunk of a CSR
// row (".warp4" metadata), accumulate into a per-warp LDS row and write it back with one
// global float atomic per feature per chunk (forward), or scatter every product with a
// global float atomic into grad_sp (backward). On MI355X global float atomics execute at
// the memory side (~1.3 TB/s of added bytes) and LDS ds_add_f32 runs at ~1/30 of the
// integer LDS atomic rate (tools/ubench_atomics.hip, profiles/r01/ubench_atomics.log), so
// both kernels are restructured:
//
//   forward : a 256- or 512-thread work-group (4 or 8 waves) owns <= 32 whole destination
//             rows (LDS accumulator rows x D); its waves take edge windows from an LDS counter
//             (or a static interleave); the edges are processed flat, k/4 lanes per edge, 4 features per
//             lane (one dwordx4 value gather + one dword selector gather; or lane chunks of
//             3 values + their selectors for k % 16 != 0), 8 independent sub-steps in
//             flight per wave (4 at k = 48); products are accumulated in LDS in exact fixed point
//             (ds_add_u64, LdsFix) or f64 (ds_add_f64), and the rows are written back once
//             with coalesced dwordx4 stores. Only rows longer than the task cap are split,
//             and only those touch global atomics.
//   backward: a 512/768/1024-thread work-group owns a block of source columns whose k-wide
//             gradients live in LDS; it sweeps the block's edges in destination-row order
//             (plan-built block-major edge list), so the lanes of one instruction gather
//             from few rows of grad_out (L1 reuse); updates are 64-bit compare-and-swaps on
//             float pairs; the block is stored once at the end (or, split over several
//             work-groups, into slabs that one combine pass adds in a fixed order). Graphs
//             whose column blocks see each grad_out row about once use a two-pass form.
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace maxk {

// Quad-shared loads: the L lanes of an edge (L % 4 == 0, quad-aligned) need the same edge
// record; lane q of a quad loads the record of sub-step 4j + q and quad_perm DPP moves
// broadcast it, so one load instruction serves four sub-steps.
template <int W>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
  static_assert(W >= 0 && W < 4, "quad lane");
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

// Forward f64 accumulator: ds_add_f64 of the f32 product val * x. Inputs with non-finite
// values take this path, so its idle lanes add 0 * 0 (fwd_edges4 zeroes their values).
struct LdsF64 {
  using T = double;
  using V = float;
  static constexpr bool kFixed = false;
  static __device__ __forceinline__ V scale(float v, double) { return v; }
  static __device__ __forceinline__ void add2(double* p, float v, float x) {
    lds_add(p, (double)(v * x));
  }
};

// Forward fixed-point accumulator (plan->fwd_fixed): ds_add_u64 runs at ~1.9x the ds_add_f64
// rate, and the f64 atomic bounds the forward at k >= 32 (profiles/r02/fwd_probe/lds_update_probes.jsonl: Reddit
// k = 32 2.46 -> 1.74 ms, k = 64 4.79 -> 3.34 with the integer atomic). A term val * x is
// scaled by 2^s (per task and call, fwd_fix_scale) and rounded to an integer by ONE fma with
// M = 1.5 * 2^52: r = fma(val * 2^s, x, M) lies in [2^52, 2^53) while |term| < 2^51, where the
// f64 bit pattern of r is bits(M) + round(term). The slot accumulates these raw patterns
// (mod 2^64); bits(M) = 0x867 * 2^51 vanishes mod 2^51, so the low 51 bits, read as a signed
// residue, are the exact integer sum as long as |sum| < 2^50 (fwd_fix_decode). The products
// are exact in f64 (24 x 24 bits) and the integer sum is exact, so the only error is the one
// rounding per term, at most 2^-(s+1).
struct LdsFix {
  using T = unsigned long long;
  using V = double;
  static constexpr bool kFixed = true;
  static __device__ __forceinline__ V scale(float v, double sc) { return (double)v * sc; }
  static __device__ __forceinline__ void add2(T* p, double v, float x) {
    const double r = __builtin_fma(v, (double)x, 0x1.8p52);
    __hip_atomic_fetch_add(p, (T)__double_as_longlong(r), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
  }
};

__device__ __forceinline__ double fwd_fix_decode(unsigned long long a, double inv) {
  const long long t = (long long)(a << 13) >> 13;  // low 51 bits as a signed residue
  return (double)t * inv;
}

// Per task and call: the scale 2^s of the fixed-point forward, or 0 (use f64). fix = {sexp,
// gexp} from fwd_fix_stats_kernel: every row of the task has sum |val| <= 2^sexp, and every
// nonzero |val| >= 2^(sexp - gexp). The statistics are xs_n pairs {B bits, 0x7fffffff - min
// nonzero |x| bits} (cbsr_stats_kernel; pair i at xs[i * stride] and xs[i * stride + off2]),
// where B bounds what one CBSR row adds to one output slot per unit of val: max |x|, or the
// row's sum |x| when its selectors repeat. With 2^ex > B and min |x| >= 2^en: s = 49 - sexp -
// ex keeps every slot's sum of |terms| below 2^49 (below 2^50 is what fwd_fix_decode needs);
// the rounding error of a term, 2^-(s+1), relative to the smallest possible nonzero term
// 2^(sexp - gexp + en), is at most 2^(gexp + ex - en - 50). The fixed path is taken when that
// is <= 2^-25, so every output whose terms do not cancel (|y| >= sum |terms| / 2) is within
// 2^-24 relative, the rounding of the f32 result itself. Non-finite or all-zero inputs take
// the f64 path.
__device__ __forceinline__ double fwd_fix_scale(int2 fix, const uint32_t* xs, int xs_n,
                                                int stride, int off2) {
  uint32_t mx = 0u, inv = 0u;
  for (int i = 0; i < xs_n; ++i) {
    mx = max(mx, xs[i * stride]);
    inv = max(inv, xs[i * stride + off2]);
  }
  const uint32_t mn = 0x7fffffffu - inv;
  if (mx == 0u || mx >= 0x7f800000u || mn == 0u || mn > mx) return 0.0;
  const int ex = (int)(mx >> 23) - 126;                      // max |x| < 2^ex
  const int en = (mn >> 23) ? (int)(mn >> 23) - 127 : -149;  // min |x| >= 2^en
  if (fix.y + ex - en > 25) return 0.0;
  const int sc = 49 - fix.x - ex;
  if (sc > 1000 || sc < -1000) return 0.0;
  return __builtin_ldexp(1.0, sc);
}

// cbsr_stats4_kernel for k % 4 == 0 (k <= 256): L = k/4 lanes per row, each loading its 4
// values (float4) and their 4 selectors (one dword), rows 64/L per wave, coalesced. Per row,
// inclusive prefix scans over its L lanes (shuffles) give the sum of |x|, the max |x|, and
// whether a lane's first nonzero selector is <= the last nonzero selector of any earlier lane
// (or its own nonzero selectors do not ascend): the same bound as the thread-per-row kernel
// below, with the row sum added in another order (its 2^-10 headroom covers that).
//
// PACK 1: the same pass also writes the forward's packed CBSR records (k values, then the k
// selector bytes, rec_bytes per row), so the per-call pack and the statistics cost one read
// of the tables; PACK 2: the pair-chunk records instead (plan->fwd_chunk2: lane q writes the
// 16-B chunks 2q and 2q + 1, {2 values, their 2 selector bytes, 0}). STATS = false: the pack
// alone. The forward's split rows (summed atomically by their segments) are zeroed here too,
// one launch before the forward.
template <int PACK, bool STATS>
__global__ __launch_bounds__(256) void cbsr_stats4_kernel(const float* __restrict__ x,
                                                          const uint8_t* __restrict__ sel,
                                                          int64_t nrows, int k, uint32_t* st0,
                                                          uint32_t* st1, uint8_t* __restrict__ rec,
                                                          int rec_bytes,
                                                          const int32_t* __restrict__ zrows,
                                                          int nz, float* __restrict__ out, int D,
                                                          int ds, int is) {
  __shared__ uint32_t smx[256 / kWave], smn[256 / kWave];
  for (int i = blockIdx.x; i < nz; i += gridDim.x)
    for (int t = threadIdx.x; t < D; t += blockDim.x) out[(size_t)zrows[i] * D + t] = 0.f;
  const int L = k >> 2;
  const int RW = kWave / L;  // rows per wave
  const int lane = threadIdx.x & (kWave - 1);
  const int slot = lane / L, q = lane - slot * L;
  const bool on = slot < RW;
  uint32_t mx = 0u, mn = 0x7fffffffu;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
  for (int64_t r0 = ((int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave) * RW;
       r0 < nrows; r0 += waves * RW) {
    const int64_t r = r0 + slot;
    const bool live = on && r < nrows;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    uint32_t s = 0u;
    if (live) {
      v = *reinterpret_cast<const float4*>(x + r * ds + 4 * q);
      s = *reinterpret_cast<const uint32_t*>(sel + r * is + 4 * q);
      if constexpr (PACK == 1) {
        uint8_t* rp = rec + r * rec_bytes;
        *reinterpret_cast<float4*>(rp + 16 * q) = v;
        *reinterpret_cast<uint32_t*>(rp + 4 * k + 4 * q) = s;
      } else if constexpr (PACK == 2) {
        uint4* rp = reinterpret_cast<uint4*>(rec + r * rec_bytes) + 2 * q;
        rp[0] = make_uint4(__float_as_uint(v.x), __float_as_uint(v.y), s & 0xffffu, 0u);
        rp[1] = make_uint4(__float_as_uint(v.z), __float_as_uint(v.w), s >> 16, 0u);
      }
    }
    if constexpr (!STATS) continue;
    const uint32_t b[4] = {__float_as_uint(v.x) & 0x7fffffffu, __float_as_uint(v.y) & 0x7fffffffu,
                           __float_as_uint(v.z) & 0x7fffffffu, __float_as_uint(v.w) & 0x7fffffffu};
    uint32_t lmax = 0u, lmin = 0x7fffffffu;
    float lsum = 0.f;
    int first = -1, last = -1;
    bool rep = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (b[i] == 0u) continue;
      const int si = (int)((s >> (8 * i)) & 0xffu);
      lmax = max(lmax, b[i]);
      lmin = min(lmin, b[i]);
      lsum += __uint_as_float(b[i]);
      rep = rep || si <= last;
      if (first < 0) first = si;
      last = si;
    }
    // inclusive prefix over the row's lanes: sum, max, repeat flag, max of last selectors
    int pl = last;  // max nonzero selector of lanes <= q
    for (int d = 1; d < L; d <<= 1) {
      const float os = __shfl(lsum, lane - d);
      const uint32_t om = (uint32_t)__shfl((int)lmax, lane - d);
      const int orp = __shfl((int)rep, lane - d);
      const int opl = __shfl(pl, lane - d);
      if (q >= d) {
        lsum += os;
        lmax = max(lmax, om);
        rep = rep || orp;
        pl = max(pl, opl);
      }
    }
    const int prev = __shfl(pl, lane - 1);  // max nonzero selector of lanes < q
    const bool cross = q > 0 && first >= 0 && first <= prev;
    // the row's repeat flag = OR over its lanes (prefix OR, taken at the last lane)
    int any = cross ? 1 : 0;
    for (int d = 1; d < L; d <<= 1) {
      const int o = __shfl(any, lane - d);
      if (q >= d) any |= o;
    }
    if (live) {
      mn = min(mn, lmin);
      if (q == L - 1) {
        const bool rrep = rep || any;
        const uint32_t rb =
            rrep ? max(lmax, __float_as_uint(lsum * (1.0f + 0x1p-10f)) & 0x7fffffffu) : lmax;
        mx = max(mx, rb);
      }
    }
  }
  if constexpr (!STATS) return;
  for (int o = kWave / 2; o > 0; o >>= 1) {
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
  }
  const int w = threadIdx.x / kWave;
  if (lane == 0) { smx[w] = mx; smn[w] = mn; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 256 / kWave; ++i) { mx = max(mx, smx[i]); mn = min(mn, smn[i]); }
    atomicMax(st0, mx);
    atomicMax(st1, 0x7fffffffu - mn);
  }
}

// Statistics of a CBSR table for fwd_fix_scale, one thread per row (bit patterns of
// non-negative floats order like integers): *st0 = max over rows of the row's slot bound B,
// *st1 = 0x7fffffff - min nonzero |x|. B is max |x| when the row's nonzero entries have
// strictly ascending selectors (every exact top-k row), else the row's sum |x| (with 2^-10 of
// headroom for the f32 sum): m nonzero entries on one selector add m terms to one LDS slot
// (maxk_hip.h: repeated selectors are summed), which a max |x| bound would not cover. Zero
// entries (ref_compat padding) add nothing and are skipped. Both words are zeroed before the
// launch; a few hundred work-groups reduce in LDS and add one atomic each per word.
__global__ __launch_bounds__(256) void cbsr_stats_kernel(const float* __restrict__ x,
                                                         const uint8_t* __restrict__ sel,
                                                         int64_t nrows, int k, uint32_t* st0,
                                                         uint32_t* st1, int ds, int is) {
  __shared__ uint32_t smx[256 / kWave], smn[256 / kWave];
  uint32_t mx = 0u, mn = 0x7fffffffu;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows;
       r += (int64_t)gridDim.x * blockDim.x) {
    uint32_t mb = 0u, lo = 0x7fffffffu;
    float sum = 0.f;
    int prev = -1;
    bool rep = false;
    const float* xr = x + r * ds;
    const uint8_t* sr = sel + r * is;
    for (int l = 0; l < k; ++l) {
      const uint32_t b = __float_as_uint(xr[l]) & 0x7fffffffu;
      if (b == 0u) continue;
      const int s = sr[l];
      mb = max(mb, b);
      lo = min(lo, b);
      sum += __uint_as_float(b);
      rep = rep || s <= prev;
      prev = s;
    }
    // a non-finite sum (or value) gives bits >= 0x7f800000: fwd_fix_scale falls back
    const uint32_t rb = rep ? max(mb, __float_as_uint(sum * (1.0f + 0x1p-10f)) & 0x7fffffffu) : mb;
    mx = max(mx, rb);
    mn = min(mn, lo);
  }
  for (int o = kWave / 2; o > 0; o >>= 1) {
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
  }
  const int w = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) { smx[w] = mx; smn[w] = mn; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 256 / kWave; ++i) { mx = max(mx, smx[i]); mn = min(mn, smn[i]); }
    atomicMax(st0, mx);
    atomicMax(st1, 0x7fffffffu - mn);
  }
}

// --------------------------------------------------------------------------------------
// forward
// --------------------------------------------------------------------------------------
// CBSR records: the API hands over two tables (sp_data [N,k] f32, sp_index [N,k] u8), so an
// edge's gather touches two cache lines. The forward first packs them into one record per
// node, {k values, k selectors, pad} of rec_bytes (128 B at k = 16): one line per edge.
// On gfx950 the gather is bound by L1/TA request count, not by bytes or by where the line
// is served from (tools/ubench_gather.hip: 2.70 ms -> 1.84 ms for Reddit at k = 16).
// cbsr_stats4_kernel<PACK = true> writes them (k % 4 == 0), fused with the statistics.

// Lane-chunk CBSR records (plan->fwd_chunk3): chunk j of column c is 16 B, {x[3j],
// x[3j+1], x[3j+2], selectors 3j..3j+2 in bytes 0..2 of the 4th word}, so ONE dwordx4 gather
// gives a lane its 3 values and their selectors (the 4-values-per-lane records need a
// second, selector, gather per lane). Padding slots (3j+i >= k) are 0.
template <int V>
__global__ void pack_cbsr3_kernel(const float* __restrict__ sp_data,
                                  const uint8_t* __restrict__ sp_index,
                                  uint8_t* __restrict__ rec, int ncols, int k, int rec_bytes,
                                  int ds, int is) {
  // V = 3: lane chunks {3 values, their 3 selector bytes}; V = 2: pair chunks {2 values, their
  // 2 selector bytes, 0} (plan->fwd_chunk2)
  const int chunks = (k + V - 1) / V;
  const int64_t total = (int64_t)ncols * chunks;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = t / chunks;
    const int j = (int)(t - c * chunks);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int l = V * j + i;
      if (l < k) {
        w[i] = __float_as_uint(sp_data[c * ds + l]);
        w[V == 3 ? 3 : 2] |= (uint32_t)sp_index[c * is + l] << (8 * i);
      }
    }
    *reinterpret_cast<uint4*>(rec + c * rec_bytes + j * 16) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// One wave's share of the forward edges [e0, e1) (4 features per lane, or lane chunks):
// U sub-steps per iteration (kFwdUnroll; 4 with 8 waves by option) with every load issued before the first LDS update.
// The chain (col, val) -> CBSR record -> LDS has two dependent global round trips, so
// memory-level parallelism comes from U independent sub-steps per wave. Idle lanes load a
// clamped (valid) edge and add 0 at its addresses instead of branching (with a branch the
// compiler sinks sub-step 0's gather below the other loads).
// FL kFwdFlagChunk3: lane-chunk records (pack_cbsr3_kernel), l0 = chunk. kFwdFlagQuad (L % 4
// == 0): edge-major windows, sub-step u of slot s takes edge base + s U + u, so lane q of a
// quad loads the whole edge word of sub-step 4j + q (the quad reads 32 contiguous bytes) and
// DPP hands it to the quad: one edge-word instruction per four sub-steps.
// (Batching the selector words the same way, 64 scattered records per instruction, ran k = 16
// 1.10 -> 1.48 ms: only contiguous loads gain from fewer instructions.)
template <class A, int FL, int U>
__device__ __forceinline__ void fwd_edges4(typename A::T* acc, int e0, int e1, int* ctr,
                                           int wave, int nwaves, int EPS, int slot, int l0,
                                           bool lane_on,
                                           const uint2* __restrict__ cv,
                                           const uint8_t* __restrict__ rec, int rec_bytes,
                                           const uint8_t* __restrict__ seltab, int ss, int D,
                                           int k, double sc) {
  using T = typename A::T;
  constexpr bool C3 = (FL & kFwdFlagChunk3) != 0;
  constexpr bool C2 = (FL & kFwdFlagChunk2) != 0;
  constexpr bool EM = (FL & kFwdFlagQuad) != 0;
  const int last = e1 - 1;
  const int qq = threadIdx.x & 3;
  // window i of this wave: wave + i * nwaves (static), or (ctr != nullptr: plan->fwd_handout
  // 2) the next one of the task's LDS counter *ctr, handed out in order one at a time
  for (int i = 0;; ++i) {
    int wi = wave + i * nwaves;
    if (ctr) {
      int c = 0;
      if ((threadIdx.x & (kWave - 1)) == 0) c = atomicAdd(ctr, 1);
      wi = __builtin_amdgcn_readlane(c, 0);
    }
    const int base = (EM && U == 8 ? (e0 & ~1) : e0) + wi * (EPS * U);
    if (base >= e1) break;
    uint32_t cw[U];
    float v[U];
    bool ok[U];
    if constexpr (EM && U == 8) {
      // eight sub-steps per quad from one 16-B load per lane (two edge words, lane q: sub-steps
      // 2q, 2q + 1). Windows start at even edges (from e0 rounded down; cv holds E + 1 words,
      // so the pair at the last edge stays in bounds); words outside [e0, e1) are masked, with
      // their row bits dropped so their zero adds land in row 0 of this tile
      const int sb = base + slot * U;
      const uint4 wq = *reinterpret_cast<const uint4*>(cv + min(sb + 2 * qq, last & ~1));
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t w0 = quad_pick((u & 1) ? wq.z : wq.x, u >> 1);
        const uint32_t w1 = quad_pick((u & 1) ? wq.w : wq.y, u >> 1);
        ok[u] = lane_on && sb + u >= e0 && sb + u < e1;
        cw[u] = ok[u] ? w0 : (w0 & kFwdColMask);
        v[u] = __uint_as_float(w1);
      }
    } else if constexpr (EM) {
      uint2 wq[U / 4];
#pragma unroll
      for (int j = 0; j < U / 4; ++j) wq[j] = cv[min(base + slot * U + 4 * j + qq, last)];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ok[u] = lane_on && base + slot * U + u < e1;
        cw[u] = quad_pick(wq[u / 4].x, u);
        v[u] = __uint_as_float(quad_pick(wq[u / 4].y, u));
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + u * EPS + slot;
        ok[u] = lane_on && e < e1;
        const uint2 w = cv[ok[u] ? e : last];
        cw[u] = w.x;
        v[u] = __uint_as_float(w.y);
      }
    }
    float4 x[U];
    uint32_t sel[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint8_t* rp = rec + (size_t)(cw[u] & kFwdColMask) * rec_bytes;
      if constexpr (C3) {  // lane chunk: 3 values + their selector bytes, one gather
        const uint4 w = *reinterpret_cast<const uint4*>(rp + l0 * 16);
        x[u] = make_float4(__uint_as_float(w.x), __uint_as_float(w.y), __uint_as_float(w.z), 0.f);
        sel[u] = w.w;
      } else if constexpr (C2) {  // pair chunk: 2 values + their selector bytes, one gather
        const uint4 w = *reinterpret_cast<const uint4*>(rp + l0 * 16);
        x[u] = make_float4(__uint_as_float(w.x), __uint_as_float(w.y), 0.f, 0.f);
        sel[u] = w.z;
      } else {
        x[u] = *reinterpret_cast<const float4*>(rp + l0 * 4);
        // two tables (plan->fwd_two_tables): values straight from sp_data, selectors from
        // sp_index (no per-call pack); else the selector word of the record (packed per call,
        // or the caller's interleaved records)
        const uint8_t* sp = seltab ? seltab + (size_t)(cw[u] & kFwdColMask) * ss + l0
                                   : rp + 4 * k + l0;
        sel[u] = *reinterpret_cast<const uint32_t*>(sp);
      }
    }
    if constexpr (!A::kFixed) {  // finite-only fixed point: 0 * x is 0 there
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (!ok[u]) x[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      T* arow = acc + (cw[u] >> kFwdColBits) * D;
      const uint32_t sv = sel[u];
      const typename A::V vu = A::scale(ok[u] ? v[u] : 0.f, sc);
      if constexpr (C3) {
        // l0 = chunk index: slots 3 l0 .. 3 l0 + 2 (the last chunk may be partly padding)
        A::add2(arow + (sv & 0xffu), vu, x[u].x);
        if (3 * l0 + 1 < k) A::add2(arow + ((sv >> 8) & 0xffu), vu, x[u].y);
        if (3 * l0 + 2 < k) A::add2(arow + ((sv >> 16) & 0xffu), vu, x[u].z);
      } else if constexpr (C2) {  // l0 = chunk index: slots 2 l0, 2 l0 + 1 (k even)
        A::add2(arow + (sv & 0xffu), vu, x[u].x);
        A::add2(arow + ((sv >> 8) & 0xffu), vu, x[u].y);
      } else {
        A::add2(arow + (sv & 0xffu), vu, x[u].x);
        A::add2(arow + ((sv >> 8) & 0xffu), vu, x[u].y);
        A::add2(arow + ((sv >> 16) & 0xffu), vu, x[u].z);
        A::add2(arow + (sv >> 24), vu, x[u].w);
      }
    }
  }
}

// Work-group = one task (FwdTask: whole rows, or one segment of a long row). Its edges are
// column-sorted; rot_ticks > 0: the sweep starts at the column window the shared 100 MHz clock
// points to and wraps around, so concurrently running tiles gather from the same columns (L2
// reuse). accum: the rows of out hold a prior sum to add to (the multi-GPU split's remote
// part). VEC == 1: k % 4 != 0 beyond the lane chunks' range (k > 192), min(k, 64) lanes per
// edge looping over the row's k entries, f64 atomics.
template <int VEC, int FL, int NT, int FU>
__global__ __launch_bounds__(NT) void spgemm_fwd_kernel(
    const FwdTask* __restrict__ tasks, const int32_t* __restrict__ phase_off, int phases,
    const uint2* __restrict__ cv, const float* __restrict__ sp_data,
    const uint8_t* __restrict__ sp_index, const uint8_t* __restrict__ rec, int rec_bytes,
    float* __restrict__ out, int D, int k, int rot_ticks, const uint8_t* __restrict__ seltab,
    int ss, int ds, int accum, const int2* __restrict__ fix_tab,
    const uint32_t* __restrict__ xstat, int xs_n, int xs_stride, int xs_off2, int handout) {
  extern __shared__ __align__(16) double smem_d[];
  double* acc = smem_d;
  unsigned long long* acc64 = reinterpret_cast<unsigned long long*>(smem_d);
  __shared__ int s_w0;
  __shared__ int s_win[2];  // window counters of the task's two sweeps (fwd_edges4)
  if (threadIdx.x == 0) {
    s_win[0] = 0;
    s_win[1] = 0;
  }
  const int ti = blockIdx.x;
  FwdTask t = tasks[ti];
  t.e0 = phase_off[ti * (phases + 1)];
  t.e1 = phase_off[ti * (phases + 1) + phases];
  int emid = -1;
  if (rot_ticks > 0) {
    // read once per work-group: every wave must split the task at the same edge
    if (threadIdx.x == 0)
      s_w0 = (int)((__builtin_amdgcn_s_memrealtime() / (uint64_t)rot_ticks) % (uint64_t)phases);
    __syncthreads();
    emid = phase_off[ti * (phases + 1) + s_w0];
  }
  if (accum && t.e0 == t.e1) return;  // nothing to add (uniform)
  // fixed-point accumulation for this task (LdsFix), else f64; the 8-byte slots are the same.
  // A continuing launch in fixed point sums its own terms from zero and adds the prior f32
  // row at the write-back (one more f32 rounding)
  double fsc = 0.0;
  if constexpr (VEC == 4) {
    if (fix_tab) fsc = fwd_fix_scale(fix_tab[ti], xstat, xs_n, xs_stride, xs_off2);
  }
  const bool fixed = fsc != 0.0;
  const bool split = t.nrows < 0;
  const int nrows = split ? 1 : t.nrows;
  const int n = nrows * D;
  const int DS = D + kFwdRowPad;  // LDS row stride (elements)
  if (accum && !split && !fixed) {  // continue from the stored rows
    const float* src = out + (size_t)t.row0 * D;
    for (int i = threadIdx.x; i < n; i += NT) {
      const int r = i / D;
      acc[r * DS + (i - r * D)] = src[i];
    }
  } else {
    for (int i = threadIdx.x; i < nrows * DS; i += NT) acc[i] = 0.0;
  }
  __syncthreads();

  constexpr bool C3 = (FL & kFwdFlagChunk3) != 0;
  constexpr bool C2 = (FL & kFwdFlagChunk2) != 0;
  const int L = (VEC == 4) ? (C3 ? (k + 2) / 3 : C2 ? k / 2 : k / 4) : (k < kWave ? k : kWave);
  const int EPS = kWave / L;  // edges per wave instruction
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int slot = lane / L;
  const int l0 = (lane - slot * L) * (C3 || C2 ? 1 : VEC);
  const bool lane_on = slot < EPS;
  constexpr int kWaves = NT / kWave;

  if constexpr (VEC == 4) {
    auto sweep = [&](auto* a, auto tag) {
      using AA = decltype(tag);
      int* c0 = handout ? &s_win[0] : nullptr;
      int* c1 = handout ? &s_win[1] : nullptr;
      if (emid >= 0) {
        fwd_edges4<AA, FL, FU>(a, emid, t.e1, c0, wave, kWaves, EPS, slot, l0, lane_on, cv, rec,
                           rec_bytes, seltab, ss, DS, k, fsc);
        fwd_edges4<AA, FL, FU>(a, t.e0, emid, c1, wave, kWaves, EPS, slot, l0, lane_on, cv, rec,
                           rec_bytes, seltab, ss, DS, k, fsc);
      } else {
        fwd_edges4<AA, FL, FU>(a, t.e0, t.e1, c0, wave, kWaves, EPS, slot, l0, lane_on, cv, rec,
                           rec_bytes, seltab, ss, DS, k, fsc);
      }
    };
    if (fixed) sweep(acc64, LdsFix{});
    else sweep(acc, LdsF64{});
  } else {
    for (int base = t.e0 + wave * EPS; base < t.e1; base += kWaves * EPS) {
      const int e = base + slot;
      if (lane_on && e < t.e1) {
        const uint2 w = cv[e];
        const float v = __uint_as_float(w.y);
        double* arow = acc + (w.x >> kFwdColBits) * DS;
        const size_t c = w.x & kFwdColMask;
        for (int l = l0; l < k; l += L)
          LdsF64::add2(arow + sp_index[c * ss + l], v, sp_data[c * ds + l]);
      }
    }
  }
  __syncthreads();

  float* dst = out + (size_t)t.row0 * D;
  const double finv = fixed ? 1.0 / fsc : 0.0;  // 2^-s, exact
  auto get = [&](int i) -> float {
    const int r = i / D;
    if (fixed) return (float)fwd_fix_decode(acc64[r * DS + (i - r * D)], finv);
    return (float)acc[r * DS + (i - r * D)];
  };
  if (!split) {
    const bool add = accum && fixed;  // the prior row is added here (see above)
    if ((D & 3) == 0) {
      for (int i = threadIdx.x * 4; i < n; i += NT * 4) {
        float4 v = make_float4(get(i), get(i + 1), get(i + 2), get(i + 3));
        if (add) {
          const float4 o = *reinterpret_cast<const float4*>(dst + i);
          v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
        }
        *reinterpret_cast<float4*>(dst + i) = v;
      }
    } else {
      for (int i = threadIdx.x; i < n; i += NT) dst[i] = add ? dst[i] + get(i) : get(i);
    }
  } else {
    for (int i = threadIdx.x; i < D; i += NT) global_add(dst + i, get(i));
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
// backward: column blocks
// --------------------------------------------------------------------------------------
// One work-group per (column block, row chunk piece, slot group) task, NT threads (8 waves,
// 12 at k >= 32: more gathers in flight per CU under the same LDS block). Lanes: L = ns / F
// per edge, lane q owns the F slots q, q + L, ... of its group, stored adjacently in LDS
// (slot l of a column at (l % L) * F + l / L), so an update is 1 ds_read_b128 + 2
// ds_cmpst_rtn_b64 (F = 4) or 1 ds_read_b64 + 1 ds_cmpst_rtn_b64 (F = 2); a pair is retried
// if either of its floats changed. The block's selectors are staged in LDS behind the
// accumulators (the G rows evict the block's 16 B/column table from the 32 KB L1), straight
// from sp_index rows (row stride `is` bytes, column corder[position] when the plan has a
// column order): dword loads of 4 selectors, scattered into lane order, so slot l of the
// group (global slot g * ns + l; >= k is padding and selects feature 0) lands in byte
// (c * L + l % L) * F + l / L and lane q reads its F selectors as one word. (Rounds 1-4 packed
// the lane-ordered words in a per-call pass, pack_sel_kernel: 7-9 us and one launch per call;
// round 3's in-kernel staging with byte gathers had cost more than that pass.)
// Per sub-step a lane loads its edge's record {row offset, column in block, val} (Q: lane q
// of a quad loads sub-step 4j + q's whole record, DPP hands it on: one record instruction
// per four sub-steps), reads its selector word from LDS and gathers F floats of the edge's
// grad_out row with buffer loads (32-bit offsets; BIG: grad_out > 4 GiB, the record holds the
// row index and the gathers are 64-bit addressed). Records past e1 (padding or a
// neighbouring task's) are loaded and ignored.
// Per-lane accumulator update of N sub-steps: lane q adds x[u][0..F) (val already applied) to
// the F adjacent slots of column cl[u] at accq + cl[u] * KS (accq = accumulators + F q): one
// ds_read_b128 / b64 of the current values, then one 64-bit compare-and-swap per float pair,
// all reads first, all CAS next, then retries for the rare pairs another lane or wave changed.
template <int N, int F>
__device__ __forceinline__ void bwd_cas_update(unsigned* accq, int KS, const uint32_t (&cl)[N],
                                               const float (&x)[N][F], const bool (&ok)[N]) {
  using u64 = unsigned long long;
  u64 old2[N][F / 2];
#pragma unroll
  for (int u = 0; u < N; ++u) {
    // one ds_read_b128 / b64 (KS % F == 0); a stale value only costs a CAS retry
    if constexpr (F == 4) {
      const uint4 o4 = *reinterpret_cast<const uint4*>(accq + cl[u] * KS);
      old2[u][0] = (u64)o4.x | ((u64)o4.y << 32);
      old2[u][1] = (u64)o4.z | ((u64)o4.w << 32);
    } else {
      const uint2 o2 = *reinterpret_cast<const uint2*>(accq + cl[u] * KS);
      old2[u][0] = (u64)o2.x | ((u64)o2.y << 32);
    }
  }
  auto addp = [](u64 o, float a0, float a1) -> u64 {
    const float lo = __uint_as_float((unsigned)o) + a0;
    const float hi = __uint_as_float((unsigned)(o >> 32)) + a1;
    return (u64)__float_as_uint(lo) | ((u64)__float_as_uint(hi) << 32);
  };
  u64 got2[N][F / 2];
#pragma unroll
  for (int u = 0; u < N; ++u) {
    u64* a = reinterpret_cast<u64*>(accq + cl[u] * KS);
#pragma unroll
    for (int h = 0; h < F / 2; ++h) {
      got2[u][h] = old2[u][h];
      if (ok[u]) {
        u64 expected = old2[u][h];
        __hip_atomic_compare_exchange_strong(a + h, &expected,
                                             addp(old2[u][h], x[u][2 * h], x[u][2 * h + 1]),
                                             __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
        got2[u][h] = expected;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < N; ++u) {
    u64* a = reinterpret_cast<u64*>(accq + cl[u] * KS);
#pragma unroll
    for (int h = 0; h < F / 2; ++h) {
      if (ok[u] && got2[u][h] != old2[u][h]) {
        u64 cur = got2[u][h];
        while (true) {
          u64 expected = cur;
          __hip_atomic_compare_exchange_strong(a + h, &expected,
                                               addp(cur, x[u][2 * h], x[u][2 * h + 1]),
                                               __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
          if (expected == cur) break;
          cur = expected;
        }
      }
    }
  }
}

// Probe hooks (tools/probe_bwd_tail.hip includes this file with them defined: per-work-group
// start / end clocks); empty in the library.
#ifndef MAXK_BWD_PROBE_BEGIN
#define MAXK_BWD_PROBE_BEGIN()
#define MAXK_BWD_PROBE_END()
#endif

template <int U, int NT, int F, bool Q, bool BIG>
__global__ __launch_bounds__(NT) void sspmm_bwd4_kernel(
    const BwdTask* __restrict__ tasks, const uint32_t* __restrict__ rec,
    const float* __restrict__ G, uint32_t g_bytes, int D, const uint8_t* __restrict__ sp_index,
    int is, float* __restrict__ grad_sp, int k, int ns, float* __restrict__ slab,
    const int32_t* __restrict__ corder, int handout) {
  static_assert(F == 2 || F == 4, "2 or 4 slots per lane");
  static_assert(!Q || U % 4 == 0, "quad record loads need U % 4 == 0");
  using SelT = std::conditional_t<F == 4, uint32_t, uint16_t>;
  extern __shared__ __align__(16) double bsmem[];
  __shared__ int s_next;  // next window of the task's edge stream to hand out
  float* bacc = reinterpret_cast<float*>(bsmem);
  const BwdTask t = tasks[blockIdx.x];
  MAXK_BWD_PROBE_BEGIN();
  // padding / nothing to add (with the slab flush every piece stores its block, zeros too)
  if (t.ncols == 0 || (t.shared && !slab && t.e0 == t.e1)) return;
  const int L = ns / F;   // lanes per edge
  const int KS = ns;      // accumulator floats per column
  const int nacc = t.ncols * KS;
  for (int i = threadIdx.x; i < nacc; i += NT) bacc[i] = 0.f;
  if (threadIdx.x == 0) s_next = 0;
  SelT* sell = reinterpret_cast<SelT*>(bacc + ((nacc + 3) & ~3));
  {
    uint8_t* sb = reinterpret_cast<uint8_t*>(sell);
    const int g0 = t.group * ns;
    auto put = [&](int c, int l, uint32_t v) { sb[(c * L + l % L) * F + l / L] = (uint8_t)v; };
    if (((is | k | ns | (int)(reinterpret_cast<uintptr_t>(sp_index) & 3)) & 3) == 0) {
      // 4 selectors per load: a dword never straddles k (k % 4 == 0), so it is all slots or
      // all padding
      const int W4 = ns >> 2;
      for (int i = threadIdx.x; i < t.ncols * W4; i += NT) {
        const int c = i / W4, l0 = 4 * (i - c * W4);
        const int col = corder ? corder[t.col0 + c] : t.col0 + c;
        const uint32_t w = g0 + l0 < k
            ? *reinterpret_cast<const uint32_t*>(sp_index + (size_t)col * is + g0 + l0) : 0u;
#pragma unroll
        for (int b = 0; b < 4; ++b) put(c, l0 + b, (w >> (8 * b)) & 0xffu);
      }
    } else {
      for (int i = threadIdx.x; i < t.ncols * ns; i += NT) {
        const int c = i / ns, l = i - c * ns;
        const int col = corder ? corder[t.col0 + c] : t.col0 + c;
        put(c, l, g0 + l < k ? sp_index[(size_t)col * is + g0 + l] : 0u);
      }
    }
  }
  __syncthreads();

  const int EPS = kWave / L;
  const int lane = threadIdx.x & (kWave - 1);
  const int slot = lane / L;
  const int q = lane - slot * L;
  const bool lane_on = slot < EPS;
  const __amdgpu_buffer_rsrc_t gr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G), (short)0, (int)g_bytes, 0x00020000);
  const SelT* selb = sell + q;
  unsigned* accq = reinterpret_cast<unsigned*>(bacc) + F * q;
  const uint3* rec3 = reinterpret_cast<const uint3*>(rec);
  const int qq = lane & 3;

  // U sub-steps of EPS edges from `base` (sub-step u, slot s: edge base + u EPS + s, or with Q
  // lane q of a quad loads sub-step 4j + q's record), gathered from G, up to edge e_end
  auto gather_window = [&](int base, int e_end) {
    uint32_t go[U], cl[U];
    float v[U];
    bool ok[U];
    if constexpr (Q) {
      uint3 rq[U / 4];
#pragma unroll
      for (int j = 0; j < U / 4; ++j) rq[j] = rec3[base + (4 * j + qq) * EPS + slot];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ok[u] = lane_on && base + u * EPS + slot < e_end;
        go[u] = quad_pick(rq[u / 4].x, u);
        cl[u] = quad_pick(rq[u / 4].y, u);
        v[u] = __uint_as_float(quad_pick(rq[u / 4].z, u));
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + u * EPS + slot;
        ok[u] = lane_on && e < e_end;
        const uint3 r3 = rec3[e];
        go[u] = r3.x;
        cl[u] = r3.y;
        v[u] = __uint_as_float(r3.z);
      }
    }
    uint32_t s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) s[u] = selb[cl[u] * L];
    float x[U][F];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int i = 0; i < F; ++i) {
        const uint32_t f = (s[u] >> (8 * i)) & 0xffu;
        if constexpr (BIG) {
          x[u][i] = G[(size_t)go[u] * D + f];
        } else {
          x[u][i] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(gr, go[u] + (f << 2), 0, 0));
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < F; ++i) x[u][i] *= v[u];
    bwd_cas_update<U, F>(accq, KS, cl, x, ok);
  };

  // Windows of U sub-steps: window i of wave w is w + i * waves (static interleave), or
  // (handout, plan->bwd_handout 2) the next one handed out, in stream order, by an LDS counter
  // (one ds_add_rtn per window per wave), so a wave slowed by CAS retries or misses takes
  // fewer windows (the LDS-staged dense-run candidate owed its gain to this).
  const int wave = threadIdx.x / kWave;
  constexpr int kWaves = NT / kWave;
  for (int i = 0;; ++i) {
    int w = wave + i * kWaves;
    if (handout) {
      int c = 0;
      if (lane == 0) c = atomicAdd(&s_next, 1);
      w = __builtin_amdgcn_readlane(c, 0);
    }
    const int base = t.e0 + w * (EPS * U);
    if (base >= t.e1) break;
    gather_window(base, t.e1);
  }
  __syncthreads();

  // store: piece 0 of a block (or an unsplit block) into grad_sp, piece p > 0 into its slab
  // region (block positions, summed by bwd_combine_kernel), or (no slabs) global atomics into
  // a zeroed grad_sp; corder maps block positions to the columns of grad_sp. Padding slots
  // (>= k) are dropped.
  const bool atomic = t.shared && !slab;
  const bool to_slab = slab && t.slab >= 0;
  float* dst = to_slab ? slab + t.slab : grad_sp;
  const int g0 = t.group * ns;
  const int n = t.ncols * ns;
  for (int i = threadIdx.x; i < n; i += NT) {
    const int c = i / ns;
    const int l = i - c * ns;
    if (g0 + l >= k) continue;
    const float a = bacc[c * KS + (l % L) * F + l / L];
    const size_t row = to_slab ? (size_t)c : (size_t)(corder ? corder[t.col0 + c] : t.col0 + c);
    if (atomic) global_add(dst + row * k + g0 + l, a);
    else dst[row * k + g0 + l] = a;
  }
  MAXK_BWD_PROBE_END();
}

// Slab flush, second step: the blocks with several pieces add their slab regions (piece 1, 2,
// ... in order) into grad_sp, which piece 0 stored, so the result does not depend on which
// work-group finished first. comb[blockIdx.y] = {float offset of the block's first region,
// regions, col0, ncols}; regions are region_floats = C * k apart; blockIdx.x picks a slice of
// kCombineSlice floats of the block (one work-group per block was 40 work-groups on
// ogbn-proteins at k = 8, about 50 us).
constexpr int kCombineSlice = 1024;
__global__ __launch_bounds__(256) void bwd_combine_kernel(float* __restrict__ grad_sp,
                                                          const float* __restrict__ slab,
                                                          const int4* __restrict__ comb, int k,
                                                          int region_floats,
                                                          const int32_t* __restrict__ corder) {
  const int4 cb = comb[blockIdx.y];
  const int n = min(cb.w * k, (int)(blockIdx.x + 1) * kCombineSlice);
  const int i0 = blockIdx.x * kCombineSlice;
  // element i of the block (position cb.z + i / k) lives in grad_sp row corder[position]
  auto gp = [&](int i) -> float* {
    const int c = i / k;
    return grad_sp + (size_t)(corder ? corder[cb.z + c] : cb.z + c) * k + (i - c * k);
  };
  const float* sl = slab + cb.x;
  if ((k & 3) == 0) {
    for (int i = i0 + threadIdx.x * 4; i < n; i += 256 * 4) {
      float* g = gp(i);  // k % 4 == 0: the 4 elements share a column
      float4 a = *reinterpret_cast<const float4*>(g);
      for (int j = 0; j < cb.y; ++j) {
        const float4 b = *reinterpret_cast<const float4*>(sl + (size_t)j * region_floats + i);
        a.x += b.x;
        a.y += b.y;
        a.z += b.z;
        a.w += b.w;
      }
      *reinterpret_cast<float4*>(g) = a;
    }
  } else {
    for (int i = i0 + threadIdx.x; i < n; i += 256) {
      float* g = gp(i);
      float a = *g;
      for (int j = 0; j < cb.y; ++j) a += sl[(size_t)j * region_floats + i];
      *g = a;
    }
  }
}

// --------------------------------------------------------------------------------------
// backward: two passes (low row reuse)
// --------------------------------------------------------------------------------------
// Pass 1: one wavefront per R consecutive destination rows stages their grad_out rows in its
// LDS once, then walks their (contiguous) edges 64/L at a time (L = k/4 lanes per edge): lane
// q of an edge on column c reads the 4 selectors sp_index[c][4q..4q+3] (one dword),
// multiplies the 4 staged features of the edge's row (row % R from the edge record) by val
// and stores them as one float4 into the edge's slot T[e][4q..] (CSR order: the slots of a
// wavefront are contiguous, the stores coalesce; in column order the scattered stores ran
// 7-18 % slower, profiles/r02/bwd_probe/twopass_store_order.jsonl). The only gathers left on
// the texture path are the k selector bytes per edge; grad_out is read once.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, int R>
__global__ __launch_bounds__(256) void sspmm_bwd_rows_kernel(
    const int32_t* __restrict__ ptr, const uint32_t* __restrict__ erec,
    const float* __restrict__ G, const uint8_t* __restrict__ sp_index, int is,
    float* __restrict__ T, int rbeg, int rend, int64_t ebase, int D, int k) {
  // R rows of kMaxDim floats per wavefront (any u8 selector stays inside the wave's rows).
  // This launch covers destination rows [rbeg, rend), whose edges [ptr[rbeg], ptr[rend])
  // have their slots at T + (e - ebase) * k (one row chunk of the workspace)
  __shared__ float grow[256 / kWave][R * kMaxDim];
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int r0 = rbeg + (blockIdx.x * (256 / kWave) + w) * R;
  if (r0 >= rend) return;
  const int N = rend;
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
      for (int i = 0; i < kMaxDim / kWave; ++i) {
        const int f = lane + i * kWave;
        const float y = g[min(f, D - 1)];  // unconditional: all R rows' loads in flight
        x[j][i] = f < D ? y : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
      for (int i = 0; i < kMaxDim / kWave; ++i) grow[w][j * kMaxDim + lane + i * kWave] = x[j][i];
  }
  // the rows are written and read by this wavefront only
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int L = k >> 2;  // power of two <= 64 (checked by the plan)
  const int EPS = kWave / L;
  const int slot = lane / L;
  const int q = lane - slot * L;
  const float* row = grow[w];
  // branchless: idle slots load the row's last edge again and their stores fall outside the
  // row's buffer range (dropped), so every load of a step is in flight together
  const __amdgpu_buffer_rsrc_t tr = __builtin_amdgcn_make_buffer_rsrc(
      T + (size_t)(e0 - ebase) * k, (short)0, (int)((uint32_t)(e1 - e0) * (uint32_t)k * 4u),
      0x00020000);
  auto compute_store = [&](int base, const uint32_t (&c)[U], const float (&v)[U],
                           const uint32_t (&sw)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * EPS + slot;
      const float* rw = row + (R > 1 ? (c[u] >> kFwdColBits) * kMaxDim : 0);
      const uint32_t off = e < e1 ? ((uint32_t)(e - e0) * (uint32_t)k + 4u * q) * 4u : 0xfffffff0u;
      u32x4 o;
      o.x = __float_as_uint(v[u] * rw[sw[u] & 0xffu]);
      o.y = __float_as_uint(v[u] * rw[(sw[u] >> 8) & 0xffu]);
      o.z = __float_as_uint(v[u] * rw[(sw[u] >> 16) & 0xffu]);
      o.w = __float_as_uint(v[u] * rw[sw[u] >> 24]);
      // nontemporal (aux = 2): the workspace is far larger than the caches (Reddit k = 16
      // 5.58 -> 5.35 ms for both passes, ogbn-products k = 32 8.71 -> 8.56)
      __builtin_amdgcn_raw_buffer_store_b128(o, tr, off, 0, 2);
    }
  };
  auto load_sel = [&](const uint32_t (&c)[U], uint32_t (&sw)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      sw[u] = *reinterpret_cast<const uint32_t*>(sp_index + (size_t)(c[u] & kFwdColMask) * is + 4 * q);
  };
  uint32_t c[U], sw[U];
  float v[U];
  if constexpr ((U & 3) == 0) {
    if ((L & 3) == 0) {
      // lane q of a quad loads the record of sub-step 4j + q (contiguous), DPP hands it on: one
      // record instruction per four sub-steps. Software-pipelined: per step i the issue order is
      // selectors of step i+1, records of step i+2, then step i's LDS reads and stores, so no
      // load's wait covers an older store (vmcnt counts stores with loads in issue order; the
      // unpipelined loop waited for the previous step's stores before every step's selectors:
      // ogbn-products k = 32 row pass 5.37 -> 5.25 ms, profiles/r04/tp_rows_pipelined.jsonl).
      // Every load is clamped to a valid edge of the rows, no branches.
      const int qq = lane & 3;
      const int S = EPS * U;
      auto load_raw = [&](int b, uint2 (&raw)[U / 4]) {
#pragma unroll
        for (int j = 0; j < U / 4; ++j)
          raw[j] = *reinterpret_cast<const uint2*>(
              erec + 2 * (size_t)min(b + (4 * j + qq) * EPS + slot, e1 - 1));
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
        for (int u = 0; u < U; ++u) {
          c[u] = cn[u];
          v[u] = vn[u];
          sw[u] = swn[u];
        }
      }
      return;
    }
  }
  for (int base = e0; base < e1; base += EPS * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = min(base + u * EPS + slot, e1 - 1);
      const uint2 cv = *reinterpret_cast<const uint2*>(erec + 2 * (size_t)e);
      c[u] = cv.x;  // column | (row % R) << kFwdColBits
      v[u] = __uint_as_float(cv.y);
    }
    load_sel(c, sw);
    compute_store(base, c, v, sw);
  }
}

// Pass 2: one wavefront per column c sums the slots of the column's in-edges perm[lo[c] ..
// hi[c]) (64/L slots per step, float4 per lane), reduces over the slots with shuffles and
// stores grad_sp[c] (every column written once: no memset, no atomics). Row chunks
// (plan->bwd_tp_chunks > 1): this pass covers the in-edges of one row chunk, whose slots are
// at T + (perm - ebase) * k; chunk 0 stores, later chunks add to the stored sums in chunk
// order (deterministic).
template <int U>
__global__ __launch_bounds__(256) void sspmm_bwd_cols_kernel(
    const int32_t* __restrict__ lo, const int32_t* __restrict__ hi,
    const int32_t* __restrict__ perm, const float* __restrict__ T, int64_t ebase,
    float* __restrict__ grad_sp, int ncols, int k, int accumulate) {
  const int lane = threadIdx.x & (kWave - 1);
  const int c = blockIdx.x * (256 / kWave) + threadIdx.x / kWave;
  if (c >= ncols) return;
  const int L = k >> 2;
  const int EPS = kWave / L;
  const int slot = lane / L;
  const int q = lane - slot * L;
  const int e0 = lo[c], e1 = hi[c];
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int base = e0; base < e1; base += EPS * U) {
    int32_t pe[U];
    if ((U & 3) == 0 && (L & 3) == 0) {
      // lane q of a quad loads the permutation entry of sub-step 4j + q, DPP hands it on
      const int qq = lane & 3;
#pragma unroll
      for (int jj = 0; jj < U / 4; ++jj) {
        const uint32_t w = (uint32_t)(perm[min(base + (4 * jj + qq) * EPS + slot, e1 - 1)] - ebase);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int u = 4 * jj + i;
          if (u >= U) break;
          pe[u] = (int32_t)quad_pick(w, i);
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u)
        pe[u] = (int32_t)(perm[min(base + u * EPS + slot, e1 - 1)] - ebase);
    }
    float4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // idle slots load a valid slot again and drop it (no branch around the loads)
      const float4 x = *reinterpret_cast<const float4*>(T + (size_t)pe[u] * k + 4 * q);
      const bool ok = base + u * EPS + slot < e1;
      t[u] = make_float4(ok ? x.x : 0.f, ok ? x.y : 0.f, ok ? x.z : 0.f, ok ? x.w : 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc.x += t[u].x;
      acc.y += t[u].y;
      acc.z += t[u].z;
      acc.w += t[u].w;
    }
  }
  for (int m = L; m < kWave; m <<= 1) {
    acc.x += __shfl_xor(acc.x, m, kWave);
    acc.y += __shfl_xor(acc.y, m, kWave);
    acc.z += __shfl_xor(acc.z, m, kWave);
    acc.w += __shfl_xor(acc.w, m, kWave);
  }
  if (slot == 0) {
    float4* dst = reinterpret_cast<float4*>(grad_sp + (size_t)c * k + 4 * q);
    if (accumulate) {
      const float4 o = *dst;
      acc.x += o.x;
      acc.y += o.y;
      acc.z += o.z;
      acc.w += o.w;
    }
    *dst = acc;
  }
}

// --------------------------------------------------------------------------------------
// dense comparator
// --------------------------------------------------------------------------------------
// Dense CSR SpMM (DGL update_all(copy_u, sum) with edge weights: the ReLU layers' dense
// aggregation and the dense comparator). One wavefront per destination row; the row's
// D/4 float4 chunks take L lanes (the next power of two, <= 64) and the wave's 64/L edge
// slots walk the row's edges in a strided order with U loads in flight, then the slots
// are summed with lane shuffles. D = 64 (Flickr hidden size): 16 lanes per edge, 4 edges
// per instruction instead of 48 idle lanes.
template <int L, int U>
__global__ __launch_bounds__(256) void dense_spmm_kernel(
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
    const float* __restrict__ val, const float* __restrict__ X, float* __restrict__ Y,
    int N, int D) {
  constexpr int S = kWave / L;  // edge slots per wave instruction
  const int lane = threadIdx.x & (kWave - 1);
  const int row = blockIdx.x * (256 / kWave) + threadIdx.x / kWave;
  if (row >= N) return;  // wave-uniform
  const int slot = lane / L;
  const int q = lane - slot * L;
  const int e0 = ptr[row], e1 = ptr[row + 1];
  const int C4 = D >> 2;
  for (int c0 = 0; c0 < C4; c0 += L) {
    const int c = c0 + q;
    const bool on = c < C4;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int base = e0 + slot; base < e1; base += S * U) {
      float v[U];
      float4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + u * S;
        const bool ok = e < e1;
        const int ec = ok ? e : e1 - 1;
        v[u] = ok ? val[ec] : 0.f;
        x[u] = on ? *reinterpret_cast<const float4*>(X + (size_t)idx[ec] * D + 4 * c)
                  : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        a.x = fmaf(v[u], x[u].x, a.x);
        a.y = fmaf(v[u], x[u].y, a.y);
        a.z = fmaf(v[u], x[u].z, a.z);
        a.w = fmaf(v[u], x[u].w, a.w);
      }
    }
#pragma unroll
    for (int m = L; m < kWave; m <<= 1) {
      a.x += __shfl_xor(a.x, m);
      a.y += __shfl_xor(a.y, m);
      a.z += __shfl_xor(a.z, m);
      a.w += __shfl_xor(a.w, m);
    }
    if (slot == 0 && on) *reinterpret_cast<float4*>(Y + (size_t)row * D + 4 * c) = a;
  }
}

size_t fwd_lds_bytes(int tile_rows, int D) {
  return (size_t)tile_rows * (D + kFwdRowPad) * sizeof(double);
}

// LDS of a column-block work-group: C x KS f32 accumulators, then C x ns selector bytes
size_t bwd_lds_bytes(int block_cols, int ks) {
  return ((size_t)block_cols * ks + 3) / 4 * 4 * sizeof(float) + (size_t)block_cols * ks;
}

template <typename K>
static hipError_t allow_lds(K* kernel, size_t bytes) {
  return hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)bytes);
}

}  // namespace maxk

using namespace maxk;

// Fixed-point statistics of a CBSR table into two zeroed words: the lane-parallel kernel
// for k % 4 == 0 (~10 us for Reddit at k = 16), one thread per row otherwise. Rows of the
// table are ds floats (values) / is bytes (selectors) apart.
// rec != nullptr (k % 4 == 0 only): also pack the forward's CBSR records (st0 == nullptr: the
// pack alone); zrows/nz/out/D (k % 4 == 0 only): split rows of the forward to zero in the
// same launch.
static int launch_cbsr_stats(const float* sp_data, int ds, const uint8_t* sp_index, int is,
                             int64_t nrows, int k, uint32_t* st0, uint32_t* st1, int cus,
                             hipStream_t s, uint8_t* rec = nullptr, int rec_bytes = 0,
                             const int32_t* zrows = nullptr, int nz = 0, float* out = nullptr,
                             int D = 0, bool pairs = false) {
  if (nrows <= 0) return MAXK_OK;
  if (k % 4 == 0) {
    const int64_t rows_per_block = (256 / kWave) * (kWave / (k / 4));
    // statistics: one work-group per CU, each adds one atomic per word, and same-address
    // atomics from every work-group serialise at the L2; the pack alone: more in flight
    const int cap = st0 ? cus * kStatsBlocksPerCu : 8 * cus;
    const int grid = (int)std::max<int64_t>(
        1, std::min<int64_t>((nrows + rows_per_block - 1) / rows_per_block, cap));
#define STATS4(PK, ST)                                                                      \
  hipLaunchKernelGGL((cbsr_stats4_kernel<PK, ST>), dim3(grid), dim3(256), 0, s, sp_data, sp_index, \
                     nrows, k, st0, st1, rec, rec_bytes, zrows, nz, out, D, ds, is)
    if (rec && st0 && pairs) STATS4(2, true);
    else if (rec && pairs) STATS4(2, false);
    else if (rec && st0) STATS4(1, true);
    else if (rec) STATS4(1, false);
    else STATS4(0, true);
#undef STATS4
  } else {
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((nrows + 255) / 256, 2 * cus));
    hipLaunchKernelGGL(cbsr_stats_kernel, dim3(grid), dim3(256), 0, s, sp_data, sp_index, nrows,
                       k, st0, st1, ds, is);
  }
  MAXK_LAUNCH_CHECK("cbsr_stats launch");
  return MAXK_OK;
}

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

// Table row strides: 0 means k; values in floats, selectors in bytes.
static int table_strides(int64_t& ds, int64_t& is, int k, const char* who) {
  if (ds == 0) ds = k;
  if (is == 0) is = k;
  MAXK_CHECK_ARG(ds >= k && is >= k && ds <= INT32_MAX / 4 && is <= INT32_MAX,
                 std::string(who) + ": table row strides must be >= k (0: k)");
  return MAXK_OK;
}

static int spgemm_forward_impl(const maxk_plan* plan, const int32_t* ptr, const int32_t* idx,
                               const float* val, const float* sp_data, int64_t ds64,
                               const uint8_t* sp_index, int64_t is64, float* out, int32_t N,
                               int64_t E, int32_t k, int32_t D, void* stream, int accum,
                               void* ws, int64_t ws_bytes, const uint32_t* stats = nullptr,
                               int n_stats = 0, int64_t stats_stride = 2) {
  MAXK_CHECK_ARG(N >= 0 && E >= 0, "maxk_spgemm_forward: negative size");
  MAXK_CHECK_ARG(stats == nullptr || (n_stats >= 1 && n_stats <= 1024),
                 "maxk_spgemm_forward_ex: n_stats must be in [1, 1024]");
  if (stats_stride == 0) stats_stride = 2;
  MAXK_CHECK_ARG(stats_stride >= 2 && stats_stride * (int64_t)n_stats < (int64_t)INT32_MAX,
                 "maxk_spgemm_forward_ex: stats_stride must be >= 2 (or 0)");
  MAXK_CHECK_ARG(D >= 1 && D <= kMaxDim, "maxk_spgemm_forward: dim_origin must be in [1, 256]");
  MAXK_CHECK_ARG(k >= 1 && k <= D, "k must be between 1 and input dimension");
  if (int rc = table_strides(ds64, is64, k, "maxk_spgemm_forward")) return rc;
  const int ds = (int)ds64, is = (int)is64;
  int rc = check_plan(plan, ptr, idx, N, E, k, D, "maxk_spgemm_forward");
  if (rc) return rc;
  if (N == 0) return MAXK_OK;
  MAXK_CHECK_ARG(out && sp_data && sp_index && (E == 0 || (idx && val)) && ptr,
                 "maxk_spgemm_forward: null pointer");
  (void)val;  // the plan holds the permuted snapshot of (idx, val)
  uint8_t* ws_base = plan->fwd_rec;  // packed CBSR records + statistics words (per call)
  if (ws) {
    MAXK_CHECK_ARG(ws_bytes >= plan->fwd_ws_bytes,
                   "maxk_spgemm_forward: workspace smaller than maxk_plan_workspace_bytes");
    ws_base = static_cast<uint8_t*>(ws);
  } else if (plan->fwd_ws_bytes > 0 && !ws_base) {
    set_error("maxk_spgemm_forward: the plan has an external workspace; use maxk_spgemm_forward_ws");
    return MAXK_ERR_INVALID_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  uint8_t* rec_ws = ws_base;
  // split rows are summed atomically into zeroed rows: zeroed by the statistics / pack launch
  // when there is one (k % 4 == 0), else by a launch of their own
  const int nz = accum ? 0 : plan->n_zero_rows;
  const size_t lds = fwd_lds_bytes(plan->fwd_tile_rows, D);
  // the caller's tables are already interleaved CBSR records {k values, k selectors} (the
  // multi-GPU path all-gathers them so): gather from them as they are, no per-call pack
  const bool inplace = k % 4 == 0 && !plan->fwd_chunk3 && !plan->fwd_chunk2 &&
                       sp_index == reinterpret_cast<const uint8_t*>(sp_data) + 4 * (size_t)k &&
                       is == 4 * ds;
  // two tables: values read straight from sp_data (ds floats per row), selectors from sp_index
  const bool two = plan->fwd_two_tables && !inplace;  // the plan only sets it with k % 4 == 0
  const uint8_t* seltab = two ? sp_index : nullptr;
  const uint8_t* recp = (two || inplace) ? reinterpret_cast<const uint8_t*>(sp_data) : rec_ws;
  const int rec_bytes = (two || inplace) ? 4 * ds : plan->fwd_rec_bytes;
  // fixed-point forward: the call's slot bound / min |x| for fwd_fix_scale (one pass over the
  // CBSR table, fused with the record pack when there is one), or the caller's per-rank pairs
  // (maxk_spgemm_forward_ex)
  const int2* fix_tab = nullptr;
  const uint32_t* xstat = nullptr;
  uint32_t* st = nullptr;
  int xs_n = 1, xs_stride = 0, xs_off2 = 32;
  if (plan->fwd_fix && plan->num_cols > 0) {
    fix_tab = plan->fwd_fix;
    if (stats) {
      xstat = stats;
      xs_n = n_stats;
      xs_stride = (int)stats_stride;
      xs_off2 = 1;
    } else {
      st = reinterpret_cast<uint32_t*>(ws_base + plan->fwd_xstat_off);
      MAXK_HIP_TRY(hipMemsetAsync(st, 0, 256, s));
      xstat = st;
    }
  }
  // pair chunks: packed by the statistics / pack pass when k % 4 == 0, else on their own;
  // interleaved records are repacked too (W = 8 shard at k = 16: 0.356 ms compute with the
  // repack against 0.358 gathering the records in place, profiles/r06/fwd_pair_chunks.jsonl)
  const bool pairs = plan->fwd_chunk2;
  const bool pack4 = !two && !inplace && !plan->fwd_chunk3 && k % 4 == 0 && plan->num_cols > 0;
  if ((plan->fwd_chunk3 || (pairs && k % 4 != 0)) && plan->num_cols > 0) {
    const int V = plan->fwd_chunk3 ? 3 : 2;
    const int64_t items = (int64_t)plan->num_cols * ((k + V - 1) / V);
    const int grid = (int)std::min<int64_t>((items + 255) / 256, 65536);
    hipLaunchKernelGGL(V == 3 ? pack_cbsr3_kernel<3> : pack_cbsr3_kernel<2>, dim3(grid), dim3(256),
                       0, s, sp_data, sp_index, rec_ws, plan->num_cols, k, plan->fwd_rec_bytes,
                       ds, is);
    MAXK_LAUNCH_CHECK("pack_cbsr3 launch");
  }
  const bool zero_in_stats = (pack4 || st) && k % 4 == 0;
  if (nz > 0 && !zero_in_stats) {
    hipLaunchKernelGGL(zero_rows_kernel, dim3(nz), dim3(256), 0, s, plan->zero_rows, nz, out, D);
    MAXK_LAUNCH_CHECK("zero_rows launch");
  }
  if (pack4 || st) {
    const int rc2 = launch_cbsr_stats(sp_data, ds, sp_index, is, plan->num_cols, k, st,
                                      st ? st + 32 : nullptr, plan->cus, s,
                                      pack4 ? rec_ws : nullptr, plan->fwd_rec_bytes,
                                      plan->zero_rows, zero_in_stats ? nz : 0, out, D, pairs);
    if (rc2) return rc2;
  }
  if (plan->n_fwd_tasks == 0) return MAXK_OK;
  const int Lf = plan->fwd_chunk3 ? (k + 2) / 3 : pairs ? k / 2 : k / 4;  // lanes per edge
  const int FL = (plan->fwd_chunk3 ? kFwdFlagChunk3 : 0) | (pairs ? kFwdFlagChunk2 : 0) |
                 (plan->fwd_quad && Lf % 4 == 0 ? kFwdFlagQuad : 0);
  const int fwaves = plan->fwd_waves;
#define FWD_LAUNCH_NT(V, FF, NT, FU)                                                        \
  do {                                                                                      \
    if (lds > 64 * 1024) MAXK_HIP_TRY(allow_lds(spgemm_fwd_kernel<V, FF, NT, FU>, lds));     \
    hipLaunchKernelGGL((spgemm_fwd_kernel<V, FF, NT, FU>), dim3(plan->n_fwd_tasks), dim3(NT), \
                       lds, s, plan->fwd_tasks, plan->fwd_phase_off, plan->fwd_phases,      \
                       plan->fwd_cv, sp_data, sp_index, recp, rec_bytes, out, D, k,         \
                       plan->fwd_rot_ticks, seltab, is, ds, accum, fix_tab, xstat, xs_n,     \
                       xs_stride, xs_off2, plan->fwd_handout == 2 ? 1 : 0);                 \
  } while (0)
#define FWD_LAUNCH(V, FF)                                                                   \
  do {                                                                                      \
    if (fwaves == 8 && plan->fwd_unroll == 4) FWD_LAUNCH_NT(V, FF, 8 * kWave, 4);            \
    else if (fwaves == 8) FWD_LAUNCH_NT(V, FF, 8 * kWave, kFwdUnroll);                      \
    else FWD_LAUNCH_NT(V, FF, kFwdThreads, kFwdUnroll);                                     \
  } while (0)
  if (k % 4 == 0 || plan->fwd_chunk3 || plan->fwd_chunk2) {
    switch (FL) {
      case 0: FWD_LAUNCH(4, 0); break;
      case kFwdFlagChunk3: FWD_LAUNCH(4, kFwdFlagChunk3); break;
      case kFwdFlagQuad: FWD_LAUNCH(4, kFwdFlagQuad); break;
      case kFwdFlagChunk2: FWD_LAUNCH(4, kFwdFlagChunk2); break;
      case kFwdFlagChunk2 | kFwdFlagQuad: FWD_LAUNCH(4, kFwdFlagChunk2 | kFwdFlagQuad); break;
      default: FWD_LAUNCH(4, kFwdFlagChunk3 | kFwdFlagQuad); break;
    }
  } else {
    FWD_LAUNCH(1, 0);
  }
#undef FWD_LAUNCH
#undef FWD_LAUNCH_NT
  MAXK_LAUNCH_CHECK("spgemm_fwd launch");
  return MAXK_OK;
}

extern "C" int maxk_spgemm_forward(const maxk_plan* plan, const int32_t* ptr,
                                   const int32_t* idx, const float* val,
                                   const float* sp_data, const uint8_t* sp_index, float* out,
                                   int32_t N, int64_t E, int32_t k, int32_t D, void* stream) {
  return spgemm_forward_impl(plan, ptr, idx, val, sp_data, 0, sp_index, 0, out, N, E, k, D,
                             stream, 0, nullptr, 0);
}

extern "C" int maxk_spgemm_forward_ws(const maxk_plan* plan, const int32_t* ptr,
                                      const int32_t* idx, const float* val,
                                      const float* sp_data, const uint8_t* sp_index, float* out,
                                      int32_t N, int64_t E, int32_t k, int32_t D,
                                      int32_t accumulate, void* workspace,
                                      int64_t workspace_bytes, void* stream) {
  MAXK_CHECK_ARG(accumulate == 0 || accumulate == 1,
                 "maxk_spgemm_forward_ws: accumulate must be 0 or 1");
  return spgemm_forward_impl(plan, ptr, idx, val, sp_data, 0, sp_index, 0, out, N, E, k, D,
                             stream, accumulate, workspace, workspace_bytes);
}

extern "C" int maxk_spgemm_forward_ex(const maxk_plan* plan, const int32_t* ptr,
                                      const int32_t* idx, const float* val,
                                      const float* sp_data, const uint8_t* sp_index, float* out,
                                      int32_t N, int64_t E, int32_t k, int32_t D,
                                      int32_t accumulate, const uint32_t* stats,
                                      int32_t n_stats, int64_t stats_stride, void* workspace,
                                      int64_t workspace_bytes, void* stream) {
  MAXK_CHECK_ARG(accumulate == 0 || accumulate == 1,
                 "maxk_spgemm_forward_ex: accumulate must be 0 or 1");
  return spgemm_forward_impl(plan, ptr, idx, val, sp_data, 0, sp_index, 0, out, N, E, k, D,
                             stream, accumulate, workspace, workspace_bytes, stats, n_stats,
                             stats_stride);
}

extern "C" int maxk_spgemm_forward_tables(const maxk_plan* plan, const int32_t* ptr,
                                          const int32_t* idx, const float* val,
                                          const float* sp_data, int64_t data_stride,
                                          const uint8_t* sp_index, int64_t index_stride,
                                          float* out, int32_t N, int64_t E, int32_t k, int32_t D,
                                          int32_t accumulate, const uint32_t* stats,
                                          int32_t n_stats, int64_t stats_stride,
                                          void* workspace, int64_t workspace_bytes,
                                          void* stream) {
  MAXK_CHECK_ARG(accumulate == 0 || accumulate == 1,
                 "maxk_spgemm_forward_tables: accumulate must be 0 or 1");
  return spgemm_forward_impl(plan, ptr, idx, val, sp_data, data_stride, sp_index, index_stride,
                             out, N, E, k, D, stream, accumulate, workspace, workspace_bytes,
                             stats, n_stats, stats_stride);
}

extern "C" int maxk_cbsr_stats_tables(const float* sp_data, int64_t data_stride,
                                      const uint8_t* sp_index, int64_t index_stride,
                                      int32_t num_rows, int32_t dim_k, uint32_t* stats,
                                      void* stream) {
  MAXK_CHECK_ARG(num_rows >= 0 && dim_k >= 1 && dim_k <= kMaxDim,
                 "maxk_cbsr_stats: bad size");
  MAXK_CHECK_ARG(stats != nullptr && (num_rows == 0 || (sp_data && sp_index)),
                 "maxk_cbsr_stats: null pointer");
  if (int rc = table_strides(data_stride, index_stride, dim_k, "maxk_cbsr_stats")) return rc;
  hipStream_t s = (hipStream_t)stream;
  MAXK_HIP_TRY(hipMemsetAsync(stats, 0, 2 * sizeof(uint32_t), s));
  if (num_rows == 0) return MAXK_OK;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  return launch_cbsr_stats(sp_data, (int)data_stride, sp_index, (int)index_stride, num_rows,
                           dim_k, stats, stats + 1, cus, s);
}

extern "C" int maxk_cbsr_stats(const float* sp_data, const uint8_t* sp_index, int32_t num_rows,
                               int32_t dim_k, uint32_t* stats, void* stream) {
  return maxk_cbsr_stats_tables(sp_data, 0, sp_index, 0, num_rows, dim_k, stats, stream);
}

extern "C" int maxk_spgemm_forward_acc(const maxk_plan* plan, const int32_t* ptr,
                                       const int32_t* idx, const float* val,
                                       const float* sp_data, const uint8_t* sp_index,
                                       float* out, int32_t N, int64_t E, int32_t k, int32_t D,
                                       void* stream) {
  return spgemm_forward_impl(plan, ptr, idx, val, sp_data, 0, sp_index, 0, out, N, E, k, D,
                             stream, 1, nullptr, 0);
}

static int sspmm_backward_impl(const maxk_plan* plan, const int32_t* ptr, const int32_t* idx,
                               const float* val, const float* grad_out,
                               const uint8_t* sp_index, int64_t is64, float* grad_sp, int32_t N,
                               int64_t E, int32_t k, int32_t D, void* stream, void* ws,
                               int64_t ws_bytes) {
  (void)val;  // the plan holds the block-major snapshot of val
  MAXK_CHECK_ARG(N >= 0 && E >= 0, "maxk_sspmm_backward: negative size");
  MAXK_CHECK_ARG(D >= 1 && D <= kMaxDim, "maxk_sspmm_backward: dim_origin must be in [1, 256]");
  MAXK_CHECK_ARG(k >= 1 && k <= D, "k must be between 1 and input dimension");
  int64_t ds_unused = 0;
  if (int rc = table_strides(ds_unused, is64, k, "maxk_sspmm_backward")) return rc;
  const int is = (int)is64;
  int rc = check_plan(plan, ptr, idx, N, E, k, D, "maxk_sspmm_backward");
  if (rc) return rc;
  if (N == 0) return MAXK_OK;
  MAXK_CHECK_ARG(grad_out && sp_index && grad_sp, "maxk_sspmm_backward: null pointer");
  // per-call scratch: selector words + flush slabs (column blocks) or the E x k products
  // (two-pass)
  uint32_t* sel_ws = plan->bwd_sel;
  float* tbuf_ws = plan->bwd_tbuf;
  if (ws) {
    MAXK_CHECK_ARG(ws_bytes >= plan->bwd_ws_bytes,
                   "maxk_sspmm_backward: workspace smaller than maxk_plan_workspace_bytes");
    sel_ws = static_cast<uint32_t*>(ws);
    tbuf_ws = static_cast<float*>(ws);
  } else if (plan->bwd_ws_bytes > 0 && !sel_ws && !tbuf_ws) {
    set_error("maxk_sspmm_backward: the plan has an external workspace; use maxk_sspmm_backward_ws");
    return MAXK_ERR_INVALID_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const int NC = plan->num_cols;
  if (plan->bwd_twopass) {
    // the plan checked k % 4 == 0, k / 4 a power of two <= 64, E > 0, NC > 0; per row chunk
    // (the workspace holds one chunk's products): row pass, then column pass
    const int R = plan->bwd_tp_rows;
    const int P = plan->bwd_tp_chunks;
    for (int p = 0; p < P; ++p) {
      const int rb = plan->tp_rows[p], re = plan->tp_rows[p + 1];
      const int64_t eb = plan->tp_edges[p];
      if (re > rb) {
        const dim3 rgrid((re - rb + 4 * R - 1) / (4 * R));
#define ROWS_LAUNCH(RR)                                                                     \
        hipLaunchKernelGGL((sspmm_bwd_rows_kernel<4, RR>), rgrid, dim3(256), 0, s, ptr,    \
                           plan->bwd_erec, grad_out, sp_index, is, tbuf_ws, rb, re, eb, D, k)
        if (R >= 8) ROWS_LAUNCH(8);
        else if (R == 4) ROWS_LAUNCH(4);
        else if (R == 2) ROWS_LAUNCH(2);
        else ROWS_LAUNCH(1);
#undef ROWS_LAUNCH
        MAXK_LAUNCH_CHECK("sspmm_bwd_rows launch");
      }
      const int32_t* lo = P > 1 ? plan->bwd_colptr2 + (size_t)p * NC : plan->bwd_colptr;
      const int32_t* hi = P > 1 ? plan->bwd_colptr2 + (size_t)(p + 1) * NC : plan->bwd_colptr + 1;
      hipLaunchKernelGGL((sspmm_bwd_cols_kernel<4>), dim3((NC + 3) / 4), dim3(256), 0, s, lo, hi,
                         plan->bwd_perm, tbuf_ws, eb, grad_sp, NC, k, p > 0 ? 1 : 0);
      MAXK_LAUNCH_CHECK("sspmm_bwd_cols launch");
    }
    return MAXK_OK;
  }
  float* slab = plan->bwd_slab_floats > 0
                    ? reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(sel_ws) + plan->bwd_slab_off)
                    : nullptr;
  // no edges: no tasks, every gradient is zero; atomic flush: split blocks add into zeros
  if (plan->n_bwd_tasks == 0 || (plan->n_bwd_shared > 0 && !slab))
    MAXK_HIP_TRY(hipMemsetAsync(grad_sp, 0, (size_t)NC * k * sizeof(float), s));
  if (plan->n_bwd_tasks == 0) return MAXK_OK;
  const int F = plan->bwd_feats, ns = plan->bwd_ks;
  const int L = ns / F;
  const uint32_t g_bytes = plan->bwd_big ? 0u : (uint32_t)((uint64_t)N * D * 4u);
  const size_t lds = bwd_lds_bytes(plan->bwd_block_cols, ns);
  const dim3 grid(plan->n_bwd_tasks);
  const bool Q = L % 4 == 0;  // quad-aligned lane groups: batched record loads
  const int U = plan->bwd_unroll, W = plan->bwd_waves;
#define BWD_LAUNCH(UU, NT, FF, QQ, BB)                                                      \
  do {                                                                                      \
    if (lds > 64 * 1024) MAXK_HIP_TRY(allow_lds(sspmm_bwd4_kernel<UU, NT, FF, QQ, BB>, lds)); \
    hipLaunchKernelGGL((sspmm_bwd4_kernel<UU, NT, FF, QQ, BB>), grid, dim3(NT), lds, s,     \
                       plan->bwd_tasks, plan->bwd_rec, grad_out, g_bytes, D, sp_index, is,  \
                       grad_sp, k, ns, slab, plan->bwd_corder, plan->bwd_handout == 2 ? 1 : 0); \
  } while (0)
#define BWD_SHAPES(FF, QQ)                                                                  \
  do {                                                                                      \
    if (plan->bwd_big) BWD_LAUNCH(8, 512, FF, QQ, true);                                    \
    else if (W == 16) BWD_LAUNCH(8, 1024, FF, QQ, false);                                   \
    else if (W == 12 && U == 12) BWD_LAUNCH(12, 768, FF, QQ, false);                       \
    else if (W == 12) BWD_LAUNCH(8, 768, FF, QQ, false);                                    \
    else if (U == 16) BWD_LAUNCH(16, 512, FF, QQ, false);                                   \
    else if (U == 12) BWD_LAUNCH(12, 512, FF, QQ, false);                                   \
    else BWD_LAUNCH(8, 512, FF, QQ, false);                                                 \
  } while (0)
  if (F == 4) {
    if (Q) BWD_SHAPES(4, true);
    else BWD_SHAPES(4, false);
  } else {
    if (Q) BWD_SHAPES(2, true);
    else BWD_SHAPES(2, false);
  }
#undef BWD_SHAPES
#undef BWD_LAUNCH
  MAXK_LAUNCH_CHECK("sspmm_bwd launch");
  if (slab) {
    const int slices = (plan->bwd_block_cols * k + kCombineSlice - 1) / kCombineSlice;
    hipLaunchKernelGGL(bwd_combine_kernel, dim3(slices, plan->n_bwd_combine), dim3(256), 0, s,
                       grad_sp, slab, plan->bwd_combine, k, plan->bwd_block_cols * k,
                       plan->bwd_corder);
    MAXK_LAUNCH_CHECK("bwd_combine launch");
  }
  return MAXK_OK;
}

extern "C" int maxk_sspmm_backward(const maxk_plan* plan, const int32_t* ptr,
                                   const int32_t* idx, const float* val,
                                   const float* grad_out, const uint8_t* sp_index,
                                   float* grad_sp, int32_t N, int64_t E, int32_t k, int32_t D,
                                   void* stream) {
  return sspmm_backward_impl(plan, ptr, idx, val, grad_out, sp_index, 0, grad_sp, N, E, k, D,
                             stream, nullptr, 0);
}

extern "C" int maxk_sspmm_backward_ws(const maxk_plan* plan, const int32_t* ptr,
                                      const int32_t* idx, const float* val,
                                      const float* grad_out, const uint8_t* sp_index,
                                      float* grad_sp, int32_t N, int64_t E, int32_t k,
                                      int32_t D, void* workspace, int64_t workspace_bytes,
                                      void* stream) {
  return sspmm_backward_impl(plan, ptr, idx, val, grad_out, sp_index, 0, grad_sp, N, E, k, D,
                             stream, workspace, workspace_bytes);
}

extern "C" int maxk_sspmm_backward_tables(const maxk_plan* plan, const int32_t* ptr,
                                          const int32_t* idx, const float* val,
                                          const float* grad_out, const uint8_t* sp_index,
                                          int64_t index_stride, float* grad_sp, int32_t N,
                                          int64_t E, int32_t k, int32_t D, void* workspace,
                                          int64_t workspace_bytes, void* stream) {
  return sspmm_backward_impl(plan, ptr, idx, val, grad_out, sp_index, index_stride, grad_sp, N,
                             E, k, D, stream, workspace, workspace_bytes);
}

extern "C" int maxk_dense_spmm_csr(const int32_t* ptr, const int32_t* idx, const float* val,
                                   const float* X, float* Y, int32_t N, int32_t D,
                                   void* stream) {
  MAXK_CHECK_ARG(N >= 0 && D >= 1, "maxk_dense_spmm_csr: bad size");
  MAXK_CHECK_ARG(D % 4 == 0, "maxk_dense_spmm_csr: dim must be a multiple of 4");
  if (N == 0) return MAXK_OK;
  MAXK_CHECK_ARG(ptr && X && Y, "maxk_dense_spmm_csr: null pointer");
  const int C4 = D / 4;
  const dim3 grid((N + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (C4 > 32)
    hipLaunchKernelGGL((dense_spmm_kernel<64, 4>), grid, block, 0, s, ptr, idx, val, X, Y, N, D);
  else if (C4 > 16)
    hipLaunchKernelGGL((dense_spmm_kernel<32, 4>), grid, block, 0, s, ptr, idx, val, X, Y, N, D);
  else if (C4 > 8)
    hipLaunchKernelGGL((dense_spmm_kernel<16, 4>), grid, block, 0, s, ptr, idx, val, X, Y, N, D);
  else if (C4 > 4)
    hipLaunchKernelGGL((dense_spmm_kernel<8, 4>), grid, block, 0, s, ptr, idx, val, X, Y, N, D);
  else
    hipLaunchKernelGGL((dense_spmm_kernel<4, 4>), grid, block, 0, s, ptr, idx, val, X, Y, N, D);
  MAXK_LAUNCH_CHECK("dense_spmm launch");
  return MAXK_OK;
}
