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
//   forward : a 256-thread work-group owns <= 32 whole destination rows (LDS accumulator
//             rows x D); its edges are processed flat, k/4 lanes per edge, 4 features per
//             lane (one dwordx4 value gather + one dword selector gather; or lane chunks of
//             3 values + their selectors for k % 16 != 0), U independent sub-steps in
//             flight per wave; products are accumulated in LDS with f64 atomics
//             (ds_add_f64, ~9x the f32 rate), and the rows are written back once with
//             coalesced dwordx4 stores. Only rows longer than the task cap are split, and
//             only those touch global atomics.
//   backward: a 512-thread work-group owns a block of source columns whose k-wide
//             gradients live in LDS; it sweeps the block's edges in destination-row order
//             (plan-built block-major edge list), so the lanes of one instruction gather
//             from few rows of grad_out (L1 reuse); updates are 64-bit compare-and-swaps on
//             float pairs; the block is stored (or atomically flushed when it is split over
//             several work-groups) once at the end.
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace maxk {

// Accumulator kinds: MAXK_ACC_F64 (double, ds_add_f64) and MAXK_ACC_F32_CAS (float,
// ds_read + ds_cmpst_rtn_b32 loop: the integer CAS path runs at the f64-atomic rate).
template <int ACC>
struct LdsAcc;

// Quad-shared loads: the L lanes of an edge (L % 4 == 0, quad-aligned) need the same edge
// record; each lane loads ONE dword of it and quad_perm DPP moves broadcast the words, so
// the texture path returns 4 B per lane instead of the whole record per lane (PMC: TD busy
// ~93 % in both kernels, the record/edge-word loads were a third of its bytes).
template <int W>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
  static_assert(W >= 0 && W < 4, "quad lane");
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, W * 0x55, 0xf, 0xf, false);
}


// add(p, v): one accumulated term. The forward's edge loop uses scale(val, sc) once per edge
// and add2(p, scaled val, x) per slot, so the fixed-point accumulator below can fold the scale
// and the rounding into one fma.
template <>
struct LdsAcc<MAXK_ACC_F64> {
  using T = double;
  using V = float;
  static __device__ __forceinline__ void add(double* p, float v) {
    lds_add(p, (double)v);
  }
  static __device__ __forceinline__ V scale(float v, double) { return v; }
  static __device__ __forceinline__ void add2(double* p, float v, float x) { add(p, v * x); }
};

template <>
struct LdsAcc<MAXK_ACC_F32_CAS> {
  using T = float;
  using V = float;
  static __device__ __forceinline__ void add(float* p, float v) {
    unsigned* u = reinterpret_cast<unsigned*>(p);
    unsigned old = *u;
    while (true) {
      const unsigned assumed = old;
      old = atomicCAS(u, assumed, __float_as_uint(__uint_as_float(assumed) + v));
      if (old == assumed) break;
    }
  }
  static __device__ __forceinline__ V scale(float v, double) { return v; }
  static __device__ __forceinline__ void add2(float* p, float v, float x) { add(p, v * x); }
};

// Forward fixed-point accumulator (plan->fwd_fixed): ds_add_u64 runs at ~1.9x the ds_add_f64
// rate, and the f64 atomic bounds the forward at k >= 32 (tools/probe_fwd_build.py: Reddit
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

// cbsr_stats_kernel for k % 4 == 0 (k <= 256): L = k/4 lanes per row, each loading its 4
// values (float4) and their 4 selectors (one dword), rows 64/L per wave, coalesced. Per row,
// inclusive prefix scans over its L lanes (shuffles) give the sum of |x|, the max |x|, and
// whether a lane's first nonzero selector is <= the last nonzero selector of any earlier lane
// (or its own nonzero selectors do not ascend): the same bound as the thread-per-row kernel
// below, with the row sum added in another order (its 2^-10 headroom covers that).
//
// PACK: the same pass also writes the forward's packed CBSR records (pack_cbsr_kernel's
// layout: k values, then the k selector bytes, rec_bytes per row), so the per-call pack and
// the statistics cost one read of the tables. STATS = false: the pack alone.
template <bool PACK, bool STATS>
__global__ __launch_bounds__(256) void cbsr_stats4_kernel(const float* __restrict__ x,
                                                          const uint8_t* __restrict__ sel,
                                                          int64_t nrows, int k, uint32_t* st0,
                                                          uint32_t* st1, uint8_t* __restrict__ rec,
                                                          int rec_bytes,
                                                          const int32_t* __restrict__ zrows,
                                                          int nz, float* __restrict__ out, int D) {
  __shared__ uint32_t smx[256 / kWave], smn[256 / kWave];
  // the forward's split rows (summed atomically by their segments) start from zero: zeroed
  // here, one launch before the forward, instead of by a zero_rows_kernel launch of their own
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
      v = *reinterpret_cast<const float4*>(x + r * k + 4 * q);
      s = *reinterpret_cast<const uint32_t*>(sel + r * k + 4 * q);
      if constexpr (PACK) {
        uint8_t* rp = rec + r * rec_bytes;
        *reinterpret_cast<float4*>(rp + 16 * q) = v;
        *reinterpret_cast<uint32_t*>(rp + 4 * k + 4 * q) = s;
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
// launch; a few hundred work-groups reduce in LDS and add one atomic each per word (one
// atomic per wave on a shared word cost ~190 us at k = 16).
__global__ __launch_bounds__(256) void cbsr_stats_kernel(const float* __restrict__ x,
                                                         const uint8_t* __restrict__ sel,
                                                         int64_t nrows, int k, uint32_t* st0,
                                                         uint32_t* st1) {
  __shared__ uint32_t smx[256 / kWave], smn[256 / kWave];
  uint32_t mx = 0u, mn = 0x7fffffffu;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows;
       r += (int64_t)gridDim.x * blockDim.x) {
    uint32_t mb = 0u, lo = 0x7fffffffu;
    float sum = 0.f;
    int prev = -1;
    bool rep = false;
    auto take = [&](float v, int s) {
      const uint32_t b = __float_as_uint(v) & 0x7fffffffu;
      if (b == 0u) return;
      mb = max(mb, b);
      lo = min(lo, b);
      sum += __uint_as_float(b);
      rep = rep || s <= prev;
      prev = s;
    };
    const float* xr = x + r * k;
    const uint8_t* sr = sel + r * k;
    if ((k & 3) == 0) {
      for (int l = 0; l < k; l += 4) {
        const float4 v = *reinterpret_cast<const float4*>(xr + l);
        const uint32_t s = *reinterpret_cast<const uint32_t*>(sr + l);
        take(v.x, s & 0xffu);
        take(v.y, (s >> 8) & 0xffu);
        take(v.z, (s >> 16) & 0xffu);
        take(v.w, s >> 24);
      }
    } else {
      for (int l = 0; l < k; ++l) take(xr[l], sr[l]);
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
// second, selector, gather per lane). The gathers are bound by L1 line lookups per
// instruction, not by bytes (tools/ubench_tcp.hip); padding slots (3j+i >= k) are 0.
__global__ void pack_cbsr3_kernel(const float* __restrict__ sp_data,
                                  const uint8_t* __restrict__ sp_index,
                                  uint8_t* __restrict__ rec, int ncols, int k, int rec_bytes) {
  const int chunks = (k + 2) / 3;
  const int64_t total = (int64_t)ncols * chunks;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = t / chunks;
    const int j = (int)(t - c * chunks);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int l = 3 * j + i;
      if (l < k) {
        w[i] = __float_as_uint(sp_data[c * k + l]);
        w[3] |= (uint32_t)sp_index[c * k + l] << (8 * i);
      }
    }
    *reinterpret_cast<uint4*>(rec + c * rec_bytes + j * 16) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// One wave's share of the forward edges [e0, e1) (VEC = 4 lanes path): U sub-steps per
// iteration with every load issued before the first LDS update. The chain (col, val) ->
// CBSR record -> LDS has two dependent global round trips, so memory-level parallelism
// comes from U independent sub-steps per wave. Out-of-range lanes load a clamped (valid)
// edge and skip the update. PF: the next iteration's edge words are loaded right after
// this iteration's record gathers (loads retire in issue order), so the edge stream's HBM
// latency overlaps the LDS updates.
// FL bit 0 (kFwdFlagPrefetch): prefetch; bit 1 (kFwdFlagBranchless): idle lanes add 0 instead
// of branching; bit 2 (kFwdFlagChunk3): lane-chunk records (pack_cbsr3_kernel), l0 = chunk.
template <int U, class A, int FL>
__device__ __forceinline__ void fwd_edges4(typename A::T* acc, int e0, int e1, int wave,
                                           int nwaves, int EPS, int slot, int l0, bool lane_on,
                                           const uint2* __restrict__ cv,
                                           const uint8_t* __restrict__ rec, int rec_bytes,
                                           const uint8_t* __restrict__ seltab, int D, int k,
                                           double sc) {
  using T = typename A::T;
  constexpr bool PF = (FL & kFwdFlagPrefetch) != 0;
  constexpr bool C3 = (FL & kFwdFlagChunk3) != 0;
  constexpr bool QL = (FL & kFwdFlagQuad) != 0;  // L % 4 == 0: lanes load one word each
  const int last = e1 - 1;
  const uint32_t* cvw = reinterpret_cast<const uint32_t*>(cv) + (threadIdx.x & 1);
  auto load_cv = [&](int e) -> uint2 {
    if constexpr (QL) return make_uint2(cvw[2 * (size_t)e], 0u);
    else return cv[e];
  };
  auto split_cv = [&](uint2 w, uint32_t& c, float& v) {
    if constexpr (QL) {
      c = quad_bcast<0>(w.x);
      v = __uint_as_float(quad_bcast<1>(w.x));
    } else {
      c = w.x;
      v = __uint_as_float(w.y);
    }
  };
  const int stride = nwaves * EPS * U;
  int base = e0 + wave * EPS * U;
  uint2 wn[U];
  if (PF) {
#pragma unroll
    for (int u = 0; u < U; ++u) wn[u] = load_cv(min(base + u * EPS + slot, last));
  }
  // Edge-major windows (quad loads without prefetch, U % 4 == 0): sub-step u of slot s takes
  // edge base + s U + u, so lane q of a quad loads the whole edge word of sub-step 4j + q
  // (the quad reads 32 contiguous bytes) and DPP hands it to the quad: one edge-word
  // instruction per four sub-steps instead of one per sub-step
  // (Batching the selector words the same way, 64 scattered records per instruction, ran k = 16
  // 1.10 -> 1.48 ms: only contiguous loads gain from fewer instructions.)
  constexpr bool EM = QL && !PF && (U % 4) == 0;
  for (; base < e1; base += stride) {  // D: the accumulator's row stride
    uint32_t cw[U];
    float v[U];
    bool ok[U];
    if constexpr (EM) {
      const int qq = threadIdx.x & 3;
      uint2 wq[U / 4];
#pragma unroll
      for (int j = 0; j < U / 4; ++j) wq[j] = cv[min(base + slot * U + 4 * j + qq, last)];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + slot * U + u;
        ok[u] = lane_on && e < e1;
        const uint2 w = wq[u / 4];
        switch (u & 3) {
          case 0: cw[u] = quad_bcast<0>(w.x); v[u] = __uint_as_float(quad_bcast<0>(w.y)); break;
          case 1: cw[u] = quad_bcast<1>(w.x); v[u] = __uint_as_float(quad_bcast<1>(w.y)); break;
          case 2: cw[u] = quad_bcast<2>(w.x); v[u] = __uint_as_float(quad_bcast<2>(w.y)); break;
          default: cw[u] = quad_bcast<3>(w.x); v[u] = __uint_as_float(quad_bcast<3>(w.y)); break;
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + u * EPS + slot;
        ok[u] = lane_on && e < e1;
        split_cv(PF ? wn[u] : load_cv(ok[u] ? e : last), cw[u], v[u]);
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
      } else {
        x[u] = *reinterpret_cast<const float4*>(rp + l0 * 4);
        // two tables (plan->fwd_two_tables): values straight from sp_data, selectors from
        // sp_index (no per-call pack); else the selector word of the packed record
        const uint8_t* sp = seltab ? seltab + (size_t)(cw[u] & kFwdColMask) * k + l0
                                   : rp + 4 * k + l0;
        sel[u] = *reinterpret_cast<const uint32_t*>(sp);
      }
    }
    if (PF) {  // unconditional (clamped), see sspmm_bwd4_kernel
      __builtin_amdgcn_sched_barrier(0);  // keep every gather ahead of these loads
#pragma unroll
      for (int u = 0; u < U; ++u) wn[u] = load_cv(min(base + stride + u * EPS + slot, last));
      __builtin_amdgcn_sched_barrier(0);
    }
    // Branchless: idle lanes add 0 at their clamped (valid) edge's addresses; with a branch
    // the compiler sinks sub-step 0's gather below the other loads (measured: faster at
    // k = 16, slower at k = 8).
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if ((FL & kFwdFlagBranchless) || ok[u]) {
        T* arow = acc + (cw[u] >> kFwdColBits) * D;
        const uint32_t sv = sel[u];
        const typename A::V vu = A::scale((FL & kFwdFlagBranchless) && !ok[u] ? 0.f : v[u], sc);
        if constexpr (C3) {
          // l0 = chunk index: slots 3 l0 .. 3 l0 + 2 (the last chunk may be partly padding)
          A::add2(arow + (sv & 0xffu), vu, x[u].x);
          if (3 * l0 + 1 < k) A::add2(arow + ((sv >> 8) & 0xffu), vu, x[u].y);
          if (3 * l0 + 2 < k) A::add2(arow + ((sv >> 16) & 0xffu), vu, x[u].z);
        } else {
          A::add2(arow + (sv & 0xffu), vu, x[u].x);
          A::add2(arow + ((sv >> 8) & 0xffu), vu, x[u].y);
          A::add2(arow + ((sv >> 16) & 0xffu), vu, x[u].z);
          A::add2(arow + (sv >> 24), vu, x[u].w);
        }
      }
    }
  }
}

// Column phases: all work-groups of one launch gather from the same 1/B of the CBSR table
// (phase b = source columns [b*NC/B, (b+1)*NC/B)), so the records they touch stay in L2
// (tools/ubench_gather.hip: ~300 vs ~63 G edges/s for a shared window vs the whole table).
// Phase 0 stores the task's rows, later phases continue from the stored partial sums.
template <int VEC, int ACC, int U, int NT, int FL>
__global__ __launch_bounds__(NT) void spgemm_fwd_kernel(
    const FwdTask* __restrict__ tasks, int ntasks, const int32_t* __restrict__ phase_off,
    int phases, int phase, const uint2* __restrict__ cv,
    const float* __restrict__ sp_data, const uint8_t* __restrict__ sp_index,
    const uint8_t* __restrict__ rec, int rec_bytes, float* __restrict__ out, int D, int k,
    int tile_rows, int rot_ticks, const uint8_t* __restrict__ seltab, int accum,
    const int2* __restrict__ fix_tab, const uint32_t* __restrict__ xstat, int xs_n,
    int xs_stride, int xs_off2) {
  using A = LdsAcc<ACC>;
  using T = typename A::T;
  extern __shared__ __align__(16) double smem_d[];
  T* acc = reinterpret_cast<T*>(smem_d);
  // Work-group w runs tasks w, w + G, ... (G = grid size; G = #tasks by default, or the
  // resident capacity with the fwd_persistent option, which measured slower on Reddit).
  // rot_ticks > 0: one launch, each task's sweep rotated to start at the window of the
  // shared 100 MHz clock, so concurrently running tiles gather from the same columns.
  for (int ti = blockIdx.x; ti < ntasks; ti += gridDim.x) {
  FwdTask t = tasks[ti];
  int emid = -1;
  __shared__ int s_w0;
  if (rot_ticks > 0) {
    // start the column-sorted sweep at the window the clock points to, wrapping around
    // (read once per work-group: every wave must split the task at the same edge)
    __syncthreads();
    if (threadIdx.x == 0)
      s_w0 = (int)((__builtin_amdgcn_s_memrealtime() / (uint64_t)rot_ticks) % (uint64_t)phases);
    __syncthreads();
    const int w0 = s_w0;
    t.e0 = phase_off[ti * (phases + 1)];
    t.e1 = phase_off[ti * (phases + 1) + phases];
    emid = phase_off[ti * (phases + 1) + w0];
  } else {
  t.e0 = phase_off[ti * (phases + 1) + phase];
  t.e1 = phase_off[ti * (phases + 1) + phase + 1];
  }
  const bool cont = phase > 0 || accum;  // rows of out hold a prior sum to add to
  if (cont && t.e0 == t.e1) continue;  // nothing to add (uniform)
  // fixed-point accumulation for this task (LdsFix), else f64; the 8-byte slots are the same.
  // A continuing launch in fixed point sums its own terms from zero and adds the prior f32
  // row at the write-back (one more f32 rounding, as a column phase of the reference would)
  double fsc = 0.0;
  if constexpr (VEC == 4 && ACC == MAXK_ACC_F64) {
    if (fix_tab) fsc = fwd_fix_scale(fix_tab[ti], xstat, xs_n, xs_stride, xs_off2);
  }
  const bool fixed = fsc != 0.0;
  unsigned long long* acc64 = reinterpret_cast<unsigned long long*>(smem_d);
  const bool split = t.nrows < 0;
  const int nrows = split ? 1 : t.nrows;
  const int n = nrows * D;
  const int DS = D + kFwdRowPad;  // LDS row stride (elements)
  __syncthreads();  // the previous task's write-back has finished reading acc
  if (cont && !split && !fixed) {  // continue from the stored rows
    const float* src = out + (size_t)t.row0 * D;
    for (int i = threadIdx.x; i < n; i += NT) {
      const int r = i / D;
      acc[r * DS + (i - r * D)] = T(src[i]);
    }
  } else {
    for (int i = threadIdx.x; i < nrows * DS; i += NT) acc[i] = T(0);
  }
  __syncthreads();

  // lanes per edge: VEC==4 => k % 4 == 0 and k/4 <= 64; VEC==1 => min(k, 64) lanes that
  // loop over the row's k entries.
  constexpr bool C3 = (FL & kFwdFlagChunk3) != 0;
  const int L = (VEC == 4) ? (C3 ? (k + 2) / 3 : k / 4) : (k < kWave ? k : kWave);
  const int EPS = kWave / L;  // edges per wave instruction
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int slot = lane / L;
  const int l0 = (lane - slot * L) * (C3 ? 1 : VEC);
  const bool lane_on = slot < EPS;
  constexpr int kWaves = NT / kWave;

  if constexpr (VEC == 4) {
    // U sub-steps per iteration with every load issued before the first LDS update: the
    // chain (col, val) -> CBSR record -> LDS has two dependent global round trips, so
    // memory-level parallelism comes from U independent sub-steps per wave. Out-of-range
    // lanes load a clamped (valid) edge and skip the update.
    auto sweep = [&](auto* a, auto tag) {
      using AA = decltype(tag);
      if (emid >= 0) {
        fwd_edges4<U, AA, FL>(a, emid, t.e1, wave, kWaves, EPS, slot, l0, lane_on, cv, rec,
                              rec_bytes, seltab, DS, k, fsc);
        fwd_edges4<U, AA, FL>(a, t.e0, emid, wave, kWaves, EPS, slot, l0, lane_on, cv, rec,
                              rec_bytes, seltab, DS, k, fsc);
      } else {
        fwd_edges4<U, AA, FL>(a, t.e0, t.e1, wave, kWaves, EPS, slot, l0, lane_on, cv, rec,
                              rec_bytes, seltab, DS, k, fsc);
      }
    };
    if constexpr (ACC == MAXK_ACC_F64) {
      if (fixed) sweep(acc64, LdsFix{});
      else sweep(acc, A{});
    } else {
      sweep(acc, A{});
    }
  } else {
    for (int base = t.e0 + wave * EPS; base < t.e1; base += kWaves * EPS) {
      const int e = base + slot;
      if (lane_on && e < t.e1) {
        const uint2 w = cv[e];
        const uint32_t cwv = w.x;
        const float v = __uint_as_float(w.y);
        T* arow = acc + (cwv >> kFwdColBits) * DS;
        const size_t rb = (size_t)(cwv & kFwdColMask) * k;
        for (int l = l0; l < k; l += L) A::add(arow + sp_index[rb + l], v * sp_data[rb + l]);
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
    const bool add = cont && fixed;  // the prior row is added here (see above)
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
  }  // task loop
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
// instruction covers share few rows of grad_out, so its gathers stay in the CU's L1. Any
// wave may update any column of the block (that is what keeps the row locality), hence the
// atomic LDS accumulation.
template <int F, int ACC, int U>
__global__ __launch_bounds__(kBwdThreads) void sspmm_bwd_kernel(
    const BwdTask* __restrict__ tasks, const int32_t* __restrict__ erow,
    const int32_t* __restrict__ ecol, const float* __restrict__ evals,
    const float* __restrict__ G, const uint8_t* __restrict__ sp_index,
    float* __restrict__ grad_sp, int D, int k) {
  using A = LdsAcc<ACC>;
  using T = typename A::T;
  extern __shared__ __align__(16) double bsmem[];
  // Accumulator of column c, slot l at c * KS + l with KS = k + 1 (odd, so different columns
  // start on different banks); the lanes of one edge update consecutive slots (the plain
  // [c][k] layout with lane-contiguous slots put a wave on 8 banks: 8-way conflicts).
  T* bacc = reinterpret_cast<T*>(bsmem);
  const BwdTask t = tasks[blockIdx.x];
  if (t.ncols == 0 || (t.shared && t.e0 == t.e1)) return;  // padding / nothing to add
  const int KS = k + 1;
  const int nacc = t.ncols * KS;
  for (int i = threadIdx.x; i < nacc; i += kBwdThreads) bacc[i] = T(0);
  __syncthreads();

  const int L = (F == 4) ? k / 4 : (k < kWave ? k : kWave);  // lanes per edge
  const int EPS = kWave / L;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int slot = lane / L;
  const int q = lane - slot * L;
  const bool lane_on = slot < EPS;
  constexpr int kWaves = kBwdThreads / kWave;
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
      // Lane q of an edge owns the selector slots q, q + L, q + 2L, q + 3L: in gather
      // instruction i the L lanes of the edge read L adjacent (sorted) selectors of the
      // row, i.e. ~1-2 cache lines of grad_out[r] instead of L lines. The selector words
      // are loaded as dwords (lane q: slots 4q..4q+3) and redistributed with shuffles.
      uint32_t sel[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(sp_index + (size_t)c[u] * k + q * 4);
        uint32_t m = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int l = q + L * i;  // slot owned by this lane in gather i
          const uint32_t wi = (uint32_t)__shfl((int)w, slot * L + (l >> 2), kWave);
          m |= ((wi >> ((l & 3) * 8)) & 0xffu) << (8 * i);
        }
        sel[u] = m;
      }
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
          T* a = bacc + (c[u] - t.col0) * KS + q;
          A::add(a, v[u] * g[u][0]);
          A::add(a + L, v[u] * g[u][1]);
          A::add(a + 2 * L, v[u] * g[u][2]);
          A::add(a + 3 * L, v[u] * g[u][3]);
        }
      }
    } else if (k <= kWave) {
      // one feature per lane: the L = k lanes of an edge read k dwords of the same
      // grad_out row in one instruction (~7 cache lines at k = 16 instead of 16 for 4
      // features per lane over 4 instructions); the gather is bound by lines per request.
      uint32_t sel[U];
#pragma unroll
      for (int u = 0; u < U; ++u) sel[u] = sp_index[(size_t)c[u] * k + q];
      float g[U];
#pragma unroll
      for (int u = 0; u < U; ++u) g[u] = G[(size_t)r[u] * D + sel[u]];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (ok[u]) A::add(bacc + (c[u] - t.col0) * KS + q, v[u] * g[u]);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (ok[u]) {
          const float* grow = G + (size_t)r[u] * D;
          const uint8_t* srow = sp_index + (size_t)c[u] * k;
          T* a = bacc + (c[u] - t.col0) * KS;
          for (int l = q; l < k; l += L) A::add(a + l, v[u] * grow[srow[l]]);
        }
      }
    }
  }
  __syncthreads();

  float* dst = grad_sp + (size_t)t.col0 * k;
  const int n = t.ncols * k;
  for (int i = threadIdx.x; i < n; i += kBwdThreads) {
    const int cl = i / k;
    const int l = i - cl * k;
    const int pos = cl * KS + l;
    if (t.shared) global_add(dst + i, (float)bacc[pos]);
    else dst[i] = (float)bacc[pos];
  }
}


// Packed backward (k % 4 == 0, f32 accumulators): the same (block, row)-ordered sweep as
// sspmm_bwd_kernel<4, ...> with the per-edge work cut to the memory operations it needs:
// one dwordx3 record load {row * D * 4, column in block, val}, one dword of four selectors
// already in lane order (pack_sel_kernel), four buffer_load_dword gathers of grad_out with
// 32-bit offsets, and the LDS compare-and-swap adds issued as a batch (all reads, then all
// CAS, then a retry loop for the rare lanes whose CAS lost a race).
__global__ void pack_sel_kernel(const uint8_t* __restrict__ sp_index, int n, int k, int S,
                                uint32_t* __restrict__ sel, const int32_t* __restrict__ corder) {
  // sel[(g * n + c) * L + q] = slots g*k/S + q + L*i, i = 0..3, of the column at block
  // position c (corder[c], or c itself) (L = k / 4S)
  const int L = k / (4 * S);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * L * S) return;
  const int g = i / (n * L);
  const int r = i - g * (n * L);
  const int c = r / L, q = r - c * L;
  const uint8_t* s = sp_index + (size_t)(corder ? corder[c] : c) * k + g * (k / S) + q;
  sel[i] = (uint32_t)s[0] | ((uint32_t)s[L] << 8) | ((uint32_t)s[2 * L] << 16) |
           ((uint32_t)s[3 * L] << 24);
}

// Two slots per lane (sspmm_bwd4_kernel<.., F = 2>): sel[(g * n + c) * L + q] = slots
// g*k/S + q and g*k/S + q + L of column c (L = k / 2S), as one u16.
__global__ void pack_sel2_kernel(const uint8_t* __restrict__ sp_index, int n, int k, int S,
                                 uint16_t* __restrict__ sel, const int32_t* __restrict__ corder) {
  const int L = k / (2 * S);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * L * S) return;
  const int g = i / (n * L);
  const int r = i - g * (n * L);
  const int c = r / L, q = r - c * L;
  const uint8_t* s = sp_index + (size_t)(corder ? corder[c] : c) * k + g * (k / S) + q;
  sel[i] = (uint16_t)(s[0] | (s[L] << 8));
}

// NT threads per work-group (8, 12 or 16 waves: more waves, more gathers in flight per CU
// under the same LDS block). PF: the next sub-steps' records are loaded right after this
// step's gathers are issued, so the record stream's HBM latency overlaps the LDS updates
// (loads retire in issue order, so they must not precede the gathers the updates wait on).
//
// V (plan->bwd_cas64): lane q's F slots are stored adjacently (slot l of a column at
// (l % L) * F + l / L), so its updates are 1 ds_read_b128 + 2 ds_cmpst_rtn_b64 (F = 4) or
// 1 ds_read_b64 + 1 ds_cmpst_rtn_b64 (F = 2) instead of F + F dword operations (KS % F == 0);
// a pair is retried if either of its floats changed.
//
// F: selector slots per lane, L = k / (F S) lanes per edge. F = 4: a gather instruction
// covers slots 4i..4i+3 (a quarter of the sorted selectors) of 64/L edges; F = 2: slots
// 8i..8i+7 of half as many edges, so of about half as many rows of G.
template <int U, int NT, bool PF, bool V, bool Q, int F = 4>
__global__ __launch_bounds__(NT) void sspmm_bwd4_kernel(
    const BwdTask* __restrict__ tasks, const uint32_t* __restrict__ rec,
    const float* __restrict__ G, uint32_t g_bytes, const uint32_t* __restrict__ sel,
    float* __restrict__ grad_sp, int k, int S, int ncols_all, int KS, int sel_lds,
    float* __restrict__ slab, const int32_t* __restrict__ corder) {
  extern __shared__ __align__(16) double bsmem[];
  float* bacc = reinterpret_cast<float*>(bsmem);
  const BwdTask t = tasks[blockIdx.x];
  // padding / nothing to add (with the slab flush every chunk stores its block, zeros too)
  if (t.ncols == 0 || (t.shared && !slab && t.e0 == t.e1)) return;
  static_assert(F == 2 || F == 4, "2 or 4 slots per lane");
  using SelT = std::conditional_t<F == 4, uint32_t, uint16_t>;  // the F selectors of a lane
  const int ns = k / S;  // slots of this group: [t.group * ns, (t.group + 1) * ns)
  const int L = ns / F;  // lanes per edge, F slots each: q, q + L, ...
  const int nacc = t.ncols * KS;
  for (int i = threadIdx.x; i < nacc; i += NT) bacc[i] = 0.f;
  // sel_lds: the block's selector words are staged in LDS behind the accumulator, so the
  // per-edge selector lookup is an LDS read instead of an L1 miss (the G rows evict the
  // block's 16 B/column table from the 32 KB L1)
  const SelT* selg = reinterpret_cast<const SelT*>(sel) + ((size_t)t.group * ncols_all + t.col0) * L;
  SelT* sell = reinterpret_cast<SelT*>(bacc + ((nacc + 3) & ~3));
  if (sel_lds)
    for (int i = threadIdx.x; i < t.ncols * L; i += NT) sell[i] = selg[i];
  __syncthreads();

  const int EPS = kWave / L;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int slot = lane / L;
  const int q = lane - slot * L;
  const bool lane_on = slot < EPS;
  constexpr int kWaves = NT / kWave;
  const int stride = kWaves * EPS * U;
  const __amdgpu_buffer_rsrc_t gr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G), (short)0, (int)g_bytes, 0x00020000);
  const SelT* selb = (sel_lds ? sell : selg) + q;
  unsigned* accq = reinterpret_cast<unsigned*>(bacc) + (V ? F * q : q);
  const uint3* rec3 = reinterpret_cast<const uint3*>(rec);

  // records past e1 (a padded or neighbouring record) are loaded and ignored
  int base = t.e0 + wave * EPS * U;
  // Q: lane loads dword min(q & 3, 2) of its edge's record (quad_bcast below)
  const uint32_t* recw = rec + min(lane & 3, 2);
  auto load_rec = [&](int e) -> uint3 {
    if constexpr (Q) return make_uint3(recw[3 * (size_t)e], 0u, 0u);
    else return rec3[e];
  };
  constexpr bool EM = Q && (U % 4) == 0;
  const int qq = lane & 3;
  // EM: lane q of a quad loads sub-step 4j + q's whole record (records past e1 exist: padding)
  auto load_rq = [&](int b, uint3 (&rq)[U / 4 > 0 ? U / 4 : 1]) {
#pragma unroll
    for (int j = 0; j < U / 4; ++j) rq[j] = rec3[b + (4 * j + qq) * EPS + slot];
  };
  uint3 rn[U];
  uint3 rqn[U / 4 > 0 ? U / 4 : 1];
  if (PF) {
    if constexpr (EM) {
      load_rq(base, rqn);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) rn[u] = load_rec(min(base + u * EPS + slot, t.e1 - 1));
    }
  }
  // Batched records (quad loads without prefetch, U % 4 == 0): lane q of a quad loads the
  // whole record of its slot's edge in sub-step 4j + q (the wave's 64 loads cover 4 sub-steps'
  // 64 consecutive records) and DPP hands each sub-step's record to the quad: one record
  // instruction per four sub-steps. The sub-steps keep their consecutive edges (edges of a
  // gather instruction share grad_out rows).
  for (; base < t.e1; base += stride) {
    uint32_t go[U], cl[U];
    float v[U];
    bool ok[U];
    if constexpr (EM) {
      uint3 rq[U / 4 > 0 ? U / 4 : 1];
      if (PF) {
#pragma unroll
        for (int j = 0; j < U / 4; ++j) rq[j] = rqn[j];
      } else {
        load_rq(base, rq);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ok[u] = lane_on && base + u * EPS + slot < t.e1;
        const uint3 r3 = rq[u / 4];
        switch (u & 3) {
          case 0: go[u] = quad_bcast<0>(r3.x); cl[u] = quad_bcast<0>(r3.y); v[u] = __uint_as_float(quad_bcast<0>(r3.z)); break;
          case 1: go[u] = quad_bcast<1>(r3.x); cl[u] = quad_bcast<1>(r3.y); v[u] = __uint_as_float(quad_bcast<1>(r3.z)); break;
          case 2: go[u] = quad_bcast<2>(r3.x); cl[u] = quad_bcast<2>(r3.y); v[u] = __uint_as_float(quad_bcast<2>(r3.z)); break;
          default: go[u] = quad_bcast<3>(r3.x); cl[u] = quad_bcast<3>(r3.y); v[u] = __uint_as_float(quad_bcast<3>(r3.z)); break;
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + u * EPS + slot;
        ok[u] = lane_on && e < t.e1;
        const uint3 r3 = PF ? rn[u] : load_rec(e);
        if constexpr (Q) {
          go[u] = quad_bcast<0>(r3.x);
          cl[u] = quad_bcast<1>(r3.x);
          v[u] = __uint_as_float(quad_bcast<2>(r3.x));
        } else {
          go[u] = r3.x;
          cl[u] = r3.y;
          v[u] = __uint_as_float(r3.z);
        }
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
        const uint32_t off = go[u] + (((s[u] >> (8 * i)) & 0xffu) << 2);
        x[u][i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(gr, off, 0, 0));
      }
    }
    if (PF) {  // unconditional (clamped): a branch here would make the updates below wait
               // for these loads too (vmcnt counts both paths)
      __builtin_amdgcn_sched_barrier(0);  // keep every gather ahead of these loads
      if constexpr (EM) {
        load_rq(base + stride, rqn);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) rn[u] = load_rec(min(base + stride + u * EPS + slot, t.e1 - 1));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < F; ++i) x[u][i] *= v[u];
    if constexpr (V) {
      using u64 = unsigned long long;
      u64 old2[U][F / 2];
#pragma unroll
      for (int u = 0; u < U; ++u) {
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
      u64 got2[U][F / 2];
#pragma unroll
      for (int u = 0; u < U; ++u) {
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
      for (int u = 0; u < U; ++u) {
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
      continue;
    }
    unsigned old[U][F];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      unsigned* a = accq + cl[u] * KS;
#pragma unroll
      for (int i = 0; i < F; ++i)
        old[u][i] = __hip_atomic_load(a + i * L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    unsigned got[U][F];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      unsigned* a = accq + cl[u] * KS;
#pragma unroll
      for (int i = 0; i < F; ++i) {
        got[u][i] = old[u][i];
        if (ok[u]) {
          unsigned expected = old[u][i];
          __hip_atomic_compare_exchange_strong(
              a + i * L, &expected, __float_as_uint(__uint_as_float(old[u][i]) + x[u][i]),
              __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          got[u][i] = expected;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      unsigned* a = accq + cl[u] * KS;
#pragma unroll
      for (int i = 0; i < F; ++i) {
        if (ok[u] && got[u][i] != old[u][i]) {
          unsigned cur = got[u][i];
          while (true) {
            unsigned expected = cur;
            __hip_atomic_compare_exchange_strong(
                a + i * L, &expected, __float_as_uint(__uint_as_float(cur) + x[u][i]),
                __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (expected == cur) break;
            cur = expected;
          }
        }
      }
    }
  }
  __syncthreads();

  // shared block: global atomics into a zeroed grad_sp, or (slab flush) piece 0 stores into
  // grad_sp and piece p > 0 into its slab region (block positions), summed by
  // bwd_combine_kernel; corder maps block positions to the columns of grad_sp
  const bool atomic = t.shared && !slab;
  const bool to_slab = slab && t.slab >= 0;
  float* dst = to_slab ? slab + t.slab + t.group * ns : grad_sp + t.group * ns;
  const int n = t.ncols * ns;
  for (int i = threadIdx.x; i < n; i += NT) {
    const int c = i / ns;
    const int l = i - c * ns;
    const float a = bacc[c * KS + (V ? (l % L) * F + l / L : l)];
    const size_t row = to_slab ? (size_t)c : (size_t)(corder ? corder[t.col0 + c] : t.col0 + c);
    if (atomic) global_add(dst + row * k + l, a);
    else dst[row * k + l] = a;
  }
}

// Packed backward with one selector slot per lane (plan->bwd_feats == 1, k <= 64): the k
// lanes of an edge gather k dwords of ONE row of grad_out in one instruction, so a wave
// instruction covers 64/k edges that are mostly of the same row (edges are row-sorted in a
// block) and touches ~8 lines of G, where the 4-slots-per-lane kernel's instructions cover
// slot group i of 64/(k/4) edges of ~k/4 rows. The gathers are bound by distinct lines per
// instruction at the L1 (tools/ubench_tcp.hip), not by lanes. The block's selector bytes are
// staged in LDS straight from sp_index (no per-call packing).
template <int U, int NT>
__global__ __launch_bounds__(NT) void sspmm_bwd1_kernel(
    const BwdTask* __restrict__ tasks, const uint32_t* __restrict__ rec,
    const float* __restrict__ G, uint32_t g_bytes, const uint8_t* __restrict__ sp_index,
    float* __restrict__ grad_sp, int k, int KS, float* __restrict__ slab,
    const int32_t* __restrict__ corder) {
  extern __shared__ __align__(16) double bsmem[];
  float* bacc = reinterpret_cast<float*>(bsmem);
  const BwdTask t = tasks[blockIdx.x];
  // padding / nothing to add (with the slab flush every chunk stores its block, zeros too)
  if (t.ncols == 0 || (t.shared && !slab && t.e0 == t.e1)) return;
  const int nacc = t.ncols * KS;
  for (int i = threadIdx.x; i < nacc; i += NT) bacc[i] = 0.f;
  uint8_t* sell = reinterpret_cast<uint8_t*>(bacc + ((nacc + 3) & ~3));
  // the block's selector rows: columns corder[col0 ..] (or col0 .. contiguous)
  auto col_of = [&](int c) -> size_t { return corder ? (size_t)corder[t.col0 + c] : (size_t)t.col0 + c; };
  const int nsel = t.ncols * k;
  if ((k & 3) == 0) {
    const int kw = k / 4;
    for (int i = threadIdx.x; i < nsel / 4; i += NT) {
      const int c = i / kw;
      reinterpret_cast<uint32_t*>(sell)[i] =
          reinterpret_cast<const uint32_t*>(sp_index + col_of(c) * k)[i - c * kw];
    }
  } else {
    for (int i = threadIdx.x; i < nsel; i += NT) {
      const int c = i / k;
      sell[i] = sp_index[col_of(c) * k + (i - c * k)];
    }
  }
  __syncthreads();

  const int L = k;  // lanes per edge
  const int EPS = kWave / L;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int slot = lane / L;
  const int q = lane - slot * L;
  const bool lane_on = slot < EPS;
  constexpr int kWaves = NT / kWave;
  const int stride = kWaves * EPS * U;
  const __amdgpu_buffer_rsrc_t gr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G), (short)0, (int)g_bytes, 0x00020000);
  const uint3* rec3 = reinterpret_cast<const uint3*>(rec);
  const uint8_t* selq = sell + q;
  unsigned* accq = reinterpret_cast<unsigned*>(bacc) + q;

  for (int base = t.e0 + wave * EPS * U; base < t.e1; base += stride) {
    uint32_t go[U], cl[U];
    float v[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * EPS + slot;  // past e1: a padded or neighbouring record
      ok[u] = lane_on && e < t.e1;
      const uint3 r3 = rec3[e];
      go[u] = r3.x;
      cl[u] = r3.y;
      v[u] = __uint_as_float(r3.z);
    }
    float x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t off = go[u] + ((uint32_t)selq[cl[u] * k] << 2);
      x[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(gr, off, 0, 0));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] *= v[u];
    unsigned old[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      old[u] = __hip_atomic_load(accq + cl[u] * KS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    unsigned got[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      got[u] = old[u];
      if (ok[u]) {
        unsigned expected = old[u];
        __hip_atomic_compare_exchange_strong(
            accq + cl[u] * KS, &expected, __float_as_uint(__uint_as_float(old[u]) + x[u]),
            __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        got[u] = expected;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (ok[u] && got[u] != old[u]) {
        unsigned cur = got[u];
        while (true) {
          unsigned expected = cur;
          __hip_atomic_compare_exchange_strong(
              accq + cl[u] * KS, &expected, __float_as_uint(__uint_as_float(cur) + x[u]),
              __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (expected == cur) break;
          cur = expected;
        }
      }
    }
  }
  __syncthreads();

  const bool atomic = t.shared && !slab;
  const bool to_slab = slab && t.slab >= 0;
  for (int i = threadIdx.x; i < nsel; i += NT) {
    const int c = i / k;
    const float a = bacc[c * KS + (i - c * k)];
    float* dst = to_slab ? slab + t.slab + i : grad_sp + col_of(c) * k + (i - c * k);
    if (atomic) global_add(dst, a);
    else *dst = a;
  }
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

// Column-major backward for sparse graphs (plan->bwd_csc): the records are sorted by column
// (stable, so rows ascend within a column) and one wavefront owns a column c. Its L = k/F
// lanes per edge (F = 4: interleaved slots q + L*i from the packed selector word; F = 1: one
// slot per lane straight from sp_index) load the column's selectors once, then the wave
// walks the column's edges 64/L at a time, gathering k features of each source row of
// grad_out and summing them in registers; a shuffle-xor reduction over the edge slots leaves
// the k sums in lanes 0..L-1, which store them. No LDS, no atomics, no memset: every column
// is written exactly once.
template <int F, int U>
__global__ __launch_bounds__(256) void sspmm_bwd_csc_kernel(
    const int32_t* __restrict__ colptr, const uint32_t* __restrict__ rec,
    const float* __restrict__ G, uint32_t g_bytes, const uint32_t* __restrict__ sel,
    const uint8_t* __restrict__ sp_index, float* __restrict__ grad_sp, int ncols, int k) {
  const int lane = threadIdx.x & (kWave - 1);
  const int c = blockIdx.x * (256 / kWave) + threadIdx.x / kWave;
  if (c >= ncols) return;
  const int L = k / F;  // power of two <= 64 (checked by the plan)
  const int EPS = kWave / L;
  const int slot = lane / L;
  const int q = lane - slot * L;
  uint32_t so[F];
  if constexpr (F == 4) {
    const uint32_t s = sel[(size_t)c * L + q];
#pragma unroll
    for (int i = 0; i < 4; ++i) so[i] = ((s >> (8 * i)) & 0xffu) << 2;
  } else {
    so[0] = (uint32_t)sp_index[(size_t)c * k + q] << 2;
  }
  const int e0 = colptr[c], e1 = colptr[c + 1];
  const __amdgpu_buffer_rsrc_t gr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G), (short)0, (int)g_bytes, 0x00020000);
  float acc[F];
#pragma unroll
  for (int i = 0; i < F; ++i) acc[i] = 0.f;
  for (int base = e0; base < e1; base += EPS * U) {
    uint32_t go[U];
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * EPS + slot;
      if (e < e1) {
        const uint3 r3 = *reinterpret_cast<const uint3*>(rec + 3 * (size_t)e);
        go[u] = r3.x;
        v[u] = __uint_as_float(r3.z);
      } else {
        go[u] = 0;
        v[u] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = base + u * EPS + slot < e1;
#pragma unroll
      for (int i = 0; i < F; ++i) {
        // out-of-range offset for the idle slots: the buffer load returns 0 (no 0 * inf)
        const uint32_t off = ok ? go[u] + so[i] : 0xfffffffcu;
        acc[i] = fmaf(v[u], __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(gr, off, 0, 0)), acc[i]);
      }
    }
  }
  for (int m = L; m < kWave; m <<= 1) {
#pragma unroll
    for (int i = 0; i < F; ++i) acc[i] += __shfl_xor(acc[i], m, kWave);
  }
  if (slot == 0) {
    float* dst = grad_sp + (size_t)c * k + q;
#pragma unroll
    for (int i = 0; i < F; ++i) dst[i * L] = acc[i];
  }
}

// Two-pass backward (plan->bwd_twopass), pass 1: one wavefront per R consecutive destination
// rows stages their grad_out rows in its LDS once, then walks their (contiguous) edges 64/L
// at a time (L = k/4 lanes per edge): lane q of an edge on column c reads the 4 selectors
// sp_index[c][4q..4q+3] (one dword), multiplies the 4 staged features of the edge's row
// (row % R from the edge record) by val and stores them as one float4 into the edge's slot
// T[e][4q..] (CSR order: the slots of a wavefront are contiguous, the stores coalesce; in
// column order the scattered 64-B stores ran at a quarter of the bandwidth). The only gathers
// left on the texture path are the k selector bytes per edge; grad_out is read once.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// CS (plan->bwd_tp_csc): each edge's k products go to its column-order slot pos[e] of the
// workspace (full 128-B lines at k = 32), so the column pass streams its slots contiguously
// instead of gathering them through bwd_perm.
template <int U, int R, bool CS = false>
__global__ __launch_bounds__(256) void sspmm_bwd_rows_kernel(
    const int32_t* __restrict__ ptr, const uint32_t* __restrict__ erec,
    const float* __restrict__ G, const uint8_t* __restrict__ sp_index, float* __restrict__ T,
    int rbeg, int rend, int64_t ebase, int D, int k, const int32_t* __restrict__ pos) {
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
  for (int base = e0; base < e1; base += EPS * U) {
    uint32_t c[U];
    float v[U];
    if ((U & 3) == 0 && (L & 3) == 0) {
      // lane q of a quad loads the record of sub-step 4j + q (contiguous), DPP hands it on:
      // one record instruction per four sub-steps
      const int qq = lane & 3;
#pragma unroll
      for (int j = 0; j < U / 4; ++j) {
        const uint2 w = *reinterpret_cast<const uint2*>(
            erec + 2 * (size_t)min(base + (4 * j + qq) * EPS + slot, e1 - 1));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int u = 4 * j + i;
          if (u >= U) break;
          switch (i) {
            case 0: c[u] = quad_bcast<0>(w.x); v[u] = __uint_as_float(quad_bcast<0>(w.y)); break;
            case 1: c[u] = quad_bcast<1>(w.x); v[u] = __uint_as_float(quad_bcast<1>(w.y)); break;
            case 2: c[u] = quad_bcast<2>(w.x); v[u] = __uint_as_float(quad_bcast<2>(w.y)); break;
            default: c[u] = quad_bcast<3>(w.x); v[u] = __uint_as_float(quad_bcast<3>(w.y)); break;
          }
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = min(base + u * EPS + slot, e1 - 1);
        const uint2 cv = *reinterpret_cast<const uint2*>(erec + 2 * (size_t)e);
        c[u] = cv.x;  // column | (row % R) << kFwdColBits
        v[u] = __uint_as_float(cv.y);
      }
    }
    uint32_t sw[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      sw[u] = *reinterpret_cast<const uint32_t*>(sp_index + (size_t)(c[u] & kFwdColMask) * k + 4 * q);
    int32_t ps[U];
    if constexpr (CS) {
#pragma unroll
      for (int u = 0; u < U; ++u) ps[u] = pos[min(base + u * EPS + slot, e1 - 1)];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * EPS + slot;
      const float* rw = row + (R > 1 ? (c[u] >> kFwdColBits) * kMaxDim : 0);
      if constexpr (CS) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        f4v o;
        o.x = v[u] * rw[sw[u] & 0xffu];
        o.y = v[u] * rw[(sw[u] >> 8) & 0xffu];
        o.z = v[u] * rw[(sw[u] >> 16) & 0xffu];
        o.w = v[u] * rw[sw[u] >> 24];
        if (e < e1)
          __builtin_nontemporal_store(o, reinterpret_cast<f4v*>(T + (size_t)ps[u] * k + 4 * q));
        continue;
      }
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
  }
}

// Two-pass backward, pass 2: one wavefront per column c sums the slots of the column's
// in-edges perm[lo[c] .. hi[c]) (64/L slots per step, float4 per lane), reduces over the
// slots with shuffles and stores grad_sp[c] (every column written once: no memset, no
// atomics). Row chunks (plan->bwd_tp_chunks > 1): this pass covers the in-edges of one row
// chunk, whose slots are at T + (perm - ebase) * k; chunk 0 stores, later chunks add to the
// stored sums in chunk order (deterministic).
template <int U, bool CS = false>
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
    if (!CS && (U & 3) == 0 && (L & 3) == 0) {
      // lane q of a quad loads the permutation entry of sub-step 4j + q, DPP hands it on
      const int qq = lane & 3;
#pragma unroll
      for (int jj = 0; jj < U / 4; ++jj) {
        const uint32_t w = (uint32_t)(perm[min(base + (4 * jj + qq) * EPS + slot, e1 - 1)] - ebase);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int u = 4 * jj + i;
          if (u >= U) break;
          switch (i) {
            case 0: pe[u] = (int32_t)quad_bcast<0>(w); break;
            case 1: pe[u] = (int32_t)quad_bcast<1>(w); break;
            case 2: pe[u] = (int32_t)quad_bcast<2>(w); break;
            default: pe[u] = (int32_t)quad_bcast<3>(w); break;
          }
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = min(base + u * EPS + slot, e1 - 1);
        pe[u] = CS ? j : (int32_t)(perm[j] - ebase);  // CS: the slots are already in column order
      }
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

size_t acc_bytes(int acc) { return acc == MAXK_ACC_F32_CAS ? sizeof(float) : sizeof(double); }

size_t fwd_lds_bytes(int tile_rows, int D, int acc) {
  return (size_t)tile_rows * (D + kFwdRowPad) * acc_bytes(acc);
}

size_t bwd_lds_bytes(int block_cols, int k, int acc) {
  return (size_t)block_cols * (k + 1) * acc_bytes(acc);
}

template <typename K>
static hipError_t allow_lds(K* kernel, size_t bytes) {
  return hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)bytes);
}

}  // namespace maxk

using namespace maxk;

// Fixed-point statistics of a CBSR table into two zeroed words: the lane-parallel kernel
// for k % 4 == 0 (~10 us for Reddit at k = 16), one thread per row otherwise.
// rec != nullptr (k % 4 == 0 only): also pack the forward's CBSR records (st0 == nullptr: the
// pack alone)
// zrows/nz/out/D (k % 4 == 0 only): split rows of the forward to zero in the same launch.
static int launch_cbsr_stats(const float* sp_data, const uint8_t* sp_index, int64_t nrows, int k,
                             uint32_t* st0, uint32_t* st1, int cus, hipStream_t s,
                             uint8_t* rec = nullptr, int rec_bytes = 0,
                             const int32_t* zrows = nullptr, int nz = 0, float* out = nullptr,
                             int D = 0) {
  if (nrows <= 0) return MAXK_OK;
  if (k % 4 == 0) {
    const int64_t rows_per_block = (256 / kWave) * (kWave / (k / 4));
    // statistics: one work-group per CU, each adds one atomic per word, and same-address
    // atomics from every work-group serialise at the L2; the pack alone: more in flight
    const int cap = st0 ? cus * kStatsBlocksPerCu : 8 * cus;
    const int grid = (int)std::max<int64_t>(
        1, std::min<int64_t>((nrows + rows_per_block - 1) / rows_per_block, cap));
    if (rec && st0)
      hipLaunchKernelGGL((cbsr_stats4_kernel<true, true>), dim3(grid), dim3(256), 0, s, sp_data,
                         sp_index, nrows, k, st0, st1, rec, rec_bytes, zrows, nz, out, D);
    else if (rec)
      hipLaunchKernelGGL((cbsr_stats4_kernel<true, false>), dim3(grid), dim3(256), 0, s, sp_data,
                         sp_index, nrows, k, st0, st1, rec, rec_bytes, zrows, nz, out, D);
    else
      hipLaunchKernelGGL((cbsr_stats4_kernel<false, true>), dim3(grid), dim3(256), 0, s, sp_data,
                         sp_index, nrows, k, st0, st1, rec, rec_bytes, zrows, nz, out, D);
  } else {
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((nrows + 255) / 256, 2 * cus));
    hipLaunchKernelGGL(cbsr_stats_kernel, dim3(grid), dim3(256), 0, s, sp_data, sp_index, nrows,
                       k, st0, st1);
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

static int spgemm_forward_impl(const maxk_plan* plan, const int32_t* ptr, const int32_t* idx,
                               const float* val, const float* sp_data, const uint8_t* sp_index,
                               float* out, int32_t N, int64_t E, int32_t k, int32_t D,
                               void* stream, int accum, void* ws, int64_t ws_bytes,
                               const uint32_t* stats = nullptr, int n_stats = 0,
                               int64_t stats_stride = 2) {
  MAXK_CHECK_ARG(N >= 0 && E >= 0, "maxk_spgemm_forward: negative size");
  MAXK_CHECK_ARG(stats == nullptr || (n_stats >= 1 && n_stats <= 1024),
                 "maxk_spgemm_forward_ex: n_stats must be in [1, 1024]");
  if (stats_stride == 0) stats_stride = 2;
  MAXK_CHECK_ARG(stats_stride >= 2 && stats_stride * (int64_t)n_stats < (int64_t)INT32_MAX,
                 "maxk_spgemm_forward_ex: stats_stride must be >= 2 (or 0)");
  MAXK_CHECK_ARG(D >= 1 && D <= kMaxDim, "maxk_spgemm_forward: dim_origin must be in [1, 256]");
  MAXK_CHECK_ARG(k >= 1 && k <= D, "k must be between 1 and input dimension");
  int rc = check_plan(plan, ptr, idx, N, E, k, D, "maxk_spgemm_forward");
  if (rc) return rc;
  if (N == 0) return MAXK_OK;
  MAXK_CHECK_ARG(out && sp_data && sp_index && (E == 0 || (idx && val)) && ptr,
                 "maxk_spgemm_forward: null pointer");
  (void)val;  // the plan holds the permuted snapshot of (idx, val)
  uint8_t* ws_base = plan->fwd_rec;  // packed CBSR records (per call)
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
  const int R = plan->fwd_tile_rows;
  const int B = plan->fwd_phases;
  const size_t lds = fwd_lds_bytes(R, D, plan->fwd_acc);
  const int rec_bytes = plan->fwd_rec_bytes;
  // two tables: values read straight from sp_data (4k-byte rows), selectors from sp_index
  const bool two = plan->fwd_two_tables;  // the plan only sets it with k % 4 == 0, no chunks
  const uint8_t* seltab = two ? sp_index : nullptr;
  const uint8_t* recp = two ? reinterpret_cast<const uint8_t*>(sp_data) : rec_ws;
  const int rec_bytes_eff = two ? 4 * k : rec_bytes;
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
  const bool pack4 = !two && !plan->fwd_chunk3 && k % 4 == 0 && plan->num_cols > 0;
  if (plan->fwd_chunk3 && plan->num_cols > 0) {
    const int64_t items = (int64_t)plan->num_cols * ((k + 2) / 3);
    const int grid = (int)std::min<int64_t>((items + 255) / 256, 65536);
    hipLaunchKernelGGL(pack_cbsr3_kernel, dim3(grid), dim3(256), 0, s, sp_data, sp_index,
                       rec_ws, plan->num_cols, k, rec_bytes);
    MAXK_LAUNCH_CHECK("pack_cbsr3 launch");
  }
  const bool zero_in_stats = (pack4 || st) && k % 4 == 0;
  if (nz > 0 && !zero_in_stats) {
    hipLaunchKernelGGL(zero_rows_kernel, dim3(nz), dim3(256), 0, s, plan->zero_rows, nz, out, D);
    MAXK_LAUNCH_CHECK("zero_rows launch");
  }
  if (pack4 || st) {
    const int rc = launch_cbsr_stats(sp_data, sp_index, plan->num_cols, k, st,
                                     st ? st + 32 : nullptr, plan->cus, s,
                                     pack4 ? rec_ws : nullptr, rec_bytes, plan->zero_rows,
                                     zero_in_stats ? nz : 0, out, D);
    if (rc) return rc;
  }
  const int rot = plan->fwd_rot_ticks;
  // persistent grid: as many work-groups as fit on the device at once (capped by tasks)
#define FWD_LAUNCH1(V, A, UU, NT, FL)                                                     \
  do {                                                                                    \
    if (lds > 64 * 1024) MAXK_HIP_TRY(allow_lds(spgemm_fwd_kernel<V, A, UU, NT, FL>, lds)); \
    int per_cu = 0;                                                                       \
    MAXK_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(                            \
        &per_cu, spgemm_fwd_kernel<V, A, UU, NT, FL>, NT, lds));                          \
    const int g = plan->fwd_persistent                                                    \
                      ? std::max(1, std::min(plan->n_fwd_tasks, std::max(per_cu, 1) * plan->cus)) \
                      : plan->n_fwd_tasks;                                                \
    for (int b = 0; b < (rot ? 1 : B); ++b)                                               \
      hipLaunchKernelGGL((spgemm_fwd_kernel<V, A, UU, NT, FL>), dim3(g), dim3(NT), lds, s, \
                         plan->fwd_tasks, plan->n_fwd_tasks, plan->fwd_phase_off, B, b,   \
                         plan->fwd_cv, sp_data, sp_index, recp,                           \
                         rec_bytes_eff, out, D, k, R, rot, seltab, accum, fix_tab, xstat, \
                         xs_n, xs_stride, xs_off2);                                       \
  } while (0)
#define FWD_LAUNCH(V, A)                                                                  \
  do {                                                                                    \
    if (plan->fwd_unroll == 16) FWD_LAUNCH1(V, A, 16, 256, 0);                            \
    else FWD_LAUNCH1(V, A, 8, 256, 0);                                                    \
  } while (0)
#define FWD_LAUNCH_FL(NT)                                                                 \
  do {                                                                                    \
    switch (FL & 7) {                                                                     \
      case 0: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, NT, 0); break;                              \
      case 1: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, NT, 1); break;                              \
      case 2: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, NT, 2); break;                              \
      case 3: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, NT, 3); break;                              \
      case 4: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, NT, 4); break;                              \
      case 5: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, NT, 5); break;                              \
      case 6: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, NT, 6); break;                              \
      default: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, NT, 7); break;                             \
    }                                                                                     \
  } while (0)
#define FWD_LAUNCH_FLQ()                                                                  \
  do {                                                                                    \
    switch (FL & 7) {                                                                     \
      case 0: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, 256, 8); break;                             \
      case 1: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, 256, 9); break;                             \
      case 2: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, 256, 10); break;                            \
      case 3: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, 256, 11); break;                            \
      case 4: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, 256, 12); break;                            \
      case 5: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, 256, 13); break;                            \
      case 6: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, 256, 14); break;                            \
      default: FWD_LAUNCH1(4, MAXK_ACC_F64, 8, 256, 15); break;                           \
    }                                                                                     \
  } while (0)
  const int W = plan->fwd_waves;
  const int Lf = plan->fwd_chunk3 ? (k + 2) / 3 : k / 4;  // lanes per edge
  const int FL = (plan->fwd_prefetch ? kFwdFlagPrefetch : 0) |
                 (plan->fwd_branchless ? kFwdFlagBranchless : 0) |
                 (plan->fwd_chunk3 ? kFwdFlagChunk3 : 0) |
                 (plan->fwd_quad && Lf % 4 == 0 && W == 4 ? kFwdFlagQuad : 0);
  if ((k % 4 == 0 || plan->fwd_chunk3) && plan->fwd_acc == MAXK_ACC_F64 &&
      plan->fwd_unroll == 16 && W == 4) {
    switch (FL & 7) {  // 16 sub-steps in flight per wave (no quad loads)
      case 0: FWD_LAUNCH1(4, MAXK_ACC_F64, 16, 256, 0); break;
      case 1: FWD_LAUNCH1(4, MAXK_ACC_F64, 16, 256, 1); break;
      case 2: FWD_LAUNCH1(4, MAXK_ACC_F64, 16, 256, 2); break;
      case 3: FWD_LAUNCH1(4, MAXK_ACC_F64, 16, 256, 3); break;
      case 4: FWD_LAUNCH1(4, MAXK_ACC_F64, 16, 256, 4); break;
      case 5: FWD_LAUNCH1(4, MAXK_ACC_F64, 16, 256, 5); break;
      case 6: FWD_LAUNCH1(4, MAXK_ACC_F64, 16, 256, 6); break;
      default: FWD_LAUNCH1(4, MAXK_ACC_F64, 16, 256, 7); break;
    }
  } else if ((k % 4 == 0 || plan->fwd_chunk3) && plan->fwd_acc == MAXK_ACC_F64 &&
      plan->fwd_unroll == 8) {
    if (FL & kFwdFlagQuad) FWD_LAUNCH_FLQ();
    else if (W == 8) FWD_LAUNCH_FL(512);
    else if (W == 6) FWD_LAUNCH_FL(384);
    else FWD_LAUNCH_FL(256);
  } else if (k % 4 == 0 && !plan->fwd_chunk3) {
    if (plan->fwd_acc == MAXK_ACC_F32_CAS) FWD_LAUNCH(4, MAXK_ACC_F32_CAS);
    else FWD_LAUNCH(4, MAXK_ACC_F64);
  } else {
    if (plan->fwd_acc == MAXK_ACC_F32_CAS) FWD_LAUNCH(1, MAXK_ACC_F32_CAS);
    else FWD_LAUNCH(1, MAXK_ACC_F64);
  }
#undef FWD_LAUNCH_FL
#undef FWD_LAUNCH_FLQ
#undef FWD_LAUNCH
#undef FWD_LAUNCH1
  MAXK_LAUNCH_CHECK("spgemm_fwd launch");
  return MAXK_OK;
}

extern "C" int maxk_spgemm_forward(const maxk_plan* plan, const int32_t* ptr,
                                   const int32_t* idx, const float* val,
                                   const float* sp_data, const uint8_t* sp_index, float* out,
                                   int32_t N, int64_t E, int32_t k, int32_t D, void* stream) {
  return spgemm_forward_impl(plan, ptr, idx, val, sp_data, sp_index, out, N, E, k, D, stream, 0,
                             nullptr, 0);
}

extern "C" int maxk_spgemm_forward_ws(const maxk_plan* plan, const int32_t* ptr,
                                      const int32_t* idx, const float* val,
                                      const float* sp_data, const uint8_t* sp_index, float* out,
                                      int32_t N, int64_t E, int32_t k, int32_t D,
                                      int32_t accumulate, void* workspace,
                                      int64_t workspace_bytes, void* stream) {
  MAXK_CHECK_ARG(accumulate == 0 || accumulate == 1,
                 "maxk_spgemm_forward_ws: accumulate must be 0 or 1");
  return spgemm_forward_impl(plan, ptr, idx, val, sp_data, sp_index, out, N, E, k, D, stream,
                             accumulate, workspace, workspace_bytes);
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
  return spgemm_forward_impl(plan, ptr, idx, val, sp_data, sp_index, out, N, E, k, D, stream,
                             accumulate, workspace, workspace_bytes, stats, n_stats,
                             stats_stride);
}

extern "C" int maxk_cbsr_stats(const float* sp_data, const uint8_t* sp_index, int32_t num_rows,
                               int32_t dim_k, uint32_t* stats, void* stream) {
  MAXK_CHECK_ARG(num_rows >= 0 && dim_k >= 1 && dim_k <= kMaxDim,
                 "maxk_cbsr_stats: bad size");
  MAXK_CHECK_ARG(stats != nullptr && (num_rows == 0 || (sp_data && sp_index)),
                 "maxk_cbsr_stats: null pointer");
  hipStream_t s = (hipStream_t)stream;
  MAXK_HIP_TRY(hipMemsetAsync(stats, 0, 2 * sizeof(uint32_t), s));
  if (num_rows == 0) return MAXK_OK;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  return launch_cbsr_stats(sp_data, sp_index, num_rows, dim_k, stats, stats + 1, cus, s);
}

extern "C" int maxk_spgemm_forward_acc(const maxk_plan* plan, const int32_t* ptr,
                                       const int32_t* idx, const float* val,
                                       const float* sp_data, const uint8_t* sp_index,
                                       float* out, int32_t N, int64_t E, int32_t k, int32_t D,
                                       void* stream) {
  return spgemm_forward_impl(plan, ptr, idx, val, sp_data, sp_index, out, N, E, k, D, stream, 1,
                             nullptr, 0);
}

static int sspmm_backward_impl(const maxk_plan* plan, const int32_t* ptr, const int32_t* idx,
                               const float* val, const float* grad_out,
                               const uint8_t* sp_index, float* grad_sp, int32_t N, int64_t E,
                               int32_t k, int32_t D, void* stream, void* ws, int64_t ws_bytes) {
  (void)val;  // the plan holds the block-major snapshot of val
  MAXK_CHECK_ARG(N >= 0 && E >= 0, "maxk_sspmm_backward: negative size");
  MAXK_CHECK_ARG(D >= 1 && D <= kMaxDim, "maxk_sspmm_backward: dim_origin must be in [1, 256]");
  MAXK_CHECK_ARG(k >= 1 && k <= D, "k must be between 1 and input dimension");
  int rc = check_plan(plan, ptr, idx, N, E, k, D, "maxk_sspmm_backward");
  if (rc) return rc;
  if (N == 0) return MAXK_OK;
  MAXK_CHECK_ARG(grad_out && sp_index && grad_sp, "maxk_sspmm_backward: null pointer");
  // per-call scratch: selector words + flush slabs (column kernels) or the E x k products
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
  float* slab = plan->bwd_slab_floats > 0
                    ? reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(sel_ws) + plan->bwd_slab_off)
                    : nullptr;
  auto combine = [&]() -> int {
    if (!slab) return MAXK_OK;
    const int slices = (plan->bwd_block_cols * k + kCombineSlice - 1) / kCombineSlice;
    hipLaunchKernelGGL(bwd_combine_kernel, dim3(slices, plan->n_bwd_combine), dim3(256), 0,
                       (hipStream_t)stream, grad_sp, slab, plan->bwd_combine, k,
                       plan->bwd_block_cols * k, plan->bwd_corder);
    MAXK_LAUNCH_CHECK("bwd_combine launch");
    return MAXK_OK;
  };
  hipStream_t s = (hipStream_t)stream;
  if (plan->bwd_twopass) {
    // the plan checked k % 4 == 0, k / 4 a power of two <= 64, E > 0, NC > 0; per row chunk
    // (the workspace holds one chunk's products): row pass, then column pass
    const int R = plan->bwd_tp_rows;
    const bool cs = plan->bwd_tp_csc;  // the plan allows it with one chunk only
    const int P = plan->bwd_tp_chunks;
    const int NC = plan->num_cols;
    for (int p = 0; p < P; ++p) {
      const int rb = plan->tp_rows[p], re = plan->tp_rows[p + 1];
      const int64_t eb = plan->tp_edges[p];
      if (re > rb) {
        const dim3 rgrid((re - rb + 4 * R - 1) / (4 * R));
#define ROWS_LAUNCH(RR)                                                                   \
        do {                                                                              \
          if (cs)                                                                         \
            hipLaunchKernelGGL((sspmm_bwd_rows_kernel<4, RR, true>), rgrid, dim3(256), 0, s, \
                               ptr, plan->bwd_erec, grad_out, sp_index, tbuf_ws, rb, re,  \
                               eb, D, k, plan->bwd_perm);                                 \
          else                                                                            \
            hipLaunchKernelGGL((sspmm_bwd_rows_kernel<4, RR>), rgrid, dim3(256), 0, s, ptr, \
                               plan->bwd_erec, grad_out, sp_index, tbuf_ws, rb, re, eb, D, \
                               k, nullptr);                                               \
        } while (0)
        if (R >= 8) ROWS_LAUNCH(8);
        else if (R == 4) ROWS_LAUNCH(4);
        else if (R == 2) ROWS_LAUNCH(2);
        else ROWS_LAUNCH(1);
#undef ROWS_LAUNCH
        MAXK_LAUNCH_CHECK("sspmm_bwd_rows launch");
      }
      const int32_t* lo = P > 1 ? plan->bwd_colptr2 + (size_t)p * NC : plan->bwd_colptr;
      const int32_t* hi = P > 1 ? plan->bwd_colptr2 + (size_t)(p + 1) * NC : plan->bwd_colptr + 1;
      if (cs)
        hipLaunchKernelGGL((sspmm_bwd_cols_kernel<4, true>), dim3((NC + 3) / 4), dim3(256), 0, s,
                           lo, hi, nullptr, tbuf_ws, (int64_t)0, grad_sp, NC, k, 0);
      else
        hipLaunchKernelGGL((sspmm_bwd_cols_kernel<4>), dim3((NC + 3) / 4), dim3(256), 0, s, lo,
                           hi, plan->bwd_perm, tbuf_ws, eb, grad_sp, NC, k, p > 0 ? 1 : 0);
      MAXK_LAUNCH_CHECK("sspmm_bwd_cols launch");
    }
    return MAXK_OK;
  }
  if (plan->bwd_csc) {
    const int F = plan->bwd_feats;
    if (F == 4) {
      const int nsel = plan->num_cols * (k / 4);
      hipLaunchKernelGGL(pack_sel_kernel, dim3((nsel + 255) / 256), dim3(256), 0, s, sp_index,
                         plan->num_cols, k, 1, sel_ws, nullptr);
    }
    const uint32_t g_bytes = (uint32_t)((uint64_t)N * D * 4u);
    const dim3 cgrid((plan->num_cols + 3) / 4);
#define CSC_LAUNCH(FF, UU)                                                                \
    hipLaunchKernelGGL((sspmm_bwd_csc_kernel<FF, UU>), cgrid, dim3(256), 0, s,            \
                       plan->bwd_colptr, plan->bwd_rec, grad_out, g_bytes, sel_ws, \
                       sp_index, grad_sp, plan->num_cols, k)
    if (F == 4) {
      if (plan->bwd_unroll >= 8) CSC_LAUNCH(4, 8);
      else CSC_LAUNCH(4, 4);
    } else {
      if (plan->bwd_unroll >= 16) CSC_LAUNCH(1, 16);
      else if (plan->bwd_unroll >= 8) CSC_LAUNCH(1, 8);
      else CSC_LAUNCH(1, 4);
    }
#undef CSC_LAUNCH
    MAXK_LAUNCH_CHECK("sspmm_bwd_csc launch");
    return MAXK_OK;
  }
  if (plan->n_bwd_shared > 0 && !slab)  // atomic flush: shared blocks add into zeros
    MAXK_HIP_TRY(hipMemsetAsync(grad_sp, 0, (size_t)plan->num_cols * k * sizeof(float), s));
  if (plan->n_bwd_tasks == 0) return MAXK_OK;
  const size_t lds = bwd_lds_bytes(plan->bwd_block_cols, k, plan->bwd_acc);
  const dim3 grid(plan->n_bwd_tasks), block(kBwdThreads);  // general path: 512 threads
  if (plan->bwd_rec && plan->bwd_feats == 1) {
    const uint32_t g_bytes = (uint32_t)((uint64_t)N * D * 4u);
    const size_t lds1 = ((size_t)plan->bwd_block_cols * plan->bwd_ks + 3) / 4 * 4 * sizeof(float) +
                        (size_t)plan->bwd_block_cols * k;
#define BWD1_LAUNCH(UU, NT)                                                               \
    do {                                                                                  \
      if (lds1 > 64 * 1024) MAXK_HIP_TRY(allow_lds(sspmm_bwd1_kernel<UU, NT>, lds1));     \
      hipLaunchKernelGGL((sspmm_bwd1_kernel<UU, NT>), grid, dim3(NT), lds1, s,            \
                         plan->bwd_tasks, plan->bwd_rec, grad_out, g_bytes, sp_index,     \
                         grad_sp, k, plan->bwd_ks, slab, plan->bwd_corder);              \
    } while (0)
    const int W = plan->bwd_waves, U = plan->bwd_unroll;
    if (W == 16) BWD1_LAUNCH(16, 1024);
    else if (W == 12) {
      if (U >= 16) BWD1_LAUNCH(16, 768);
      else BWD1_LAUNCH(8, 768);
    } else if (U >= 16) BWD1_LAUNCH(16, 512);
    else if (U >= 12) BWD1_LAUNCH(12, 512);
    else BWD1_LAUNCH(8, 512);
#undef BWD1_LAUNCH
    MAXK_LAUNCH_CHECK("sspmm_bwd1 launch");
    return combine();
  }
  if (plan->bwd_rec && plan->bwd_feats == 2) {  // two slots per lane
    const int S = plan->bwd_slot_groups;
    const int nsel = plan->num_cols * (k / 2);
    hipLaunchKernelGGL(pack_sel2_kernel, dim3((nsel + 255) / 256), dim3(256), 0, s, sp_index,
                       plan->num_cols, k, S, reinterpret_cast<uint16_t*>(sel_ws),
                       plan->bwd_corder);
    const uint32_t g_bytes = (uint32_t)((uint64_t)N * D * 4u);
    const size_t lds2 = ((size_t)plan->bwd_block_cols * plan->bwd_ks + 3) / 4 * 4 * sizeof(float) +
                        (plan->bwd_sel_lds ? (size_t)plan->bwd_block_cols * (k / S) : 0);
#define BWD2_LAUNCH(UU, NT, V, Q)                                                         \
    do {                                                                                  \
      if (lds2 > 64 * 1024)                                                               \
        MAXK_HIP_TRY(allow_lds(sspmm_bwd4_kernel<UU, NT, false, V, Q, 2>, lds2));         \
      hipLaunchKernelGGL((sspmm_bwd4_kernel<UU, NT, false, V, Q, 2>), grid, dim3(NT), lds2, s, \
                         plan->bwd_tasks, plan->bwd_rec, grad_out, g_bytes, sel_ws,       \
                         grad_sp, k, S, plan->num_cols, plan->bwd_ks, plan->bwd_sel_lds,  \
                         slab, plan->bwd_corder);                                         \
    } while (0)
    const int U = plan->bwd_unroll;
    const bool QL = plan->bwd_quad && (k / S / 2) % 4 == 0;
    if (plan->bwd_cas64) {
      if (U >= 16) {
        if (QL) BWD2_LAUNCH(16, 512, true, true);
        else BWD2_LAUNCH(16, 512, true, false);
      } else if (U >= 12) {
        if (QL) BWD2_LAUNCH(12, 512, true, true);
        else BWD2_LAUNCH(12, 512, true, false);
      } else {
        if (QL) BWD2_LAUNCH(8, 512, true, true);
        else BWD2_LAUNCH(8, 512, true, false);
      }
    } else {
      if (QL) BWD2_LAUNCH(8, 512, false, true);
      else BWD2_LAUNCH(8, 512, false, false);
    }
#undef BWD2_LAUNCH
    MAXK_LAUNCH_CHECK("sspmm_bwd2 launch");
    return combine();
  }
  if (plan->bwd_rec) {
    const int S = plan->bwd_slot_groups;
    const int nsel = plan->num_cols * (k / 4);
    hipLaunchKernelGGL(pack_sel_kernel, dim3((nsel + 255) / 256), dim3(256), 0, s, sp_index,
                       plan->num_cols, k, S, sel_ws, plan->bwd_corder);
    const uint32_t g_bytes = (uint32_t)((uint64_t)N * D * 4u);
    const size_t lds4 = ((size_t)plan->bwd_block_cols * plan->bwd_ks + 3) / 4 * 4 * sizeof(float) +
                        (plan->bwd_sel_lds ? (size_t)plan->bwd_block_cols * (k / S) : 0);
#define BWD4_LAUNCH(UU, NT, PF, V, Q)                                                     \
    do {                                                                                  \
      if (lds4 > 64 * 1024) MAXK_HIP_TRY(allow_lds(sspmm_bwd4_kernel<UU, NT, PF, V, Q>, lds4)); \
      hipLaunchKernelGGL((sspmm_bwd4_kernel<UU, NT, PF, V, Q>), grid, dim3(NT), lds4, s,  \
                         plan->bwd_tasks, plan->bwd_rec, grad_out, g_bytes, sel_ws, \
                         grad_sp, k, S, plan->num_cols, plan->bwd_ks, plan->bwd_sel_lds,  \
                         slab, plan->bwd_corder);                                         \
    } while (0)
    const int W = plan->bwd_waves, U = plan->bwd_unroll;
    const bool PFon = plan->bwd_prefetch != 0;
    const bool QL = plan->bwd_quad && (k / S / 4) % 4 == 0;  // quad-aligned edge lane groups
    if (plan->bwd_cas64) {
      if (W == 16) {
        if (QL) BWD4_LAUNCH(6, 1024, false, true, true);
        else BWD4_LAUNCH(6, 1024, false, true, false);
      } else if (W == 12) {
        if (QL) BWD4_LAUNCH(8, 768, false, true, true);
        else BWD4_LAUNCH(8, 768, false, true, false);
      } else if (PFon) {
        if (QL) BWD4_LAUNCH(8, 512, true, true, true);
        else BWD4_LAUNCH(8, 512, true, true, false);
      } else if (U == 12) {
        if (QL) BWD4_LAUNCH(12, 512, false, true, true);
        else BWD4_LAUNCH(12, 512, false, true, false);
      } else if (U == 16) {
        BWD4_LAUNCH(16, 512, false, true, false);
      } else {
        if (QL) BWD4_LAUNCH(8, 512, false, true, true);
        else BWD4_LAUNCH(8, 512, false, true, false);
      }
    } else if (W == 16) {
      if (PFon) BWD4_LAUNCH(6, 1024, true, false, false);
      else BWD4_LAUNCH(6, 1024, false, false, false);
    } else if (W == 12) {
      if (PFon) BWD4_LAUNCH(8, 768, true, false, false);
      else BWD4_LAUNCH(8, 768, false, false, false);
    } else if (PFon) {
      BWD4_LAUNCH(8, 512, true, false, false);
    } else if (U == 16) BWD4_LAUNCH(16, 512, false, false, false);
    else if (U == 12) BWD4_LAUNCH(12, 512, false, false, false);
    else if (U == 4) BWD4_LAUNCH(4, 512, false, false, false);
    else BWD4_LAUNCH(8, 512, false, false, false);
#undef BWD4_LAUNCH
    MAXK_LAUNCH_CHECK("sspmm_bwd launch");
    return combine();
  }
#define BWD_LAUNCH1(F, A, UU)                                                             \
  do {                                                                                    \
    if (lds > 64 * 1024) MAXK_HIP_TRY(allow_lds(sspmm_bwd_kernel<F, A, UU>, lds));       \
    hipLaunchKernelGGL((sspmm_bwd_kernel<F, A, UU>), grid, block, lds, s, plan->bwd_tasks, \
                       plan->bwd_row, plan->bwd_col, plan->bwd_val, grad_out, sp_index,   \
                       grad_sp, D, k);                                                    \
  } while (0)
#define BWD_LAUNCH(F, A)                                                                  \
  do {                                                                                    \
    if (plan->bwd_unroll >= 12) BWD_LAUNCH1(F, A, 16);                                    \
    else BWD_LAUNCH1(F, A, 8);                                                            \
  } while (0)
  if (plan->bwd_feats == 4) {
    if (plan->bwd_acc == MAXK_ACC_F32_CAS) BWD_LAUNCH(4, MAXK_ACC_F32_CAS);
    else BWD_LAUNCH(4, MAXK_ACC_F64);
  } else {
    if (plan->bwd_acc == MAXK_ACC_F32_CAS) BWD_LAUNCH(1, MAXK_ACC_F32_CAS);
    else BWD_LAUNCH(1, MAXK_ACC_F64);
  }
#undef BWD_LAUNCH
#undef BWD_LAUNCH1
  MAXK_LAUNCH_CHECK("sspmm_bwd launch");
  return MAXK_OK;
}

extern "C" int maxk_sspmm_backward(const maxk_plan* plan, const int32_t* ptr,
                                   const int32_t* idx, const float* val,
                                   const float* grad_out, const uint8_t* sp_index,
                                   float* grad_sp, int32_t N, int64_t E, int32_t k, int32_t D,
                                   void* stream) {
  return sspmm_backward_impl(plan, ptr, idx, val, grad_out, sp_index, grad_sp, N, E, k, D,
                             stream, nullptr, 0);
}

extern "C" int maxk_sspmm_backward_ws(const maxk_plan* plan, const int32_t* ptr,
                                      const int32_t* idx, const float* val,
                                      const float* grad_out, const uint8_t* sp_index,
                                      float* grad_sp, int32_t N, int64_t E, int32_t k,
                                      int32_t D, void* workspace, int64_t workspace_bytes,
                                      void* stream) {
  return sspmm_backward_impl(plan, ptr, idx, val, grad_out, sp_index, grad_sp, N, E, k, D,
                             stream, workspace, workspace_bytes);
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
