// Exact top-k probes (tooling, round 5): where the product kernel's time goes and whether a
// pipelined row loop or an LDS-free selection is faster. Includes the product source, so the
// variants reuse its exact_select / emit_staged. Build here, run on the GPU box:
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -shared -fPIC -Iinclude -Ispgemm-gnn_amd/csrc \
//         tools/probe_topk2.hip spgemm-gnn_amd/csrc/capi.cpp -o tools/libprobe_topk2.so
//   python tools/probe_topk2.py
//
// variant 0: the library kernel (maxk_topk_cbsr)
//         1: pipelined rows: a wave owns R rows, keeps P row loads in flight (row r + P is
//            issued before row r is selected), D = 256
//         2: compute only: R rows loaded once, exact_select run REP times per row, one dword
//            per wave stored (selection throughput without the loads and the emit)
//         4: lean_select + emit_lean (fewer scalar instructions), pipelined like 1
//         3: LDS-free selection: after the top-byte walk, a bit descent on ballots of the
//            surviving candidates (no histogram round trips), pipelined like 1
#include "../spgemm-gnn_amd/csrc/maxk_topk.hip"

namespace probe {
using namespace maxk;

// Bit descent: the same contract as exact_select. The walk fixes the top byte (and how many
// keys are still needed inside its bin); then each lower bit splits the surviving candidates
// (lane masks in SGPRs) in two, keeping the half that holds the need-th largest, until the
// surviving bin holds exactly the keys needed or every bit is fixed (ties).
__device__ __forceinline__ void descent_select(const float x[4], int k, int lane, bool sel[4]) {
  uint32_t u[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) u[i] = order_key(x[i]);
  uint32_t m = max(max(u[0], u[1]), max(u[2], u[3]));
  m = wave_umax(m);
  const int top = (int)(m >> 24);
  uint32_t need = (uint32_t)k;
  uint64_t alive[4], above[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) above[i] = 0;
  uint32_t ctot = 0;
  // top byte walk: keys above the threshold byte are selected outright
  for (int b = top;; --b) {
    uint32_t cnt = 0;
    uint64_t in_b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      in_b[i] = __ballot((u[i] >> 24) == (uint32_t)b);
      cnt += __popcll(in_b[i]);
    }
    if (cnt >= need) {
#pragma unroll
      for (int i = 0; i < 4; ++i) alive[i] = in_b[i];
      ctot = cnt;
      break;
    }
    need -= cnt;
#pragma unroll
    for (int i = 0; i < 4; ++i) above[i] |= in_b[i];
  }
  for (int bit = 23; bit >= 0 && ctot != need; --bit) {
    uint64_t one[4];
    uint32_t cnt = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      one[i] = alive[i] & __ballot((u[i] >> bit) & 1u);
      cnt += __popcll(one[i]);
    }
    if (cnt >= need) {
#pragma unroll
      for (int i = 0; i < 4; ++i) alive[i] = one[i];
      ctot = cnt;
    } else {
      need -= cnt;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        above[i] |= one[i];
        alive[i] &= ~one[i];
      }
      ctot -= cnt;
    }
  }
  // alive: the keys equal to the threshold (all of them when ctot == need); take the lowest
  // feature indices among them
  const uint64_t me = 1ull << lane;
  int rank = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) rank += (int)lanes_below(alive[i]);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool a = (alive[i] & me) != 0;
    sel[i] = ((above[i] & me) != 0) || (a && rank < (int)need);
    rank += a ? 1 : 0;
  }
}


__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t v) {
  return wave_reduce_dpp(v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
}

// Fewer scalar instructions (the scalar unit, one per CU, bounds exact_select): the top byte
// from packed per-bin counts summed with DPP (no ballot per bin), histogram adds unconditional
// (+0 for keys outside the prefix: no exec-mask branches), the rest as exact_select.
__device__ __forceinline__ void lean_select(const float x[4], int k, uint32_t* hist, int lane,
                                            bool sel[4]) {
  uint32_t u[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) u[i] = order_key(x[i]);
  const uint32_t top = wave_umax(max(max(u[0], u[1]), max(u[2], u[3]))) >> 24;
  // bins top, top-1, top-2 counted in 10-bit fields of one word
  uint32_t w = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t d = top - (u[i] >> 24);
    w += d < 3u ? 1u << (10u * d) : 0u;
  }
  w = wave_sum_dpp(w);
  uint32_t need = (uint32_t)k, prefix = 0, pmask = 0;
  bool whole_bin = false;
  int first_shift = 24;
  {
    const uint32_t c0 = w & 1023u, c1 = (w >> 10) & 1023u, c2 = w >> 20;
    if (c0 >= need) { prefix = top; whole_bin = c0 == need; }
    else if (c0 + c1 >= need) { need -= c0; prefix = top - 1; whole_bin = c1 == need; }
    else if (c0 + c1 + c2 >= need) { need -= c0 + c1; prefix = top - 2; whole_bin = c2 == need; }
    else { need -= c0 + c1 + c2; prefix = 0xffffffffu; }  // below top-2: histogram of the top byte
    if (prefix != 0xffffffffu) {
      prefix <<= 24;
      pmask = 0xff000000u;
      first_shift = 16;
    } else {
      // keys in bins top..top-2 are above the threshold: histogram the rest's top byte
      prefix = 0;
      first_shift = 24;
    }
  }
  const uint32_t below = top >= 3u ? (top - 2u) << 24 : 0u;  // keys < below: candidates of the fallback
#pragma unroll
  for (int shift = 24; shift >= 0; shift -= 8) {
    if (shift > first_shift || whole_bin) continue;  // uniform
    reinterpret_cast<uint4*>(hist)[lane] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool in = shift == 24 ? u[i] < below : (u[i] & pmask) == prefix;
      __hip_atomic_fetch_add(&hist[(u[i] >> shift) & 255u], in ? 1u : 0u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    const uint4 h = reinterpret_cast<const uint4*>(hist)[lane];
    const uint32_t lsum = h.x + h.y + h.z + h.w;
    const uint32_t pre = wave_prefix_sum(lsum);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)pre, kWave - 1);
    const uint32_t ge3 = total - pre + h.w;
    const uint32_t ge2 = ge3 + h.z, ge1 = ge2 + h.y, ge0 = ge1 + h.x;
    const uint64_t m = __ballot(ge0 >= need);
    const int ls = 63 - __builtin_clzll(m);
    uint32_t d, above, inbin;
    if (ge3 >= need) { d = 3; above = ge3 - h.w; inbin = h.w; }
    else if (ge2 >= need) { d = 2; above = ge3; inbin = h.z; }
    else if (ge1 >= need) { d = 1; above = ge2; inbin = h.y; }
    else { d = 0; above = ge1; inbin = h.x; }
    d = (uint32_t)__builtin_amdgcn_readlane((int)(4 * lane + d), ls);
    above = (uint32_t)__builtin_amdgcn_readlane((int)above, ls);
    inbin = (uint32_t)__builtin_amdgcn_readlane((int)inbin, ls);
    need -= above;
    prefix |= d << shift;
    pmask |= 255u << shift;
    if (inbin == need) {
      whole_bin = true;
      break;
    }
  }
  if (whole_bin) {
#pragma unroll
    for (int i = 0; i < 4; ++i) sel[i] = (u[i] & pmask) >= prefix;
  } else {
    const uint32_t T = prefix;
    uint64_t meq[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) meq[i] = __ballot(u[i] == T);
    int rank = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) rank += (int)lanes_below(meq[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool eq = u[i] == T;
      sel[i] = u[i] > T || (eq && rank < (int)need);
      rank += eq ? 1 : 0;
    }
  }
}

// emit_staged<false> without divergent branches: every element writes its stage slot, the
// unselected (and those past k) into a per-lane dummy slot 64 + lane (k <= 64).
__device__ __forceinline__ void emit_lean(const float x[4], const bool sel[4], int lane, int row,
                                          int k, float* stage_v, uint8_t* stage_i,
                                          float* __restrict__ sp_data,
                                          uint8_t* __restrict__ sp_index) {
  uint64_t m[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) m[i] = __ballot(sel[i]);
  int pos = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) pos += (int)lanes_below(m[i]);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int at = sel[i] && pos < k ? pos : 64 + lane;
    stage_v[at] = x[i];
    stage_i[at] = (uint8_t)(lane * 4 + i);
    pos += sel[i] ? 1 : 0;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float* drow = sp_data + (size_t)row * k;
  uint8_t* irow = sp_index + (size_t)row * k;
  if (lane < k) drow[lane] = stage_v[lane];
  if ((k & 3) == 0) {
    if (lane < k / 4)
      reinterpret_cast<uint32_t*>(irow)[lane] = reinterpret_cast<const uint32_t*>(stage_i)[lane];
  } else if (lane < k) {
    irow[lane] = stage_i[lane];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int R, int P, int SELECT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void topk_pipe_kernel(
    const float* __restrict__ in, float* __restrict__ sp_data, uint8_t* __restrict__ sp_index,
    int N, int k) {
  __shared__ __align__(16) uint32_t hist_all[4][256];
  __shared__ __align__(16) float stage_v[4][kMaxDim];
  __shared__ __align__(16) uint8_t stage_i[4][kMaxDim];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x / 64;
  const int row0 = (blockIdx.x * 4 + w) * R;
  if (row0 >= N) return;
  float ring[P][4];
  const bool valid[4] = {true, true, true, true};
  auto load = [&](int r, float (&dst)[4]) {
    const float4 v = *reinterpret_cast<const float4*>(in + (size_t)min(r, N - 1) * 256 + 4 * lane);
    dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
  };
#pragma unroll
  for (int p = 0; p < P; ++p) load(row0 + p, ring[p]);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int row = row0 + r;
    float x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = ring[r % P][i];
    if (r + P < R) load(row0 + r + P, ring[r % P]);
    if (row >= N) break;
    bool sel[4];
    if constexpr (SELECT == 0) exact_select(x, valid, k, hist_all[w], lane, sel);
    else if constexpr (SELECT == 1) descent_select(x, k, lane, sel);
    else lean_select(x, k, hist_all[w], lane, sel);
    if constexpr (SELECT >= 2) emit_lean(x, sel, lane, row, k, stage_v[w], stage_i[w], sp_data, sp_index);
    else emit_staged<false>(x, sel, lane, row, k, stage_v[w], stage_i[w], sp_data, sp_index, k, k);
  }
}


// Two rows selected in lockstep by one wave: their dependency chains (DPP scans, LDS
// round trips, readlanes) are independent, so the compiler interleaves them and each wave has
// twice the latency-hiding work (the selection is latency-bound at full occupancy: its time did
// not change when the scalar instructions were cut, lean_select).
struct RowSel {
  uint32_t u[4];
  uint32_t need, prefix, pmask;
  int first_shift;
  bool whole;
};

__device__ __forceinline__ void row_top(RowSel& S, const float x[4], int k) {
#pragma unroll
  for (int i = 0; i < 4; ++i) S.u[i] = order_key(x[i]);
  const uint32_t top = wave_umax(max(max(S.u[0], S.u[1]), max(S.u[2], S.u[3]))) >> 24;
  uint32_t w = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t d = top - (S.u[i] >> 24);
    w += d < 3u ? 1u << (10u * d) : 0u;
  }
  w = wave_sum_dpp(w);
  const uint32_t c0 = w & 1023u, c1 = (w >> 10) & 1023u, c2 = w >> 20;
  uint32_t need = (uint32_t)k;
  S.whole = false;
  S.first_shift = 16;
  S.pmask = 0xff000000u;
  if (c0 >= need) { S.prefix = top << 24; S.whole = c0 == need; }
  else if (c0 + c1 >= need) { need -= c0; S.prefix = (top - 1) << 24; S.whole = c1 == need; }
  else if (c0 + c1 + c2 >= need) { need -= c0 + c1; S.prefix = (top - 2) << 24; S.whole = c2 == need; }
  else { need -= c0 + c1 + c2; S.prefix = (top - 2) << 24; S.pmask = 0; S.first_shift = 24; }
  S.need = need;
}

// one radix pass of 8 bits at `shift` for row S (act: the row takes part; else its adds are
// +0 and its state is left alone). shift 24 = the fallback below bin top-2 (prefix holds
// (top - 2) << 24 and pmask 0 then: candidates are the keys below it).
__device__ __forceinline__ void row_pass(RowSel& S, int shift, uint32_t* hist, int lane, bool act) {
  reinterpret_cast<uint4*>(hist)[lane] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool in = shift == 24 ? S.u[i] < S.prefix : (S.u[i] & S.pmask) == S.prefix;
    __hip_atomic_fetch_add(&hist[(S.u[i] >> shift) & 255u], act && in ? 1u : 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  const uint4 h = reinterpret_cast<const uint4*>(hist)[lane];
  const uint32_t lsum = h.x + h.y + h.z + h.w;
  const uint32_t pre = wave_prefix_sum(lsum);
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)pre, kWave - 1);
  const uint32_t need = S.need;
  const uint32_t ge3 = total - pre + h.w;
  const uint32_t ge2 = ge3 + h.z, ge1 = ge2 + h.y, ge0 = ge1 + h.x;
  const uint64_t m = __ballot(ge0 >= need);
  const int ls = m ? 63 - __builtin_clzll(m) : 0;
  uint32_t d, above, inbin;
  if (ge3 >= need) { d = 3; above = ge3 - h.w; inbin = h.w; }
  else if (ge2 >= need) { d = 2; above = ge3; inbin = h.z; }
  else if (ge1 >= need) { d = 1; above = ge2; inbin = h.y; }
  else { d = 0; above = ge1; inbin = h.x; }
  d = (uint32_t)__builtin_amdgcn_readlane((int)(4 * lane + d), ls);
  above = (uint32_t)__builtin_amdgcn_readlane((int)above, ls);
  inbin = (uint32_t)__builtin_amdgcn_readlane((int)inbin, ls);
  if (act) {
    S.need = need - above;
    if (shift == 24) S.prefix = 0;
    S.prefix |= d << shift;
    S.pmask |= 255u << shift;
    S.whole = inbin == S.need;
  }
}

__device__ __forceinline__ void row_finish(const RowSel& S, bool sel[4]) {
  if (S.whole) {
#pragma unroll
    for (int i = 0; i < 4; ++i) sel[i] = (S.u[i] & S.pmask) >= S.prefix;
  } else {
    const uint32_t T = S.prefix;
    uint64_t meq[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) meq[i] = __ballot(S.u[i] == T);
    int rank = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) rank += (int)lanes_below(meq[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool eq = S.u[i] == T;
      sel[i] = S.u[i] > T || (eq && rank < (int)S.need);
      rank += eq ? 1 : 0;
    }
  }
}

__device__ __forceinline__ void dual_select(const float xa[4], const float xb[4], int k,
                                            uint32_t* ha, uint32_t* hb, int lane, bool sa[4],
                                            bool sb[4]) {
  RowSel A, B;
  row_top(A, xa, k);
  row_top(B, xb, k);
#pragma unroll
  for (int shift = 24; shift >= 0; shift -= 8) {
    const bool aa = !A.whole && shift <= A.first_shift;
    const bool ab = !B.whole && shift <= B.first_shift;
    if (!aa && !ab) continue;  // uniform
    row_pass(A, shift, ha, lane, aa);
    row_pass(B, shift, hb, lane, ab);
  }
  row_finish(A, sa);
  row_finish(B, sb);
}

template <int R, int P>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void topk_dual_kernel(
    const float* __restrict__ in, float* __restrict__ sp_data, uint8_t* __restrict__ sp_index,
    int N, int k) {
  static_assert(R % 2 == 0 && P % 2 == 0, "row pairs");
  __shared__ __align__(16) uint32_t hist_all[4][2][256];
  __shared__ __align__(16) float stage_v[4][kMaxDim];
  __shared__ __align__(16) uint8_t stage_i[4][kMaxDim];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x / 64;
  const int row0 = (blockIdx.x * 4 + w) * R;
  if (row0 >= N) return;
  float ring[P][4];
  auto load = [&](int r, float (&dst)[4]) {
    const float4 v = *reinterpret_cast<const float4*>(in + (size_t)min(r, N - 1) * 256 + 4 * lane);
    dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
  };
#pragma unroll
  for (int p = 0; p < P; ++p) load(row0 + p, ring[p]);
#pragma unroll
  for (int r = 0; r < R; r += 2) {
    float xa[4], xb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      xa[i] = ring[r % P][i];
      xb[i] = ring[(r + 1) % P][i];
    }
    if (r + P < R) {
      load(row0 + r + P, ring[r % P]);
      load(row0 + r + 1 + P, ring[(r + 1) % P]);
    }
    if (row0 + r >= N) break;
    bool sa[4], sb[4];
    dual_select(xa, xb, k, hist_all[w][0], hist_all[w][1], lane, sa, sb);
    emit_lean(xa, sa, lane, row0 + r, k, stage_v[w], stage_i[w], sp_data, sp_index);
    if (row0 + r + 1 < N)
      emit_lean(xb, sb, lane, row0 + r + 1, k, stage_v[w], stage_i[w], sp_data, sp_index);
  }
}

template <int R, int REP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void topk_compute_kernel(
    const float* __restrict__ in, uint32_t* __restrict__ sink, int N, int k, int select) {
  __shared__ __align__(16) uint32_t hist_all[4][256];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x / 64;
  const int row0 = (blockIdx.x * 4 + w) * R;
  if (row0 >= N) return;
  float xs[R][4];
  const bool valid[4] = {true, true, true, true};
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float4 v = *reinterpret_cast<const float4*>(in + (size_t)min(row0 + r, N - 1) * 256 + 4 * lane);
    xs[r][0] = v.x; xs[r][1] = v.y; xs[r][2] = v.z; xs[r][3] = v.w;
  }
  uint32_t acc = 0;
  for (int rep = 0; rep < REP; ++rep) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float x[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = xs[r][i] + (float)rep * 0.0f;
      bool sel[4];
      if (select == 0) exact_select(x, valid, k, hist_all[w], lane, sel);
      else if (select == 1) descent_select(x, k, lane, sel);
      else lean_select(x, k, hist_all[w], lane, sel);
      acc += (uint32_t)sel[0] + 2u * sel[1] + 4u * sel[2] + 8u * sel[3];
    }
  }
  acc = wave_umax(acc);
  if (lane == 0) sink[blockIdx.x * 4 + w] = acc;
}

}  // namespace probe

extern "C" float probe_topk2(int variant, int R, int P, int rep, const float* in, float* d,
                             uint8_t* i, uint32_t* sink, int N, int k, int iters) {
  using namespace probe;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto launch = [&]() {
    const int rpb = 4 * R;
    const dim3 grid((N + rpb - 1) / rpb);
#define PIPE(RR, PP, SS) hipLaunchKernelGGL((topk_pipe_kernel<RR, PP, SS>), grid, dim3(256), 0, 0, in, d, i, N, k)
#define COMP(RR, RE) hipLaunchKernelGGL((topk_compute_kernel<RR, RE>), grid, dim3(256), 0, 0, in, sink, N, k, P)
    if (variant == 0) {
      maxk_topk_cbsr(in, d, i, N, 256, k, 0, nullptr);
    } else if (variant == 5) {
#define DUAL(RR, PP) hipLaunchKernelGGL((topk_dual_kernel<RR, PP>), grid, dim3(256), 0, 0, in, d, i, N, k)
      if (R == 2 && P == 2) DUAL(2, 2);
      else if (R == 4 && P == 4) DUAL(4, 4);
      else if (R == 8 && P == 4) DUAL(8, 4);
      else if (R == 8 && P == 8) DUAL(8, 8);
      else if (R == 4 && P == 2) DUAL(4, 2);
#undef DUAL
    } else if (variant == 4) {
      if (R == 4 && P == 4) PIPE(4, 4, 2);
      else if (R == 2 && P == 2) PIPE(2, 2, 2);
      else if (R == 8 && P == 4) PIPE(8, 4, 2);
      else if (R == 8 && P == 8) PIPE(8, 8, 2);
      else if (R == 1 && P == 1) PIPE(1, 1, 2);
    } else if (variant == 1 || variant == 3) {
      const int S = variant == 3 ? 1 : 0;
      if (R == 4 && P == 1) { if (S) PIPE(4, 1, 1); else PIPE(4, 1, 0); }
      else if (R == 4 && P == 2) { if (S) PIPE(4, 2, 1); else PIPE(4, 2, 0); }
      else if (R == 8 && P == 2) { if (S) PIPE(8, 2, 1); else PIPE(8, 2, 0); }
      else if (R == 8 && P == 4) { if (S) PIPE(8, 4, 1); else PIPE(8, 4, 0); }
      else if (R == 4 && P == 4) { if (S) PIPE(4, 4, 1); else PIPE(4, 4, 0); }
      else if (R == 2 && P == 2) { if (S) PIPE(2, 2, 1); else PIPE(2, 2, 0); }
    } else if (variant == 2) {  // P = select kind here
      if (R == 4 && rep == 1) COMP(4, 1);
      else if (R == 4 && rep == 4) COMP(4, 4);
    }
#undef PIPE
#undef COMP
  };
  launch();
  hipDeviceSynchronize();
  hipEventRecord(a, 0);
  for (int t = 0; t < iters; ++t) launch();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms / iters;
}
