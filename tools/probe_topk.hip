// Probe (tooling, not product): where the exact top-k's time goes and what a different emit /
// rows-per-wave would buy. Reuses the product kernel's helpers by including its source; the
// probe kernel is the product algorithm with switches:
//   MODE 0: load + reduce only (the HBM floor of this launch shape)
//   MODE 1: no selection, emit the first k features (load + emit)
//   MODE 2: full selection, no emit (lane 0 stores the threshold)
//   MODE 3: full selection, product emit (per-lane scattered stores)
//   MODE 4: full selection, emit staged through LDS (one coalesced store per table)
//   MODE 5: MODE 4 with the selection run phase by phase across the wave's R rows
//   MODE 6/7: MODE 4 in persistent waves (8 / 4 work-groups per CU), next rows prefetched
// R = rows per wave. Assumes D == 256 and k <= 64 (checked by the caller).
#include "../spgemm-gnn_amd/csrc/maxk_topk.hip"

namespace maxk {
void set_error(const std::string&) {}  // the product's error slot lives in capi.cpp
}  // namespace maxk

namespace {

template <int R, int MODE>
__global__ __launch_bounds__(256) void topk_probe(const float* __restrict__ in,
                                                  float* __restrict__ sp_data,
                                                  uint8_t* __restrict__ sp_index, int N, int k) {
  __shared__ __align__(16) uint32_t hist_all[4][256];
  __shared__ __align__(16) float stage_v[4][64];
  __shared__ __align__(16) uint8_t stage_i[4][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x / 64;
  const int row0 = (blockIdx.x * 4 + w) * R;
  if (row0 >= N) return;
  uint32_t* hist = hist_all[w];
  float xs[R][4];
  bool valid[4];
#pragma unroll
  for (int r = 0; r < R; ++r) load_row4(in, min(row0 + r, N - 1), 256, lane, xs[r], valid);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int row = row0 + r;
    if (row >= N) break;
    const float* x = xs[r];
    if constexpr (MODE == 0) {
      float s = x[0] + x[1] + x[2] + x[3];
      s = wave_max(s);
      if (lane == 0) sp_data[(size_t)row * k] = s;
      continue;
    }
    bool sel[4];
    uint32_t prefix = 0, pmask = 0;
    if constexpr (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i) sel[i] = lane * 4 + i < k;
    } else {
      uint32_t u[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) u[i] = order_key(x[i]);
      uint32_t need = (uint32_t)k;
      bool whole_bin = false;
      int first_shift = 24;
      {
        uint32_t m = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) m = max(m, u[i]);
        m = wave_umax(m);
        const int top = (int)(m >> 24);
        uint32_t left = need;
        for (int it = 0; it < kTopkWalk && top - it >= 0; ++it) {
          const uint32_t b = (uint32_t)(top - it);
          uint32_t cnt = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) cnt += (uint32_t)wave_count((u[i] >> 24) == b);
          if (cnt >= left) {
            prefix = b << 24;
            pmask = 0xff000000u;
            need = left;
            whole_bin = cnt == left;
            first_shift = 16;
            break;
          }
          left -= cnt;
        }
      }
#pragma unroll
      for (int shift = 24; shift >= 0; shift -= 8) {
        if (shift > first_shift || whole_bin) continue;
        reinterpret_cast<uint4*>(hist)[lane] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if ((u[i] & pmask) == prefix)
            __hip_atomic_fetch_add(&hist[(u[i] >> shift) & 255u], 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WAVEFRONT);
        const uint4 h = reinterpret_cast<const uint4*>(hist)[lane];
        const uint32_t lsum = h.x + h.y + h.z + h.w;
        const uint32_t pre = wave_prefix_sum(lsum);
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)pre, 63);
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
        bool gt[4], eq[4];
        uint64_t meq[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          gt[i] = u[i] > T;
          eq[i] = u[i] == T;
          meq[i] = __ballot(eq[i]);
        }
        int rank = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) rank += (int)lanes_below(meq[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sel[i] = gt[i] || (eq[i] && rank < (int)need);
          rank += eq[i] ? 1 : 0;
        }
      }
    }
    if constexpr (MODE == 2) {
      uint32_t any = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) any += sel[i] ? 1u : 0u;
      any = __popcll(__ballot(any != 0));
      if (lane == 0) sp_data[(size_t)row * k] = (float)(any + prefix);
    } else if constexpr (MODE == 4) {
      uint64_t m[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) m[i] = __ballot(sel[i]);
      int pos = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) pos += (int)lanes_below(m[i]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (sel[i]) {
          if (pos < k) {
            stage_v[w][pos] = x[i];
            stage_i[w][pos] = (uint8_t)(lane * 4 + i);
          }
          ++pos;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lane < k) sp_data[(size_t)row * k + lane] = stage_v[w][lane];
      if (lane < k / 4)
        reinterpret_cast<uint32_t*>(sp_index + (size_t)row * k)[lane] =
            reinterpret_cast<const uint32_t*>(stage_i[w])[lane];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
      emit_selected(x, sel, lane, row, k, sp_data, sp_index);
    }
  }
}

// MODE 5: the selection of the wave's R rows run phase by phase across the rows (walk for all
// rows, then each histogram pass for all rows still open), so the R dependent chains of LDS
// round trips and DPP scans overlap; emit staged through LDS.
template <int R>
__device__ __forceinline__ void topk_rows_batched(const float (&xs)[R][4], int row0, int N, int k,
                                                  int lane, uint32_t* hist /* [R][256] */,
                                                  float* stage_v /* [R][64] */,
                                                  uint8_t* stage_i /* [R][64] */,
                                                  float* __restrict__ sp_data,
                                                  uint8_t* __restrict__ sp_index) {
  uint32_t u[R][4];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) u[r][i] = order_key(xs[r][i]);
  uint32_t prefix[R], pmask[R], need[R];
  bool open[R];   // histogram passes still needed
  bool whole[R];  // selection = keys whose fixed high digits are >= prefix
  int top[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    uint32_t m = max(max(u[r][0], u[r][1]), max(u[r][2], u[r][3]));
    top[r] = (int)(wave_umax(m) >> 24);
    prefix[r] = 0; pmask[r] = 0; need[r] = (uint32_t)k; open[r] = true; whole[r] = false;
  }
  // top byte: walk bins top, top-1, ... (all rows each step, scalar selects)
  bool walked[R];
#pragma unroll
  for (int r = 0; r < R; ++r) walked[r] = false;
#pragma unroll
  for (int it = 0; it < kTopkWalk; ++it) {
    bool any = false;
#pragma unroll
    for (int r = 0; r < R; ++r) any |= !walked[r];
    if (!any) break;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t b = (uint32_t)(top[r] - it);
      uint32_t cnt = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) cnt += (uint32_t)wave_count((u[r][i] >> 24) == b);
      const bool take = !walked[r] && top[r] - it >= 0 && cnt >= need[r];
      if (take) {
        prefix[r] = b << 24;
        pmask[r] = 0xff000000u;
        whole[r] = cnt == need[r];
        open[r] = !whole[r];
      }
      if (!walked[r] && !take) need[r] -= (top[r] - it >= 0) ? cnt : 0u;
      walked[r] = walked[r] || take || top[r] - it < 0;
    }
  }
  // rows whose walk did not fix the top byte restart from the full count at shift 24
  bool from24[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    from24[r] = pmask[r] == 0;
    if (from24[r]) need[r] = (uint32_t)k;
  }
#pragma unroll
  for (int shift = 24; shift >= 0; shift -= 8) {
    bool act[R];
    bool any = false;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      act[r] = open[r] && (shift < 24 || from24[r]);
      any |= act[r];
    }
    if (!any) continue;
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (act[r]) reinterpret_cast<uint4*>(hist + r * 256)[lane] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (act[r] && (u[r][i] & pmask[r]) == prefix[r])
          __hip_atomic_fetch_add(&hist[r * 256 + ((u[r][i] >> shift) & 255u)], 1u,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    uint4 h[R];
#pragma unroll
    for (int r = 0; r < R; ++r) h[r] = reinterpret_cast<const uint4*>(hist + r * 256)[lane];
    uint32_t pre[R];
#pragma unroll
    for (int r = 0; r < R; ++r) pre[r] = wave_prefix_sum(h[r].x + h[r].y + h[r].z + h[r].w);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!act[r]) continue;
      const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)pre[r], 63);
      const uint32_t ge3 = total - pre[r] + h[r].w;
      const uint32_t ge2 = ge3 + h[r].z, ge1 = ge2 + h[r].y, ge0 = ge1 + h[r].x;
      const uint32_t nd = need[r];
      const uint64_t m = __ballot(ge0 >= nd);
      const int ls = 63 - __builtin_clzll(m);
      uint32_t d, above, inbin;
      if (ge3 >= nd) { d = 3; above = ge3 - h[r].w; inbin = h[r].w; }
      else if (ge2 >= nd) { d = 2; above = ge3; inbin = h[r].z; }
      else if (ge1 >= nd) { d = 1; above = ge2; inbin = h[r].y; }
      else { d = 0; above = ge1; inbin = h[r].x; }
      d = (uint32_t)__builtin_amdgcn_readlane((int)(4 * lane + d), ls);
      above = (uint32_t)__builtin_amdgcn_readlane((int)above, ls);
      inbin = (uint32_t)__builtin_amdgcn_readlane((int)inbin, ls);
      need[r] = nd - above;
      prefix[r] |= d << shift;
      pmask[r] |= 255u << shift;
      if (inbin == need[r]) { whole[r] = true; open[r] = false; }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    bool sel[4];
    if (whole[r]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) sel[i] = (u[r][i] & pmask[r]) >= prefix[r];
    } else {
      const uint32_t T = prefix[r];
      uint64_t meq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) meq[i] = __ballot(u[r][i] == T);
      int rank = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) rank += (int)lanes_below(meq[i]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool eq = u[r][i] == T;
        sel[i] = u[r][i] > T || (eq && rank < (int)need[r]);
        rank += eq ? 1 : 0;
      }
    }
    uint64_t m[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) m[i] = __ballot(sel[i]);
    int pos = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) pos += (int)lanes_below(m[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (sel[i]) {
        if (pos < k) {
          stage_v[r * 64 + pos] = xs[r][i];
          stage_i[r * 64 + pos] = (uint8_t)(lane * 4 + i);
        }
        ++pos;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int row = row0 + r;
    if (row >= N) break;
    if (lane < k) sp_data[(size_t)row * k + lane] = stage_v[r * 64 + lane];
    if (lane < k / 4)
      reinterpret_cast<uint32_t*>(sp_index + (size_t)row * k)[lane] =
          reinterpret_cast<const uint32_t*>(stage_i + r * 64)[lane];
  }
}

template <int R>
__global__ __launch_bounds__(256) void topk_probe_batched(const float* __restrict__ in,
                                                          float* __restrict__ sp_data,
                                                          uint8_t* __restrict__ sp_index, int N,
                                                          int k) {
  __shared__ __align__(16) uint32_t hist_all[4][R * 256];
  __shared__ __align__(16) float stage_v[4][R * 64];
  __shared__ __align__(16) uint8_t stage_i[4][R * 64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x / 64;
  const int row0 = (blockIdx.x * 4 + w) * R;
  if (row0 >= N) return;
  float xs[R][4];
  bool valid[4];
#pragma unroll
  for (int r = 0; r < R; ++r) load_row4(in, min(row0 + r, N - 1), 256, lane, xs[r], valid);
  topk_rows_batched<R>(xs, row0, N, k, lane, hist_all[w], stage_v[w], stage_i[w], sp_data,
                       sp_index);
}

// MODE 6/7: persistent waves (8 / 4 work-groups per CU) that load the next batch of R rows
// into registers before selecting the current one, so each wave overlaps its own loads with
// its selection (mode 4's select + LDS-staged emit).
template <int R>
__device__ __forceinline__ void select_emit_row(const float (&x)[4], int row, int k, int lane,
                                                uint32_t* hist, float* stage_v, uint8_t* stage_i,
                                                float* __restrict__ sp_data,
                                                uint8_t* __restrict__ sp_index) {
  uint32_t u[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) u[i] = order_key(x[i]);
  uint32_t prefix = 0, pmask = 0, need = (uint32_t)k;
  bool whole_bin = false;
  int first_shift = 24;
  {
    uint32_t m = max(max(u[0], u[1]), max(u[2], u[3]));
    m = wave_umax(m);
    const int top = (int)(m >> 24);
    uint32_t left = need;
    for (int it = 0; it < kTopkWalk && top - it >= 0; ++it) {
      const uint32_t b = (uint32_t)(top - it);
      uint32_t cnt = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) cnt += (uint32_t)wave_count((u[i] >> 24) == b);
      if (cnt >= left) {
        prefix = b << 24; pmask = 0xff000000u; need = left; whole_bin = cnt == left;
        first_shift = 16;
        break;
      }
      left -= cnt;
    }
  }
#pragma unroll
  for (int shift = 24; shift >= 0; shift -= 8) {
    if (shift > first_shift || whole_bin) continue;
    reinterpret_cast<uint4*>(hist)[lane] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if ((u[i] & pmask) == prefix)
        __hip_atomic_fetch_add(&hist[(u[i] >> shift) & 255u], 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WAVEFRONT);
    const uint4 h = reinterpret_cast<const uint4*>(hist)[lane];
    const uint32_t pre = wave_prefix_sum(h.x + h.y + h.z + h.w);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)pre, 63);
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
    if (inbin == need) { whole_bin = true; break; }
  }
  bool sel[4];
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
  uint64_t mm[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) mm[i] = __ballot(sel[i]);
  int pos = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) pos += (int)lanes_below(mm[i]);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (sel[i]) {
      if (pos < k) { stage_v[pos] = x[i]; stage_i[pos] = (uint8_t)(lane * 4 + i); }
      ++pos;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane < k) sp_data[(size_t)row * k + lane] = stage_v[lane];
  if (lane < k / 4)
    reinterpret_cast<uint32_t*>(sp_index + (size_t)row * k)[lane] =
        reinterpret_cast<const uint32_t*>(stage_i)[lane];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int R>
__global__ __launch_bounds__(256) void topk_probe_persistent(const float* __restrict__ in,
                                                             float* __restrict__ sp_data,
                                                             uint8_t* __restrict__ sp_index,
                                                             int N, int k) {
  __shared__ __align__(16) uint32_t hist_all[4][256];
  __shared__ __align__(16) float stage_v[4][64];
  __shared__ __align__(16) uint8_t stage_i[4][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x / 64;
  const int nb = (N + R - 1) / R;
  const int stride = gridDim.x * 4;
  int b = blockIdx.x * 4 + w;
  if (b >= nb) return;
  float cur[R][4], nxt[R][4];
  bool valid[4];
#pragma unroll
  for (int r = 0; r < R; ++r) load_row4(in, min(b * R + r, N - 1), 256, lane, cur[r], valid);
  for (; b < nb; b += stride) {
    const int bn = b + stride;
    if (bn < nb) {
#pragma unroll
      for (int r = 0; r < R; ++r) load_row4(in, min(bn * R + r, N - 1), 256, lane, nxt[r], valid);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = b * R + r;
      if (row >= N) break;
      select_emit_row<R>(cur[r], row, k, lane, hist_all[w], stage_v[w], stage_i[w], sp_data,
                         sp_index);
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) cur[r][i] = nxt[r][i];
  }
}

template <int R>
void launch(int mode, const float* in, float* d, uint8_t* i, int N, int k, hipStream_t s) {
  const int grid = (N + 4 * R - 1) / (4 * R);
  switch (mode) {
    case 0: hipLaunchKernelGGL((topk_probe<R, 0>), dim3(grid), dim3(256), 0, s, in, d, i, N, k); break;
    case 1: hipLaunchKernelGGL((topk_probe<R, 1>), dim3(grid), dim3(256), 0, s, in, d, i, N, k); break;
    case 2: hipLaunchKernelGGL((topk_probe<R, 2>), dim3(grid), dim3(256), 0, s, in, d, i, N, k); break;
    case 3: hipLaunchKernelGGL((topk_probe<R, 3>), dim3(grid), dim3(256), 0, s, in, d, i, N, k); break;
    case 4: hipLaunchKernelGGL((topk_probe<R, 4>), dim3(grid), dim3(256), 0, s, in, d, i, N, k); break;
    case 5: hipLaunchKernelGGL((topk_probe_batched<R>), dim3(grid), dim3(256), 0, s, in, d, i, N, k); break;
    default: {
      int dev = 0, cus = 0;
      hipGetDevice(&dev);
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      const int g = std::min(grid, cus * (mode == 6 ? 8 : 4));
      hipLaunchKernelGGL((topk_probe_persistent<R>), dim3(g), dim3(256), 0, s, in, d, i, N, k);
    }
  }
}

}  // namespace

// Mean ms per launch over `reps` launches after 3 warm-ups; < 0 on a bad argument.
extern "C" float probe_topk(int mode, int R, const float* in, float* sp_data, uint8_t* sp_index,
                            int N, int k, int reps) {
  if (N <= 0 || k < 4 || k > 64 || (k & 3) || mode < 0 || mode > 7 || reps <= 0) return -1.f;
  auto run = [&]() {
    switch (R) {
      case 1: launch<1>(mode, in, sp_data, sp_index, N, k, nullptr); break;
      case 2: launch<2>(mode, in, sp_data, sp_index, N, k, nullptr); break;
      case 8: launch<8>(mode, in, sp_data, sp_index, N, k, nullptr); break;
      default: launch<4>(mode, in, sp_data, sp_index, N, k, nullptr); break;
    }
  };
  for (int i = 0; i < 3; ++i) run();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, nullptr);
  for (int i = 0; i < reps; ++i) run();
  hipEventRecord(b, nullptr);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return hipGetLastError() == hipSuccess ? ms / reps : -2.f;
}
