// Shared helpers for the gfx950 MaxK kernels and the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "maxk_hip.h"

namespace maxk {

constexpr int kWave = 64;               // CDNA wavefront width (never 32)
constexpr int kFwdTileRows = 32;        // default destination rows per forward work-group
constexpr int kFwdMaxTileRows = 64;
// forward LDS accumulator row stride D + kFwdRowPad elements: rows start on different banks,
// so lanes of different edges with nearby selectors (sorted CBSR slots) spread over banks
// (Reddit: k = 16 1.354 -> 1.341 ms, k = 32 2.500 -> 2.470, k = 8 0.898 -> 0.905)
constexpr int kFwdRowPad = 1;
// forward edge word: source column in the low kFwdColBits bits, row within the tile above
constexpr int kFwdColBits = 26;
constexpr uint32_t kFwdColMask = (1u << kFwdColBits) - 1;
constexpr int kFwdThreads = 256;        // 4 waves per forward work-group
constexpr int kBwdThreads = 512;        // 8 waves per backward work-group (12 at k >= 32)
constexpr int kMaxDim = 256;            // u8 selectors => D <= 256
constexpr int kFwdUnroll = 8;           // independent sub-steps in flight per wave
constexpr int kFwdFlagChunk3 = 1;       // forward kernel flags (template FL): lane-chunk records
constexpr int kFwdFlagQuad = 2;         // quad-shared edge-word loads
constexpr int kFwdFlagChunk2 = 4;       // pair-chunk records: 2 values + their selectors per 16 B
constexpr int kBwdTasksPerCu = 2;
constexpr int kBwdMinTaskEdges = 100000;  // a chunk's flush (C*k stores) vs its edges
constexpr int kXcds = 8;
constexpr int kFwdRotWindows = 16;         // column windows of the rotated forward sweep
constexpr double kFwdSlotEdgeRate = 1.6e8;  // edges/s one forward slot sustains at k = 16
constexpr double kFwdSlotEdgeRateFixed = 3.0e8;  // the same with the fixed-point update
// (round 4: 2.6e8 -> 3.0e8 with the 1.5 x task cap, Reddit k = 16 / 32 / 64 -1.0 / -0.2 / -0.3 %;
// 3.5e8 and above slower, profiles/r04/fwd_rot_rate_ab.jsonl)
// CBSR tables (5k bytes per column) above these sizes get packed one-line forward records
// even where two tables would otherwise be used (plan.hip: k >= 32 / k < 32)
constexpr double kFwdPackedTableBytes = 150e6;
constexpr double kFwdPackedTableBytes16 = 32e6;
// k < 32: below kFwdPackMinEdgesPerCol edges per column the forward gathers from the two API
// tables instead of packing one record per column per call; below kFwdPackMinEdgesPerColL2
// too while the selector table (k bytes per column) stays L2-resident, where the second
// (selector) touch of an edge is cheap (plan.hip)
constexpr long long kFwdPackMinEdgesPerCol = 40;
constexpr long long kFwdPackMinEdgesPerColL2 = 128;
constexpr double kFwdSelL2Bytes = 3e6;
// two-pass backward below this many expected edges per (row, column block), i.e. when a
// column block sees each grad_out row it fetches about once. Measured (blocks vs two-pass,
// ms): ogbn-products k = 16 (0.04) 13.4 / 6.0, k = 32 (0.02) 16.0 / 8.3; yelp k = 64 (0.015)
// 1.98 / 1.81; flickr k = 8 (0.50) 0.25 / 0.06; Reddit k = 64 (0.96) 4.86 / 15.2, k = 16 (3.8)
// 1.70 / 5.35; ogbn-proteins k = 8 (15) 0.94 / 2.68
constexpr double kBwdTwoPassReuse = 0.75;
constexpr int kBwdRowsPerWave = 4;  // row pass: most destination rows one wavefront stages
// two-pass backward: the E x k product workspace is cut into row chunks of at most this many
// bytes (one row pass + one column pass per chunk; bwd_tp_chunks overrides)
// (ogbn-products k = 32, 15.8 GB in one chunk: 1 / 2 / 4 / 8 chunks ran 8.11 / 8.68 / 10.49 /
// 14.60 ms; every chunk's column pass visits every column)
constexpr double kBwdTwoPassWorkspaceCap = 16.0 * (1ull << 30);
// work-groups per CU of the fused CBSR pack + statistics pass (each adds one atomic per
// statistics word, and same-address atomics serialise at the L2). Reddit, pack+stats at
// k = 16 / stats at k = 32, 64: 1 -> 24.5 / 54.5 us, 4 -> 20.8 / 26.6 us, 8 -> 31.5 / 33.7 us
// (the separate pack + stats passes took 21 + 17 us at k = 16)
constexpr int kStatsBlocksPerCu = 4;
// Records past the end of the backward edge list that a wave may read (and ignore): one
// iteration of a wave covers at most 16 sub-steps x 64 edges.
constexpr int kBwdRecPad = 16 * kWave + kWave;
constexpr int kBwdLdsBudget = 160 * 1024; // all of a CU's LDS: one work-group per CU

// Thread-local error message plumbing for maxk_last_error().
void set_error(const std::string& msg);

#define MAXK_CHECK_ARG(cond, msg)                 \
  do {                                            \
    if (!(cond)) {                                \
      ::maxk::set_error(msg);                     \
      return MAXK_ERR_INVALID_ARG;                \
    }                                             \
  } while (0)

#define MAXK_HIP_TRY(expr)                                                      \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) {                                                     \
      ::maxk::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));     \
      return (int)_e;                                                           \
    }                                                                           \
  } while (0)

#define MAXK_LAUNCH_CHECK(what)                                                 \
  do {                                                                          \
    hipError_t _e = hipGetLastError();                                          \
    if (_e != hipSuccess) {                                                     \
      ::maxk::set_error(std::string(what) + ": " + hipGetErrorString(_e));      \
      return (int)_e;                                                           \
    }                                                                           \
  } while (0)

// Forward work item: a run of whole destination rows [row0, row0+nrows) (or, nrows < 0, one
// segment of a long row whose partial sum is added atomically into a row pre-zeroed by
// zero_rows), with edge range [e0, e1) of the plan's permuted edge order (the task's CSR
// edges sorted by column).
struct FwdTask {
  int32_t row0;
  int32_t nrows;
  int32_t e0;
  int32_t e1;
};
static_assert(sizeof(FwdTask) == 16, "FwdTask is loaded as one dwordx4");

// Packed CBSR record size for k (k % 4 == 0): k f32 values + k u8 selectors, rounded to
// 64 B when that fits one 64-B sector, to one 128-B line when it fits one, else to 16 B
// (k = 32: 160-B records ran 2.73 ms against 3.24 ms for 256-B ones on Reddit).
inline int cbsr_record_bytes(int k) {
  const int b = 5 * k;
  return b <= 64 ? 64 : b <= 128 ? 128 : (b + 15) / 16 * 16;
}

// Backward work item: edges [e0, e1) of the column-block-major, row-sorted edge list, all
// with source column in [col0, col0 + ncols). shared != 0: the block is split over several
// work-groups, so its LDS accumulator is flushed with float atomics into a pre-zeroed
// grad_sp; otherwise it is stored.
struct BwdTask {
  int32_t col0;
  int32_t ncols;
  int32_t e0;
  int32_t e1;
  int32_t shared;
  int32_t group;  // selector slot group (packed path): slots [group * k/S, (group+1) * k/S)
  int32_t chunk;  // piece index within its block (0 .. pieces - 1)
  int32_t slab;   // slab flush: float offset of this piece's [C][k] slab region; -1: piece
                  // 0 (stores straight into grad_sp)
};
static_assert(sizeof(BwdTask) == 32, "BwdTask is 2 x dwordx4");


__device__ __forceinline__ void lds_add(double* p, double v) {
  // ds_add_f64 (no return).
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void global_add(float* p, float v) {
  // One global_atomic_add_f32 (no CAS loop on gfx950).
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace maxk

// Opaque plan (definition shared by plan.hip and the kernels' launchers).
struct maxk_plan {
  int32_t num_nodes = 0;   // destination rows
  int32_t num_cols = 0;    // source columns (rows of the CBSR tables / grad_sp)
  int64_t num_edges = 0;
  int32_t dim_origin = 0;
  int32_t dim_k = 0;
  const int32_t* src_ptr = nullptr;  // identity of the graph the plan was built for
  const int32_t* src_idx = nullptr;
  int32_t cus = 256;             // compute units of the device the plan was built on
  // ---- forward: tiles of whole rows (FwdTask), edges column-sorted per tile
  int32_t fwd_tile_rows = 32;
  int32_t fwd_waves = 4;        // wavefronts per forward work-group (4 or 8)
  int32_t fwd_unroll = 8;       // forward sub-steps in flight per wave (4 only with 8 waves)
  int32_t fwd_rec_bytes = 0;     // packed CBSR record size (per-call pack)
  uint8_t* fwd_rec = nullptr;    // [num_cols][fwd_rec_bytes] plan-owned workspace
  // fixed-point forward (LdsFix): per task {sexp, gexp} (fwd_fix_stats_kernel); the call's
  // {max |x|, min |x|} words live at fwd_xstat_off of the forward workspace
  int32_t fwd_fixed = 0;
  int2* fwd_fix = nullptr;
  int32_t* fwd_rowptr = nullptr;  // plan copy of ptr for the bounds' row sums
  int64_t fwd_xstat_off = 0;
  maxk::FwdTask* fwd_tasks = nullptr;   // e0/e1 index the permuted edge order below
  int32_t fwd_phases = 1;        // column windows of the rotated sweep (1: no rotation)
  int32_t fwd_rot_ticks = 0;     // > 0: rotated sweeps, s_memrealtime ticks per window
  int32_t fwd_chunk3 = 0;        // lane-chunk records: 3 values + their selectors per 16 B
  int32_t fwd_chunk2 = 0;        // pair-chunk records: 2 values + their selectors per 16 B
  int32_t fwd_quad = 0;          // quad-shared edge-word loads
  int32_t fwd_two_tables = 0;    // gather from sp_data / sp_index directly (no pack)
  int32_t* fwd_phase_off = nullptr;  // [tasks][phases + 1] edge offsets per window
  int32_t* fwd_perm = nullptr;   // CSR edge id of each permuted forward edge
  uint2* fwd_cv = nullptr;       // {column | (row within the task << kFwdColBits), val bits}
  int32_t n_fwd_tasks = 0;
  int32_t* zero_rows = nullptr;  // rows written by split tasks (atomic), zeroed first
  int32_t n_zero_rows = 0;
  // ---- backward, column blocks (sspmm_bwd4_kernel): one 12-B record per reordered edge
  // {row * D * 4 (or the row index when grad_out exceeds 4 GiB), column within its block,
  // val}; F selector slots per lane, S slot groups, k padded to bwd_kp (a multiple of F * S;
  // the padding slots gather feature 0 into accumulators that are never stored)
  int32_t bwd_feats = 4;         // F: 4 or 2
  int32_t bwd_slot_groups = 1;   // S
  int32_t bwd_kp = 0;            // padded slots per column
  int32_t bwd_ks = 0;            // accumulator floats per column and group (= bwd_kp / S)
  int32_t bwd_unroll = 8;
  int32_t bwd_waves = 8;
  int32_t bwd_big = 0;           // grad_out > 4 GiB: 64-bit row addressing
  int32_t bwd_block_cols = 0;
  int32_t n_bwd_blocks = 0;
  maxk::BwdTask* bwd_tasks = nullptr;
  int32_t n_bwd_tasks = 0;
  int32_t n_bwd_shared = 0;
  int32_t* bwd_perm = nullptr;   // CSR edge id of each reordered edge
  uint32_t* bwd_rec = nullptr;   // [num_edges + kBwdRecPad][3]
  uint32_t* bwd_sel = nullptr;   // plan-owned workspace: the slabs (bwd_slab_floats)
  // two-pass backward (low row reuse): a row pass writes each edge's k products val *
  // grad_out[r, sel(c)] into the edge's slot of bwd_tbuf (CSR order), a column pass sums the
  // slots of each column's in-edges (bwd_perm, bwd_colptr)
  int32_t bwd_twopass = 0;
  int32_t bwd_tp_rows = 1;       // R: destination rows per wavefront of the row pass
  uint32_t* bwd_erec = nullptr;  // [num_edges][2] CSR order: {column | (row % R) << 26, val}
  float* bwd_tbuf = nullptr;     // [max chunk edges][k] plan-owned workspace
  int32_t* bwd_colptr = nullptr; // [num_cols + 1] offsets of the column-sorted edges
  // row chunks of the two-pass backward (workspace bounded by kBwdTwoPassWorkspaceCap):
  // chunk p covers destination rows [tp_rows[p], tp_rows[p+1]) = CSR edges [tp_edges[p],
  // tp_edges[p+1]); bwd_colptr2[p * NC + c] = first column-sorted position of column c whose
  // row is >= tp_rows[p] (rows ascend within a column), p = 0 .. P (P = 1: bwd_colptr)
  int32_t bwd_tp_chunks = 1;
  std::vector<int32_t> tp_rows;
  std::vector<int64_t> tp_edges;
  int32_t* bwd_colptr2 = nullptr;
  // column order of the column blocks (maxk_plan_options.col_order): bwd_corder[p] = the
  // source column placed at position p of the blocks (nullptr: identity)
  int32_t col_order = 1;
  int32_t* bwd_corder = nullptr;
  // slab flush of split blocks: piece 0 of a block stores into grad_sp, piece p > 0 into its
  // [C][k] slab region (bwd_slab_floats f32 in all, at byte bwd_slab_off of the backward
  // workspace, behind the selector words); bwd_combine_kernel adds each block's regions in
  // piece order. bwd_combine: one int4 {slab offset, regions, col0, ncols} per block with
  // more than one piece. bwd_slab_floats == 0 with split blocks: global float atomics
  int64_t bwd_slab_floats = 0;
  int64_t bwd_slab_off = 0;
  int4* bwd_combine = nullptr;
  int32_t n_bwd_combine = 0;
  int64_t device_bytes = 0;
  // per-call scratch: the forward's packed CBSR records and statistics words, the backward's
  // selector words + flush slabs or two-pass product workspace. external_ws: the plan
  // allocates none of them and the *_ws entry points take the caller's buffer
  int32_t external_ws = 0;
  int64_t fwd_ws_bytes = 0;
  int64_t bwd_ws_bytes = 0;
  int32_t bwd_row_order = 1;     // rows in the block streams: 1 ascending, 2 scattered
  // windows of the forward / column-block backward waves: 1 static interleave, 2 handed out
  // by a per-work-group LDS counter (maxk_plan_options.fwd_handout / bwd_handout)
  int32_t fwd_handout = 1;
  int32_t bwd_handout = 1;
};
