/*
 * maxk_baseline.h — comparator entry points (libmaxk_baseline.so), not on the MaxK path.
 *
 * Replaces the reference's cuSPARSE baselines spmm_cusparse (maxk_kernels.so SO@0x243a0,
 * SURVEY §8(a) a10) and spmm_cusparse_coo (SO@0x24700): Y = 1 * A * X + 0 * Y, A CSR (int32 row pointers and columns, base 0,
 * f32 values), X and Y dense row-major [n, d], rocsparse_spmm with the given algorithm, one
 * warm-up call then `times` timed calls on `stream`. Kept in its own library so the product
 * library (libmaxk_hip.so) does not link rocSPARSE.
 */
#ifndef MAXK_BASELINE_H
#define MAXK_BASELINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Message of the last failed call on this thread. */
const char* maxk_baseline_last_error(void);

/* alg: rocsparse_spmm_alg value (0 = default). *ms = mean time of one timed call (or of the
 * warm-up when times == 0). Returns 0 on success, -1 bad argument, -4 rocSPARSE/HIP error. */
int maxk_spmm_rocsparse(const int32_t* ptr, const int32_t* idx, const float* val,
                        const float* x, float* y, int32_t n, int64_t nnz, int32_t d,
                        int32_t alg, int32_t times, float* ms, void* stream);

/* The same with A in COO form (row[i], col[i], val[i], i < nnz; rows ascending, as a CSR's
 * expanded row ids), replacing the reference's spmm_cusparse_coo (SO@0x24700). alg: 0
 * default, 2 segmented, 3 atomic, 6 segmented + atomics. */
int maxk_spmm_rocsparse_coo(const int32_t* row, const int32_t* col, const float* val,
                            const float* x, float* y, int32_t n, int64_t nnz, int32_t d,
                            int32_t alg, int32_t times, float* ms, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MAXK_BASELINE_H */
