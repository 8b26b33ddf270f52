// rocSPARSE sparse x dense SpMM comparators (config 2's "vs rocSPARSE SpMM"): the MI355X
// counterparts of the reference's cuSPARSE baselines spmm_cusparse (CSR, SO@0x243a0) and
// spmm_cusparse_coo (COO, SO@0x24700): Y = 1 * A * X + 0 * Y with A
// int32 indices/base 0/f32, X and Y row-major, one warm-up call and `times` timed calls. Built into its own library
// (maxk_kernels/libmaxk_baseline.so) so the product library does not link rocSPARSE.
#include <hip/hip_runtime.h>
#include <rocsparse/rocsparse.h>

#include "maxk_baseline.h"

#include <cstdint>
#include <string>

namespace {
thread_local std::string g_err;

#define RS_TRY(x)                                                                       \
  do {                                                                                  \
    rocsparse_status s_ = (x);                                                          \
    if (s_ != rocsparse_status_success) {                                               \
      g_err = std::string(#x) + " -> rocsparse status " + std::to_string((int)s_);      \
      rc = -4;                                                                          \
      goto done;                                                                        \
    }                                                                                   \
  } while (0)
#define HIP_TRY(x)                                                                      \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      g_err = std::string(#x) + " -> " + hipGetErrorString(e_);                          \
      rc = -4;                                                                          \
      goto done;                                                                        \
    }                                                                                   \
  } while (0)
}  // namespace

extern "C" const char* maxk_baseline_last_error() { return g_err.c_str(); }

// Times rocsparse_spmm on the matrix descriptor a: Y = 1 * A * X + 0 * Y, X and Y row-major
// [n, d]; one warm-up call and `times` timed calls, *ms = the mean of one timed call (or the
// warm-up's time when times == 0). Takes ownership of a.
static int time_spmm(rocsparse_handle h, rocsparse_spmat_descr a, const float* x, float* y,
                     int32_t n, int32_t d, int32_t alg, int32_t times, float* ms,
                     void* stream) {
  int rc = 0;
  rocsparse_dnmat_descr b = nullptr, c = nullptr;
  void* buf = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  size_t bytes = 0;
  const float alpha = 1.f, beta = 0.f;
  const auto A = rocsparse_operation_none;
  const auto al = (rocsparse_spmm_alg)alg;
  float t = 0.f;
  RS_TRY(rocsparse_create_dnmat_descr(&b, n, d, d, const_cast<float*>(x),
                                      rocsparse_datatype_f32_r, rocsparse_order_row));
  RS_TRY(rocsparse_create_dnmat_descr(&c, n, d, d, y, rocsparse_datatype_f32_r,
                                      rocsparse_order_row));
  RS_TRY(rocsparse_spmm(h, A, A, &alpha, a, b, &beta, c, rocsparse_datatype_f32_r, al,
                        rocsparse_spmm_stage_buffer_size, &bytes, nullptr));
  if (bytes) HIP_TRY(hipMalloc(&buf, bytes));
  RS_TRY(rocsparse_spmm(h, A, A, &alpha, a, b, &beta, c, rocsparse_datatype_f32_r, al,
                        rocsparse_spmm_stage_preprocess, &bytes, buf));
  HIP_TRY(hipEventCreate(&e0));
  HIP_TRY(hipEventCreate(&e1));
  HIP_TRY(hipEventRecord(e0, (hipStream_t)stream));
  RS_TRY(rocsparse_spmm(h, A, A, &alpha, a, b, &beta, c, rocsparse_datatype_f32_r, al,
                        rocsparse_spmm_stage_compute, &bytes, buf));  // warm-up
  HIP_TRY(hipEventRecord(e1, (hipStream_t)stream));
  if (times > 0) {
    HIP_TRY(hipEventSynchronize(e1));
    HIP_TRY(hipEventRecord(e0, (hipStream_t)stream));
    for (int i = 0; i < times; ++i)
      RS_TRY(rocsparse_spmm(h, A, A, &alpha, a, b, &beta, c, rocsparse_datatype_f32_r, al,
                            rocsparse_spmm_stage_compute, &bytes, buf));
    HIP_TRY(hipEventRecord(e1, (hipStream_t)stream));
  }
  HIP_TRY(hipEventSynchronize(e1));
  HIP_TRY(hipEventElapsedTime(&t, e0, e1));
  *ms = times > 0 ? t / times : t;
done:
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (buf) (void)hipFree(buf);
  if (c) rocsparse_destroy_dnmat_descr(c);
  if (b) rocsparse_destroy_dnmat_descr(b);
  rocsparse_destroy_spmat_descr(a);
  return rc;
}

static bool bad_args(int32_t n, int64_t nnz, int32_t d, int32_t times, float* ms,
                     const char* who) {
  if (n < 0 || nnz < 0 || d < 1 || times < 0 || !ms) {
    g_err = std::string(who) + ": bad argument";
    return true;
  }
  return false;
}

extern "C" int maxk_spmm_rocsparse(const int32_t* ptr, const int32_t* idx, const float* val,
                                   const float* x, float* y, int32_t n, int64_t nnz, int32_t d,
                                   int32_t alg, int32_t times, float* ms, void* stream) {
  if (bad_args(n, nnz, d, times, ms, "maxk_spmm_rocsparse")) return -1;
  int rc = 0;
  rocsparse_handle h = nullptr;
  rocsparse_spmat_descr a = nullptr;
  RS_TRY(rocsparse_create_handle(&h));
  RS_TRY(rocsparse_set_stream(h, (hipStream_t)stream));
  RS_TRY(rocsparse_create_csr_descr(&a, n, n, nnz, const_cast<int32_t*>(ptr),
                                    const_cast<int32_t*>(idx), const_cast<float*>(val),
                                    rocsparse_indextype_i32, rocsparse_indextype_i32,
                                    rocsparse_index_base_zero, rocsparse_datatype_f32_r));
  rc = time_spmm(h, a, x, y, n, d, alg, times, ms, stream);
done:
  if (h) rocsparse_destroy_handle(h);
  return rc;
}

extern "C" int maxk_spmm_rocsparse_coo(const int32_t* row, const int32_t* col, const float* val,
                                       const float* x, float* y, int32_t n, int64_t nnz,
                                       int32_t d, int32_t alg, int32_t times, float* ms,
                                       void* stream) {
  if (bad_args(n, nnz, d, times, ms, "maxk_spmm_rocsparse_coo")) return -1;
  int rc = 0;
  rocsparse_handle h = nullptr;
  rocsparse_spmat_descr a = nullptr;
  RS_TRY(rocsparse_create_handle(&h));
  RS_TRY(rocsparse_set_stream(h, (hipStream_t)stream));
  RS_TRY(rocsparse_create_coo_descr(&a, n, n, nnz, const_cast<int32_t*>(row),
                                    const_cast<int32_t*>(col), const_cast<float*>(val),
                                    rocsparse_indextype_i32, rocsparse_index_base_zero,
                                    rocsparse_datatype_f32_r));
  rc = time_spmm(h, a, x, y, n, d, alg, times, ms, stream);
done:
  if (h) rocsparse_destroy_handle(h);
  return rc;
}
