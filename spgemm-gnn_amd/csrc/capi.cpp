// C ABI housekeeping: version, thread-local error text, .warp4 compatibility export.
#include <string>

#include "common.h"

namespace maxk {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace maxk

extern "C" int maxk_abi_version(void) { return MAXK_ABI_VERSION; }

extern "C" const char* maxk_last_error(void) { return maxk::g_last_error.c_str(); }

// Reference chunk rule (path "../w12_nz64_warp_4/<name>.warp4" at
// SO@0x292ad-0x292c1, consumed by SPMM_MAXK::do_test SO@0x24d16-0x24f32): every CSR row is
// cut into consecutive chunks of <= max_nz (64) nonzeros, one int4 {row, first_nz, len, 0}
// per chunk, rows in order, no header. Empty rows produce no chunk.
extern "C" int maxk_warp4_build(const int32_t* host_ptr, int32_t num_nodes, int32_t max_nz,
                                int32_t* out, int64_t out_capacity_chunks,
                                int64_t* num_chunks) {
  MAXK_CHECK_ARG(host_ptr != nullptr && num_chunks != nullptr, "maxk_warp4_build: null pointer");
  MAXK_CHECK_ARG(num_nodes >= 0 && max_nz >= 1, "maxk_warp4_build: bad size");
  int64_t n = 0;
  for (int32_t r = 0; r < num_nodes; ++r) {
    const int64_t b = host_ptr[r], e = host_ptr[r + 1];
    MAXK_CHECK_ARG(e >= b, "maxk_warp4_build: ptr must be non-decreasing");
    for (int64_t s = b; s < e; s += max_nz) {
      if (out) {
        MAXK_CHECK_ARG(n < out_capacity_chunks, "maxk_warp4_build: output too small");
        int32_t* q = out + 4 * n;
        q[0] = r;
        q[1] = (int32_t)s;
        q[2] = (int32_t)((e - s) < max_nz ? (e - s) : max_nz);
        q[3] = 0;
      }
      ++n;
    }
  }
  *num_chunks = n;
  return MAXK_OK;
}
