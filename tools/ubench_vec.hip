// Micro-benchmark (tooling, not product): cost of one wave64 gather instruction by load width
// and lanes per record, to choose CBSR record layouts. Every "edge" is a random 128-B-aligned
// record of the table; the LPE lanes of an edge read consecutive BYTES-wide pieces of it
// (starting at byte OFF of the record), idle lanes (64 % LPE) repeat lane 0's piece.
// Timed with events; ns per instruction per CU and per edge.
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int ITERS = 512;

template <int BYTES>
struct Piece;
template <> struct Piece<4> { typedef uint32_t T; };
template <> struct Piece<8> { typedef uint2 T; };
template <> struct Piece<12> { typedef uint3 T; };
template <> struct Piece<16> { typedef uint4 T; };

__device__ __forceinline__ uint32_t fold(uint32_t x) { return x; }
__device__ __forceinline__ uint32_t fold(uint2 x) { return x.x ^ x.y; }
__device__ __forceinline__ uint32_t fold(uint3 x) { return x.x ^ x.y ^ x.z; }
__device__ __forceinline__ uint32_t fold(uint4 x) { return x.x ^ x.y ^ x.z ^ x.w; }

template <int BYTES, int LPE, int OFF>
__global__ __launch_bounds__(256) void vec_kern(const uint8_t* __restrict__ table, int nrec,
                                                uint32_t* __restrict__ out) {
  typedef typename Piece<BYTES>::T P;
  const int lane = threadIdx.x & 63;
  const int EPI = 64 / LPE;
  const int slot = lane / LPE < EPI ? lane / LPE : 0;
  const int j = lane / LPE < EPI ? lane - (lane / LPE) * LPE : 0;
  const uint32_t wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  uint32_t s = (wid * 64 + slot) * 2654435761u + 12345u;
  uint32_t acc = 0;
#pragma unroll 8
  for (int it = 0; it < ITERS; ++it) {
    s = s * 1664525u + 1013904223u;
    const uint32_t rec = __umulhi(s, (uint32_t)nrec);
    const P v = *reinterpret_cast<const P*>(table + (size_t)rec * 128 + OFF + j * BYTES);
    acc ^= fold(v);
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

extern "C" float ubench_vec(int pattern, const uint8_t* table, int nrec, uint32_t* out, int nwg,
                            int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto launch = [&]() {
    switch (pattern) {
#define CASE(n, by, lpe, off) \
  case n: hipLaunchKernelGGL((vec_kern<by, lpe, off>), nwg, 256, 0, 0, table, nrec, out); break;
      CASE(0, 16, 4, 0)    // packed k=16 values: 64 B of the record, 16 edges
      CASE(1, 4, 4, 64)    // packed k=16 selectors: 16 B at +64, 16 edges
      CASE(2, 16, 6, 0)    // lane chunks k=16: 96 B, 10 edges
      CASE(3, 16, 8, 0)    // 128 B per edge (k=32 values), 8 edges
      CASE(4, 16, 5, 0)    // 80 B per edge (values + selectors, 5 lanes), 12 edges
      CASE(5, 12, 8, 0)    // 96 B as 8 x 12 B, 8 edges
      CASE(6, 16, 2, 0)    // 32 B per edge, 32 edges
      CASE(7, 16, 1, 0)    // 16 B per edge, 64 edges
      CASE(8, 4, 1, 0)     // 4 B per edge, 64 edges
      CASE(9, 4, 16, 0)    // 64 B as 16 x 4 B, 4 edges
      CASE(10, 8, 4, 0)    // 32 B as 4 x 8 B, 16 edges
      CASE(11, 4, 4, 0)    // 16 B as 4 x 4 B, 16 edges
#undef CASE
    }
  };
  launch();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}
