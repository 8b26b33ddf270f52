// Micro-benchmark (tooling, not product): vector-L1 (TCP) cost of one wave64 dword-gather
// instruction by address pattern, to calibrate the SSpMM backward's G gathers.
// Each wave issues ITERS dword loads from a table (L1/L2-resident by default), the address of
// lane l in iteration i given by the pattern; run under rocprofv3 --pmc
// TCP_TOTAL_CACHE_ACCESSES_sum to count L1 tag accesses per instruction, and timed with events.
//   0 all 64 lanes read one dword
//   1 64 consecutive dwords (256 B)
//   2 16 groups of 4 lanes; group g reads 4 consecutive dwords of its own 128-B line
//   3 16 groups of 4 lanes; group g reads 4 random dwords of its own 1-KB row (the current
//     backward: 4 slots of one edge)
//   4 4 groups of 16 lanes (4 edges of one row); random dwords in one 256-B quarter of the row
//   5 4 groups of 16 lanes; group g reads 16 random dwords of its own 1-KB row
//   6 every lane a distinct random 128-B line
//   7 16 groups of 4 lanes; group g reads 4 random dwords of one 256-B quarter of its own row
//     (the interleaved backward: slots 4i..4i+3 of sorted selectors)
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int ITERS = 512;

// per-lane LCGs keep the address arithmetic to a few VALU ops per load (the TCP, not the
// VALU, must be the bottleneck): s_g is shared by the lanes of a group (same row), s_l is
// per lane (position in the row)
template <int G, int MODE>  // G lanes per group; MODE 0 one dword, 1 consecutive,
                            // 2 16-B chunk, 3 random in row, 4 random in row quarter
__global__ __launch_bounds__(256) void tcp_kern(const float* __restrict__ table, int rows_1k,
                                                float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint32_t wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  uint32_t sg = (wid * 64 + lane / G) * 2654435761u + 12345u;
  uint32_t sl = (wid * 64 + lane) * 2246822519u + 777u;
  float acc = 0.f;
#pragma unroll 8
  for (int it = 0; it < ITERS; ++it) {
    sg = sg * 1664525u + 1013904223u;
    sl = sl * 22695477u + 1u;
    const uint32_t row = __umulhi(sg, (uint32_t)rows_1k);
    uint32_t col;
    if (MODE == 0) col = 0;
    else if (MODE == 1) col = lane;
    else if (MODE == 2) col = ((sg >> 8) & 63) * 4 + (lane & 3);
    else if (MODE == 3) col = sl >> 24;
    else col = (it & 3) * 64 + (sl >> 26);
    acc += table[row * 256 + col];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

extern "C" float ubench_tcp(int pattern, const float* table, int rows_1k, float* out, int nwg,
                            int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto launch = [&]() {
    switch (pattern) {
#define CASE(n, g, m) case n: hipLaunchKernelGGL((tcp_kern<g, m>), nwg, 256, 0, 0, table, rows_1k, out); break;
      CASE(0, 64, 0) CASE(1, 64, 1) CASE(2, 4, 2) CASE(3, 4, 3) CASE(4, 16, 4) CASE(5, 16, 3)
      CASE(6, 1, 0) CASE(7, 4, 4)
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
