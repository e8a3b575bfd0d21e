// Column reduction of per-block partial rows: out[c] (+)= sum_r part[r][c].
//
// Used to finalize the per-block column partials written by the LayerNorm /
// GELU / bias-gradient kernels (no atomics, deterministic order).  A block of
// 32 columns x 8 row-groups (256 threads): each thread sums nparts/8 rows with
// 4 independent accumulators (the loads issue back to back instead of forming
// one dependent chain), and the 8 partial sums are combined through LDS in a
// fixed order.  grid = (ceil(N/32), n_arrays).  Small blocks on purpose: these
// run beside the weight-gradient GEMM blocks of the side stream, where a
// 1024-thread block waits for a whole CU to drain (12 us per call inside the
// step vs 4.6 us alone).
#pragma once
#include "common.h"

namespace hs {
namespace {  // internal linkage: the header is compiled into several TUs

struct ReduceArgs {
  const float* part[3];
  float* out[3];
};

__global__ void __launch_bounds__(256) reduce_rows_kernel(ReduceArgs args, int nparts, int N, int accumulate) {
  __shared__ float red[8][33];
  const float* part = args.part[blockIdx.y];
  float* out = args.out[blockIdx.y];
  const int cx = threadIdx.x & 31, ry = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cx;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < N) {
    int r = ry;
    for (; r + 24 < nparts; r += 32) {
      s0 += part[(int64_t)r * N + c];
      s1 += part[(int64_t)(r + 8) * N + c];
      s2 += part[(int64_t)(r + 16) * N + c];
      s3 += part[(int64_t)(r + 24) * N + c];
    }
    for (; r < nparts; r += 8) s0 += part[(int64_t)r * N + c];
  }
  red[ry][cx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ry == 0 && c < N) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += red[i][cx];
    out[c] = accumulate ? out[c] + t : t;
  }
}

inline void launch_reduce_rows(const float* const* parts, float* const* outs, int n, int nparts, int N,
                               int accumulate, hipStream_t st) {
  ReduceArgs a{};
  for (int i = 0; i < n; ++i) {
    a.part[i] = parts[i];
    a.out[i] = outs[i];
  }
  hipLaunchKernelGGL(reduce_rows_kernel, dim3((N + 31) / 32, n), dim3(256), 0, st, a, nparts, N, accumulate);
}

}  // namespace
}  // namespace hs
