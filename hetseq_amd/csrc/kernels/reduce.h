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

// The same reduction with 16-byte loads (N % 4 == 0, 16-B aligned rows): a thread owns 4 columns
// and rows ry, ry + 32, ... (32 row groups), 4 independent float4 accumulators, so 512 partial
// rows (the 8-row LayerNorm-backward workgroups of a 4096-row batch) are 4 rounds of 4 loads per
// thread instead of 16 dependent rounds; the 32 group sums are combined in a fixed order.
__global__ void __launch_bounds__(256) reduce_rows4_kernel(ReduceArgs args, int nparts, int N, int accumulate) {
  __shared__ float4 red[32][8];
  __shared__ float4 red4[4][8];
  const float* part = args.part[blockIdx.y];
  float* out = args.out[blockIdx.y];
  const int cq = threadIdx.x & 7, ry = threadIdx.x >> 3;
  const int c = blockIdx.x * 32 + 4 * cq;
  float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0, s2 = s0, s3 = s0;
  auto ld = [&](int r) { return *reinterpret_cast<const float4*>(part + (int64_t)r * N + c); };
  auto add = [](float4& a, const float4& b) {
    a.x += b.x;
    a.y += b.y;
    a.z += b.z;
    a.w += b.w;
  };
  if (c < N) {
    int r = ry;
    for (; r + 96 < nparts; r += 128) {
      const float4 a = ld(r), b = ld(r + 32), d = ld(r + 64), e = ld(r + 96);
      add(s0, a);
      add(s1, b);
      add(s2, d);
      add(s3, e);
    }
    for (; r < nparts; r += 32) add(s0, ld(r));
  }
  add(s0, s1);
  add(s2, s3);
  add(s0, s2);
  red[ry][cq] = s0;
  __syncthreads();
  if (ry < 4) {  // four sums of eight row groups each, then those four (fixed order)
    float4 t = red[8 * ry][cq];
#pragma unroll
    for (int i = 1; i < 8; ++i) add(t, red[8 * ry + i][cq]);
    red4[ry][cq] = t;
  }
  __syncthreads();
  if (ry == 0 && c < N) {
    float4 t = red4[0][cq];
    add(t, red4[1][cq]);
    add(t, red4[2][cq]);
    add(t, red4[3][cq]);
    float4* o = reinterpret_cast<float4*>(out + c);
    if (accumulate) add(t, *o);
    *o = t;
  }
}

inline void launch_reduce_rows(const float* const* parts, float* const* outs, int n, int nparts, int N,
                               int accumulate, hipStream_t st) {
  if (g_hs_skip & kSkipReduceRows) return;
  ReduceArgs a{};
  for (int i = 0; i < n; ++i) {
    a.part[i] = parts[i];
    a.out[i] = outs[i];
  }
  bool vec = N % 4 == 0;
  for (int i = 0; i < n; ++i)
    vec = vec && (reinterpret_cast<uintptr_t>(parts[i]) & 15) == 0 && (reinterpret_cast<uintptr_t>(outs[i]) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(reduce_rows4_kernel, dim3((N + 31) / 32, n), dim3(256), 0, st, a, nparts, N, accumulate);
  else
    hipLaunchKernelGGL(reduce_rows_kernel, dim3((N + 31) / 32, n), dim3(256), 0, st, a, nparts, N, accumulate);
}

}  // namespace
}  // namespace hs
