// Fused softmax cross-entropy with ignore_index (K07/K08 loss part).
//
// Reference: CrossEntropyLoss(ignore_index=-1) over [B*S, V] MLM logits and
// [B, 2] NSP logits, mean over non-ignored rows (bert_modeling.py:880-886).
// Forward: one block per row, single pass online max/sum-exp -> per-row loss
// and logsumexp; a one-block reduce writes mean loss and valid count to
// device memory (no host sync).  Backward: dlogits = (softmax - onehot) *
// dloss / count computed IN PLACE over the logits buffer (the logits are not
// needed after the loss), the upstream dloss read from device memory.
#include "common.h"

namespace hs {

template <typename T>
__global__ void __launch_bounds__(256) xent_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       int V, int64_t ldv, int ignore, float* __restrict__ row_loss,
                                                       float* __restrict__ lse_out) {
  const int row = blockIdx.x;
  const int64_t lab = labels[row];
  const T* x = logits + (int64_t)row * ldv;
  float m = -INFINITY, s = 0.f;
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float v = to_f(x[i]);
    if (v > m) {
      s = s * __expf(m - v) + 1.f;
      m = v;
    } else {
      s += __expf(v - m);
    }
  }
  // combine (m, s) across the block
  __shared__ float sm[4], ss[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    const float mm = fmaxf(m, m2);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mm)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mm));
    m = mm;
  }
  if (lane == 0) {
    sm[w] = m;
    ss[w] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) M = fmaxf(M, sm[i]);
    float Ssum = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) Ssum += ss[i] * __expf(sm[i] - M);
    const float lse = M + __logf(Ssum);
    lse_out[row] = lse;
    if (lab == ignore || lab < 0 || lab >= V)
      row_loss[row] = 0.f;
    else
      row_loss[row] = lse - to_f(x[lab]);
  }
}

// out[0] = mean loss over valid rows (NaN if none, like torch); out[1] = count
__global__ void xent_reduce_kernel(const float* __restrict__ row_loss, const int64_t* __restrict__ labels, int rows,
                                   int V, int ignore, float* __restrict__ out) {
  float s = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < rows; i += blockDim.x) {
    const int64_t lab = labels[i];
    if (lab != ignore && lab >= 0 && lab < V) {
      s += row_loss[i];
      c += 1.f;
    }
  }
  s = wave_sum(s);
  c = wave_sum(c);
  __shared__ float rs[16], rc[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    rs[w] = s;
    rc[w] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float S = 0.f, C = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
      S += rs[i];
      C += rc[i];
    }
    out[0] = S / C;
    out[1] = C;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) xent_bwd_kernel(T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       const float* __restrict__ lse, int V, int64_t ldv, int ignore,
                                                       const float* __restrict__ dloss, const float* __restrict__ stats) {
  const int row = blockIdx.x;
  const int64_t lab = labels[row];
  T* x = logits + (int64_t)row * ldv;
  const bool valid = !(lab == ignore || lab < 0 || lab >= V);
  const float g = valid ? dloss[0] / stats[1] : 0.f;
  const float L = lse[row];
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float pr = __expf(to_f(x[i]) - L);
    const float d = valid ? g * (pr - (i == lab ? 1.f : 0.f)) : 0.f;
    x[i] = from_f<T>(d);
  }
}

}  // namespace hs

using namespace hs;

void launch_xent_fwd(int dtype, const void* logits, const int64_t* labels, int rows, int V, int64_t ldv, int ignore,
                     float* row_loss, float* lse, float* out, hipStream_t st) {
  if (rows <= 0) return;
  const int threads = V >= 1024 ? 256 : 64;
  if (dtype == 0)
    hipLaunchKernelGGL(xent_fwd_kernel<float>, dim3(rows), dim3(threads), 0, st, (const float*)logits, labels, V, ldv,
                       ignore, row_loss, lse);
  else
    hipLaunchKernelGGL(xent_fwd_kernel<bf16_t>, dim3(rows), dim3(threads), 0, st, (const bf16_t*)logits, labels, V,
                       ldv, ignore, row_loss, lse);
  hipLaunchKernelGGL(xent_reduce_kernel, dim3(1), dim3(1024), 0, st, row_loss, labels, rows, V, ignore, out);
}

void launch_xent_bwd(int dtype, void* logits, const int64_t* labels, const float* lse, int rows, int V, int64_t ldv,
                     int ignore, const float* dloss, const float* stats, hipStream_t st) {
  if (rows <= 0) return;
  const int threads = V >= 1024 ? 256 : 64;
  if (dtype == 0)
    hipLaunchKernelGGL(xent_bwd_kernel<float>, dim3(rows), dim3(threads), 0, st, (float*)logits, labels, lse, V, ldv,
                       ignore, dloss, stats);
  else
    hipLaunchKernelGGL(xent_bwd_kernel<bf16_t>, dim3(rows), dim3(threads), 0, st, (bf16_t*)logits, labels, lse, V, ldv,
                       ignore, dloss, stats);
}
