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
                                                       const float* __restrict__ dloss, const float* __restrict__ stats,
                                                       float* __restrict__ amax) {
  const int row = blockIdx.x;
  const int64_t lab = labels[row];
  T* x = logits + (int64_t)row * ldv;
  const bool valid = !(lab == ignore || lab < 0 || lab >= V);
  const float g = valid ? dloss[0] / stats[1] : 0.f;
  const float L = lse[row];
  uint32_t mb = 0u;
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float pr = __expf(to_f(x[i]) - L);
    const float d = valid ? g * (pr - (i == lab ? 1.f : 0.f)) : 0.f;
    mb = amax_bits(mb, d);
    x[i] = from_f<T>(d);
  }
  if (amax) amax_commit(amax, mb);  // (block-uniform: every lane of every wave reaches it)
}

// fp32 rows with 16-B aligned starts (ldv % 4 == 0): float4 loads, two independent (max, sum)
// chains per thread (two loads in flight instead of one dependent scalar chain), the max taken per
// quad before one rescale.  The MLM head's [640, 30522] logits: one row of ~120 KB per block.
HS_DEVICE void xent_quad(const float4 a, float& m, float& s) {
  const float mq = fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w));
  if (mq > m) {
    s *= __expf(m - mq);  // (m = -inf at the start: s = 0)
    m = mq;
  }
  s += (__expf(a.x - m) + __expf(a.y - m)) + (__expf(a.z - m) + __expf(a.w - m));
}

__global__ void __launch_bounds__(256) xent_fwd_vec_kernel(const float* __restrict__ logits,
                                                           const int64_t* __restrict__ labels, int V, int64_t ldv,
                                                           int ignore, float* __restrict__ row_loss,
                                                           float* __restrict__ lse_out) {
  const int row = blockIdx.x;
  const int64_t lab = labels[row];
  const float* x = logits + (int64_t)row * ldv;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const int n4 = V >> 2, bd = blockDim.x;
  float m0 = -INFINITY, s0 = 0.f, m1 = -INFINITY, s1 = 0.f;
  int i = threadIdx.x;
  for (; i + bd < n4; i += 2 * bd) {
    const float4 a = x4[i], b = x4[i + bd];
    xent_quad(a, m0, s0);
    xent_quad(b, m1, s1);
  }
  if (i < n4) xent_quad(x4[i], m0, s0);
  const int t = (n4 << 2) + threadIdx.x;  // the last V % 4 elements
  if (t < V) {
    const float v = x[t];
    if (v > m1) {
      s1 = s1 * __expf(m1 - v) + 1.f;
      m1 = v;
    } else {
      s1 += __expf(v - m1);
    }
  }
  float m = fmaxf(m0, m1);
  float s = (m0 == -INFINITY ? 0.f : s0 * __expf(m0 - m)) + (m1 == -INFINITY ? 0.f : s1 * __expf(m1 - m));
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
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) M = fmaxf(M, sm[k]);
    float Ssum = 0.f;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) Ssum += ss[k] * __expf(sm[k] - M);
    const float lse = M + __logf(Ssum);
    lse_out[row] = lse;
    row_loss[row] = (lab == ignore || lab < 0 || lab >= V) ? 0.f : lse - x[lab];
  }
}

__global__ void __launch_bounds__(256) xent_bwd_vec_kernel(float* __restrict__ logits,
                                                           const int64_t* __restrict__ labels,
                                                           const float* __restrict__ lse, int V, int64_t ldv,
                                                           int ignore, const float* __restrict__ dloss,
                                                           const float* __restrict__ stats, float* __restrict__ amax) {
  const int row = blockIdx.x;
  const int64_t lab = labels[row];
  float* x = logits + (int64_t)row * ldv;
  float4* x4 = reinterpret_cast<float4*>(x);
  const bool valid = !(lab == ignore || lab < 0 || lab >= V);
  const float g = valid ? dloss[0] / stats[1] : 0.f;
  const float L = lse[row];
  const int n4 = V >> 2, bd = blockDim.x;
  uint32_t mb = 0u;  // |max| of the written gradient (the decoder products' operand scale)
  auto grad = [&](float v, int idx) {
    const float d = valid ? g * (__expf(v - L) - (idx == lab ? 1.f : 0.f)) : 0.f;
    mb = amax_bits(mb, d);
    return d;
  };
  int i = threadIdx.x;
  for (; i + bd < n4; i += 2 * bd) {
    const float4 a = x4[i], b = x4[i + bd];
    const int ia = 4 * i, ib = 4 * (i + bd);
    x4[i] = make_float4(grad(a.x, ia), grad(a.y, ia + 1), grad(a.z, ia + 2), grad(a.w, ia + 3));
    x4[i + bd] = make_float4(grad(b.x, ib), grad(b.y, ib + 1), grad(b.z, ib + 2), grad(b.w, ib + 3));
  }
  if (i < n4) {
    const float4 a = x4[i];
    const int ia = 4 * i;
    x4[i] = make_float4(grad(a.x, ia), grad(a.y, ia + 1), grad(a.z, ia + 2), grad(a.w, ia + 3));
  }
  const int t = (n4 << 2) + threadIdx.x;
  if (t < V) x[t] = grad(x[t], t);
  if (amax) amax_commit(amax, mb);
}

}  // namespace hs

using namespace hs;

static bool xent_vec_ok(const void* logits, int64_t ldv, int threads) {
  return threads == 256 && ldv % 4 == 0 && (reinterpret_cast<uintptr_t>(logits) & 15) == 0;
}

void launch_xent_fwd(int dtype, const void* logits, const int64_t* labels, int rows, int V, int64_t ldv, int ignore,
                     float* row_loss, float* lse, float* out, hipStream_t st) {
  if (rows <= 0) return;
  const int threads = V >= 1024 ? 256 : 64;
  if (dtype == 0 && xent_vec_ok(logits, ldv, threads))
    hipLaunchKernelGGL(xent_fwd_vec_kernel, dim3(rows), dim3(threads), 0, st, (const float*)logits, labels, V, ldv,
                       ignore, row_loss, lse);
  else if (dtype == 0)
    hipLaunchKernelGGL(xent_fwd_kernel<float>, dim3(rows), dim3(threads), 0, st, (const float*)logits, labels, V, ldv,
                       ignore, row_loss, lse);
  else
    hipLaunchKernelGGL(xent_fwd_kernel<bf16_t>, dim3(rows), dim3(threads), 0, st, (const bf16_t*)logits, labels, V,
                       ldv, ignore, row_loss, lse);
  hipLaunchKernelGGL(xent_reduce_kernel, dim3(1), dim3(1024), 0, st, row_loss, labels, rows, V, ignore, out);
}

// amax (optional, a zeroed |max| slot): |max| of the written dlogits
void launch_xent_bwd(int dtype, void* logits, const int64_t* labels, const float* lse, int rows, int V, int64_t ldv,
                     int ignore, const float* dloss, const float* stats, hipStream_t st, float* amax) {
  if (rows <= 0) return;
  const int threads = V >= 1024 ? 256 : 64;
  if (dtype == 0 && xent_vec_ok(logits, ldv, threads))
    hipLaunchKernelGGL(xent_bwd_vec_kernel, dim3(rows), dim3(threads), 0, st, (float*)logits, labels, lse, V, ldv,
                       ignore, dloss, stats, amax);
  else if (dtype == 0)
    hipLaunchKernelGGL(xent_bwd_kernel<float>, dim3(rows), dim3(threads), 0, st, (float*)logits, labels, lse, V, ldv,
                       ignore, dloss, stats, amax);
  else
    hipLaunchKernelGGL(xent_bwd_kernel<bf16_t>, dim3(rows), dim3(threads), 0, st, (bf16_t*)logits, labels, lse, V, ldv,
                       ignore, dloss, stats, amax);
}
