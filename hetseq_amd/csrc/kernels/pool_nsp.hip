// Pooler + NSP classifier + NSP cross-entropy, forward and backward (K08).
//
// Reference (bert_modeling.py:506-516, 572-581, 880-886):
//   pooled = tanh(seq[:, 0] @ Wp^T + bp)          BertPooler (LinearActivation, act tanh)
//   logits = pooled @ Wn^T + bn                   seq_relationship, Linear(H, 2)
//   loss   = mlm_loss + CE(logits, label, ignore_index=-1)
// There the pooler is a GEMM + a TorchScript bias-tanh kernel, the NSP head
// another GEMM + bias, the CE two more kernels and the final add a fifth.  The
// work is tiny ([B, H] x [H, H] with B = 32 or 8), so it is launch- and
// latency-bound: here it is four kernels for forward + backward together,
// all in fp32 whatever the encoder's compute dtype, reading the first-token
// rows straight out of the [B*S, H] sequence output (no gather copy).
//
//   pool_nsp_fwd_kernel   grid B: pooled[b], logits[b] (one workgroup per sequence;
//                         Wp rows are dotted by whole waves, 4 rows per pass)
//   nsp_loss_kernel       1 wave: mean CE over labelled rows, + mlm_loss -> total
//   pool_nsp_bwd_kernel   grid B: dlogits, dpre = (dlogits Wn) o (1 - pooled^2),
//                         dx = dpre Wp added into dseq's first-token row
//   pool_nsp_wgrad_kernel grid H + 2: dWp / dbp rows, then dWn / dbn, summed over b
//                         in a fixed order (deterministic), written or accumulated
//                         into the flat gradient buffer
#include "common.h"

namespace hs {

constexpr int kPoolThreads = 256;

// pooled[b, :] and logits[b, :].  x = seq row b*S (the first token).
template <typename T>
__global__ void __launch_bounds__(kPoolThreads)
    pool_nsp_fwd_kernel(const T* __restrict__ seq, int S, int H, const float* __restrict__ Wp,
                        const float* __restrict__ bp, const float* __restrict__ Wn, const float* __restrict__ bn,
                        float* __restrict__ pooled, float* __restrict__ logits) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* xs = sm;      // [H] first-token row
  float* ps = sm + H;  // [H] pooled row
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = kPoolThreads / 64;
  const T* x = seq + (int64_t)b * S * H;
  for (int k = threadIdx.x * 4; k < H; k += kPoolThreads * 4) {
    float v[4];
    load4(x + k, v);
    *reinterpret_cast<float4*>(xs + k) = make_float4(v[0], v[1], v[2], v[3]);
  }
  __syncthreads();
  // each wave takes 4 rows of Wp at a time: 4 independent dot products per lane, one shuffle tree
  for (int i0 = 4 * w; i0 < H; i0 += 4 * nw) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = lane * 4; k < H; k += 256) {
      const float4 xv = *reinterpret_cast<const float4*>(xs + k);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (i0 + r < H) {
          const float4 wv = *reinterpret_cast<const float4*>(Wp + (int64_t)(i0 + r) * H + k);
          acc[r] = fmaf(wv.x, xv.x, fmaf(wv.y, xv.y, fmaf(wv.z, xv.z, fmaf(wv.w, xv.w, acc[r]))));
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = wave_sum(acc[r]);
    if (lane < 4 && i0 + lane < H) {
      const float a = lane == 0 ? acc[0] : lane == 1 ? acc[1] : lane == 2 ? acc[2] : acc[3];
      const float y = tanhf(a + bp[i0 + lane]);
      ps[i0 + lane] = y;
      pooled[(int64_t)b * H + i0 + lane] = y;
    }
  }
  __syncthreads();
  if (w < 2) {  // wave c: logit c
    float acc = 0.f;
    for (int k = lane; k < H; k += 64) acc = fmaf(ps[k], Wn[(int64_t)w * H + k], acc);
    acc = wave_sum(acc);
    if (lane == 0) logits[b * 2 + w] = acc + bn[w];
  }
}

// total[0] = mlm_loss[0] + mean_b CE(logits[b], label[b]) over labels != -1 (NaN if none, as
// torch); lse[b] kept for the backward, stats[0] = count of labelled rows.
__global__ void __launch_bounds__(64)
    nsp_loss_kernel(const float* __restrict__ logits, const int64_t* __restrict__ label, int B,
                    const float* __restrict__ mlm_loss, float* __restrict__ lse, float* __restrict__ stats,
                    float* __restrict__ total) {
  float s = 0.f, c = 0.f;
  for (int b = threadIdx.x; b < B; b += 64) {
    const float l0 = logits[2 * b], l1 = logits[2 * b + 1];
    const float m = fmaxf(l0, l1);
    const float z = m + __logf(__expf(l0 - m) + __expf(l1 - m));
    lse[b] = z;
    const int64_t y = label[b];
    if (y == 0 || y == 1) {
      s += z - (y == 0 ? l0 : l1);
      c += 1.f;
    }
  }
  s = wave_sum(s);
  c = wave_sum(c);
  if (threadIdx.x == 0) {
    stats[0] = c;
    stats[1] = s / c;
    total[0] = (mlm_loss ? mlm_loss[0] : 0.f) + s / c;
  }
}

// dlogits[b] = dloss / count * (softmax - onehot) (0 for ignored rows); dpre[b] = (dlogits Wn) o
// (1 - pooled^2); dseq[b*S, :] += dpre Wp.
template <typename T>
__global__ void __launch_bounds__(kPoolThreads)
    pool_nsp_bwd_kernel(const float* __restrict__ dloss, const float* __restrict__ logits,
                        const float* __restrict__ lse, const int64_t* __restrict__ label,
                        const float* __restrict__ stats, const float* __restrict__ pooled,
                        const float* __restrict__ Wn, const float* __restrict__ Wp, int S, int H,
                        float* __restrict__ dlogits, float* __restrict__ dpre, T* __restrict__ dseq) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* dps = sm;  // [H]
  const int b = blockIdx.x;
  const int64_t y = label[b];
  const bool valid = y == 0 || y == 1;
  const float g = valid ? dloss[0] / stats[0] : 0.f;
  const float z = lse[b];
  const float d0 = g * (__expf(logits[2 * b] - z) - (y == 0 ? 1.f : 0.f));
  const float d1 = g * (__expf(logits[2 * b + 1] - z) - (y == 1 ? 1.f : 0.f));
  if (threadIdx.x == 0) {
    dlogits[2 * b] = d0;
    dlogits[2 * b + 1] = d1;
  }
  for (int k = threadIdx.x; k < H; k += kPoolThreads) {
    const float p = pooled[(int64_t)b * H + k];
    const float d = (d0 * Wn[k] + d1 * Wn[H + k]) * (1.f - p * p);
    dps[k] = d;
    dpre[(int64_t)b * H + k] = d;
  }
  __syncthreads();
  // dx[j] = sum_i dpre[i] Wp[i][j]: threads own 4 consecutive columns, rows streamed in order
  T* row = dseq + (int64_t)b * S * H;
  for (int j = threadIdx.x * 4; j < H; j += kPoolThreads * 4) {
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < H; ++i) {
      const float4 wv = *reinterpret_cast<const float4*>(Wp + (int64_t)i * H + j);
      const float d = dps[i];
      a[0] = fmaf(d, wv.x, a[0]);
      a[1] = fmaf(d, wv.y, a[1]);
      a[2] = fmaf(d, wv.z, a[2]);
      a[3] = fmaf(d, wv.w, a[3]);
    }
    float old[4];
    load4(row + j, old);
    const float v[4] = {old[0] + a[0], old[1] + a[1], old[2] + a[2], old[3] + a[3]};
    store4(row + j, v);
  }
}

// blocks 0..H-1: dWp[i, :] (+)= sum_b dpre[b, i] x[b, :], dbp[i] (+)= sum_b dpre[b, i];
// blocks H, H+1: dWn[c, :] (+)= sum_b dlogits[b, c] pooled[b, :], dbn[c] (+)= sum_b dlogits[b, c].
template <typename T>
__global__ void __launch_bounds__(kPoolThreads)
    pool_nsp_wgrad_kernel(const T* __restrict__ seq, const float* __restrict__ dpre, const float* __restrict__ dlogits,
                          const float* __restrict__ pooled, int B, int S, int H, float* __restrict__ dWp,
                          float* __restrict__ dbp, float* __restrict__ dWn, float* __restrict__ dbn, int accumulate) {
  const int i = blockIdx.x;
  const bool nsp = i >= H;
  const int c = i - H;
  float* out = nsp ? dWn + (int64_t)c * H : dWp + (int64_t)i * H;
  for (int j = threadIdx.x * 4; j < H; j += kPoolThreads * 4) {
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    for (int b = 0; b < B; ++b) {
      const float d = nsp ? dlogits[2 * b + c] : dpre[(int64_t)b * H + i];
      float v[4];
      if (nsp) load4(pooled + (int64_t)b * H + j, v);
      else load4(seq + (int64_t)b * S * H + j, v);
      a[0] = fmaf(d, v[0], a[0]);
      a[1] = fmaf(d, v[1], a[1]);
      a[2] = fmaf(d, v[2], a[2]);
      a[3] = fmaf(d, v[3], a[3]);
    }
    if (accumulate) {
      float o[4];
      load4(out + j, o);
      a[0] += o[0];
      a[1] += o[1];
      a[2] += o[2];
      a[3] += o[3];
    }
    store4(out + j, a);
  }
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += nsp ? dlogits[2 * b + c] : dpre[(int64_t)b * H + i];
    float* bo = nsp ? dbn + c : dbp + i;
    *bo = accumulate ? *bo + s : s;
  }
}

}  // namespace hs

using namespace hs;

// dtype: 0 fp32, 1 bf16 sequence output.  H % 4 == 0 (checked by the caller too).
int launch_pool_nsp_fwd(int dtype, const void* seq, int B, int S, int H, const float* Wp, const float* bp,
                        const float* Wn, const float* bn, const int64_t* label, const float* mlm_loss, float* pooled,
                        float* logits, float* lse, float* stats, float* total, hipStream_t st) {
  if (B <= 0 || H <= 0 || H % 4) return -1;
  const size_t lds = 2 * (size_t)H * sizeof(float);
  if (dtype == 0)
    hipLaunchKernelGGL(pool_nsp_fwd_kernel<float>, dim3(B), dim3(kPoolThreads), lds, st, (const float*)seq, S, H, Wp,
                       bp, Wn, bn, pooled, logits);
  else
    hipLaunchKernelGGL(pool_nsp_fwd_kernel<bf16_t>, dim3(B), dim3(kPoolThreads), lds, st, (const bf16_t*)seq, S, H,
                       Wp, bp, Wn, bn, pooled, logits);
  hipLaunchKernelGGL(nsp_loss_kernel, dim3(1), dim3(64), 0, st, logits, label, B, mlm_loss, lse, stats, total);
  return 0;
}

int launch_pool_nsp_bwd(int dtype, const float* dloss, const void* seq, void* dseq, int B, int S, int H,
                        const float* Wp, const float* Wn, const int64_t* label, const float* pooled,
                        const float* logits, const float* lse, const float* stats, float* dlogits, float* dpre,
                        float* dWp, float* dbp, float* dWn, float* dbn, int accumulate, hipStream_t st) {
  if (B <= 0 || H <= 0 || H % 4) return -1;
  const size_t lds = (size_t)H * sizeof(float);
  if (dtype == 0) {
    hipLaunchKernelGGL(pool_nsp_bwd_kernel<float>, dim3(B), dim3(kPoolThreads), lds, st, dloss, logits, lse, label,
                       stats, pooled, Wn, Wp, S, H, dlogits, dpre, (float*)dseq);
    hipLaunchKernelGGL(pool_nsp_wgrad_kernel<float>, dim3(H + 2), dim3(kPoolThreads), 0, st, (const float*)seq, dpre,
                       dlogits, pooled, B, S, H, dWp, dbp, dWn, dbn, accumulate);
  } else {
    hipLaunchKernelGGL(pool_nsp_bwd_kernel<bf16_t>, dim3(B), dim3(kPoolThreads), lds, st, dloss, logits, lse, label,
                       stats, pooled, Wn, Wp, S, H, dlogits, dpre, (bf16_t*)dseq);
    hipLaunchKernelGGL(pool_nsp_wgrad_kernel<bf16_t>, dim3(H + 2), dim3(kPoolThreads), 0, st, (const bf16_t*)seq,
                       dpre, dlogits, pooled, B, S, H, dWp, dbp, dWn, dbn, accumulate);
  }
  return 0;
}
