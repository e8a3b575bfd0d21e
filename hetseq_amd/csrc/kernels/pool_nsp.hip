// Pooler + NSP classifier + NSP cross-entropy, forward and backward (K08).
//
// Reference (bert_modeling.py:506-516, 572-581, 880-886):
//   pooled = tanh(seq[:, 0] @ Wp^T + bp)          BertPooler (LinearActivation, act tanh)
//   logits = pooled @ Wn^T + bn                   seq_relationship, Linear(H, 2)
//   loss   = mlm_loss + CE(logits, label, ignore_index=-1)
// There the pooler is a GEMM + a TorchScript bias-tanh kernel, the NSP head
// another GEMM + bias, the CE two more kernels and the final add a fifth.  The
// work is tiny ([B, H] x [H, H] with B = 32 or 8), so it is latency-bound: the
// kernels below spread it over hundreds of waves (one per pooler row / row chunk),
// all in fp32 whatever the encoder's compute dtype, reading the first-token
// rows straight out of the [B*S, H] sequence output (no gather copy).
//
//   pool_fwd_kernel       grid H/4: one wave per pooler row, all B first-token rows past it
//   nsp_loss_kernel       1 workgroup: logits, mean CE over labelled rows, + mlm_loss -> total
//   nsp_bwd_kernel        grid B: dlogits, dpre = (dlogits Wn) o (1 - pooled^2)
//   pool_dx_partial/finish grid (B, 8) + B: dx = dpre Wp in 8 row chunks, summed in fixed
//                         order and added into dseq's first-token rows
//   pool_nsp_wgrad_kernel grid H + 2: dWp / dbp rows, then dWn / dbn, summed over b
//                         in a fixed order (deterministic), written or accumulated
//                         into the flat gradient buffer
#include "common.h"

namespace hs {

constexpr int kPoolThreads = 256;

// pooled[b, i] = tanh(x_b . Wp[i] + bp[i]) for every b: one wave per row i (its Wp row stays in
// registers, 3 x 16 B per lane at H = 768) and the B first-token rows streamed past it, four in
// flight; grid H / 4 workgroups of 4 waves fill the chip instead of one workgroup per sequence.
template <typename T>
__global__ void __launch_bounds__(kPoolThreads)
    pool_fwd_kernel(const T* __restrict__ seq, int B, int S, int H, const float* __restrict__ Wp,
                    const float* __restrict__ bp, float* __restrict__ pooled) {
  constexpr int kMaxV = 4;  // float4 per lane: H <= 1024
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * (kPoolThreads / 64) + (threadIdx.x >> 6);
  if (i >= H) return;
  float w[kMaxV][4];
#pragma unroll
  for (int v = 0; v < kMaxV; ++v) {
    const int k = 4 * (lane + 64 * v);
    if (k < H) load4(Wp + (int64_t)i * H + k, w[v]);
    else w[v][0] = w[v][1] = w[v][2] = w[v][3] = 0.f;
  }
  const float bias = bp[i];
  for (int b0 = 0; b0 < B; b0 += 4) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int b = min(b0 + u, B - 1);
#pragma unroll
      for (int v = 0; v < kMaxV; ++v) {
        const int k = 4 * (lane + 64 * v);
        if (k < H) {
          float x[4];
          load4(seq + (int64_t)b * S * H + k, x);
          acc[u] = fmaf(w[v][0], x[0], fmaf(w[v][1], x[1], fmaf(w[v][2], x[2], fmaf(w[v][3], x[3], acc[u]))));
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = wave_sum(acc[u]);
    if (lane < 4 && b0 + lane < B) {
      const float a = lane == 0 ? acc[0] : lane == 1 ? acc[1] : lane == 2 ? acc[2] : acc[3];
      pooled[(int64_t)(b0 + lane) * H + i] = tanhf(a + bias);
    }
  }
}

// logits[b] = pooled[b] Wn^T + bn (one wave per b), then total[0] = mlm_loss[0] + mean_b
// CE(logits[b], label[b]) over labels != -1 (NaN if none, as torch); lse[b] kept for the
// backward, stats[0] = count of labelled rows, stats[1] = NSP loss.  One workgroup.
__global__ void __launch_bounds__(kPoolThreads)
    nsp_loss_kernel(const float* __restrict__ pooled, const float* __restrict__ Wn, const float* __restrict__ bn,
                    const int64_t* __restrict__ label, int B, int H, const float* __restrict__ mlm_loss,
                    float* __restrict__ logits, float* __restrict__ lse, float* __restrict__ stats,
                    float* __restrict__ total) {
  __shared__ float red[2][kPoolThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = kPoolThreads / 64;
  float s = 0.f, c = 0.f;
  for (int b = w; b < B; b += nw) {
    float a0 = 0.f, a1 = 0.f;
    for (int k = lane; k < H; k += 64) {
      const float p = pooled[(int64_t)b * H + k];
      a0 = fmaf(p, Wn[k], a0);
      a1 = fmaf(p, Wn[H + k], a1);
    }
    const float l0 = wave_sum(a0) + bn[0], l1 = wave_sum(a1) + bn[1];
    const float m = fmaxf(l0, l1);
    const float z = m + __logf(__expf(l0 - m) + __expf(l1 - m));
    const int64_t y = label[b];
    if (lane == 0) {
      logits[2 * b] = l0;
      logits[2 * b + 1] = l1;
      lse[b] = z;
      if (y == 0 || y == 1) {
        s += z - (y == 0 ? l0 : l1);
        c += 1.f;
      }
    }
  }
  if (lane == 0) {
    red[0][w] = s;
    red[1][w] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float ts = 0.f, tc = 0.f;
    for (int i = 0; i < nw; ++i) {  // fixed order: deterministic
      ts += red[0][i];
      tc += red[1][i];
    }
    stats[0] = tc;
    stats[1] = ts / tc;
    total[0] = (mlm_loss ? mlm_loss[0] : 0.f) + ts / tc;
  }
}

// dlogits[b] = dloss / count * (softmax - onehot) (0 for ignored rows);
// dpre[b] = (dlogits Wn) o (1 - pooled^2).  Grid B.
__global__ void __launch_bounds__(kPoolThreads)
    nsp_bwd_kernel(const float* __restrict__ dloss, const float* __restrict__ logits, const float* __restrict__ lse,
                   const int64_t* __restrict__ label, const float* __restrict__ stats,
                   const float* __restrict__ pooled, const float* __restrict__ Wn, int H,
                   float* __restrict__ dlogits, float* __restrict__ dpre) {
  const int b = blockIdx.x;
  const int64_t y = label[b];
  const float g = (y == 0 || y == 1) ? dloss[0] / stats[0] : 0.f;
  const float z = lse[b];
  const float d0 = g * (__expf(logits[2 * b] - z) - (y == 0 ? 1.f : 0.f));
  const float d1 = g * (__expf(logits[2 * b + 1] - z) - (y == 1 ? 1.f : 0.f));
  if (threadIdx.x == 0) {
    dlogits[2 * b] = d0;
    dlogits[2 * b + 1] = d1;
  }
  for (int k = threadIdx.x; k < H; k += kPoolThreads) {
    const float p = pooled[(int64_t)b * H + k];
    dpre[(int64_t)b * H + k] = (d0 * Wn[k] + d1 * Wn[H + k]) * (1.f - p * p);
  }
}

// dx = dpre Wp in kChunks row chunks of Wp: workgroup (b, c) sums rows [c H/kChunks, (c+1) H/kChunks)
// of Wp weighted by dpre[b] (each wave a quarter of them, lanes over all columns, then the waves
// combined in LDS in fixed order) -> part[b][c][:]
constexpr int kChunks = 8;

__global__ void __launch_bounds__(kPoolThreads)
    pool_dx_partial_kernel(const float* __restrict__ dpre, const float* __restrict__ Wp, int H,
                           float* __restrict__ part) {
  constexpr int kMaxV = 4;  // H <= 1024
  extern __shared__ __attribute__((aligned(16))) float smp[];  // [4 waves][H]
  const int b = blockIdx.x, c = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = kPoolThreads / 64;
  const int rows = H / kChunks, r0 = c * rows + w * (rows / nw), r1 = (w == nw - 1) ? (c + 1) * rows : r0 + rows / nw;
  float acc[kMaxV][4] = {};
  for (int i = r0; i < r1; ++i) {
    const float d = dpre[(int64_t)b * H + i];
#pragma unroll
    for (int v = 0; v < kMaxV; ++v) {
      const int k = 4 * (lane + 64 * v);
      if (k < H) {
        float wv[4];
        load4(Wp + (int64_t)i * H + k, wv);
        acc[v][0] = fmaf(d, wv[0], acc[v][0]);
        acc[v][1] = fmaf(d, wv[1], acc[v][1]);
        acc[v][2] = fmaf(d, wv[2], acc[v][2]);
        acc[v][3] = fmaf(d, wv[3], acc[v][3]);
      }
    }
  }
#pragma unroll
  for (int v = 0; v < kMaxV; ++v) {
    const int k = 4 * (lane + 64 * v);
    if (k < H) store4(smp + w * H + k, acc[v]);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < H; k += kPoolThreads) {
    float t = 0.f;
    for (int q = 0; q < nw; ++q) t += smp[q * H + k];
    part[((int64_t)b * kChunks + c) * H + k] = t;
  }
}

// dseq[b*S, :] += sum_c part[b][c][:] (fixed order).  Grid B.
template <typename T>
__global__ void __launch_bounds__(kPoolThreads)
    pool_dx_finish_kernel(const float* __restrict__ part, int S, int H, T* __restrict__ dseq) {
  const int b = blockIdx.x;
  T* row = dseq + (int64_t)b * S * H;
  for (int j = threadIdx.x * 4; j < H; j += kPoolThreads * 4) {
    float a[4];
    load4(row + j, a);
    for (int c = 0; c < kChunks; ++c) {
      float v[4];
      load4(part + ((int64_t)b * kChunks + c) * H + j, v);
      a[0] += v[0];
      a[1] += v[1];
      a[2] += v[2];
      a[3] += v[3];
    }
    store4(row + j, a);
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

// dtype: 0 fp32, 1 bf16 sequence output.  H % 4 == 0, H <= 1024 (checked by the caller too).
int launch_pool_nsp_fwd(int dtype, const void* seq, int B, int S, int H, const float* Wp, const float* bp,
                        const float* Wn, const float* bn, const int64_t* label, const float* mlm_loss, float* pooled,
                        float* logits, float* lse, float* stats, float* total, hipStream_t st) {
  if (B <= 0 || H <= 0 || H % 4 || H > 1024) return -1;
  const dim3 grid((H + 3) / 4);
  if (dtype == 0)
    hipLaunchKernelGGL(pool_fwd_kernel<float>, grid, dim3(kPoolThreads), 0, st, (const float*)seq, B, S, H, Wp, bp,
                       pooled);
  else
    hipLaunchKernelGGL(pool_fwd_kernel<bf16_t>, grid, dim3(kPoolThreads), 0, st, (const bf16_t*)seq, B, S, H, Wp,
                       bp, pooled);
  hipLaunchKernelGGL(nsp_loss_kernel, dim3(1), dim3(kPoolThreads), 0, st, pooled, Wn, bn, label, B, H, mlm_loss,
                     logits, lse, stats, total);
  return 0;
}

// scratch: dlogits [B, 2], dpre [B, H], part [B, 8, H] floats
int launch_pool_nsp_bwd(int dtype, const float* dloss, const void* seq, void* dseq, int B, int S, int H,
                        const float* Wp, const float* Wn, const int64_t* label, const float* pooled,
                        const float* logits, const float* lse, const float* stats, float* dlogits, float* dpre,
                        float* part, float* dWp, float* dbp, float* dWn, float* dbn, int accumulate,
                        hipStream_t st) {
  if (B <= 0 || H <= 0 || H % 4 || H > 1024 || H % (kChunks * 4)) return -1;
  hipLaunchKernelGGL(nsp_bwd_kernel, dim3(B), dim3(kPoolThreads), 0, st, dloss, logits, lse, label, stats, pooled, Wn,
                     H, dlogits, dpre);
  hipLaunchKernelGGL(pool_dx_partial_kernel, dim3(B, kChunks), dim3(kPoolThreads), 4 * (size_t)H * sizeof(float), st,
                     dpre, Wp, H, part);
  if (dtype == 0) {
    hipLaunchKernelGGL(pool_dx_finish_kernel<float>, dim3(B), dim3(kPoolThreads), 0, st, part, S, H, (float*)dseq);
    hipLaunchKernelGGL(pool_nsp_wgrad_kernel<float>, dim3(H + 2), dim3(kPoolThreads), 0, st, (const float*)seq, dpre,
                       dlogits, pooled, B, S, H, dWp, dbp, dWn, dbn, accumulate);
  } else {
    hipLaunchKernelGGL(pool_dx_finish_kernel<bf16_t>, dim3(B), dim3(kPoolThreads), 0, st, part, S, H, (bf16_t*)dseq);
    hipLaunchKernelGGL(pool_nsp_wgrad_kernel<bf16_t>, dim3(H + 2), dim3(kPoolThreads), 0, st, (const bf16_t*)seq,
                       dpre, dlogits, pooled, B, S, H, dWp, dbp, dWn, dbn, accumulate);
  }
  return 0;
}
