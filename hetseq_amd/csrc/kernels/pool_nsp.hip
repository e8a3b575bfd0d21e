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
//   pool_fwd_kernel       one wave per (4 pooler rows, 8 sequences): 32 dot products per wave
//   nsp_loss_kernel       1 workgroup of 16 waves (one per sequence): logits, mean CE over labelled
//                         rows, + mlm_loss -> total
//   nsp_bwd_kernel        grid B: dlogits, dpre = (dlogits Wn) o (1 - pooled^2)
//   pool_dx_partial/finish grid (8, B/8) + B: dx = dpre Wp in 8 row chunks, summed in fixed
//                         order and added into dseq's first-token rows
//   pool_nsp_wgrad_kernel grid H/4 + 2: dWp / dbp rows (4 per block), then dWn / dbn, summed over b
//                         in a fixed order (deterministic), written or accumulated
//                         into the flat gradient buffer
#include "common.h"

namespace hs {

constexpr int kPoolThreads = 256;

// pooled[b, i] = tanh(x_b . Wp[i] + bp[i]): one wave per (4 pooler rows, 8 sequences) -- its
// 4 x 8 dot products read each Wp row and each first-token row once, all loads of a 256-column
// slice issued together (no load -> reduce -> load chain); grid (H / 4) x ceil(B / 8) waves.
constexpr int kPoolRows = 4, kPoolSeqs = 8;

template <typename T>
__global__ void __launch_bounds__(kPoolThreads)
    pool_fwd_kernel(const T* __restrict__ seq, int B, int S, int H, const float* __restrict__ Wp,
                    const float* __restrict__ bp, float* __restrict__ pooled) {
  const int lane = threadIdx.x & 63;
  const int wv = blockIdx.x * (kPoolThreads / 64) + (threadIdx.x >> 6);
  const int ngrp = (B + kPoolSeqs - 1) / kPoolSeqs;
  const int i0 = (wv / ngrp) * kPoolRows, b0 = (wv % ngrp) * kPoolSeqs;
  if (i0 >= H) return;
  float acc[kPoolRows][kPoolSeqs];
#pragma unroll
  for (int r = 0; r < kPoolRows; ++r)
#pragma unroll
    for (int u = 0; u < kPoolSeqs; ++u) acc[r][u] = 0.f;
  for (int k = 4 * lane; k < H; k += 256) {
    float w[kPoolRows][4], x[kPoolSeqs][4];
#pragma unroll
    for (int r = 0; r < kPoolRows; ++r) load4(Wp + (int64_t)(i0 + r) * H + k, w[r]);
#pragma unroll
    for (int u = 0; u < kPoolSeqs; ++u) load4(seq + (int64_t)min(b0 + u, B - 1) * S * H + k, x[u]);
#pragma unroll
    for (int r = 0; r < kPoolRows; ++r)
#pragma unroll
      for (int u = 0; u < kPoolSeqs; ++u)
        acc[r][u] = fmaf(w[r][0], x[u][0], fmaf(w[r][1], x[u][1], fmaf(w[r][2], x[u][2], fmaf(w[r][3], x[u][3], acc[r][u]))));
  }
#pragma unroll
  for (int r = 0; r < kPoolRows; ++r)
#pragma unroll
    for (int u = 0; u < kPoolSeqs; ++u) acc[r][u] = wave_sum(acc[r][u]);
  if (lane < kPoolRows * kPoolSeqs) {
    const int r = lane / kPoolSeqs, u = lane % kPoolSeqs;
    float a = 0.f;
#pragma unroll
    for (int rr = 0; rr < kPoolRows; ++rr)
#pragma unroll
      for (int uu = 0; uu < kPoolSeqs; ++uu)
        if (rr == r && uu == u) a = acc[rr][uu];
    if (b0 + u < B) pooled[(int64_t)(b0 + u) * H + i0 + r] = tanhf(a + bp[i0 + r]);
  }
}

// logits[b] = pooled[b] Wn^T + bn (one wave per b), then total[0] = mlm_loss[0] + mean_b
// CE(logits[b], label[b]) over labels != -1 (NaN if none, as torch); lse[b] kept for the
// backward, stats[0] = count of labelled rows, stats[1] = NSP loss.  One workgroup.
constexpr int kNspThreads = 1024;

__global__ void __launch_bounds__(kNspThreads)
    nsp_loss_kernel(const float* __restrict__ pooled, const float* __restrict__ Wn, const float* __restrict__ bn,
                    const int64_t* __restrict__ label, int B, int H, const float* __restrict__ mlm_loss,
                    float* __restrict__ logits, float* __restrict__ lse, float* __restrict__ stats,
                    float* __restrict__ total) {
  __shared__ float red[2][kNspThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = kNspThreads / 64;
  float s = 0.f, c = 0.f;
  for (int b = w; b < B; b += nw) {  // one wave per sequence: 16-B loads, both classes at once
    float a0 = 0.f, a1 = 0.f;
    for (int k = 4 * lane; k < H; k += 256) {
      float pv[4], w0[4], w1[4];
      load4(pooled + (int64_t)b * H + k, pv);
      load4(Wn + k, w0);
      load4(Wn + H + k, w1);
      a0 = fmaf(pv[0], w0[0], fmaf(pv[1], w0[1], fmaf(pv[2], w0[2], fmaf(pv[3], w0[3], a0))));
      a1 = fmaf(pv[0], w1[0], fmaf(pv[1], w1[1], fmaf(pv[2], w1[2], fmaf(pv[3], w1[3], a1))));
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

// dx = dpre Wp in kChunks row chunks of Wp: workgroup (c, g) covers rows [c H/kChunks, (c+1)
// H/kChunks) of Wp for the 8 sequences of group g -- each of its 8 waves an eighth of the rows, a
// Wp row loaded once for all 8 sequences -- then the waves are combined in LDS in fixed order
// -> part[b][c][:]
constexpr int kChunks = 8;
constexpr int kDxThreads = 512, kDxSeqs = 8;

__global__ void __launch_bounds__(kDxThreads)
    pool_dx_partial_kernel(const float* __restrict__ dpre, const float* __restrict__ Wp, int B, int H,
                           float* __restrict__ part) {
  constexpr int kMaxV = 4;  // H <= 1024
  constexpr int nw = kDxThreads / 64;
  extern __shared__ __attribute__((aligned(16))) float smp[];  // [8 waves][H]
  const int c = blockIdx.x, b0 = blockIdx.y * kDxSeqs, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rows = H / kChunks, per = (rows + nw - 1) / nw;
  const int r0 = c * rows + w * per, r1 = min(c * rows + rows, r0 + per);
  float acc[kDxSeqs][kMaxV][4];
#pragma unroll
  for (int u = 0; u < kDxSeqs; ++u)
#pragma unroll
    for (int v = 0; v < kMaxV; ++v) acc[u][v][0] = acc[u][v][1] = acc[u][v][2] = acc[u][v][3] = 0.f;
  for (int i = r0; i < r1; ++i) {
    float wv[kMaxV][4];
#pragma unroll
    for (int v = 0; v < kMaxV; ++v) {
      const int k = 4 * (lane + 64 * v);
      if (k < H) load4(Wp + (int64_t)i * H + k, wv[v]);
      else wv[v][0] = wv[v][1] = wv[v][2] = wv[v][3] = 0.f;
    }
#pragma unroll
    for (int u = 0; u < kDxSeqs; ++u) {
      const float d = b0 + u < B ? dpre[(int64_t)(b0 + u) * H + i] : 0.f;
#pragma unroll
      for (int v = 0; v < kMaxV; ++v)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[u][v][e] = fmaf(d, wv[v][e], acc[u][v][e]);
    }
  }
#pragma unroll
  for (int u = 0; u < kDxSeqs; ++u) {
    __syncthreads();
#pragma unroll
    for (int v = 0; v < kMaxV; ++v) {
      const int k = 4 * (lane + 64 * v);
      if (k < H) store4(smp + w * H + k, acc[u][v]);
    }
    __syncthreads();
    if (b0 + u < B)
      for (int k = threadIdx.x; k < H; k += kDxThreads) {
        float t = 0.f;
        for (int q = 0; q < nw; ++q) t += smp[q * H + k];  // fixed order
        part[((int64_t)(b0 + u) * kChunks + c) * H + k] = t;
      }
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

// blocks 0..H/4-1: dWp[i, :] (+)= sum_b dpre[b, i] x[b, :], dbp[i] (+)= sum_b dpre[b, i] for the
// block's 4 rows i (each first-token row x[b] loaded once for all four);
// blocks H/4, H/4+1: dWn[c, :] (+)= sum_b dlogits[b, c] pooled[b, :], dbn[c] (+)= sum_b dlogits[b, c].
constexpr int kWgRows = 4;

template <typename T>
__global__ void __launch_bounds__(kPoolThreads)
    pool_nsp_wgrad_kernel(const T* __restrict__ seq, const float* __restrict__ dpre, const float* __restrict__ dlogits,
                          const float* __restrict__ pooled, int B, int S, int H, float* __restrict__ dWp,
                          float* __restrict__ dbp, float* __restrict__ dWn, float* __restrict__ dbn, int accumulate) {
  constexpr int U = 8;  // sequences whose rows are loaded together
  const int nblk = H / kWgRows;
  const bool nsp = (int)blockIdx.x >= nblk;
  const int c = blockIdx.x - nblk;
  const int i0 = nsp ? 0 : blockIdx.x * kWgRows;
  for (int j = threadIdx.x * 4; j < H; j += kPoolThreads * 4) {
    float a[kWgRows][4];
#pragma unroll
    for (int r = 0; r < kWgRows; ++r) a[r][0] = a[r][1] = a[r][2] = a[r][3] = 0.f;
    for (int b0 = 0; b0 < B; b0 += U) {
      float v[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // all U row loads in flight before the FMAs
        const int b = min(b0 + u, B - 1);
        if (nsp) load4(pooled + (int64_t)b * H + j, v[u]);
        else load4(seq + (int64_t)b * S * H + j, v[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (b0 + u >= B) break;
#pragma unroll
        for (int r = 0; r < kWgRows; ++r) {
          const float d = nsp ? (r == 0 ? dlogits[2 * (b0 + u) + c] : 0.f) : dpre[(int64_t)(b0 + u) * H + i0 + r];
#pragma unroll
          for (int e = 0; e < 4; ++e) a[r][e] = fmaf(d, v[u][e], a[r][e]);
        }
      }
    }
    const int nr = nsp ? 1 : kWgRows;
#pragma unroll
    for (int r = 0; r < kWgRows; ++r) {
      if (r < nr) {
        float* out = nsp ? dWn + (int64_t)c * H : dWp + (int64_t)(i0 + r) * H;
        if (accumulate) {
          float o[4];
          load4(out + j, o);
          a[r][0] += o[0];
          a[r][1] += o[1];
          a[r][2] += o[2];
          a[r][3] += o[3];
        }
        store4(out + j, a[r]);
      }
    }
  }
  const int nr = nsp ? 1 : kWgRows;
  if ((int)threadIdx.x < nr) {
    const int r = threadIdx.x;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += nsp ? dlogits[2 * b + c] : dpre[(int64_t)b * H + i0 + r];
    float* bo = nsp ? dbn + c : dbp + i0 + r;
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
  const int waves = ((H + kPoolRows - 1) / kPoolRows) * ((B + kPoolSeqs - 1) / kPoolSeqs);
  const dim3 grid((waves + kPoolThreads / 64 - 1) / (kPoolThreads / 64));
  if (H % kPoolRows) return -1;
  if (dtype == 0)
    hipLaunchKernelGGL(pool_fwd_kernel<float>, grid, dim3(kPoolThreads), 0, st, (const float*)seq, B, S, H, Wp, bp,
                       pooled);
  else
    hipLaunchKernelGGL(pool_fwd_kernel<bf16_t>, grid, dim3(kPoolThreads), 0, st, (const bf16_t*)seq, B, S, H, Wp,
                       bp, pooled);
  hipLaunchKernelGGL(nsp_loss_kernel, dim3(1), dim3(kNspThreads), 0, st, pooled, Wn, bn, label, B, H, mlm_loss,
                     logits, lse, stats, total);
  return 0;
}

// the pooler / NSP parameter gradients alone (after the backward's nsp_bwd wrote dpre / dlogits):
// the fused BERT head runs them on the weight-gradient stream, off the data-gradient chain
void launch_pool_nsp_wgrad(int dtype, const void* seq, const float* dpre, const float* dlogits, const float* pooled,
                           int B, int S, int H, float* dWp, float* dbp, float* dWn, float* dbn, int accumulate,
                           hipStream_t st) {
  if (dtype == 0)
    hipLaunchKernelGGL(pool_nsp_wgrad_kernel<float>, dim3(H / kWgRows + 2), dim3(kPoolThreads), 0, st,
                       (const float*)seq, dpre, dlogits, pooled, B, S, H, dWp, dbp, dWn, dbn, accumulate);
  else
    hipLaunchKernelGGL(pool_nsp_wgrad_kernel<bf16_t>, dim3(H / kWgRows + 2), dim3(kPoolThreads), 0, st,
                       (const bf16_t*)seq, dpre, dlogits, pooled, B, S, H, dWp, dbp, dWn, dbn, accumulate);
}

// scratch: dlogits [B, 2], dpre [B, H], part [B, 8, H] floats
int launch_pool_nsp_bwd(int dtype, const float* dloss, const void* seq, void* dseq, int B, int S, int H,
                        const float* Wp, const float* Wn, const int64_t* label, const float* pooled,
                        const float* logits, const float* lse, const float* stats, float* dlogits, float* dpre,
                        float* part, float* dWp, float* dbp, float* dWn, float* dbn, int accumulate,
                        hipStream_t st, int with_wgrad) {
  if (B <= 0 || H <= 0 || H % 4 || H > 1024 || H % (kChunks * 4)) return -1;
  hipLaunchKernelGGL(nsp_bwd_kernel, dim3(B), dim3(kPoolThreads), 0, st, dloss, logits, lse, label, stats, pooled, Wn,
                     H, dlogits, dpre);
  hipLaunchKernelGGL(pool_dx_partial_kernel, dim3(kChunks, (B + kDxSeqs - 1) / kDxSeqs), dim3(kDxThreads),
                     (kDxThreads / 64) * (size_t)H * sizeof(float), st, dpre, Wp, B, H, part);
  if (dtype == 0)
    hipLaunchKernelGGL(pool_dx_finish_kernel<float>, dim3(B), dim3(kPoolThreads), 0, st, part, S, H, (float*)dseq);
  else
    hipLaunchKernelGGL(pool_dx_finish_kernel<bf16_t>, dim3(B), dim3(kPoolThreads), 0, st, part, S, H, (bf16_t*)dseq);
  if (with_wgrad)
    launch_pool_nsp_wgrad(dtype, seq, dpre, dlogits, pooled, B, S, H, dWp, dbp, dWn, dbn, accumulate, st);
  return 0;
}
