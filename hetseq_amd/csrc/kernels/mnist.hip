// MNISTNet on gfx950 (K15; reference tasks.py:337-362, eval_mnist.py:9-37), fp32 throughout:
//   conv(1->32, 3x3) + ReLU -> conv(32->64, 3x3) + ReLU -> maxpool 2 -> Dropout2d(0.25)
//   -> flatten -> fc(9216->128) + ReLU -> dropout(0.5) -> fc(128->10) -> log_softmax -> NLL.
//
// The network is a few MFLOP per image, so it is organised around the two products that carry
// the work -- conv2 as an implicit GEMM over an im2col matrix [R, 320] (R = B*576 rows padded to
// a multiple of 2048 so the weight-gradient product splits K 64 ways; K = 9*32 = 288 padded to
// 320 with zero columns so every GEMM dimension tiles by 64/32) and fc1 -- which run on the
// exact-fp32 MFMA GEMM (gemm.hip), with every elementwise stage fused into a small kernel around
// them.  Activations are channel-last (NHWC), so every gather / scatter is a run of 32 or 64
// contiguous floats:
//   conv1_fwd_kernel      direct 3x3 conv + bias + ReLU -> h1 [B,26,26,32] (one thread per output)
//   im2col_kernel         h1 -> [R, 320] rows (b, y, x), columns (ky*3 + kx)*32 + ci (float4 runs)
//   pool_fwd_kernel       conv2 GEMM output [R, 64] -> ReLU -> 2x2 max (first max wins, as torch)
//                         -> Dropout2d keep per (b, c) -> [Bp, 9216] in (y, x, c) order (fc1's
//                         weight columns are permuted to match); the argmax slot is kept
//   head_fwd_kernel       one wave per row: ReLU + dropout on fc1 output, fc2, log_softmax, NLL
//   head_bwd_kernel       dlogits = (softmax - onehot) * g, dh = dlogits W2, ReLU / dropout masks
//   fc2_wgrad_*_kernel    dW2 = dlogits^T h, db2: 64 batch chunks, then a fixed-order sum
//   pool_bwd_kernel       route the pooled gradient to each window's argmax (others 0)
//   col2im_kernel         dh1[b,iy,ix,:] = sum of the dcol runs that read it (a gather in a fixed
//                         order: no atomics), times conv1's ReLU mask
//   conv1_wgrad_*_kernel  dW1 / db1: 1024 position chunks x 32 channels, then a fixed-order sum
//   perm_cols_kernel      weight layout glue (conv2 filter <-> padded (ky,kx,ci) columns, fc1
//                         columns (c,y,x) <-> (y,x,c))
// Dropout keep decisions are Philox draws (common.h keep4) keyed by (seed, site offset, element),
// so a step is reproducible from its seed.
#include <algorithm>

#include "common.h"

namespace hs {

constexpr int kC1 = 32, kC2 = 64, kIn = 28, kO1 = 26, kO2 = 24, kP = 12;
constexpr int kKc = kC1 * 9, kKp = 320;     // conv2 reduction length, padded
constexpr int kFlat = kC2 * kP * kP;       // 9216
constexpr int kHid = 128, kCls = 10;

__global__ void __launch_bounds__(256) conv1_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ b, float* __restrict__ y, int B) {
  const int64_t n = (int64_t)B * kO1 * kO1 * kC1;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i & (kC1 - 1));
    const int64_t pos = i >> 5;
    const int xo = (int)(pos % kO1), yo = (int)((pos / kO1) % kO1);
    const int64_t bb = pos / (kO1 * kO1);
    const float* in = x + bb * kIn * kIn + yo * kIn + xo;
    const float* f = w + c * 9;
    float a = b[c];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) a = fmaf(f[ky * 3 + kx], in[ky * kIn + kx], a);
    y[i] = fmaxf(a, 0.f);
  }
}

// rows r < B*576 gather 9 runs of 32 channels; pad columns and pad rows r >= B*576 are zero
__global__ void __launch_bounds__(256) im2col_kernel(const float* __restrict__ h1, float* __restrict__ col, int B,
                                                     int R) {
  const int64_t n = (int64_t)R * (kKp / 4), valid = (int64_t)B * kO2 * kO2;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int k4 = (int)(i % (kKp / 4));
    const int64_t r = i / (kKp / 4);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (k4 < kKc / 4 && r < valid) {
      const int kk = k4 >> 3, ci = (k4 & 7) * 4, ky = kk / 3, kx = kk % 3;
      const int xo = (int)(r % kO2), yo = (int)((r / kO2) % kO2);
      const int64_t bb = r / (kO2 * kO2);
      v = *reinterpret_cast<const float4*>(h1 + ((bb * kO1 + yo + ky) * kO1 + xo + kx) * kC1 + ci);
    }
    *reinterpret_cast<float4*>(col + i * 4) = v;
  }
}

// dst[r][j] = src[r][source column of j] (0 where there is none); mode 0: conv2 filter
// [64, (ci,ky,kx)=288] -> [64, (ky,kx,ci) + 32 zero = 320]; 1: its inverse (320 -> 288);
// 2: fc1 columns (c, y, x) -> (y, x, c); 3: the inverse
__global__ void __launch_bounds__(256) perm_cols_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                        int rows, int mode) {
  const int dcols = mode == 0 ? kKp : mode == 1 ? kKc : kFlat;
  const int scols = mode == 0 ? kKc : mode == 1 ? kKp : kFlat;
  const int64_t n = (int64_t)rows * dcols;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / dcols;
    const int j = (int)(i % dcols);
    int sj;
    if (mode == 0)
      sj = j < kKc ? (j & 31) * 9 + (j >> 5) : -1;
    else if (mode == 1)
      sj = (j % 9) * kC1 + j / 9;
    else if (mode == 2)
      sj = (j & (kC2 - 1)) * (kP * kP) + (j >> 6);
    else
      sj = (j % (kP * kP)) * kC2 + j / (kP * kP);
    dst[i] = sj >= 0 ? src[r * scols + sj] : 0.f;
  }
}

// one thread per pooled element (b, y, x, c) -- channel fastest, so the four window reads and the
// write are contiguous runs; rows >= B of the [Bp, 9216] output are zero
__global__ void __launch_bounds__(256) pool_fwd_kernel(const float* __restrict__ c2, float* __restrict__ pooled,
                                                       uint8_t* __restrict__ arg, int B, int Bp, float p,
                                                       uint64_t seed, uint64_t off) {
  const int64_t n = (int64_t)Bp * kFlat;
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int j = (int)(i % kFlat), c = j & (kC2 - 1), px = (j >> 6) % kP, py = (j >> 6) / kP;
    const int64_t bb = i / kFlat;
    if (bb >= B) {
      pooled[i] = 0.f;
      continue;
    }
    const float* base = c2 + ((bb * kO2 + 2 * py) * kO2 + 2 * px) * kC2 + c;
    float m = base[0];
    int a = 0;
    const float v1 = base[kC2], v2 = base[kO2 * kC2], v3 = base[kO2 * kC2 + kC2];
    if (v1 > m) { m = v1; a = 1; }
    if (v2 > m) { m = v2; a = 2; }
    if (v3 > m) { m = v3; a = 3; }
    float keep = 1.f;
    if (p > 0.f) {  // Dropout2d: one draw per (b, c) channel
      const int64_t q = bb * kC2 + c;
      float k4[4];
      keep4(seed, off, (uint64_t)(q >> 2), p, scale, k4);
      keep = k4[q & 3];
    }
    pooled[i] = fmaxf(m, 0.f) * keep;
    arg[i] = static_cast<uint8_t>(a | (m > 0.f ? 4 : 0) | (keep != 0.f ? 8 : 0));
  }
}

// dc2 rows B*576 .. R-1 (GEMM padding) are written as zero
__global__ void __launch_bounds__(256) pool_bwd_kernel(const float* __restrict__ dpooled,
                                                       const uint8_t* __restrict__ arg, float* __restrict__ dc2, int B,
                                                       int R, float p) {
  const int64_t n = (int64_t)B * kFlat;
  const float scale = p > 0.f && p < 1.f ? 1.f / (1.f - p) : 1.f;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int j = (int)(i % kFlat), c = j & (kC2 - 1), px = (j >> 6) % kP, py = (j >> 6) / kP;
    const int64_t bb = i / kFlat;
    const int a = arg[i];
    const float g = ((a & 4) && (a & 8)) ? dpooled[i] * scale : 0.f;
    float* base = dc2 + ((bb * kO2 + 2 * py) * kO2 + 2 * px) * kC2 + c;
    base[0] = (a & 3) == 0 ? g : 0.f;
    base[kC2] = (a & 3) == 1 ? g : 0.f;
    base[kO2 * kC2] = (a & 3) == 2 ? g : 0.f;
    base[kO2 * kC2 + kC2] = (a & 3) == 3 ? g : 0.f;
  }
  const int64_t v0 = (int64_t)B * kO2 * kO2 * kC2, v1 = (int64_t)R * kC2;
  for (int64_t i = v0 + blockIdx.x * 256ll + threadIdx.x; i < v1; i += (int64_t)gridDim.x * 256) dc2[i] = 0.f;
}

// one wave per row b < B: h = relu(pre + 0) * keep (fc1 bias already in pre), logits = h W2^T + b2,
// logp = log_softmax(logits); nll[b] = -logp[target] (0 for ignored targets < 0)
__global__ void __launch_bounds__(256) head_fwd_kernel(const float* __restrict__ pre, const float* __restrict__ w2,
                                                       const float* __restrict__ b2, const int64_t* __restrict__ target,
                                                       float* __restrict__ h, float* __restrict__ logp,
                                                       float* __restrict__ nll, int B, float p, uint64_t seed,
                                                       uint64_t off) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  float hv[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int j = lane + 64 * e;
    float keep = 1.f;
    if (p > 0.f) {
      const int64_t q = (int64_t)row * kHid + j;
      float k4[4];
      keep4(seed, off, (uint64_t)(q >> 2), p, scale, k4);
      keep = k4[q & 3];
    }
    hv[e] = fmaxf(pre[(int64_t)row * kHid + j], 0.f) * keep;
    h[(int64_t)row * kHid + j] = hv[e];
  }
  float lg[kCls];
  float mx = -3.4e38f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) {
    lg[c] = wave_sum(hv[0] * w2[c * kHid + lane] + hv[1] * w2[c * kHid + 64 + lane]) + b2[c];
    mx = fmaxf(mx, lg[c]);
  }
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) se += __expf(lg[c] - mx);
  const float lse = mx + __logf(se);
  if (lane < kCls) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c)
      if (c == lane) v = lg[c] - lse;
    logp[(int64_t)row * kCls + lane] = v;
  }
  if (lane == 0) {
    const int64_t t = target[row];
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c)
      if (c == t) v = lse - lg[c];
    nll[row] = t >= 0 && t < kCls ? v : 0.f;
  }
}

// loss[0] = sum (or mean over valid targets) of nll; correct[0] = argmax hits (eval) -- one
// workgroup, fixed-order reduction
__global__ void __launch_bounds__(256) loss_reduce_kernel(const float* __restrict__ nll, const float* __restrict__ logp,
                                                          const int64_t* __restrict__ target, int B, int mean,
                                                          float* __restrict__ loss, float* __restrict__ correct,
                                                          float* __restrict__ count) {
  __shared__ float r0[256], r1[256], r2[256];
  float s = 0.f, cor = 0.f, cnt = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) {
    const int64_t t = target[b];
    if (t < 0 || t >= kCls) continue;
    s += nll[b];
    cnt += 1.f;
    int am = 0;
    float best = logp[(int64_t)b * kCls];
    for (int c = 1; c < kCls; ++c)
      if (logp[(int64_t)b * kCls + c] > best) { best = logp[(int64_t)b * kCls + c]; am = c; }
    cor += am == t ? 1.f : 0.f;
  }
  r0[threadIdx.x] = s;
  r1[threadIdx.x] = cor;
  r2[threadIdx.x] = cnt;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      r0[threadIdx.x] += r0[threadIdx.x + w];
      r1[threadIdx.x] += r1[threadIdx.x + w];
      r2[threadIdx.x] += r2[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    loss[0] = mean ? r0[0] / r2[0] : r0[0];
    correct[0] = r1[0];
    count[0] = r2[0];
  }
}

// one wave per row b < Bp: dlogits = (softmax - onehot) * g (g = dloss / count for the mean),
// dpre = (dlogits W2) * relu'(pre) * keep; rows >= B write zeros
__global__ void __launch_bounds__(256) head_bwd_kernel(const float* __restrict__ dloss, const float* __restrict__ count,
                                                       const float* __restrict__ logp, const int64_t* __restrict__ target,
                                                       const float* __restrict__ pre, const float* __restrict__ h,
                                                       const float* __restrict__ w2, float* __restrict__ dlogits,
                                                       float* __restrict__ dpre, int B, int Bp, int mean, float p) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= Bp) return;
  if (row >= B) {
    if (lane < kCls) dlogits[(int64_t)row * kCls + lane] = 0.f;
    dpre[(int64_t)row * kHid + lane] = 0.f;
    dpre[(int64_t)row * kHid + 64 + lane] = 0.f;
    return;
  }
  const int64_t t = target[row];
  const bool valid = t >= 0 && t < kCls;
  const float g = valid ? (mean ? dloss[0] / count[0] : dloss[0]) : 0.f;
  float dl[kCls];
#pragma unroll
  for (int c = 0; c < kCls; ++c) dl[c] = g * (__expf(logp[(int64_t)row * kCls + c]) - (c == t ? 1.f : 0.f));
  if (lane < kCls) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c)
      if (c == lane) v = dl[c];
    dlogits[(int64_t)row * kCls + lane] = v;
  }
  const float scale = p > 0.f && p < 1.f ? 1.f / (1.f - p) : 1.f;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int j = lane + 64 * e;
    float dh = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c) dh = fmaf(dl[c], w2[c * kHid + j], dh);
    // h = relu(pre) * keep: d/dpre = keep * [pre > 0]; keep = h / relu(pre) (0 or scale)
    const float pr = pre[(int64_t)row * kHid + j];
    const float keep = p > 0.f ? (h[(int64_t)row * kHid + j] != 0.f ? scale : 0.f) : 1.f;
    dpre[(int64_t)row * kHid + j] = pr > 0.f ? dh * keep : 0.f;
  }
}

// dW2[c][j] = sum_b dlogits[b][c] h[b][j], db2[c] = sum_b dlogits[b][c].  Stage 1: block g owns a
// contiguous chunk of the batch rows, thread j accumulates all 10 classes of hidden unit j (threads
// 0..9 also the bias partial of class j) -> part[g][c*128 + j], part[g][1280 + c]; stage 2 sums the
// chunks in order: deterministic.
constexpr int kFcChunks = 64, kFcPart = kCls * kHid + kCls;
__global__ void __launch_bounds__(kHid) fc2_wgrad_part_kernel(const float* __restrict__ dlogits,
                                                             const float* __restrict__ h, float* __restrict__ part,
                                                             int B) {
  const int j = threadIdx.x, per = (B + kFcChunks - 1) / kFcChunks;
  const int b0 = blockIdx.x * per, b1 = min(B, b0 + per);
  float acc[kCls], sb = 0.f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) acc[c] = 0.f;
  for (int b = b0; b < b1; ++b) {
    const float hv = h[(int64_t)b * kHid + j];
    const float* d = dlogits + (int64_t)b * kCls;
#pragma unroll
    for (int c = 0; c < kCls; ++c) acc[c] = fmaf(d[c], hv, acc[c]);
    if (j < kCls) sb += d[j];
  }
  float* out = part + (int64_t)blockIdx.x * kFcPart;
#pragma unroll
  for (int c = 0; c < kCls; ++c) out[c * kHid + j] = acc[c];
  if (j < kCls) out[kCls * kHid + j] = sb;
}

__global__ void __launch_bounds__(256) fc2_wgrad_final_kernel(const float* __restrict__ part, float* __restrict__ dw2,
                                                              float* __restrict__ db2) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= kFcPart) return;
  float s = 0.f;
  for (int g = 0; g < kFcChunks; ++g) s += part[g * kFcPart + e];
  if (e < kCls * kHid)
    dw2[e] = s;
  else
    db2[e - kCls * kHid] = s;
}

// one thread per 4 channels of one h1 position: 9 float4 reads of the dcol runs that read it
__global__ void __launch_bounds__(256) col2im_kernel(const float* __restrict__ dcol, const float* __restrict__ h1,
                                                     float* __restrict__ dh1, int B) {
  const int64_t n = (int64_t)B * kO1 * kO1 * (kC1 / 4);
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int ci = (int)(i & 7) * 4;
    const int64_t pos = i >> 3;
    const int ix = (int)(pos % kO1), iy = (int)((pos / kO1) % kO1);
    const int64_t bb = pos / (kO1 * kO1);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int y = iy - ky, x = ix - kx;
        if (y >= 0 && y < kO2 && x >= 0 && x < kO2) {
          const float4 d =
              *reinterpret_cast<const float4*>(dcol + ((bb * kO2 + y) * kO2 + x) * kKp + (ky * 3 + kx) * kC1 + ci);
          s.x += d.x;
          s.y += d.y;
          s.z += d.z;
          s.w += d.w;
        }
      }
    const float4 h = *reinterpret_cast<const float4*>(h1 + i * 4);
    float4 o;
    o.x = h.x > 0.f ? s.x : 0.f;
    o.y = h.y > 0.f ? s.y : 0.f;
    o.z = h.z > 0.f ? s.z : 0.f;
    o.w = h.w > 0.f ? s.w : 0.f;
    *reinterpret_cast<float4*>(dh1 + i * 4) = o;
  }
}

// dW1[co][k] = sum_{b,y,x} dh1[b][y][x][co] x[b][y+ky][x+kx], db1[co] = sum dh1.  Stage 1: block g
// owns a contiguous chunk of the B*676 positions; thread (sub, c) walks every 8th position of it
// for channel c (a 128-B run of dh1 per position, x broadcast), then the 8 sub-partials are summed
// in a fixed order -> part[g][k*32 + c].  Stage 2 sums the chunks in order: deterministic.
constexpr int kWgChunks = 1024;
__global__ void __launch_bounds__(256) conv1_wgrad_part_kernel(const float* __restrict__ dh1,
                                                               const float* __restrict__ x, float* __restrict__ part,
                                                               int B) {
  __shared__ float red[8][10 * kC1];
  const int c = threadIdx.x & (kC1 - 1), sub = threadIdx.x >> 5;
  const int64_t npos = (int64_t)B * kO1 * kO1, per = (npos + kWgChunks - 1) / kWgChunks;
  const int64_t p0 = blockIdx.x * per, p1 = std::min<int64_t>(npos, p0 + per);
  float acc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = 0.f;
  for (int64_t q = p0 + sub; q < p1; q += 8) {
    const int xo = (int)(q % kO1), yo = (int)((q / kO1) % kO1);
    const int64_t bb = q / (kO1 * kO1);
    const float g = dh1[q * kC1 + c];
    const float* in = x + bb * kIn * kIn + yo * kIn + xo;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) acc[ky * 3 + kx] = fmaf(g, in[ky * kIn + kx], acc[ky * 3 + kx]);
    acc[9] += g;
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) red[sub][k * kC1 + c] = acc[k];
  __syncthreads();
  for (int j = threadIdx.x; j < 10 * kC1; j += 256) {
    float s = red[0][j];
#pragma unroll
    for (int t = 1; t < 8; ++t) s += red[t][j];
    part[(int64_t)blockIdx.x * 10 * kC1 + j] = s;
  }
}

// block k (0..9) finishes entry k of every channel: thread (sub, c) sums chunks sub, sub+8, ...,
// then the 8 partials are added in a fixed order
__global__ void __launch_bounds__(256) conv1_wgrad_final_kernel(const float* __restrict__ part,
                                                                float* __restrict__ dw1, float* __restrict__ db1) {
  __shared__ float red[8][kC1];
  const int k = blockIdx.x, c = threadIdx.x & (kC1 - 1), sub = threadIdx.x >> 5, j = k * kC1 + c;
  float s = 0.f;
  for (int g = sub; g < kWgChunks; g += 8) s += part[g * 10 * kC1 + j];
  red[sub][c] = s;
  __syncthreads();
  if (sub == 0) {
#pragma unroll
    for (int t = 1; t < 8; ++t) s += red[t][c];
    if (k < 9)
      dw1[c * 9 + k] = s;
    else
      db1[c] = s;
  }
}

static int grid_for(int64_t n) { return (int)std::min<int64_t>((n + 255) / 256, 8192); }

}  // namespace hs

using namespace hs;

void launch_mnist_conv1_fwd(const float* x, const float* w, const float* b, float* y, int B, hipStream_t st) {
  hipLaunchKernelGGL(conv1_fwd_kernel, dim3(grid_for((int64_t)B * kC1 * kO1 * kO1)), dim3(256), 0, st, x, w, b, y, B);
}
void launch_mnist_im2col(const float* h1, float* col, int B, int R, hipStream_t st) {
  hipLaunchKernelGGL(im2col_kernel, dim3(grid_for((int64_t)R * (kKp / 4))), dim3(256), 0, st, h1, col, B, R);
}
void launch_mnist_perm(const float* src, float* dst, int rows, int mode, hipStream_t st) {
  const int dcols = mode == 0 ? kKp : mode == 1 ? kKc : kFlat;
  hipLaunchKernelGGL(perm_cols_kernel, dim3(grid_for((int64_t)rows * dcols)), dim3(256), 0, st, src, dst, rows, mode);
}
void launch_mnist_pool_fwd(const float* c2, float* pooled, uint8_t* arg, int B, int Bp, float p, uint64_t seed,
                           uint64_t off, hipStream_t st) {
  hipLaunchKernelGGL(pool_fwd_kernel, dim3(grid_for((int64_t)Bp * kFlat)), dim3(256), 0, st, c2, pooled, arg, B, Bp, p,
                     seed, off);
}
void launch_mnist_pool_bwd(const float* dpooled, const uint8_t* arg, float* dc2, int B, int R, float p,
                           hipStream_t st) {
  hipLaunchKernelGGL(pool_bwd_kernel, dim3(grid_for((int64_t)B * kFlat)), dim3(256), 0, st, dpooled, arg, dc2, B, R, p);
}
void launch_mnist_head_fwd(const float* pre, const float* w2, const float* b2, const int64_t* target, float* h,
                           float* logp, float* nll, int B, float p, uint64_t seed, uint64_t off, hipStream_t st) {
  hipLaunchKernelGGL(head_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, st, pre, w2, b2, target, h, logp, nll, B, p,
                     seed, off);
}
void launch_mnist_loss(const float* nll, const float* logp, const int64_t* target, int B, int mean, float* loss,
                       float* correct, float* count, hipStream_t st) {
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(256), 0, st, nll, logp, target, B, mean, loss, correct, count);
}
void launch_mnist_head_bwd(const float* dloss, const float* count, const float* logp, const int64_t* target,
                           const float* pre, const float* h, const float* w2, float* dlogits, float* dpre, int B,
                           int Bp, int mean, float p, hipStream_t st) {
  hipLaunchKernelGGL(head_bwd_kernel, dim3((Bp + 3) / 4), dim3(256), 0, st, dloss, count, logp, target, pre, h, w2,
                     dlogits, dpre, B, Bp, mean, p);
}
// part: kFcChunks * kFcPart floats of scratch (the conv1 weight-gradient scratch is larger and reused)
void launch_mnist_fc2_wgrad(const float* dlogits, const float* h, float* part, float* dw2, float* db2, int B,
                            hipStream_t st) {
  hipLaunchKernelGGL(fc2_wgrad_part_kernel, dim3(kFcChunks), dim3(kHid), 0, st, dlogits, h, part, B);
  hipLaunchKernelGGL(fc2_wgrad_final_kernel, dim3((kFcPart + 255) / 256), dim3(256), 0, st, part, dw2, db2);
}
void launch_mnist_col2im(const float* dcol, const float* h1, float* dh1, int B, hipStream_t st) {
  hipLaunchKernelGGL(col2im_kernel, dim3(grid_for((int64_t)B * kO1 * kO1 * (kC1 / 4))), dim3(256), 0, st, dcol, h1,
                     dh1, B);
}
// part: kWgChunks * 320 floats of scratch
void launch_mnist_conv1_wgrad(const float* dh1, const float* x, float* part, float* dw1, float* db1, int B,
                              hipStream_t st) {
  hipLaunchKernelGGL(conv1_wgrad_part_kernel, dim3(kWgChunks), dim3(256), 0, st, dh1, x, part, B);
  hipLaunchKernelGGL(conv1_wgrad_final_kernel, dim3(10), dim3(256), 0, st, part, dw1, db1);
}
