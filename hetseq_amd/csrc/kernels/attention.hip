// Fused scaled-dot-product attention for BERT on CDNA4 MFMA (K02, K09, K10).
//
// Reference (bert_modeling.py:351-377, 798-806): per head
//   scores = (Q K^T)/sqrt(d) + (1-mask)*-10000 ; probs = softmax(scores)
//   probs  = dropout(probs, p)                 ; ctx = probs V
// with Q/K/V produced by three separate Linear layers and permuted copies.
//
// Here the kernels read Q, K, V straight out of the fused QKV projection
// output [B*S, 3H] (no permute/contiguous copies), never materialise the
// [B,nh,S,S] probability tensor (online softmax, flash style), keep only a
// 1-bit-per-probability dropout mask (Philox keep decisions packed into one
// 32-bit word per query x 32 keys, 786 KB per BERT-base layer) for the
// backward pass, and write the context in the [B*S, H] layout the output
// projection consumes.  The QKV bias is added on load (no biased copy).
//
// MFMA mapping (v_mfma_f32_32x32x2_f32, exact fp32 -- the reference is fp32):
//  * a wave owns 32 rows (queries in fwd/dQ, keys in dK/dV); lane l holds row
//    (l & 31) and half of the head dim, d = 32*(l>>5) + kk, kk = 0..31, which is
//    exactly the A/B operand map of the 32x32x2 MFMA with a permuted k order;
//  * products are oriented ("swapped") so that the softmax row is the MFMA
//    COLUMN: the row max/sum is 15 in-register ops + one lane^32 shuffle, and
//    the score accumulator feeds the next MFMA as an operand with no LDS trip
//    (key order inside a k-step follows the C layout row(r) = (r&3)+8(r>>2)+4h);
//  * K/V (fwd, dQ) or Q/dO (dK/dV) are staged through LDS in chunks of up to
//    128 rows with a 68-float row stride (16-B reads conflict-free).
// Backward = two kernels, no atomics: dQ (also emits D = rowsum(dO*O)), then
// dK/dV.  Supports S % 32 == 0, S <= 512 chunked, head dim 64.
#include "common.h"

namespace hs {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kD = 64;    // head dim
constexpr int kLD = 68;   // LDS row stride (floats)
constexpr int kCH = 128;  // rows per LDS chunk

HS_DEVICE f32x16 mfma32(float a, float b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0); }

// key/query offset (within a 32-tile) held in accumulator register r by lane half hf
HS_DEVICE int crow(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }

// out[kk] = (src[kk] + bias[kk]) * scale for a 32-wide half row (bias may be null).
// The QKV projection bias is folded in here, so the projection GEMM runs
// without a bias epilogue and no biased copy of Q/K/V is ever written.
template <typename T>
HS_DEVICE void load_row_half(const T* src, const float* bias, float scale, float (&out)[32]) {
#pragma unroll
  for (int kk = 0; kk < 32; kk += 4) {
    float v[4], b[4] = {0.f, 0.f, 0.f, 0.f};
    load4(src + kk, v);
    if (bias) load4(bias + kk, b);
    out[kk] = (v[0] + b[0]) * scale;
    out[kk + 1] = (v[1] + b[1]) * scale;
    out[kk + 2] = (v[2] + b[2]) * scale;
    out[kk + 3] = (v[3] + b[3]) * scale;
  }
}

// Stage rows [r0, r0+n) of a head slice (column offset col) into LDS (fp32),
// adding the (nullable) per-column bias `bias` (already offset to `col`).
template <typename T>
HS_DEVICE void stage_rows(float* lds, const T* base, int64_t ld, int r0, int n, int col, const float* bias,
                          float scale) {
  for (int i = threadIdx.x; i < n * 16; i += blockDim.x) {
    const int r = i >> 4, c4 = (i & 15) * 4;
    float v[4], b[4] = {0.f, 0.f, 0.f, 0.f};
    load4(base + (int64_t)(r0 + r) * ld + col + c4, v);
    if (bias) load4(bias + c4, b);
    *reinterpret_cast<float4*>(lds + r * kLD + c4) =
        make_float4((v[0] + b[0]) * scale, (v[1] + b[1]) * scale, (v[2] + b[2]) * scale, (v[3] + b[3]) * scale);
  }
}

HS_DEVICE const float* boff(const float* b, int off) { return b ? b + off : nullptr; }

template <typename T>
__global__ void __launch_bounds__(256, 2)
    attn_fwd_kernel(const T* __restrict__ qkv, const int64_t* __restrict__ mask, const float* __restrict__ bqkv,
                    T* __restrict__ ctx, float* __restrict__ lse, uint32_t* __restrict__ dmask, int S, int NH, float p,
                    uint64_t seed, uint64_t off) {
  __shared__ __attribute__((aligned(16))) float Ks[kCH * kLD];
  __shared__ __attribute__((aligned(16))) float Vs[kCH * kLD];
  __shared__ float Ms[kCH];
  const int H = NH * kD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.y, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int q0 = blockIdx.x * 128 + w * 32;
  const bool active = q0 < S;
  const T* rows = qkv + (int64_t)b * S * ld;
  const float dscale = p < 1.f ? 1.f / (1.f - p) : 0.f;

  float qr[32];
  if (active) load_row_half(rows + (int64_t)(q0 + li) * ld + h * kD + hf * 32, boff(bqkv, h * kD + hf * 32), 0.125f, qr);
  f32x16 o0 = {}, o1 = {};
  float m = -1e30f, l = 0.f;
  const uint64_t erow = ((uint64_t)bh * S + (q0 + li)) * (uint64_t)S;

  for (int c0 = 0; c0 < S; c0 += kCH) {
    const int clen = min(kCH, S - c0);
    __syncthreads();
    stage_rows(Ks, rows, ld, c0, clen, H + h * kD, boff(bqkv, H + h * kD), 1.f);
    stage_rows(Vs, rows, ld, c0, clen, 2 * H + h * kD, boff(bqkv, 2 * H + h * kD), 1.f);
    for (int i = threadIdx.x; i < clen; i += blockDim.x)
      Ms[i] = (1.f - (float)mask[(int64_t)b * S + c0 + i]) * -10000.f;
    __syncthreads();
    if (!active) continue;
    for (int t = 0; t < clen; t += 32) {
      f32x16 s = {};
      const float* kp = Ks + (t + li) * kLD + hf * 32;
#pragma unroll
      for (int kk = 0; kk < 32; kk += 4) {
        const float4 k4 = *reinterpret_cast<const float4*>(kp + kk);
        s = mfma32(k4.x, qr[kk], s);
        s = mfma32(k4.y, qr[kk + 1], s);
        s = mfma32(k4.z, qr[kk + 2], s);
        s = mfma32(k4.w, qr[kk + 3], s);
      }
      float mt = -1e30f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[r] += Ms[t + crow(r, hf)];
        mt = fmaxf(mt, s[r]);
      }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m, mt);
      const float alpha = __expf(m - mn);
      m = mn;
      float pr[16];
      float ps = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        pr[r] = __expf(s[r] - mn);
        ps += pr[r];
      }
      ps += __shfl_xor(ps, 32, 64);
      l = l * alpha + ps;
      o0 *= alpha;
      o1 *= alpha;
      if (p > 0.f) {
        uint32_t bits = 0u;  // keep-bit of key (c0+t+k) at bit k, this lane's half
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float mk[4];
          keep4(seed, off, (erow + c0 + t + 8 * g + 4 * hf) >> 2, p, dscale, mk);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pr[4 * g + j] *= mk[j];
            bits |= (mk[j] != 0.f ? 1u : 0u) << (8 * g + 4 * hf + j);
          }
        }
        // one 32-bit word per (query, 32-key tile) for the backward kernels
        bits |= static_cast<uint32_t>(__shfl_xor(static_cast<int>(bits), 32, 64));
        if (dmask && hf == 0) dmask[((uint64_t)bh * S + q0 + li) * (uint64_t)(S >> 5) + ((c0 + t) >> 5)] = bits;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float* vp = Vs + (t + crow(r, hf)) * kLD;
        o0 = mfma32(vp[li], pr[r], o0);
        o1 = mfma32(vp[32 + li], pr[r], o1);
      }
    }
  }
  if (!active) return;
  const float inv = 1.f / l;
  T* out = ctx + ((int64_t)b * S + q0 + li) * H + h * kD;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * hf;
    float v0[4] = {o0[4 * g] * inv, o0[4 * g + 1] * inv, o0[4 * g + 2] * inv, o0[4 * g + 3] * inv};
    float v1[4] = {o1[4 * g] * inv, o1[4 * g + 1] * inv, o1[4 * g + 2] * inv, o1[4 * g + 3] * inv};
    store4(out + d, v0);
    store4(out + 32 + d, v1);
  }
  if (hf == 0) lse[(int64_t)bh * S + q0 + li] = m + __logf(l);
}

template <typename T>
__global__ void __launch_bounds__(256, 2)
    attn_bwd_dq_kernel(const T* __restrict__ qkv, const int64_t* __restrict__ mask, const float* __restrict__ bqkv,
                       const T* __restrict__ ctx,
                       const T* __restrict__ dctx, const float* __restrict__ lse, float* __restrict__ Dout,
                       T* __restrict__ dqkv, int S, int NH, float p, const uint32_t* __restrict__ dmask) {
  __shared__ __attribute__((aligned(16))) float Ks[kCH * kLD];
  __shared__ __attribute__((aligned(16))) float Vs[kCH * kLD];
  __shared__ float Ms[kCH];
  const int H = NH * kD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.y, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int q0 = blockIdx.x * 128 + w * 32;
  const bool active = q0 < S;
  const T* rows = qkv + (int64_t)b * S * ld;
  const float dscale = p < 1.f ? 1.f / (1.f - p) : 0.f;

  float qr[32], dor[32];
  float dsum = 0.f, lq = 0.f;
  if (active) {
    const int64_t tok = (int64_t)b * S + q0 + li;
    load_row_half(rows + (int64_t)(q0 + li) * ld + h * kD + hf * 32, boff(bqkv, h * kD + hf * 32), 0.125f, qr);
    load_row_half(dctx + tok * H + h * kD + hf * 32, nullptr, 1.f, dor);
    float orow[32];
    load_row_half(ctx + tok * H + h * kD + hf * 32, nullptr, 1.f, orow);
#pragma unroll
    for (int kk = 0; kk < 32; ++kk) dsum = fmaf(dor[kk], orow[kk], dsum);
    dsum += __shfl_xor(dsum, 32, 64);
    if (hf == 0) Dout[(int64_t)bh * S + q0 + li] = dsum;
    lq = lse[(int64_t)bh * S + q0 + li];
  }
  f32x16 dq0 = {}, dq1 = {};

  for (int c0 = 0; c0 < S; c0 += kCH) {
    const int clen = min(kCH, S - c0);
    __syncthreads();
    stage_rows(Ks, rows, ld, c0, clen, H + h * kD, boff(bqkv, H + h * kD), 1.f);
    stage_rows(Vs, rows, ld, c0, clen, 2 * H + h * kD, boff(bqkv, 2 * H + h * kD), 1.f);
    for (int i = threadIdx.x; i < clen; i += blockDim.x)
      Ms[i] = (1.f - (float)mask[(int64_t)b * S + c0 + i]) * -10000.f;
    __syncthreads();
    if (!active) continue;
    for (int t = 0; t < clen; t += 32) {
      f32x16 s = {}, dp = {};
      const float* kp = Ks + (t + li) * kLD + hf * 32;
      const float* vp = Vs + (t + li) * kLD + hf * 32;
#pragma unroll
      for (int kk = 0; kk < 32; kk += 4) {
        const float4 k4 = *reinterpret_cast<const float4*>(kp + kk);
        const float4 v4 = *reinterpret_cast<const float4*>(vp + kk);
        s = mfma32(k4.x, qr[kk], s);
        dp = mfma32(v4.x, dor[kk], dp);
        s = mfma32(k4.y, qr[kk + 1], s);
        dp = mfma32(v4.y, dor[kk + 1], dp);
        s = mfma32(k4.z, qr[kk + 2], s);
        dp = mfma32(v4.z, dor[kk + 2], dp);
        s = mfma32(k4.w, qr[kk + 3], s);
        dp = mfma32(v4.w, dor[kk + 3], dp);
      }
      float ds[16];
      if (p > 0.f) {
        const uint32_t word = dmask[((uint64_t)bh * S + q0 + li) * (uint64_t)(S >> 5) + ((c0 + t) >> 5)];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float mk = ((word >> crow(r, hf)) & 1u) ? dscale : 0.f;
          const float pv = __expf(s[r] + Ms[t + crow(r, hf)] - lq);
          ds[r] = pv * (dp[r] * mk - dsum);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pv = __expf(s[r] + Ms[t + crow(r, hf)] - lq);
          ds[r] = pv * (dp[r] - dsum);
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float* kr = Ks + (t + crow(r, hf)) * kLD;
        dq0 = mfma32(kr[li], ds[r], dq0);
        dq1 = mfma32(kr[32 + li], ds[r], dq1);
      }
    }
  }
  if (!active) return;
  T* out = dqkv + ((int64_t)b * S + q0 + li) * ld + h * kD;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * hf;
    float v0[4] = {dq0[4 * g] * 0.125f, dq0[4 * g + 1] * 0.125f, dq0[4 * g + 2] * 0.125f, dq0[4 * g + 3] * 0.125f};
    float v1[4] = {dq1[4 * g] * 0.125f, dq1[4 * g + 1] * 0.125f, dq1[4 * g + 2] * 0.125f, dq1[4 * g + 3] * 0.125f};
    store4(out + d, v0);
    store4(out + 32 + d, v1);
  }
}

template <typename T>
__global__ void __launch_bounds__(256, 2)
    attn_bwd_dkv_kernel(const T* __restrict__ qkv, const int64_t* __restrict__ mask, const float* __restrict__ bqkv,
                        const T* __restrict__ dctx,
                        const float* __restrict__ lse, const float* __restrict__ Dd, T* __restrict__ dqkv, int S,
                        int NH, float p, const uint32_t* __restrict__ dmask) {
  __shared__ __attribute__((aligned(16))) float Qs[kCH * kLD];
  __shared__ __attribute__((aligned(16))) float Os[kCH * kLD];
  __shared__ float Ls[kCH];
  __shared__ float Ds[kCH];
  const int H = NH * kD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.y, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int k0 = blockIdx.x * 128 + w * 32;
  const bool active = k0 < S;
  const int key = k0 + li;
  const T* rows = qkv + (int64_t)b * S * ld;
  const T* drows = dctx + (int64_t)b * S * H;
  const float dscale = p < 1.f ? 1.f / (1.f - p) : 0.f;

  float kr[32], vr[32];
  float madd = 0.f;
  if (active) {
    load_row_half(rows + (int64_t)key * ld + H + h * kD + hf * 32, boff(bqkv, H + h * kD + hf * 32), 1.f, kr);
    load_row_half(rows + (int64_t)key * ld + 2 * H + h * kD + hf * 32, boff(bqkv, 2 * H + h * kD + hf * 32), 1.f,
                  vr);
    madd = (1.f - (float)mask[(int64_t)b * S + key]) * -10000.f;
  }
  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};

  for (int c0 = 0; c0 < S; c0 += kCH) {
    const int clen = min(kCH, S - c0);
    __syncthreads();
    stage_rows(Qs, rows, ld, c0, clen, h * kD, boff(bqkv, h * kD), 0.125f);
    stage_rows(Os, drows, H, c0, clen, h * kD, nullptr, 1.f);
    for (int i = threadIdx.x; i < clen; i += blockDim.x) {
      Ls[i] = lse[(int64_t)bh * S + c0 + i];
      Ds[i] = Dd[(int64_t)bh * S + c0 + i];
    }
    __syncthreads();
    if (!active) continue;
    for (int t = 0; t < clen; t += 32) {
      f32x16 s = {}, dp = {};
      const float* qp = Qs + (t + li) * kLD + hf * 32;
      const float* op = Os + (t + li) * kLD + hf * 32;
#pragma unroll
      for (int kk = 0; kk < 32; kk += 4) {
        const float4 q4 = *reinterpret_cast<const float4*>(qp + kk);
        const float4 o4 = *reinterpret_cast<const float4*>(op + kk);
        s = mfma32(q4.x, kr[kk], s);
        dp = mfma32(o4.x, vr[kk], dp);
        s = mfma32(q4.y, kr[kk + 1], s);
        dp = mfma32(o4.y, vr[kk + 1], dp);
        s = mfma32(q4.z, kr[kk + 2], s);
        dp = mfma32(o4.z, vr[kk + 2], dp);
        s = mfma32(q4.w, kr[kk + 3], s);
        dp = mfma32(o4.w, vr[kk + 3], dp);
      }
      float pd[16], ds[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qi = t + crow(r, hf);
        const float pv = __expf(s[r] + madd - Ls[qi]);
        const float mk = p > 0.f ? (((dmask[((uint64_t)bh * S + c0 + qi) * (uint64_t)(S >> 5) + (key >> 5)] >>
                                       (key & 31)) & 1u) ? dscale : 0.f)
                                 : 1.f;
        pd[r] = pv * mk;
        ds[r] = pv * (dp[r] * mk - Ds[qi]);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qi = t + crow(r, hf);
        const float* orow = Os + qi * kLD;
        const float* qrow = Qs + qi * kLD;
        dv0 = mfma32(orow[li], pd[r], dv0);
        dv1 = mfma32(orow[32 + li], pd[r], dv1);
        dk0 = mfma32(qrow[li], ds[r], dk0);
        dk1 = mfma32(qrow[32 + li], ds[r], dk1);
      }
    }
  }
  if (!active) return;
  T* outk = dqkv + ((int64_t)b * S + key) * ld + H + h * kD;
  T* outv = dqkv + ((int64_t)b * S + key) * ld + 2 * H + h * kD;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * hf;
    float a0[4] = {dk0[4 * g], dk0[4 * g + 1], dk0[4 * g + 2], dk0[4 * g + 3]};
    float a1[4] = {dk1[4 * g], dk1[4 * g + 1], dk1[4 * g + 2], dk1[4 * g + 3]};
    float c0v[4] = {dv0[4 * g], dv0[4 * g + 1], dv0[4 * g + 2], dv0[4 * g + 3]};
    float c1v[4] = {dv1[4 * g], dv1[4 * g + 1], dv1[4 * g + 2], dv1[4 * g + 3]};
    store4(outk + d, a0);
    store4(outk + 32 + d, a1);
    store4(outv + d, c0v);
    store4(outv + 32 + d, c1v);
  }
}

}  // namespace hs

using namespace hs;

// dmask: uint32 keep-bits [B*NH*S*(S/32)] written by the forward when p > 0
// and read by both backward kernels (required when p > 0).
int launch_attn_fwd(int dtype, const void* qkv, const int64_t* mask, const float* bqkv, void* ctx, float* lse,
                    uint32_t* dmask, int B, int S, int NH, int D, float p, uint64_t seed, uint64_t off,
                    hipStream_t st) {
  if (D != kD || S % 32 != 0 || S <= 0) return -1;
  dim3 grid((S + 127) / 128, B * NH);
  if (dtype == 0)
    hipLaunchKernelGGL(attn_fwd_kernel<float>, grid, dim3(256), 0, st, (const float*)qkv, mask, bqkv, (float*)ctx,
                       lse, dmask, S, NH, p, seed, off);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)qkv, mask, bqkv,
                       (bf16_t*)ctx, lse, dmask, S, NH, p, seed, off);
  return 0;
}

int launch_attn_bwd(int dtype, const void* qkv, const int64_t* mask, const float* bqkv, const void* ctx,
                    const void* dctx, const float* lse, float* Dbuf, void* dqkv, const uint32_t* dmask, int B, int S,
                    int NH, int D, float p, hipStream_t st) {
  if (D != kD || S % 32 != 0 || S <= 0 || (p > 0.f && dmask == nullptr)) return -1;
  dim3 grid((S + 127) / 128, B * NH);
  if (dtype == 0) {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<float>, grid, dim3(256), 0, st, (const float*)qkv, mask, bqkv,
                       (const float*)ctx, (const float*)dctx, lse, Dbuf, (float*)dqkv, S, NH, p, dmask);
    hipLaunchKernelGGL(attn_bwd_dkv_kernel<float>, grid, dim3(256), 0, st, (const float*)qkv, mask, bqkv,
                       (const float*)dctx, lse, Dbuf, (float*)dqkv, S, NH, p, dmask);
  } else {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)qkv, mask, bqkv,
                       (const bf16_t*)ctx, (const bf16_t*)dctx, lse, Dbuf, (bf16_t*)dqkv, S, NH, p, dmask);
    hipLaunchKernelGGL(attn_bwd_dkv_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)qkv, mask, bqkv,
                       (const bf16_t*)dctx, lse, Dbuf, (bf16_t*)dqkv, S, NH, p, dmask);
  }
  return 0;
}
