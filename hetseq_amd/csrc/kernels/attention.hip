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
#include <cstdlib>
#include <string>

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

// Stage rows [r0, r0+n) (n <= 128) of a head slice (column offset col) into LDS
// (fp32), adding the (nullable) per-column bias `bias` (already offset to `col`).
// All of a thread's global loads are issued before any LDS store (one memory
// round trip per staging instead of one per row group).  NT = block size.
template <int NT, typename T>
HS_DEVICE void stage_rows(float* lds, const T* base, int64_t ld, int r0, int n, int col, const float* bias,
                          float scale) {
  constexpr int kPer = 128 * 16 / NT;  // float4 units per thread for a full 128-row chunk
  const int c4 = (threadIdx.x & 15) * 4;  // NT % 16 == 0: a thread always owns the same 4 columns
  float b[4] = {0.f, 0.f, 0.f, 0.f};
  if (bias) load4(bias + c4, b);
  float v[kPer][4];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {  // unconditional loads (row clamped): keeps v[] in registers
    const int r = min((threadIdx.x + i * NT) >> 4, n - 1);
    load4(base + (int64_t)(r0 + r) * ld + col + c4, v[i]);
  }
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int r = (threadIdx.x + i * NT) >> 4;
    if (r < n)
      *reinterpret_cast<float4*>(lds + r * kLD + c4) = make_float4((v[i][0] + b[0]) * scale, (v[i][1] + b[1]) * scale,
                                                                   (v[i][2] + b[2]) * scale, (v[i][3] + b[3]) * scale);
  }
}

// Two stagings with all loads of both in flight before the first LDS store.
template <int NT, typename T1, typename T2>
HS_DEVICE void stage_rows2(float* l1, const T1* b1, int64_t ld1, int col1, const float* bias1, float sc1, float* l2,
                           const T2* b2, int64_t ld2, int col2, const float* bias2, float sc2, int r0, int n) {
  constexpr int kPer = 128 * 16 / NT;
  const int c4 = (threadIdx.x & 15) * 4;
  float ba[4] = {0.f, 0.f, 0.f, 0.f}, bb[4] = {0.f, 0.f, 0.f, 0.f};
  if (bias1) load4(bias1 + c4, ba);
  if (bias2) load4(bias2 + c4, bb);
  float v1[kPer][4], v2[kPer][4];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {  // unconditional loads (row clamped): keeps v1/v2 in registers
    const int r = min((threadIdx.x + i * NT) >> 4, n - 1);
    load4(b1 + (int64_t)(r0 + r) * ld1 + col1 + c4, v1[i]);
    load4(b2 + (int64_t)(r0 + r) * ld2 + col2 + c4, v2[i]);
  }
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int r = (threadIdx.x + i * NT) >> 4;
    if (r < n) {
      *reinterpret_cast<float4*>(l1 + r * kLD + c4) = make_float4((v1[i][0] + ba[0]) * sc1, (v1[i][1] + ba[1]) * sc1,
                                                                  (v1[i][2] + ba[2]) * sc1, (v1[i][3] + ba[3]) * sc1);
      *reinterpret_cast<float4*>(l2 + r * kLD + c4) = make_float4((v2[i][0] + bb[0]) * sc2, (v2[i][1] + bb[1]) * sc2,
                                                                  (v2[i][2] + bb[2]) * sc2, (v2[i][3] + bb[3]) * sc2);
    }
  }
}

HS_DEVICE const float* boff(const float* b, int off) { return b ? b + off : nullptr; }

template <typename T>
__global__ void __launch_bounds__(256, 2)
    attn_fwd_kernel(const T* __restrict__ qkv, const int64_t* __restrict__ mask, const float* __restrict__ bqkv,
                    T* __restrict__ ctx, float* __restrict__ lse, uint32_t* __restrict__ dmask, int S, int NH, float p,
                    uint64_t seed, uint64_t off, const uint64_t* __restrict__ seed_dev, int bh0) {
  seed = resolve_seed(seed, seed_dev);
  __shared__ __attribute__((aligned(16))) float Ks[kCH * kLD];
  __shared__ __attribute__((aligned(16))) float Vs[kCH * kLD];
  __shared__ float Ms[kCH];
  const int H = NH * kD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int q0 = blockIdx.y * 128 + w * 32;
  const bool active = q0 < S;
  const T* rows = qkv + (int64_t)b * S * ld;
  const uint32_t thr = drop_thr16(p);
  const float dscale = drop_scale16(thr);

  float qr[32];
  if (active) load_row_half(rows + (int64_t)(q0 + li) * ld + h * kD + hf * 32, boff(bqkv, h * kD + hf * 32), 0.125f, qr);
  f32x16 o0 = {}, o1 = {};
  float m = -1e30f, l = 0.f;
  const uint64_t erow = ((uint64_t)(bh0 + bh) * S + (q0 + li)) * (uint64_t)S;  // bh0: a batch slice's first head

  for (int c0 = 0; c0 < S; c0 += kCH) {
    const int clen = min(kCH, S - c0);
    __syncthreads();
    stage_rows2<256>(Ks, rows, ld, H + h * kD, boff(bqkv, H + h * kD), 1.f, Vs, rows, ld, 2 * H + h * kD,
                     boff(bqkv, 2 * H + h * kD), 1.f, c0, clen);
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
        // keep bits of the 32-key tile: this lane half draws key groups 2hf and 2hf+1 (8 keys
        // per Philox call, 16-bit uniforms) and swaps them with the partner lane (l ^ 32)
        const uint64_t e0 = (erow + c0 + t) >> 3;  // group index of key 0 of the tile
        const uint32_t mine = keep8_bits(seed, off, e0 + 2 * hf, thr) | (keep8_bits(seed, off, e0 + 2 * hf + 1, thr) << 8);
        const uint32_t other = static_cast<uint32_t>(__shfl_xor(static_cast<int>(mine), 32, 64));
        const uint32_t bits = hf == 0 ? (mine | (other << 16)) : (other | (mine << 16));  // bit k: key t+k
#pragma unroll
        for (int r = 0; r < 16; ++r) pr[r] = ((bits >> crow(r, hf)) & 1u) ? pr[r] * dscale : 0.f;
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
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int q0 = blockIdx.y * 128 + w * 32;
  const bool active = q0 < S;
  const T* rows = qkv + (int64_t)b * S * ld;
  const float dscale = drop_scale16(drop_thr16(p));

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
    stage_rows2<256>(Ks, rows, ld, H + h * kD, boff(bqkv, H + h * kD), 1.f, Vs, rows, ld, 2 * H + h * kD,
                     boff(bqkv, 2 * H + h * kD), 1.f, c0, clen);
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
  __shared__ uint32_t Wd[kCH][4];  // keep-bit words of the chunk's queries for this block's 4 key words
  const int H = NH * kD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int k0 = blockIdx.y * 128 + w * 32;
  const bool active = k0 < S;
  const int key = k0 + li;
  const T* rows = qkv + (int64_t)b * S * ld;
  const T* drows = dctx + (int64_t)b * S * H;
  const float dscale = drop_scale16(drop_thr16(p));

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
    stage_rows2<256>(Qs, rows, ld, h * kD, boff(bqkv, h * kD), 0.125f, Os, drows, H, h * kD, nullptr, 1.f, c0, clen);
    for (int i = threadIdx.x; i < clen; i += blockDim.x) {
      Ls[i] = lse[(int64_t)bh * S + c0 + i];
      Ds[i] = Dd[(int64_t)bh * S + c0 + i];
    }
    if (p > 0.f)
      for (int i = threadIdx.x; i < clen * 4; i += blockDim.x) {
        const int qi = i >> 2, kw = blockIdx.y * 4 + (i & 3);
        Wd[qi][i & 3] = kw < (S >> 5) ? dmask[((uint64_t)bh * S + c0 + qi) * (uint64_t)(S >> 5) + kw] : 0u;
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
        const float mk = p > 0.f ? (((Wd[qi][w] >> li) & 1u) ? dscale : 0.f) : 1.f;
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

// Fused backward for S <= 128: one block per (batch, head) owns every query and
// every key, so the seven products of the two-kernel path become five.  8 waves
// (2 per SIMD):
//   phase 1, wave (kg = w&3, qh = w>>2): keys 32kg..32kg+31, query tiles {64qh, 64qh+32}:
//     S^T = K Q^T, dP^T = V dO^T, dS^T = P^T o (dP^T - D); dV += P^T dO, dK += dS^T Q
//     (partials over the two query halves), dS written to LDS ([query][key], 132-float rows);
//   phase 2, wave (qt = w&3, kh = w>>2): dQ[queries 32qt..] partial over keys 64kh..64kh+63,
//     dQ = dS K with K re-staged from registers into LDS (72-float rows);
//   combine: waves 4..7 hand their dK/dV and dQ partials to waves 0..3 through the
//     freed LDS (fixed order: deterministic), which write the results.
// No recompute of S and dP, no atomics.  D = rowsum(dO o O) in the prologue.
// LDS 142 KB -> 1 block (8 waves) per CU.
constexpr int kLDS = 132;  // dS row stride (floats): conflict-free b128 reads in phase 2
constexpr int kLDK = 72;   // K row stride in phase 2

template <typename T>
__global__ void __launch_bounds__(512, 1)
    attn_bwd_fused_kernel(const T* __restrict__ qkv, const int64_t* __restrict__ mask, const float* __restrict__ bqkv,
                          const T* __restrict__ ctx, const T* __restrict__ dctx, const float* __restrict__ lse,
                          T* __restrict__ dqkv, int S, int NH, float p, const uint32_t* __restrict__ dmask) {
  __shared__ __attribute__((aligned(16))) float QKs[128 * kLDK];  // Q (stride kLD) in phase 1, K (kLDK) in phase 2
  __shared__ __attribute__((aligned(16))) float Os[128 * kLD];    // dO; then dQ partials
  __shared__ __attribute__((aligned(16))) float dSs[128 * kLDS];  // dS; then dK/dV partials
  __shared__ float Ls[128];
  __shared__ float Ds[128];
  __shared__ uint32_t Wd[128][4];
  const int H = NH * kD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int g4 = w & 3, half = w >> 2;  // phase 1: key group / query half; phase 2: query tile / key half
  const bool kactive = 32 * g4 < S;
  const int key = 32 * g4 + li;
  const T* rows = qkv + (int64_t)b * S * ld;
  const T* drows = dctx + (int64_t)b * S * H;
  const float dscale = drop_scale16(drop_thr16(p));

  // ---- prologue: stage Q (biased, scaled), dO, lse, keep words; D = rowsum(dO o O)
  stage_rows2<512>(QKs, rows, ld, h * kD, boff(bqkv, h * kD), 0.125f, Os, drows, H, h * kD, nullptr, 1.f, 0, S);
  for (int i = threadIdx.x; i < S; i += blockDim.x) Ls[i] = lse[(int64_t)bh * S + i];
  if (p > 0.f)
    for (int i = threadIdx.x; i < S * (S >> 5); i += blockDim.x)
      Wd[i / (S >> 5)][i % (S >> 5)] = dmask[((uint64_t)bh * S) * (uint64_t)(S >> 5) + i];
  float kr[32], vr[32];
  float madd = 0.f;
  if (kactive) {
    load_row_half(rows + (int64_t)key * ld + H + h * kD + hf * 32, boff(bqkv, H + h * kD + hf * 32), 1.f, kr);
    load_row_half(rows + (int64_t)key * ld + 2 * H + h * kD + hf * 32, boff(bqkv, 2 * H + h * kD + hf * 32), 1.f,
                  vr);
    madd = (1.f - (float)mask[(int64_t)b * S + key]) * -10000.f;
  }
  __syncthreads();  // Os staged
  {
    const int r = threadIdx.x >> 2, qtr = threadIdx.x & 3;  // 4 threads per query row
    float dsum = 0.f;
    if (r < S) {
      const T* orow = ctx + ((int64_t)b * S + r) * H + h * kD + qtr * 16;
      const float* dor = Os + r * kLD + qtr * 16;
#pragma unroll
      for (int kk = 0; kk < 16; kk += 4) {
        float o[4];
        load4(orow + kk, o);
        dsum = fmaf(dor[kk], o[0], fmaf(dor[kk + 1], o[1], fmaf(dor[kk + 2], o[2], fmaf(dor[kk + 3], o[3], dsum))));
      }
    }
    dsum += __shfl_xor(dsum, 1, 64);
    dsum += __shfl_xor(dsum, 2, 64);
    if (r < S && qtr == 0) Ds[r] = dsum;
  }
  __syncthreads();

  // ---- phase 1: dK, dV partials for this wave's keys over its query half; dS tiles to LDS
  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  if (kactive) {
    for (int t = 64 * half; t < min(S, 64 * half + 64); t += 32) {
      f32x16 s = {}, dp = {};
      const float* qp = QKs + (t + li) * kLD + hf * 32;
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
        const float mk = p > 0.f ? (((Wd[qi][g4] >> li) & 1u) ? dscale : 0.f) : 1.f;
        pd[r] = pv * mk;
        ds[r] = pv * (dp[r] * mk - Ds[qi]);
        dSs[qi * kLDS + key] = ds[r];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qi = t + crow(r, hf);
        const float* orow = Os + qi * kLD;
        const float* qrow = QKs + qi * kLD;
        dv0 = mfma32(orow[li], pd[r], dv0);
        dv1 = mfma32(orow[32 + li], pd[r], dv1);
        dk0 = mfma32(qrow[li], ds[r], dk0);
        dk1 = mfma32(qrow[32 + li], ds[r], dk1);
      }
    }
  }
  __syncthreads();  // every wave done with Q and dO; dS complete
  if (kactive && half == 0) {  // K rows (biased) from registers into LDS for phase 2
    float* kd = QKs + key * kLDK + hf * 32;
#pragma unroll
    for (int kk = 0; kk < 32; kk += 4)
      *reinterpret_cast<float4*>(kd + kk) = make_float4(kr[kk], kr[kk + 1], kr[kk + 2], kr[kk + 3]);
  }
  __syncthreads();

  // ---- phase 2: dQ partial for queries 32*g4.. over keys 64*half..64*half+63
  const bool qactive = 32 * g4 < S;
  f32x16 dq0 = {}, dq1 = {};
  if (qactive) {
    const float* dsr = dSs + (32 * g4 + li) * kLDS + 4 * hf;
    for (int k0 = 64 * half; k0 < min(S, 64 * half + 64); k0 += 8) {
      const float4 b4 = *reinterpret_cast<const float4*>(dsr + k0);
      const float bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const float* kp = QKs + (k0 + 4 * hf + s2) * kLDK;
        dq0 = mfma32(kp[li], bv[s2], dq0);
        dq1 = mfma32(kp[32 + li], bv[s2], dq1);
      }
    }
  }
  __syncthreads();  // dS and K consumed: LDS free for the hand-off

  // ---- combine: waves 4..7 hand their partials to waves 0..3 (lane-private slots, fixed order)
  float* xq = Os + g4 * 64 * 32 + lane;   // dq partial: 32 floats per lane, element r at xq[64 r]
  float* xk = dSs + g4 * 64 * 64 + lane;  // dk/dv partials: 64 floats per lane (conflict-free slots)
  if (half == 1) {
    if (qactive)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        xq[64 * r] = dq0[r];
        xq[64 * (16 + r)] = dq1[r];
      }
    if (kactive)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        xk[64 * r] = dk0[r];
        xk[64 * (16 + r)] = dk1[r];
        xk[64 * (32 + r)] = dv0[r];
        xk[64 * (48 + r)] = dv1[r];
      }
  }
  __syncthreads();
  if (half == 1) return;
  if (qactive)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dq0[r] += xq[64 * r];
      dq1[r] += xq[64 * (16 + r)];
    }
  if (kactive)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dk0[r] += xk[64 * r];
      dk1[r] += xk[64 * (16 + r)];
      dv0[r] += xk[64 * (32 + r)];
      dv1[r] += xk[64 * (48 + r)];
    }
  if (!qactive) return;  // qactive == kactive here (both 32*g4 < S)
  const int64_t tok = (int64_t)b * S + key;  // key == query index 32*g4 + li
  T* outq = dqkv + tok * ld + h * kD;
  T* outk = dqkv + tok * ld + H + h * kD;
  T* outv = dqkv + tok * ld + 2 * H + h * kD;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * hf;
    float q0v[4] = {dq0[4 * g] * 0.125f, dq0[4 * g + 1] * 0.125f, dq0[4 * g + 2] * 0.125f, dq0[4 * g + 3] * 0.125f};
    float q1v[4] = {dq1[4 * g] * 0.125f, dq1[4 * g + 1] * 0.125f, dq1[4 * g + 2] * 0.125f, dq1[4 * g + 3] * 0.125f};
    float a0[4] = {dk0[4 * g], dk0[4 * g + 1], dk0[4 * g + 2], dk0[4 * g + 3]};
    float a1[4] = {dk1[4 * g], dk1[4 * g + 1], dk1[4 * g + 2], dk1[4 * g + 3]};
    float c0v[4] = {dv0[4 * g], dv0[4 * g + 1], dv0[4 * g + 2], dv0[4 * g + 3]};
    float c1v[4] = {dv1[4 * g], dv1[4 * g + 1], dv1[4 * g + 2], dv1[4 * g + 3]};
    store4(outq + d, q0v);
    store4(outq + 32 + d, q1v);
    store4(outk + d, a0);
    store4(outk + 32 + d, a1);
    store4(outv + d, c0v);
    store4(outv + 32 + d, c1v);
  }
}

}  // namespace hs

using namespace hs;

int launch_attn_fwd_bf16(const void* qkv, const int64_t* mask, const float* bqkv, void* ctx, float* lse,
                         uint32_t* dmask, int B, int S, int NH, int D, float p, uint64_t seed, uint64_t off,
                         hipStream_t st, int bh0);

int launch_attn_bwd_fused_bf16(const void* qkv, const int64_t* mask, const float* bqkv, const void* ctx,
                               const void* dctx, const float* lse, void* dqkv, const uint32_t* dmask, int B, int S,
                               int NH, int D, float p, hipStream_t st);

int launch_attn_fwd_h3(const float* qkv, const int64_t* mask, const float* bqkv, float* ctx, float* lse,
                       uint32_t* dmask, int B, int S, int NH, int D, float p, uint64_t seed, uint64_t off,
                       hipStream_t st, int bh0, float* amax, void* pl = nullptr, int64_t ps = 0, int8_t* ex = nullptr);

int launch_attn_bwd_h3(const float* qkv, const int64_t* mask, const float* bqkv, const float* ctx, const float* dctx,
                       const float* lse, float* Dbuf, float* dqkv, const uint32_t* dmask, int B, int S, int NH, int D,
                       float p, hipStream_t st, float* amax, void* pl = nullptr, int64_t ps = 0,
                       int8_t* ex = nullptr, float* dsbuf = nullptr);

// fp32 attention products: 2 "h3" (three split-fp16 products with in-kernel power-of-two scales,
// attention_h3.hip; default) or 0 "native" (exact-fp32 MFMA, the oracle) -- HETSEQ_ATTN_FP32.  (The
// six-term split-bf16 kernels were retired in round 6: the h3 kernels' per-row / per-chunk scales
// cover their range role, the exact kernels their accuracy role.)
static int g_attn_fp32 = [] {
  const char* e = std::getenv("HETSEQ_ATTN_FP32");
  return e && std::string(e) == "native" ? 0 : 2;
}();

void set_attn_fp32_mode(int mode) { g_attn_fp32 = mode == 0 ? 0 : 2; }
int attn_fp32_mode() { return g_attn_fp32; }

// HETSEQ_ATTN_BF16_MFMA=0 keeps bf16 attention on the fp32-MFMA kernels (A/B and tests)
static bool bf16_mfma_enabled() {
  const char* e = std::getenv("HETSEQ_ATTN_BF16_MFMA");
  return !(e && std::string(e) == "0");
}

// HETSEQ_ATTN_BWD=split forces the two-kernel backward (A/B and tests)
static bool fused_bwd_enabled() {
  const char* e = std::getenv("HETSEQ_ATTN_BWD");
  return !(e && std::string(e) == "split");
}

// dmask: uint32 keep-bits [B*NH*S*(S/32)] written by the forward when p > 0
// and read by both backward kernels (required when p > 0).
// bh0: index of the launch's first (batch, head) in the whole batch -- the dropout keep bits of a
// batch slice are the ones the whole-batch launch would draw for those heads.
// amax (optional): |max| slot of the output; *amax_done = 1 when the kernel wrote it (the h3 engine),
// else the caller runs a |max| pass
int launch_attn_fwd(int dtype, const void* qkv, const int64_t* mask, const float* bqkv, void* ctx, float* lse,
                    uint32_t* dmask, int B, int S, int NH, int D, float p, uint64_t seed, uint64_t off,
                    hipStream_t st, int bh0, float* amax, int* amax_done) {
  if (amax_done) *amax_done = 0;
  if (D != kD || S % 32 != 0 || S <= 0 || bh0 < 0) return -1;
  dim3 grid(B * NH, (S + 127) / 128);  // head-major: a head's blocks share one XCD's L2
  if (dtype != 0 && bf16_mfma_enabled())  // bf16 matrix cores (attention_bf16.hip)
    return launch_attn_fwd_bf16(qkv, mask, bqkv, ctx, lse, dmask, B, S, NH, D, p, seed, off, st, bh0);
  if (dtype == 0 && g_attn_fp32 == 2) {  // fp32 as split-fp16 products (attention_h3.hip)
    const int rc = launch_attn_fwd_h3((const float*)qkv, mask, bqkv, (float*)ctx, lse, dmask, B, S, NH, D, p, seed, off,
                                      st, bh0, amax);
    if (rc == 0 && amax_done) *amax_done = amax != nullptr;
    return rc;
  }
  if (dtype == 0)
    hipLaunchKernelGGL(attn_fwd_kernel<float>, grid, dim3(256), 0, st, (const float*)qkv, mask, bqkv, (float*)ctx,
                       lse, dmask, S, NH, p, seed, off, g_seed_dev, bh0);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)qkv, mask, bqkv,
                       (bf16_t*)ctx, lse, dmask, S, NH, p, seed, off, g_seed_dev, bh0);
  return 0;
}

int launch_attn_bwd(int dtype, const void* qkv, const int64_t* mask, const float* bqkv, const void* ctx,
                    const void* dctx, const float* lse, float* Dbuf, void* dqkv, const uint32_t* dmask, int B, int S,
                    int NH, int D, float p, hipStream_t st, float* amax, int* amax_done) {
  if (amax_done) *amax_done = 0;
  if (D != kD || S % 32 != 0 || S <= 0 || (p > 0.f && dmask == nullptr)) return -1;
  if (dtype == 0 && g_attn_fp32 == 2) {
    const int rc = launch_attn_bwd_h3((const float*)qkv, mask, bqkv, (const float*)ctx, (const float*)dctx, lse, Dbuf,
                                      (float*)dqkv, dmask, B, S, NH, D, p, st, amax);
    if (rc == 0 && amax_done) *amax_done = amax != nullptr;
    return rc;
  }
  if (S <= 128 && fused_bwd_enabled()) {  // one block per (batch, head): 5 products instead of 7
    if (dtype != 0 && bf16_mfma_enabled())
      return launch_attn_bwd_fused_bf16(qkv, mask, bqkv, ctx, dctx, lse, dqkv, dmask, B, S, NH, D, p, st);
    if (dtype == 0)
      hipLaunchKernelGGL(attn_bwd_fused_kernel<float>, dim3(B * NH), dim3(512), 0, st, (const float*)qkv, mask, bqkv,
                         (const float*)ctx, (const float*)dctx, lse, (float*)dqkv, S, NH, p, dmask);
    else
      hipLaunchKernelGGL(attn_bwd_fused_kernel<bf16_t>, dim3(B * NH), dim3(512), 0, st, (const bf16_t*)qkv, mask,
                         bqkv, (const bf16_t*)ctx, (const bf16_t*)dctx, lse, (bf16_t*)dqkv, S, NH, p, dmask);
    return 0;
  }
  dim3 grid(B * NH, (S + 127) / 128);  // head-major: a head's blocks share one XCD's L2
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
