// fp32 attention forward on the bf16 matrix cores (split-bf16 products, fp32-level error).
//
// Same contract as attn_fwd_kernel (attention.hip; reference bert_modeling.py:351-377):
// Q/K/V read from the fused QKV projection output [B*S, 3H] (fp32) with the projection
// bias folded into the loads, additive -10000 mask, Philox dropout with the 1-bit keep mask
// for the backward (identical bit stream and word layout), context out in [B*S, H], per-row
// log-sum-exp saved.
//
// Products: every fp32 operand x is split (round-to-nearest-even) into three bf16 terms
// x = hi + mid + lo (exact to 2^-27) and each product a*b is accumulated from the six cross
// terms of order <= 2^-16 -- the GEMM engine's scheme (gemm.hip, docs/kernels.md) -- on
// v_mfma_f32_32x32x16_bf16: a 32-key x 32-query score tile costs 24 bf16 MFMAs (768 cycles)
// instead of 32 exact-fp32 v_mfma_f32_32x32x2_f32 (2048 cycles), and so does P V.
// Orientation and fragment maps are those of attention_bf16.hip (a wave owns 32 queries, the
// score tile is S^T[key][query], the probability accumulator registers 8s..8s+7 are the B
// fragment of k-step s).  K and V^T are split once per block while staged into LDS (three
// planes each, 64-key chunks: 54 KB, two blocks per CU); the lane's Q row is split once in
// registers; probabilities are split in registers per tile.
#include "common.h"

namespace hs {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bfx2 __attribute__((ext_vector_type(2)));
typedef float fx2 __attribute__((ext_vector_type(2)));

constexpr int kXD = 64;    // head dim
constexpr int kXCH = 64;   // keys per LDS chunk
constexpr int kXKLD = 72;  // K plane row stride (bf16): 144 B
constexpr int kXVLD = 72;  // V^T plane row stride (bf16): 144 B

HS_DEVICE f32x16 mma(bfx8 a, bfx8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0); }
HS_DEVICE int xrow(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }

// 8 fp32 -> three bf16x8 planes (hi, mid, lo), RNE at every step
HS_DEVICE void split8(const float (&v)[8], bfx8& hi, bfx8& mi, bfx8& lo) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const fx2 x = {v[2 * i], v[2 * i + 1]};
    const bfx2 h = __builtin_convertvector(x, bfx2);
    const fx2 r = x - __builtin_convertvector(h, fx2);
    const bfx2 m = __builtin_convertvector(r, bfx2);
    const bfx2 l = __builtin_convertvector(r - __builtin_convertvector(m, fx2), bfx2);
    hi[2 * i] = h[0];
    hi[2 * i + 1] = h[1];
    mi[2 * i] = m[0];
    mi[2 * i + 1] = m[1];
    lo[2 * i] = l[0];
    lo[2 * i + 1] = l[1];
  }
}

// acc += a * b over the six split terms, smallest first (a, b: planes hi/mid/lo)
HS_DEVICE f32x16 mma6(const bfx8 (&a)[3], const bfx8 (&b)[3], f32x16 acc) {
  acc = mma(a[2], b[0], acc);
  acc = mma(a[0], b[2], acc);
  acc = mma(a[1], b[1], acc);
  acc = mma(a[1], b[0], acc);
  acc = mma(a[0], b[1], acc);
  return mma(a[0], b[0], acc);
}

// 8 consecutive fp32 (+ bias) * scale
HS_DEVICE void ld8(const float* src, const float* bias, float scale, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  if (bias) {
    const float4 c = *reinterpret_cast<const float4*>(bias), d = *reinterpret_cast<const float4*>(bias + 4);
    v[0] += c.x; v[1] += c.y; v[2] += c.z; v[3] += c.w; v[4] += d.x; v[5] += d.y; v[6] += d.z; v[7] += d.w;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] *= scale;
}

// two 8-B runs 8 elements apart -> one k-step fragment
HS_DEVICE bfx8 frag2x4(const __bf16* p) {
  const uint2 x = *reinterpret_cast<const uint2*>(p), y = *reinterpret_cast<const uint2*>(p + 8);
  const uint4 u = make_uint4(x.x, x.y, y.x, y.y);
  return __builtin_bit_cast(bfx8, u);
}

HS_DEVICE const float* bofs(const float* b, int off) { return b ? b + off : nullptr; }

}  // namespace

__global__ void __launch_bounds__(256, 2)
    attn_fwd_x6_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ mask, const float* __restrict__ bqkv,
                       float* __restrict__ ctx, float* __restrict__ lse, uint32_t* __restrict__ dmask, int S, int NH,
                       float p, uint64_t seed, uint64_t off, const uint64_t* __restrict__ seed_dev) {
  seed = resolve_seed(seed, seed_dev);
  __shared__ __attribute__((aligned(16))) __bf16 Ks[3][kXCH * kXKLD];
  __shared__ __attribute__((aligned(16))) __bf16 Vt[3][kXD * kXVLD];
  __shared__ float Ms[kXCH];
  const int H = NH * kXD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.y, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int q0 = blockIdx.x * 128 + w * 32;
  const bool active = q0 < S;
  const float* rows = qkv + (int64_t)b * S * ld;
  const uint32_t thr = drop_thr16(p);
  const float dscale = drop_scale16(thr);

  // the lane's Q row, dims 16s + 8hf + j (k-step s), biased, * 1/sqrt(64) (exact), split
  bfx8 qf[4][3];
  if (active) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float v[8];
      const int d = 16 * s + 8 * hf;
      ld8(rows + (int64_t)(q0 + li) * ld + h * kXD + d, bofs(bqkv, h * kXD + d), 0.125f, v);
      split8(v, qf[s][0], qf[s][1], qf[s][2]);
    }
  }
  f32x16 o0 = {}, o1 = {};
  float m = -1e30f, l = 0.f;
  const uint64_t erow = ((uint64_t)bh * S + (q0 + li)) * (uint64_t)S;

  for (int c0 = 0; c0 < S; c0 += kXCH) {
    const int clen = min(kXCH, S - c0);
    __syncthreads();
    // K chunk -> three row-major planes; unit = (key row, 8-dim chunk)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int u = threadIdx.x + 256 * i, r = u >> 3, c8 = (u & 7) * 8;
      if (r < clen) {
        float v[8];
        ld8(rows + (int64_t)(c0 + r) * ld + H + h * kXD + c8, bofs(bqkv, H + h * kXD + c8), 1.f, v);
        bfx8 a, bb, c;
        split8(v, a, bb, c);
        *reinterpret_cast<bfx8*>(&Ks[0][r * kXKLD + c8]) = a;
        *reinterpret_cast<bfx8*>(&Ks[1][r * kXKLD + c8]) = bb;
        *reinterpret_cast<bfx8*>(&Ks[2][r * kXKLD + c8]) = c;
      }
    }
    // V chunk -> three transposed planes Vt[d][key]; consecutive lanes take consecutive keys
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int u = threadIdx.x + 256 * i, r = u & (kXCH - 1), c8 = (u / kXCH) * 8;
      if (r < clen) {
        float v[8];
        ld8(rows + (int64_t)(c0 + r) * ld + 2 * H + h * kXD + c8, bofs(bqkv, 2 * H + h * kXD + c8), 1.f, v);
        bfx8 a, bb, c;
        split8(v, a, bb, c);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          Vt[0][(c8 + j) * kXVLD + r] = a[j];
          Vt[1][(c8 + j) * kXVLD + r] = bb[j];
          Vt[2][(c8 + j) * kXVLD + r] = c[j];
        }
      }
    }
    for (int i = threadIdx.x; i < clen; i += blockDim.x)
      Ms[i] = (1.f - (float)mask[(int64_t)b * S + c0 + i]) * -10000.f;
    __syncthreads();
    if (!active) continue;
    for (int t = 0; t < clen; t += 32) {
      f32x16 s = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bfx8 kf[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          kf[pl] = *reinterpret_cast<const bfx8*>(&Ks[pl][(t + li) * kXKLD + 16 * ks + 8 * hf]);
        s = mma6(kf, qf[ks], s);
      }
      float mt = -1e30f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[r] += Ms[t + xrow(r, hf)];
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
      if (p > 0.f) {  // the fp32 kernel's keep-bit stream and word layout (the backward reads them)
        const uint64_t e0 = (erow + c0 + t) >> 3;
        const uint32_t mine = keep8_bits(seed, off, e0 + 2 * hf, thr) | (keep8_bits(seed, off, e0 + 2 * hf + 1, thr) << 8);
        const uint32_t other = static_cast<uint32_t>(__shfl_xor(static_cast<int>(mine), 32, 64));
        const uint32_t bits = hf == 0 ? (mine | (other << 16)) : (other | (mine << 16));
#pragma unroll
        for (int r = 0; r < 16; ++r) pr[r] = ((bits >> xrow(r, hf)) & 1u) ? pr[r] * dscale : 0.f;
        if (dmask && hf == 0) dmask[((uint64_t)bh * S + q0 + li) * (uint64_t)(S >> 5) + ((c0 + t) >> 5)] = bits;
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float pv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) pv[j] = pr[8 * ks + j];
        bfx8 pf[3];
        split8(pv, pf[0], pf[1], pf[2]);
        const int k0 = t + 16 * ks + 4 * hf;
        bfx8 a0[3], a1[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          a0[pl] = frag2x4(&Vt[pl][li * kXVLD + k0]);
          a1[pl] = frag2x4(&Vt[pl][(32 + li) * kXVLD + k0]);
        }
        o0 = mma6(a0, pf, o0);
        o1 = mma6(a1, pf, o1);
      }
    }
  }
  if (!active) return;
  const float inv = 1.f / l;
  float* out = ctx + ((int64_t)b * S + q0 + li) * H + h * kXD;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * hf;
    *reinterpret_cast<float4*>(out + d) = make_float4(o0[4 * g] * inv, o0[4 * g + 1] * inv, o0[4 * g + 2] * inv,
                                                      o0[4 * g + 3] * inv);
    *reinterpret_cast<float4*>(out + 32 + d) = make_float4(o1[4 * g] * inv, o1[4 * g + 1] * inv,
                                                           o1[4 * g + 2] * inv, o1[4 * g + 3] * inv);
  }
  if (hf == 0) lse[(int64_t)bh * S + q0 + li] = m + __logf(l);
}

}  // namespace hs

using namespace hs;

int launch_attn_fwd_x6(const float* qkv, const int64_t* mask, const float* bqkv, float* ctx, float* lse,
                       uint32_t* dmask, int B, int S, int NH, int D, float p, uint64_t seed, uint64_t off,
                       hipStream_t st) {
  if (D != kXD || S % 32 != 0 || S <= 0) return -1;
  dim3 grid((S + 127) / 128, B * NH);
  hipLaunchKernelGGL(attn_fwd_x6_kernel, grid, dim3(256), 0, st, qkv, mask, bqkv, ctx, lse, dmask, S, NH, p, seed, off,
                     g_seed_dev);
  return 0;
}
