// bf16 attention on the bf16 matrix cores (v_mfma_f32_32x32x16_bf16) for
// --dtype bf16.  Same contract as attention.hip (reference bert_modeling.py:
// 351-377): Q/K/V read from the fused QKV projection output [B*S, 3H] with the
// projection bias folded into the loads, additive -10000 mask, Philox dropout
// on the probabilities with a 1-bit keep mask for the backward, context out in
// [B*S, H], per-row log-sum-exp saved.  fp32 accumulation and softmax
// statistics; MFMA operands bf16 (the QK scale 1/8 is exact in bf16).
//
// Orientation (same as the fp32 kernels): a wave owns 32 queries; the score
// tile is S^T[key][query] so a lane holds one query's scores in registers.
//   S^T = K Q^T : A = K rows from LDS (16-B reads, 144-B rows: conflict-free),
//                 B = the lane's own Q row (registers, 4 k-steps of 16 dims);
//   O^T = V^T P^T: B = the probability accumulator itself, converted to bf16 --
//                 registers 8s..8s+7 are exactly the B fragment of k-step s
//                 (key 16s + 8(j>>2) + 4*half + (j&3) for element j);
//                 A = V^T from a transposed LDS image (two 8-B reads per step).
// 8 MFMAs per 32-key tile instead of 128 fp32 ones: the kernel is bound by the
// softmax/dropout VALU work, not the matrix cores.
#include "common.h"

namespace hs {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kBD = 64;        // head dim
constexpr int kKLD = 72;       // K image row stride (bf16): 144 B
constexpr int kVLD = 132;      // V^T image row stride (bf16): 264 B -> lanes d, d+1 on adjacent bank pairs
constexpr int kBCH = 128;      // keys per LDS chunk

HS_DEVICE f32x16 mfma16(bf16x8 a, bf16x8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0); }
HS_DEVICE int crow16(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }
HS_DEVICE short bfbits(float v) { return static_cast<short>(from_f<bf16_t>(v).x); }
HS_DEVICE float bfval(uint16_t b) { return __uint_as_float(static_cast<uint32_t>(b) << 16); }

// 8 consecutive bf16 of a row (16-B load) -> fp32, + bias, * scale
HS_DEVICE void load8(const bf16_t* src, const float* bias, float scale, float (&v)[8]) {
  const uint4 t = *reinterpret_cast<const uint4*>(src);
  const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
  if (bias) {
    const float4 b0 = *reinterpret_cast<const float4*>(bias), b1 = *reinterpret_cast<const float4*>(bias + 4);
    v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
    v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] *= scale;
}

HS_DEVICE bf16x8 pack8(const float (&v)[8]) {
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = bfbits(v[i]);
  return r;
}

HS_DEVICE const float* boff16(const float* b, int off) { return b ? b + off : nullptr; }

__global__ void __launch_bounds__(256, 2)
    attn_fwd_bf16_kernel(const bf16_t* __restrict__ qkv, const int64_t* __restrict__ mask,
                         const float* __restrict__ bqkv, bf16_t* __restrict__ ctx, float* __restrict__ lse,
                         uint32_t* __restrict__ dmask, int S, int NH, float p, uint64_t seed, uint64_t off,
                         const uint64_t* __restrict__ seed_dev, int bh0) {
  seed = resolve_seed(seed, seed_dev);
  __shared__ __attribute__((aligned(16))) uint16_t Ks[kBCH * kKLD];
  __shared__ __attribute__((aligned(16))) uint16_t Vt[kBD * kVLD];
  __shared__ float Ms[kBCH];
  const int H = NH * kBD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int q0 = blockIdx.y * 128 + w * 32;
  const bool active = q0 < S;
  const bf16_t* rows = qkv + (int64_t)b * S * ld;
  const uint32_t thr = drop_thr16(p);
  const float dscale = drop_scale16(thr);

  // the lane's Q row, dims 16s + 8hf + j (k-step s), biased and scaled by 1/sqrt(64)
  bf16x8 qf[4];
  if (active) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float v[8];
      const int d = 16 * s + 8 * hf;
      load8(rows + (int64_t)(q0 + li) * ld + h * kBD + d, boff16(bqkv, h * kBD + d), 0.125f, v);
      qf[s] = pack8(v);
    }
  }
  f32x16 o0 = {}, o1 = {};
  float m = -1e30f, l = 0.f;
  const uint64_t erow = ((uint64_t)(bh0 + bh) * S + (q0 + li)) * (uint64_t)S;  // bh0: a batch slice's first head

  for (int c0 = 0; c0 < S; c0 += kBCH) {
    const int clen = min(kBCH, S - c0);
    __syncthreads();
    // K chunk: row-major image; thread unit = (row, 8-dim chunk)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = threadIdx.x + 256 * i, r = u >> 3, c8 = (u & 7) * 8;
      if (r < clen) {
        float v[8];
        load8(rows + (int64_t)(c0 + r) * ld + H + h * kBD + c8, boff16(bqkv, H + h * kBD + c8), 1.f, v);
        *reinterpret_cast<bf16x8*>(Ks + r * kKLD + c8) = pack8(v);
      }
    }
    // V chunk, transposed: Vt[d][key]; consecutive lanes take consecutive keys (conflict-free 2-B writes)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = threadIdx.x + 256 * i, r = u & 127, c8 = (u >> 7) * 8;
      if (r < clen) {
        float v[8];
        load8(rows + (int64_t)(c0 + r) * ld + 2 * H + h * kBD + c8, boff16(bqkv, 2 * H + h * kBD + c8), 1.f, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) Vt[(c8 + j) * kVLD + r] = static_cast<uint16_t>(bfbits(v[j]));
      }
    }
    for (int i = threadIdx.x; i < clen; i += blockDim.x)
      Ms[i] = (1.f - (float)mask[(int64_t)b * S + c0 + i]) * -10000.f;
    __syncthreads();
    if (!active) continue;
    for (int t = 0; t < clen; t += 32) {
      f32x16 s = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        s = mfma16(*reinterpret_cast<const bf16x8*>(Ks + (t + li) * kKLD + 16 * ks + 8 * hf), qf[ks], s);
      float mt = -1e30f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[r] += Ms[t + crow16(r, hf)];
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
      if (p > 0.f) {  // same keep-bit stream and word layout as the fp32 kernel
        const uint64_t e0 = (erow + c0 + t) >> 3;
        const uint32_t mine = keep8_bits(seed, off, e0 + 2 * hf, thr) | (keep8_bits(seed, off, e0 + 2 * hf + 1, thr) << 8);
        const uint32_t other = static_cast<uint32_t>(__shfl_xor(static_cast<int>(mine), 32, 64));
        const uint32_t bits = hf == 0 ? (mine | (other << 16)) : (other | (mine << 16));
#pragma unroll
        for (int r = 0; r < 16; ++r) pr[r] = ((bits >> crow16(r, hf)) & 1u) ? pr[r] * dscale : 0.f;
        if (dmask && hf == 0) dmask[((uint64_t)bh * S + q0 + li) * (uint64_t)(S >> 5) + ((c0 + t) >> 5)] = bits;
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = bfbits(pr[8 * ks + j]);
        const int k0 = t + 16 * ks + 4 * hf;
        // A = V^T rows d = li (o0) and 32 + li (o1), keys k0..k0+3 and k0+8..k0+11
        const uint16_t* v0 = Vt + li * kVLD + k0;
        const uint16_t* v1 = Vt + (32 + li) * kVLD + k0;
        bf16x8 a0, a1;
        const uint2 x0 = *reinterpret_cast<const uint2*>(v0), y0 = *reinterpret_cast<const uint2*>(v0 + 8);
        const uint2 x1 = *reinterpret_cast<const uint2*>(v1), y1 = *reinterpret_cast<const uint2*>(v1 + 8);
        a0[0] = (short)(x0.x & 0xffff); a0[1] = (short)(x0.x >> 16); a0[2] = (short)(x0.y & 0xffff); a0[3] = (short)(x0.y >> 16);
        a0[4] = (short)(y0.x & 0xffff); a0[5] = (short)(y0.x >> 16); a0[6] = (short)(y0.y & 0xffff); a0[7] = (short)(y0.y >> 16);
        a1[0] = (short)(x1.x & 0xffff); a1[1] = (short)(x1.x >> 16); a1[2] = (short)(x1.y & 0xffff); a1[3] = (short)(x1.y >> 16);
        a1[4] = (short)(y1.x & 0xffff); a1[5] = (short)(y1.x >> 16); a1[6] = (short)(y1.y & 0xffff); a1[7] = (short)(y1.y >> 16);
        o0 = mfma16(a0, pf, o0);
        o1 = mfma16(a1, pf, o1);
      }
    }
  }
  if (!active) return;
  const float inv = 1.f / l;
  bf16_t* out = ctx + ((int64_t)b * S + q0 + li) * H + h * kBD;
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

// ---------------------------------------------------------------------------
// Fused backward on the bf16 matrix cores, S <= 128: one block (8 waves) per
// (batch, head), the bf16 counterpart of attn_bwd_fused_kernel (attention.hip).
//   phase 1, wave (kg = w&3, qh = w>>2): keys 32kg.., query tiles {64qh, 64qh+32}:
//     S = Q K^T, dP = dO V^T  (A = Q / dO rows from LDS, B = the lane's own K / V row);
//     P, dS = P o (dP - D) in registers (lane = key, registers = queries);
//     dV^T += dO^T P, dK^T += Q^T dS with P / dS used directly as the B operand
//     (registers 8s..8s+7 = k-step s) and A from transposed dO / Q images;
//     dS (bf16) stored to LDS [query][key];
//   phase 2, wave (qt = w&3, kh = w>>2): dQ^T = K^T dS^T over keys 64kh..64kh+63,
//     A = K^T image (written from the waves' K registers), B = dS rows;
//   combine: waves 4..7 hand dK/dV/dQ partials to waves 0..3 through the freed LDS.
// 20 bf16 MFMAs per 32x32 tile pair instead of 160 fp32 ones.  LDS 110 KB.
constexpr int kTLD = 136;  // transposed images: [64 d][128 + 8] bf16 (272-B rows)

HS_DEVICE bf16x8 ld8x2(const uint16_t* p) {  // two 8-B runs 8 elements apart -> one k-step fragment
  const uint2 x = *reinterpret_cast<const uint2*>(p), y = *reinterpret_cast<const uint2*>(p + 8);
  bf16x8 a;
  a[0] = (short)(x.x & 0xffff); a[1] = (short)(x.x >> 16); a[2] = (short)(x.y & 0xffff); a[3] = (short)(x.y >> 16);
  a[4] = (short)(y.x & 0xffff); a[5] = (short)(y.x >> 16); a[6] = (short)(y.y & 0xffff); a[7] = (short)(y.y >> 16);
  return a;
}

__global__ void __launch_bounds__(512, 1)
    attn_bwd_fused_bf16_kernel(const bf16_t* __restrict__ qkv, const int64_t* __restrict__ mask,
                               const float* __restrict__ bqkv, const bf16_t* __restrict__ ctx,
                               const bf16_t* __restrict__ dctx, const float* __restrict__ lse,
                               bf16_t* __restrict__ dqkv, int S, int NH, float p, const uint32_t* __restrict__ dmask) {
  constexpr int kR1 = 128 * kKLD + kBD * kTLD;  // Q rows + Q^T (bf16 elements); K^T in phase 2
  constexpr int kRS = 128 * kTLD;               // dS [query][key]
  constexpr int kR2 = 128 * kKLD + kBD * kTLD;  // dO rows + dO^T
  __shared__ __attribute__((aligned(16))) uint16_t smem[kR1 + kRS + kR2];
  __shared__ float Ls[128];
  __shared__ float Ds[128];
  __shared__ uint32_t Wd[128][4];
  uint16_t* Qs = smem;
  uint16_t* Qt = smem + 128 * kKLD;
  uint16_t* Kt = smem;  // phase 2 (Q consumed)
  uint16_t* dSs = smem + kR1;
  uint16_t* Os = smem + kR1 + kRS;
  uint16_t* Ot = Os + 128 * kKLD;

  const int H = NH * kBD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int g4 = w & 3, half = w >> 2;
  const bool kactive = 32 * g4 < S;
  const int key = 32 * g4 + li;
  const bf16_t* rows = qkv + (int64_t)b * S * ld;
  const bf16_t* drows = dctx + (int64_t)b * S * H;
  const float dscale = drop_scale16(drop_thr16(p));

  // ---- prologue: Q (biased, * 1/8) and dO, row-major and transposed; lse, keep words
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int u = threadIdx.x + 512 * i, r = u & 127, c8 = (u >> 7) * 8;
    if (r < S) {
      float v[8], o[8];
      load8(rows + (int64_t)r * ld + h * kBD + c8, boff16(bqkv, h * kBD + c8), 0.125f, v);
      load8(drows + (int64_t)r * H + h * kBD + c8, nullptr, 1.f, o);
      const bf16x8 vb = pack8(v), ob = pack8(o);
      *reinterpret_cast<bf16x8*>(Qs + r * kKLD + c8) = vb;
      *reinterpret_cast<bf16x8*>(Os + r * kKLD + c8) = ob;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        Qt[(c8 + j) * kTLD + r] = static_cast<uint16_t>(vb[j]);
        Ot[(c8 + j) * kTLD + r] = static_cast<uint16_t>(ob[j]);
      }
    }
  }
  for (int i = threadIdx.x; i < S; i += blockDim.x) Ls[i] = lse[(int64_t)bh * S + i];
  if (p > 0.f)
    for (int i = threadIdx.x; i < S * (S >> 5); i += blockDim.x)
      Wd[i / (S >> 5)][i % (S >> 5)] = dmask[((uint64_t)bh * S) * (uint64_t)(S >> 5) + i];
  // the lane's K and V rows (biased), d = 16s + 8hf + j
  bf16x8 kf[4], vf[4];
  float madd = 0.f;
  if (kactive) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float v[8];
      const int d = 16 * s + 8 * hf;
      load8(rows + (int64_t)key * ld + H + h * kBD + d, boff16(bqkv, H + h * kBD + d), 1.f, v);
      kf[s] = pack8(v);
      load8(rows + (int64_t)key * ld + 2 * H + h * kBD + d, boff16(bqkv, 2 * H + h * kBD + d), 1.f, v);
      vf[s] = pack8(v);
    }
    madd = (1.f - (float)mask[(int64_t)b * S + key]) * -10000.f;
  }
  {  // D = rowsum(dO o O) from the bf16 inputs, 4 threads per row
    const int r = threadIdx.x >> 2, qtr = threadIdx.x & 3;
    float dsum = 0.f;
    if (r < S) {
      float o[8], g[8];
#pragma unroll
      for (int c = 0; c < 16; c += 8) {
        load8(ctx + ((int64_t)b * S + r) * H + h * kBD + qtr * 16 + c, nullptr, 1.f, o);
        load8(drows + (int64_t)r * H + h * kBD + qtr * 16 + c, nullptr, 1.f, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum = fmaf(g[j], o[j], dsum);
      }
    }
    dsum += __shfl_xor(dsum, 1, 64);
    dsum += __shfl_xor(dsum, 2, 64);
    if (r < S && qtr == 0) Ds[r] = dsum;
  }
  __syncthreads();

  // ---- phase 1
  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  if (kactive) {
    for (int t = 64 * half; t < min(S, 64 * half + 64); t += 32) {
      f32x16 sc = {}, dp = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        sc = mfma16(*reinterpret_cast<const bf16x8*>(Qs + (t + li) * kKLD + 16 * ks + 8 * hf), kf[ks], sc);
        dp = mfma16(*reinterpret_cast<const bf16x8*>(Os + (t + li) * kKLD + 16 * ks + 8 * hf), vf[ks], dp);
      }
      float pd[16], ds[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qi = t + crow16(r, hf);
        const float pv = __expf(sc[r] + madd - Ls[qi]);
        const float mk = p > 0.f ? (((Wd[qi][g4] >> li) & 1u) ? dscale : 0.f) : 1.f;
        pd[r] = pv * mk;
        ds[r] = pv * (dp[r] * mk - Ds[qi]);
        dSs[qi * kTLD + key] = static_cast<uint16_t>(bfbits(ds[r]));
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 pb, sb;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pb[j] = bfbits(pd[8 * ks + j]);
          sb[j] = bfbits(ds[8 * ks + j]);
        }
        const int q = t + 16 * ks + 4 * hf;  // queries q..q+3, q+8..q+11 for this lane half
        dv0 = mfma16(ld8x2(Ot + li * kTLD + q), pb, dv0);
        dv1 = mfma16(ld8x2(Ot + (32 + li) * kTLD + q), pb, dv1);
        dk0 = mfma16(ld8x2(Qt + li * kTLD + q), sb, dk0);
        dk1 = mfma16(ld8x2(Qt + (32 + li) * kTLD + q), sb, dk1);
      }
    }
  }
  __syncthreads();  // Q, dO consumed; dS complete
  if (kactive && half == 0)  // K^T from the lanes' K rows
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) Kt[(16 * s + 8 * hf + j) * kTLD + key] = static_cast<uint16_t>(kf[s][j]);
  __syncthreads();

  // ---- phase 2: dQ^T partial for queries 32*g4.. over keys 64*half..
  const bool qactive = 32 * g4 < S;
  f32x16 dq0 = {}, dq1 = {};
  if (qactive) {
    const uint16_t* dsr = dSs + (32 * g4 + li) * kTLD + 8 * hf;
    for (int k0 = 64 * half; k0 < min(S, 64 * half + 64); k0 += 16) {
      const bf16x8 bq = *reinterpret_cast<const bf16x8*>(dsr + k0);
      dq0 = mfma16(*reinterpret_cast<const bf16x8*>(Kt + li * kTLD + k0 + 8 * hf), bq, dq0);
      dq1 = mfma16(*reinterpret_cast<const bf16x8*>(Kt + (32 + li) * kTLD + k0 + 8 * hf), bq, dq1);
    }
  }
  __syncthreads();  // LDS free for the hand-off

  // ---- combine (fixed order) and store
  float* xk = reinterpret_cast<float*>(smem) + g4 * 64 * 64 + lane;          // dk/dv: R1 + dS regions
  float* xq = reinterpret_cast<float*>(smem + kR1 + kRS) + g4 * 64 * 32 + lane;  // dq: R2 region
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
  if (half == 1 || !qactive) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    dq0[r] += xq[64 * r];
    dq1[r] += xq[64 * (16 + r)];
    dk0[r] += xk[64 * r];
    dk1[r] += xk[64 * (16 + r)];
    dv0[r] += xk[64 * (32 + r)];
    dv1[r] += xk[64 * (48 + r)];
  }
  const int64_t tok = (int64_t)b * S + key;  // key == query index 32*g4 + li
  bf16_t* outq = dqkv + tok * ld + h * kBD;
  bf16_t* outk = dqkv + tok * ld + H + h * kBD;
  bf16_t* outv = dqkv + tok * ld + 2 * H + h * kBD;
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
                         hipStream_t st, int bh0) {
  if (D != kBD || S % 32 != 0 || S <= 0) return -1;
  dim3 grid(B * NH, (S + 127) / 128);  // head-major: a head's blocks share one XCD's L2
  hipLaunchKernelGGL(attn_fwd_bf16_kernel, grid, dim3(256), 0, st, (const bf16_t*)qkv, mask, bqkv, (bf16_t*)ctx, lse,
                     dmask, S, NH, p, seed, off, g_seed_dev, bh0);
  return 0;
}

int launch_attn_bwd_fused_bf16(const void* qkv, const int64_t* mask, const float* bqkv, const void* ctx,
                               const void* dctx, const float* lse, void* dqkv, const uint32_t* dmask, int B, int S,
                               int NH, int D, float p, hipStream_t st) {
  if (D != kBD || S % 32 != 0 || S <= 0 || S > 128 || (p > 0.f && dmask == nullptr)) return -1;
  hipLaunchKernelGGL(attn_bwd_fused_bf16_kernel, dim3(B * NH), dim3(512), 0, st, (const bf16_t*)qkv, mask, bqkv,
                     (const bf16_t*)ctx, (const bf16_t*)dctx, lse, (bf16_t*)dqkv, S, NH, p, dmask);
  return 0;
}
