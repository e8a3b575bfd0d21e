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
#include <cstdlib>

#include "common.h"

namespace hs {

int launch_attn_bwd_dsum(const float* ctx, const float* dctx, float* Dout, int B, int S, int NH, hipStream_t st);

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bfx2 __attribute__((ext_vector_type(2)));
typedef float fx2 __attribute__((ext_vector_type(2)));

constexpr int kXD = 64;    // head dim
constexpr int kXCH = 64;   // keys per LDS chunk

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

HS_DEVICE const float* bofs(const float* b, int off) { return b ? b + off : nullptr; }

// the lane's K / V row halves in fragment order: r[s][j] = row[16 s + 8 hf + j] (+ bias)
HS_DEVICE void row_frags(const float* row, const float* bias, int hf, float (&r)[4][8]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) ld8(row + 16 * s + 8 * hf, bias ? bias + 16 * s + 8 * hf : nullptr, 1.f, r[s]);
}

// 16 accumulator registers of two 32x32 C tiles (rows d = crow, lane column) -> 64 fp32 of a
// token row: out[d] for d = 8g + 4hf + (0..3), out[32 + d]
HS_DEVICE void store_rows(float* out, const f32x16& c0, const f32x16& c1, int hf, float scale) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * hf;
    *reinterpret_cast<float4*>(out + d) =
        make_float4(c0[4 * g] * scale, c0[4 * g + 1] * scale, c0[4 * g + 2] * scale, c0[4 * g + 3] * scale);
    *reinterpret_cast<float4*>(out + 32 + d) =
        make_float4(c1[4 * g] * scale, c1[4 * g + 1] * scale, c1[4 * g + 2] * scale, c1[4 * g + 3] * scale);
  }
}

// ---- pre-split plane images of 64-row chunks (the "p" backward kernels) ----
// A chunk of Q / dO (or K / V) rows is split ONCE per block into three bf16 planes [row][64 d]
// (128-B rows, 8 KB per plane), read two ways: row fragments (k = d) by one ds_read_b128 each,
// transposed fragments (rows = d, k = rows of the chunk, in the score-register order) by two
// ds_read_b64_tr_b16.  The 16-B chunk swizzle pswz makes both patterns conflict-free (searched
// exhaustively over 3-bit row-bit selections: the b128 lane groups and the 32-lane tr16 halves).
constexpr int kPRow = 128;            // bytes per plane row
constexpr int kPPlane = 64 * kPRow;   // bytes per plane (64 rows)
constexpr int kPImg = 3 * kPPlane;    // one operand's three planes: 24 KB

typedef short ps4 __attribute__((ext_vector_type(4)));
typedef short ps8 __attribute__((ext_vector_type(8)));

HS_DEVICE int pswz(int r) { return ((r >> 2) & 1) | (((r >> 3) & 1) << 1) | (((r >> 1) & 1) << 2); }

// rows [r0, r0 + n) (n <= 64) of a head slice, (x + bias) * scale, split into the plane image;
// unit = (row, 16-d segment): four float4 loads, two 16-B chunks per plane
template <int NT>
HS_DEVICE void stage_planes(char* img, const float* base, int64_t ld, int r0, int n, const float* bias, float scale) {
  for (int u = threadIdx.x; u < 64 * 4; u += NT) {
    const int row = u >> 2, seg = u & 3;
    if (row >= n) continue;
    float v[2][8];
    ld8(base + (int64_t)(r0 + row) * ld + 16 * seg, bias ? bias + 16 * seg : nullptr, scale, v[0]);
    ld8(base + (int64_t)(r0 + row) * ld + 16 * seg + 8, bias ? bias + 16 * seg + 8 : nullptr, scale, v[1]);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      bfx8 f[3];
      split8(v[e], f[0], f[1], f[2]);
      const int off = row * kPRow + 16 * ((2 * seg + e) ^ pswz(row));
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<bfx8*>(img + pl * kPPlane + off) = f[pl];
    }
  }
}

// stage_planes for dO rows that also writes D[row] = rowsum(dO o O) of the head (O rows at orows,
// row stride ld): the four threads of a row (16 d each) reduce their partial dots by shuffles
template <int NT>
HS_DEVICE void stage_planes_dsum(char* img, const float* base, const float* obase, int64_t ld, int r0, int n,
                                 float* Dsm) {
  for (int u = threadIdx.x; u < 64 * 4; u += NT) {
    const int row = u >> 2, seg = u & 3;
    float dsum = 0.f;
    if (row < n) {
      float v[2][8], o[8];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        ld8(base + (int64_t)(r0 + row) * ld + 16 * seg + 8 * e, nullptr, 1.f, v[e]);
        ld8(obase + (int64_t)(r0 + row) * ld + 16 * seg + 8 * e, nullptr, 1.f, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum = fmaf(v[e][j], o[j], dsum);
        bfx8 f[3];
        split8(v[e], f[0], f[1], f[2]);
        const int off = row * kPRow + 16 * ((2 * seg + e) ^ pswz(row));
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<bfx8*>(img + pl * kPPlane + off) = f[pl];
      }
    }
    dsum += __shfl_xor(dsum, 1, 64);
    dsum += __shfl_xor(dsum, 2, 64);
    if (row < n && seg == 0) Dsm[row] = dsum;
  }
}

// row fragment of plane pl: row `row` (this lane's), 16-B chunk c (= 2 ks + lane half)
HS_DEVICE bfx8 prow_frag(const char* img, int pl, int row, int c) {
  return *reinterpret_cast<const bfx8*>(img + pl * kPPlane + row * kPRow + 16 * (c ^ pswz(row)));
}

// transposed fragment of plane pl: lane (r, h) gets column d0 + r of rows q0 + 4h + 8(j>>2) + (j&3)
// (j = 0..7: the order of score registers 8ks..8ks+7, so it pairs with P / dS as the B operand)
HS_DEVICE bfx8 ptr_frag(const char* img, int pl, int d0, int q0, int lane) {
  const int l16 = lane & 15, qq = l16 >> 2, pp = l16 & 3, g = lane >> 4;
  const int col = d0 + 16 * (g & 1) + 4 * pp;
  const char* plb = img + pl * kPPlane;
  ps4 v[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int row = q0 + 4 * (g >> 1) + 8 * jj + qq;
    const char* a = plb + row * kPRow + 16 * ((col >> 3) ^ pswz(row)) + 2 * (col & 7);
    v[jj] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) ps4*)(a));
  }
  const ps8 u = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
  return __builtin_bit_cast(bfx8, u);
}

}  // namespace

// ---------------------------------------------------------------------------
// Backward on pre-split plane images ("p" kernels; any S % 32 == 0): like the dQ / dKV pair
// above, but each 64-row chunk of the shared operand is split into planes once per block
// (instead of once per wave and fragment) and the transposed fragments come from the same
// image through ds_read_b64_tr_b16 (no scalar gathers, no second split).  Per 32x32 tile a
// wave splits only its own K / V (or Q / dO) fragments and the P / dS registers.  48 KB of
// LDS, two blocks per CU.

// LDS of one block of the backward pair: the dKV role's Q / dO plane images + per-query lse, D
// and keep words, or the dQ role's K / V plane images + key mask (the larger layout: 50.7 KB)
constexpr int kBwdSmem = 2 * kPImg + 64 * 4 * 2 + 64 * 4 * 4;

// dK / dV for 32 keys per wave (lane = key) over 64-query chunks of Q (biased, * 1/8) and dO;
// bx = the block's 128-key group.
HS_DEVICE void dkv_x6p_body(char* __restrict__ smem, int bx, int bh, const float* __restrict__ qkv,
                            const int64_t* __restrict__ mask, const float* __restrict__ bqkv,
                            const float* __restrict__ dctx, const float* __restrict__ lse,
                            const float* __restrict__ Dd, float* __restrict__ dqkv, int S, int NH, float p,
                            const uint32_t* __restrict__ dmask, const float* __restrict__ ctx) {
  char* const Qp = smem;
  char* const Op = smem + kPImg;
  float* const Ls = reinterpret_cast<float*>(smem + 2 * kPImg);
  float* const Ds = Ls + 64;
  uint32_t(*const Wd)[4] = reinterpret_cast<uint32_t(*)[4]>(Ds + 64);
  const int H = NH * kXD;
  const int64_t ld = 3 * (int64_t)H;
  const int b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int k0 = bx * 128 + w * 32;
  const bool active = k0 < S;
  const int key = k0 + li;
  const float* rows = qkv + (int64_t)b * S * ld;
  const float* drows = dctx + (int64_t)b * S * H;
  const float dscale = drop_scale16(drop_thr16(p));

  // the lane's K / V rows, split once (they are the B operand of every tile)
  bfx8 kb[4][3], vb[4][3];
  float madd = 0.f;
  {
    float kr[4][8], vr[4][8];
    if (active) {
      row_frags(rows + (int64_t)key * ld + H + h * kXD, bofs(bqkv, H + h * kXD), hf, kr);
      row_frags(rows + (int64_t)key * ld + 2 * H + h * kXD, bofs(bqkv, 2 * H + h * kXD), hf, vr);
      madd = (1.f - (float)mask[(int64_t)b * S + key]) * -10000.f;
    } else {
#pragma unroll
      for (int ss = 0; ss < 4; ++ss)
#pragma unroll
        for (int j = 0; j < 8; ++j) kr[ss][j] = vr[ss][j] = 0.f;
    }
#pragma unroll
    for (int ss = 0; ss < 4; ++ss) {
      split8(kr[ss], kb[ss][0], kb[ss][1], kb[ss][2]);
      split8(vr[ss], vb[ss][0], vb[ss][1], vb[ss][2]);
    }
  }
  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  for (int c0 = 0; c0 < S; c0 += 64) {
    const int clen = min(64, S - c0);
    __syncthreads();
    stage_planes<256>(Qp, rows + h * kXD, ld, c0, clen, bofs(bqkv, h * kXD), 0.125f);
    if (ctx) {  // D = rowsum(dO o O) of the chunk's queries computed while dO is staged
      stage_planes_dsum<256>(Op, drows + h * kXD, ctx + (int64_t)b * S * H + h * kXD, H, c0, clen, Ds);
      for (int i = threadIdx.x; i < clen; i += blockDim.x) Ls[i] = lse[(int64_t)bh * S + c0 + i];
    } else {
      stage_planes<256>(Op, drows + h * kXD, H, c0, clen, nullptr, 1.f);
      for (int i = threadIdx.x; i < clen; i += blockDim.x) {
        Ls[i] = lse[(int64_t)bh * S + c0 + i];
        Ds[i] = Dd[(int64_t)bh * S + c0 + i];
      }
    }
    if (p > 0.f)
      for (int i = threadIdx.x; i < clen * 4; i += blockDim.x) {
        const int qi = i >> 2, kw = bx * 4 + (i & 3);
        Wd[qi][i & 3] = kw < (S >> 5) ? dmask[((uint64_t)bh * S + c0 + qi) * (uint64_t)(S >> 5) + kw] : 0u;
      }
    __syncthreads();
    if (!active) continue;
    for (int t = 0; t < clen; t += 32) {
      f32x16 sc = {}, dp = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bfx8 a[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a[pl] = prow_frag(Qp, pl, t + li, 2 * ks + hf);
        sc = mma6(a, kb[ks], sc);
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bfx8 a[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a[pl] = prow_frag(Op, pl, t + li, 2 * ks + hf);
        dp = mma6(a, vb[ks], dp);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float pd[8], ds[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int r = 8 * ks + j, qi = t + xrow(r, hf);
          const float pv = __expf(sc[r] + madd - Ls[qi]);
          const float mk = p > 0.f ? (((Wd[qi][w] >> li) & 1u) ? dscale : 0.f) : 1.f;
          pd[j] = pv * mk;
          ds[j] = pv * (dp[r] * mk - Ds[qi]);
        }
        bfx8 pb[3], a[3];
        split8(pd, pb[0], pb[1], pb[2]);
        const int q0 = t + 16 * ks;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a[pl] = ptr_frag(Op, pl, 0, q0, lane);
        dv0 = mma6(a, pb, dv0);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a[pl] = ptr_frag(Op, pl, 32, q0, lane);
        dv1 = mma6(a, pb, dv1);
        split8(ds, pb[0], pb[1], pb[2]);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a[pl] = ptr_frag(Qp, pl, 0, q0, lane);
        dk0 = mma6(a, pb, dk0);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a[pl] = ptr_frag(Qp, pl, 32, q0, lane);
        dk1 = mma6(a, pb, dk1);
      }
    }
  }
  if (!active) return;
  float* out = dqkv + ((int64_t)b * S + key) * ld + h * kXD;
  store_rows(out + H, dk0, dk1, hf, 1.f);
  store_rows(out + 2 * H, dv0, dv1, hf, 1.f);
}

// dQ for 32 queries per wave (lane = query) over 64-key chunks of K / V (biased); bx = the
// block's 128-query group; D = rowsum(dO o O) read from attn_bwd_dsum_kernel's output.
HS_DEVICE void dq_x6p_body(char* __restrict__ smem, int bx, int bh, const float* __restrict__ qkv,
                           const int64_t* __restrict__ mask, const float* __restrict__ bqkv,
                           const float* __restrict__ dctx, const float* __restrict__ lse, const float* __restrict__ Dd,
                           float* __restrict__ dqkv, int S, int NH, float p, const uint32_t* __restrict__ dmask,
                           const float* __restrict__ ctx) {
  char* const Kp = smem;
  char* const Vp = smem + kPImg;
  float* const Ms = reinterpret_cast<float*>(smem + 2 * kPImg);
  const int H = NH * kXD;
  const int64_t ld = 3 * (int64_t)H;
  const int b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int q0 = bx * 128 + w * 32;
  const bool active = q0 < S;
  const float* rows = qkv + (int64_t)b * S * ld;
  const float dscale = drop_scale16(drop_thr16(p));

  // the lane's Q (biased, * 1/8) and dO rows, split once (the B operand of every tile)
  bfx8 qb[4][3], ob[4][3];
  float dsum = 0.f, lq = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    float qr[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, dor[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (active) {
      const int64_t tok = (int64_t)b * S + q0 + li;
      const int d = 16 * s + 8 * hf;
      ld8(rows + (int64_t)(q0 + li) * ld + h * kXD + d, bofs(bqkv, h * kXD + d), 0.125f, qr);
      ld8(dctx + tok * H + h * kXD + d, nullptr, 1.f, dor);
      if (ctx) {  // D = rowsum(dO o O): this lane's half of the row, the other half from lane ^ 32
        float o[8];
        ld8(ctx + tok * H + h * kXD + d, nullptr, 1.f, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum = fmaf(dor[j], o[j], dsum);
      }
    }
    split8(qr, qb[s][0], qb[s][1], qb[s][2]);
    split8(dor, ob[s][0], ob[s][1], ob[s][2]);
  }
  if (ctx) dsum += __shfl_xor(dsum, 32, 64);
  if (active) {
    if (!ctx) dsum = Dd[(int64_t)bh * S + q0 + li];
    lq = lse[(int64_t)bh * S + q0 + li];
  }
  f32x16 dq0 = {}, dq1 = {};
  for (int c0 = 0; c0 < S; c0 += 64) {
    const int clen = min(64, S - c0);
    __syncthreads();
    stage_planes<256>(Kp, rows + H + h * kXD, ld, c0, clen, bofs(bqkv, H + h * kXD), 1.f);
    stage_planes<256>(Vp, rows + 2 * H + h * kXD, ld, c0, clen, bofs(bqkv, 2 * H + h * kXD), 1.f);
    for (int i = threadIdx.x; i < clen; i += blockDim.x) Ms[i] = (1.f - (float)mask[(int64_t)b * S + c0 + i]) * -10000.f;
    __syncthreads();
    if (!active) continue;
    for (int t = 0; t < clen; t += 32) {
      f32x16 sc = {}, dp = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bfx8 a[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a[pl] = prow_frag(Kp, pl, t + li, 2 * ks + hf);
        sc = mma6(a, qb[ks], sc);
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bfx8 a[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a[pl] = prow_frag(Vp, pl, t + li, 2 * ks + hf);
        dp = mma6(a, ob[ks], dp);
      }
      const uint32_t word = p > 0.f ? dmask[((uint64_t)bh * S + q0 + li) * (uint64_t)(S >> 5) + ((c0 + t) >> 5)] : 0u;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float ds[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int r = 8 * ks + j, kj = xrow(r, hf);
          const float mk = p > 0.f ? (((word >> kj) & 1u) ? dscale : 0.f) : 1.f;
          const float pv = __expf(sc[r] + Ms[t + kj] - lq);
          ds[j] = pv * (dp[r] * mk - dsum);
        }
        bfx8 sb[3], a[3];
        split8(ds, sb[0], sb[1], sb[2]);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a[pl] = ptr_frag(Kp, pl, 0, t + 16 * ks, lane);
        dq0 = mma6(a, sb, dq0);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) a[pl] = ptr_frag(Kp, pl, 32, t + 16 * ks, lane);
        dq1 = mma6(a, sb, dq1);
      }
    }
  }
  if (!active) return;
  store_rows(dqkv + ((int64_t)b * S + q0 + li) * ld + h * kXD, dq0, dq1, hf, 0.125f);
}

// D[bh][q] = rowsum(dO o O) over the head's 64 dims: 16 lanes per (token, head), float4 each.
__global__ void __launch_bounds__(256) attn_bwd_dsum_kernel(const float* __restrict__ ctx,
                                                            const float* __restrict__ dctx, float* __restrict__ Dout,
                                                            int B, int S, int NH) {
  const int64_t u = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);  // (token, head) unit
  const int l = threadIdx.x & 15;
  const int64_t units = (int64_t)B * S * NH;
  const int64_t tok = u / NH;
  const int h = (int)(u % NH);
  float v = 0.f;
  if (u < units) {
    const int64_t o = tok * NH * kXD + h * kXD + 4 * l;
    const float4 a = *reinterpret_cast<const float4*>(dctx + o), c = *reinterpret_cast<const float4*>(ctx + o);
    v = a.x * c.x + a.y * c.y + a.z * c.z + a.w * c.w;
  }
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) v += __shfl_xor(v, m, 16);
  if (u < units && l == 0) {
    const int64_t b = tok / S, q = tok % S;
    Dout[(b * NH + h) * S + q] = v;
  }
}

// The backward pair as ONE launch: blocks x < nq run the dQ role, the rest the dK / dV role (both
// only read D, computed beforehand).  Sequential dQ and dKV launches each ran (S/128) * B*NH blocks
// on 512 two-per-CU slots -- 0.75 of a round at S = 512, B = 8, NH = 12, half the CUs holding one
// block -- and waited for each other; one launch of both roles fills the slots the first round
// leaves and backfills the second.
__global__ void __launch_bounds__(256, 2)
    attn_bwd_x6p_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ mask,
                        const float* __restrict__ bqkv, const float* __restrict__ dctx,
                        const float* __restrict__ lse, const float* __restrict__ Dd, float* __restrict__ dqkv, int S,
                        int NH, float p, const uint32_t* __restrict__ dmask, int dkv_first,
                        const float* __restrict__ ctx) {
  // ctx != nullptr: both roles compute D = rowsum(dO o O) themselves (no attn_bwd_dsum pass; S <= 128,
  // where each head's one dK / dV block stages every query once)
  __shared__ __attribute__((aligned(16))) char smem[kBwdSmem];
  // grid (B*NH, 2 * nq): blocks dispatch x-fastest, so every head's dK / dV blocks (the longer
  // role) go out before the dQ ones and the shorter blocks fill the tail of the last round
  const int nq = (S + 127) / 128, bh = blockIdx.x;
  const int y = blockIdx.y, first = y < nq, g = first ? y : y - nq;  // role group, block in the role
  if (first == (dkv_first != 0))
    dkv_x6p_body(smem, g, bh, qkv, mask, bqkv, dctx, lse, Dd, dqkv, S, NH, p, dmask, ctx);
  else
    dq_x6p_body(smem, g, bh, qkv, mask, bqkv, dctx, lse, Dd, dqkv, S, NH, p, dmask, ctx);
}

// ---------------------------------------------------------------------------
// Plane-image fragment helpers of the forward below.
// Lane byte offsets of ptr_frag's two ds_read_b64_tr_b16 per (d0 = 0 / 32, jj) in a 64-d plane image,
// relative to row q0 (a multiple of 16: the swizzle depends on row bits 1..3 only), so every
// transposed fragment of a phase is one of four base registers + an immediate offset.
struct TrBase {
  int o[2][2];
};
HS_DEVICE TrBase tr_base(int lane) {
  TrBase t;
  const int l16 = lane & 15, qq = l16 >> 2, pp = l16 & 3, g = lane >> 4;
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int row = 4 * (g >> 1) + 8 * jj + qq, col = 32 * dh + 16 * (g & 1) + 4 * pp;
      t.o[dh][jj] = row * kPRow + 16 * ((col >> 3) ^ pswz(row)) + 2 * (col & 7);
    }
  return t;
}
// ptr_frag with the offsets precomputed: plb = plane base + q0 rows
HS_DEVICE bfx8 ptr_frag_b(const char* plb, const TrBase& t, int dh) {
  ps4 v[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj)
    v[jj] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) ps4*)(plb + t.o[dh][jj]));
  const ps8 u = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
  return __builtin_bit_cast(bfx8, u);
}

// A value the compiler must treat as new at this point: lane-derived LDS addresses are recomputed
// per phase instead of being hoisted out of the slice loop (and spilled around it).
HS_DEVICE int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// 8 fp32 -> planes at 16-B chunk c of row `row` of a plane image (plane stride ps)
HS_DEVICE void put_planes(char* img, int ps, int row, int c, const float (&v)[8]) {
  bfx8 f[3];
  split8(v, f[0], f[1], f[2]);
  const int off = row * kPRow + 16 * (c ^ pswz(row));
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<bfx8*>(img + pl * ps + off) = f[pl];
}

// ---------------------------------------------------------------------------
// Forward on plane images ("p" forward, fp32 default): attn_fwd_x6_kernel's algorithm (a wave owns
// 32 queries, S^T tiles with the key on the registers, online softmax, the same keep bits) with
// the backward kernels' operand staging: each 64-key chunk of K and of V is split once into
// [key][64 d] plane images (16-B b128 stores, the pswz swizzle) -- S = K Q^T reads K fragments by
// rows, P V reads V^T fragments transposed (ds_read_b64_tr_b16) from the same row-major image.
// The first x6 forward staged V^T by 2-byte scalar stores (48 per thread and chunk, 28 % LDS bank
// conflicts).  The next chunk's K / V rows are loaded under the current chunk's MFMAs.  48 KB LDS.
__global__ void __launch_bounds__(256, 2)
    attn_fwd_x6p_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ mask,
                        const float* __restrict__ bqkv, float* __restrict__ ctx, float* __restrict__ lse,
                        uint32_t* __restrict__ dmask, int S, int NH, float p, uint64_t seed, uint64_t off,
                        const uint64_t* __restrict__ seed_dev, int bh0) {
  seed = resolve_seed(seed, seed_dev);
  __shared__ __attribute__((aligned(16))) char smem[2 * kPImg];
  __shared__ float Ms[kXCH];
  __shared__ __attribute__((aligned(16))) float KVb[2 * kXD];  // K and V bias of the head
  char* const Kimg = smem;
  char* const Vimg = smem + kPImg;
  const int H = NH * kXD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5, li = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q0 = blockIdx.y * 128 + w * 32;
  const bool active = q0 < S;
  const float* rows = qkv + (int64_t)b * S * ld;
  const uint32_t thr = drop_thr16(p);
  const float dscale = drop_scale16(thr);
  if (tid < 2 * kXD) KVb[tid] = bqkv ? bqkv[(1 + (tid >> 6)) * H + h * kXD + (tid & 63)] : 0.f;

  // the lane's Q row, dims 16s + 8hf + j (k-step s), biased, * 1/sqrt(64) (exact), split
  bfx8 qf[4][3];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int d = 16 * s + 8 * hf;
    if (active) ld8(rows + (int64_t)(q0 + li) * ld + h * kXD + d, bofs(bqkv, h * kXD + d), 0.125f, v);
    split8(v, qf[s][0], qf[s][1], qf[s][2]);
  }
  f32x16 o0 = {}, o1 = {};
  float m = -1e30f, l = 0.f;
  const uint64_t erow = ((uint64_t)(bh0 + bh) * S + (q0 + li)) * (uint64_t)S;  // bh0: a batch slice's first head

  // staging units of this thread: (key row u >> 3, 8-d chunk u & 7) for u = tid, tid + 256, of K and V
  float4 kv[2][2][2];  // [K / V][unit][half]
  auto load = [&](int c0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int u = tid + 256 * i, r = u >> 3, c8 = (u & 7) * 8;
      const bool ok = c0 + r < S;
#pragma unroll
      for (int kvs = 0; kvs < 2; ++kvs) {
        const float* src = rows + (int64_t)(c0 + r) * ld + (1 + kvs) * H + h * kXD + c8;
        kv[kvs][i][0] = ok ? *reinterpret_cast<const float4*>(src) : make_float4(0.f, 0.f, 0.f, 0.f);
        kv[kvs][i][1] = ok ? *reinterpret_cast<const float4*>(src + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  load(0);
  __syncthreads();  // KVb
  for (int c0 = 0; c0 < S; c0 += kXCH) {
    const int clen = min(kXCH, S - c0);
    if (c0 > 0) __syncthreads();  // every wave done with the previous chunk's images
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int u = tid + 256 * i, r = u >> 3, c = u & 7;
#pragma unroll
      for (int kvs = 0; kvs < 2; ++kvs) {
        const float* bb = KVb + kvs * kXD + 8 * c;
        const float4 x = kv[kvs][i][0], y = kv[kvs][i][1];
        const float v[8] = {x.x + bb[0], x.y + bb[1], x.z + bb[2], x.w + bb[3],
                            y.x + bb[4], y.y + bb[5], y.z + bb[6], y.w + bb[7]};
        put_planes(kvs ? Vimg : Kimg, kPPlane, r, c, v);
      }
    }
    for (int i = tid; i < clen; i += blockDim.x) Ms[i] = (1.f - (float)mask[(int64_t)b * S + c0 + i]) * -10000.f;
    __syncthreads();
    if (c0 + kXCH < S) load(c0 + kXCH);  // the next chunk's rows fly under this chunk's MFMAs
    if (!active) continue;
    const int ln = opaque(lane);
    const TrBase tb = tr_base(ln);
    for (int t = 0; t < clen; t += 32) {
      f32x16 s = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bfx8 kf[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) kf[pl] = prow_frag(Kimg, pl, t + li, 2 * ks + hf);
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
        const char* vb = Vimg + (t + 16 * ks) * kPRow;
        bfx8 a0[3], a1[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          a0[pl] = ptr_frag_b(vb + pl * kPPlane, tb, 0);
          a1[pl] = ptr_frag_b(vb + pl * kPPlane, tb, 1);
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

// The strict-fp32 (x6) attention: the plane-image forward and the plane-image dQ / dKV backward pair,
// both roles in one launch (dK / dV blocks dispatched first).  (The key-block backward kernels, the
// first x6 forward and the separate-D option were measured slower and removed in round 5:
// profiles/r3_attention.md.)
int launch_attn_bwd_x6(const float* qkv, const int64_t* mask, const float* bqkv, const float* ctx, const float* dctx,
                       const float* lse, float* Dbuf, float* dqkv, const uint32_t* dmask, int B, int S, int NH,
                       int D, float p, hipStream_t st) {
  if (D != kXD || S % 32 != 0 || S <= 0 || (p > 0.f && dmask == nullptr)) return -1;
  const bool fused_d = S <= 128;  // the roles compute D = rowsum(dO o O) themselves; else a separate pass
  if (!fused_d) {
    const int64_t units = (int64_t)B * S * NH;
    hipLaunchKernelGGL(attn_bwd_dsum_kernel, dim3((unsigned)((units + 15) / 16)), dim3(256), 0, st, ctx, dctx, Dbuf,
                       B, S, NH);
  }
  dim3 grid(B * NH, 2 * ((S + 127) / 128));
  hipLaunchKernelGGL(attn_bwd_x6p_kernel, grid, dim3(256), 0, st, qkv, mask, bqkv, dctx, lse, Dbuf, dqkv, S, NH, p,
                     dmask, 1, fused_d ? ctx : nullptr);
  return 0;
}

// D = rowsum(dO o O) per (batch, head, query) for the S > 128 backward of either fp32 engine
int hs::launch_attn_bwd_dsum(const float* ctx, const float* dctx, float* Dout, int B, int S, int NH, hipStream_t st) {
  const int64_t units = (int64_t)B * S * NH;
  hipLaunchKernelGGL(attn_bwd_dsum_kernel, dim3((unsigned)((units + 15) / 16)), dim3(256), 0, st, ctx, dctx, Dout, B, S,
                     NH);
  return 0;
}

int launch_attn_fwd_x6(const float* qkv, const int64_t* mask, const float* bqkv, float* ctx, float* lse,
                       uint32_t* dmask, int B, int S, int NH, int D, float p, uint64_t seed, uint64_t off,
                       hipStream_t st, int bh0) {
  if (D != kXD || S % 32 != 0 || S <= 0) return -1;
  // grid (B*NH, S/128): consecutive blocks are different heads, so (B*NH a multiple of 8) every
  // query block of a head lands on the same XCD and its K / V come through one L2
  dim3 grid(B * NH, (S + 127) / 128);
  hipLaunchKernelGGL(attn_fwd_x6p_kernel, grid, dim3(256), 0, st, qkv, mask, bqkv, ctx, lse, dmask, S, NH, p, seed,
                     off, g_seed_dev, bh0);
  return 0;
}
