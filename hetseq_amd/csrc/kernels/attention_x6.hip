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

// ---- backward helpers (fp32 tiles in LDS, split into planes as fragments are read) ----
constexpr int kBLD = 68;    // fp32 row stride of staged Q / dO / K / V rows: conflict-free b128 fragment reads
constexpr int kBLS = 132;   // fp32 row stride of dS [query][key] and K^T [d][key] (fused kernel)

// 8 consecutive fp32 of an LDS row (two b128 reads) -> hi/mid/lo fragment planes
HS_DEVICE void lds_planes(const float* p, bfx8 (&f)[3]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  split8(v, f[0], f[1], f[2]);
}

// k-step fragment of a transposed operand: column `col` of rows r0 + {0..3, 8..11} (the
// accumulator-register order of a 16-row k-step) -> planes
HS_DEVICE void lds_col_planes(const float* base, int r0, int col, bfx8 (&f)[3]) {
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = base[(r0 + (j & 3) + 8 * (j >> 2)) * kBLD + col];
  split8(v, f[0], f[1], f[2]);
}

// rows [r0, r0 + n) of a head slice -> LDS (fp32, kBLD stride), (x + bias) * scale; 256 or 512
// threads, 16 per row (4 floats each); rows past n are not written
template <int NT>
HS_DEVICE void stage_x6(float* lds, const float* base, int64_t ld, int r0, int n, const float* bias, float scale) {
  const int c4 = (threadIdx.x & 15) * 4;
  float4 bb = make_float4(0.f, 0.f, 0.f, 0.f);
  if (bias) bb = *reinterpret_cast<const float4*>(bias + c4);
  constexpr int kPer = 128 * 16 / NT;
  float4 v[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int r = min((int)(threadIdx.x + i * NT) >> 4, n - 1);
    v[i] = *reinterpret_cast<const float4*>(base + (int64_t)(r0 + r) * ld + c4);
  }
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int r = (threadIdx.x + i * NT) >> 4;
    if (r < n)
      *reinterpret_cast<float4*>(lds + r * kBLD + c4) = make_float4((v[i].x + bb.x) * scale, (v[i].y + bb.y) * scale,
                                                                    (v[i].z + bb.z) * scale, (v[i].w + bb.w) * scale);
  }
}

// One 32-key x 32-query tile of the key-side backward (dK / dV), lane = key:
//   S^T-tile sc[query][key] = Q K^T, dp = dO V^T (A = Q / dO rows from LDS, B = the lane's K / V row),
//   P and dS = P o (dP o keep - D) in registers, then dV^T += dO^T P, dK^T += Q^T dS with the
//   registers as the B operand and dO^T / Q^T gathered from the row-major LDS images.
// Qs / Os: staged rows (Q scaled by 1/8), t: tile's first row in them; Lq / Dq / keep: per-row
// lse, D and keep word of row t + i.  ds_out: optional dS sink (fused kernel), row stride kBLS.
struct KeyTile {
  const float* Qs;
  const float* Os;
  const float* Ls;
  const float* Ds;
  const uint32_t* Wd;  // keep word of (row, this wave's key word), stride wstride
  int wstride;
  float p, dscale;
};

HS_DEVICE void key_tile(const KeyTile& k, int t, const float (&kr)[4][8], const float (&vr)[4][8], float madd, int li,
                        int hf, f32x16& dk0, f32x16& dk1, f32x16& dv0, f32x16& dv1, float* ds_out, int key) {
  // one product at a time and P / dS built per k-step: the live fragments stay under the
  // 256-VGPR budget of two waves per SIMD
  f32x16 sc = {}, dp = {};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    bfx8 a[3], bb[3];
    lds_planes(k.Qs + (t + li) * kBLD + 16 * ks + 8 * hf, a);
    split8(kr[ks], bb[0], bb[1], bb[2]);
    sc = mma6(a, bb, sc);
  }
  __builtin_amdgcn_sched_barrier(0);  // bound the live fragments (no spills at 256 VGPRs)
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    bfx8 a[3], bb[3];
    lds_planes(k.Os + (t + li) * kBLD + 16 * ks + 8 * hf, a);
    split8(vr[ks], bb[0], bb[1], bb[2]);
    dp = mma6(a, bb, dp);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    float pd[8], ds[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = 8 * ks + j, qi = t + xrow(r, hf);
      const float pv = __expf(sc[r] + madd - k.Ls[qi]);
      const float mk = k.p > 0.f ? (((k.Wd[qi * k.wstride] >> li) & 1u) ? k.dscale : 0.f) : 1.f;
      pd[j] = pv * mk;
      ds[j] = pv * (dp[r] * mk - k.Ds[qi]);
      if (ds_out) ds_out[qi * kBLS + key] = ds[j];
    }
    bfx8 pb[3], a[3];
    split8(pd, pb[0], pb[1], pb[2]);
    const int q = t + 16 * ks + 4 * hf;
    lds_col_planes(k.Os, q, li, a);
    dv0 = mma6(a, pb, dv0);
    lds_col_planes(k.Os, q, 32 + li, a);
    dv1 = mma6(a, pb, dv1);
    split8(ds, pb[0], pb[1], pb[2]);
    lds_col_planes(k.Qs, q, li, a);
    dk0 = mma6(a, pb, dk0);
    lds_col_planes(k.Qs, q, 32 + li, a);
    dk1 = mma6(a, pb, dk1);
  }
}

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

__global__ void __launch_bounds__(256, 2)
    attn_fwd_x6_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ mask, const float* __restrict__ bqkv,
                       float* __restrict__ ctx, float* __restrict__ lse, uint32_t* __restrict__ dmask, int S, int NH,
                       float p, uint64_t seed, uint64_t off, const uint64_t* __restrict__ seed_dev, int bh0) {
  seed = resolve_seed(seed, seed_dev);
  __shared__ __attribute__((aligned(16))) __bf16 Ks[3][kXCH * kXKLD];
  __shared__ __attribute__((aligned(16))) __bf16 Vt[3][kXD * kXVLD];
  __shared__ float Ms[kXCH];
  const int H = NH * kXD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int q0 = blockIdx.y * 128 + w * 32;
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
  const uint64_t erow = ((uint64_t)(bh0 + bh) * S + (q0 + li)) * (uint64_t)S;  // bh0: a batch slice's first head

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

// ---------------------------------------------------------------------------
// Backward, fp32 operands as split-bf16 products (the forward's scheme; reference
// bert_modeling.py:361-376).  Staged tiles stay fp32 in LDS (the most compact image: one
// plane set would take 1.5x the bytes) and every fragment is split into hi/mid/lo planes in
// registers as it is read, so a 32x32 product costs 6 x 2 bf16 MFMAs per 16-deep k-step
// (24 x 32 cycles per 64-deep tile) instead of 32 exact-fp32 v_mfma_f32_32x32x2_f32 (2048).
//
// Fused, S <= 128: one block (8 waves) per (batch, head), the x6 counterpart of
// attn_bwd_fused_kernel (attention.hip): phase 1 wave (kg = w & 3, half = w >> 2) runs key_tile
// over query tiles {64 half, 64 half + 32} for keys 32 kg.. and stores dS [query][key]; phase 2
// dQ^T = K^T dS^T for queries 32 kg.. over keys 64 half.. with K^T staged from the registers;
// waves 4..7 hand their partials to waves 0..3 (fixed order).  LDS 140 KB, one block per CU.
__global__ void __launch_bounds__(512, 1)
    attn_bwd_fused_x6_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ mask,
                             const float* __restrict__ bqkv, const float* __restrict__ ctx,
                             const float* __restrict__ dctx, const float* __restrict__ lse, float* __restrict__ dqkv,
                             int S, int NH, float p, const uint32_t* __restrict__ dmask) {
  __shared__ __attribute__((aligned(16))) float QKs[128 * kBLD];  // Q rows; K^T [64][kBLS] in phase 2
  __shared__ __attribute__((aligned(16))) float Os[128 * kBLD];   // dO rows; then dQ partials
  __shared__ __attribute__((aligned(16))) float dSs[128 * kBLS];  // dS; then dK / dV partials
  __shared__ float Ls[128];
  __shared__ float Ds[128];
  __shared__ uint32_t Wd[128][4];
  static_assert(64 * kBLS <= 128 * kBLD, "K^T image fits the Q region");
  const int H = NH * kXD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int g4 = w & 3, half = w >> 2;
  const bool kactive = 32 * g4 < S;
  const int key = 32 * g4 + li;
  const float* rows = qkv + (int64_t)b * S * ld;
  const float* drows = dctx + (int64_t)b * S * H;

  stage_x6<512>(QKs, rows + h * kXD, ld, 0, S, bofs(bqkv, h * kXD), 0.125f);
  stage_x6<512>(Os, drows + h * kXD, H, 0, S, nullptr, 1.f);
  for (int i = threadIdx.x; i < S; i += blockDim.x) Ls[i] = lse[(int64_t)bh * S + i];
  if (p > 0.f)
    for (int i = threadIdx.x; i < S * (S >> 5); i += blockDim.x)
      Wd[i / (S >> 5)][i % (S >> 5)] = dmask[((uint64_t)bh * S) * (uint64_t)(S >> 5) + i];
  float kr[4][8], vr[4][8];
  float madd = 0.f;
  if (kactive) {
    row_frags(rows + (int64_t)key * ld + H + h * kXD, bofs(bqkv, H + h * kXD), hf, kr);
    row_frags(rows + (int64_t)key * ld + 2 * H + h * kXD, bofs(bqkv, 2 * H + h * kXD), hf, vr);
    madd = (1.f - (float)mask[(int64_t)b * S + key]) * -10000.f;
  }
  {  // D = rowsum(dO o O), 4 threads per query row
    const int r = threadIdx.x >> 2, qtr = threadIdx.x & 3;
    float dsum = 0.f;
    if (r < S) {
      const float* orow = ctx + ((int64_t)b * S + r) * H + h * kXD + qtr * 16;
      const float* grow = drows + (int64_t)r * H + h * kXD + qtr * 16;
#pragma unroll
      for (int c = 0; c < 16; c += 4) {
        const float4 o = *reinterpret_cast<const float4*>(orow + c), g = *reinterpret_cast<const float4*>(grow + c);
        dsum = fmaf(g.x, o.x, fmaf(g.y, o.y, fmaf(g.z, o.z, fmaf(g.w, o.w, dsum))));
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
    const KeyTile kt{QKs, Os, Ls, Ds, &Wd[0][g4], 4, p, drop_scale16(drop_thr16(p))};
    for (int t = 64 * half; t < min(S, 64 * half + 64); t += 32)
      key_tile(kt, t, kr, vr, madd, li, hf, dk0, dk1, dv0, dv1, dSs, key);
  }
  __syncthreads();  // Q, dO consumed; dS complete
  if (kactive && half == 0)  // K^T [d][key] from the lanes' K rows
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) QKs[(16 * s + 8 * hf + j) * kBLS + key] = kr[s][j];
  __syncthreads();

  // ---- phase 2: dQ^T partial for queries 32 g4.. over keys 64 half..
  f32x16 dq0 = {}, dq1 = {};
  if (kactive) {
    const float* dsr = dSs + (32 * g4 + li) * kBLS + 8 * hf;
    for (int k0 = 64 * half; k0 < min(S, 64 * half + 64); k0 += 16) {
      bfx8 bq[3], a[3];
      lds_planes(dsr + k0, bq);
      lds_planes(QKs + li * kBLS + k0 + 8 * hf, a);
      dq0 = mma6(a, bq, dq0);
      lds_planes(QKs + (32 + li) * kBLS + k0 + 8 * hf, a);
      dq1 = mma6(a, bq, dq1);
    }
  }
  __syncthreads();  // LDS free for the hand-off

  // ---- combine (fixed order) and store
  float* xq = Os + g4 * 64 * 32 + lane;
  float* xk = dSs + g4 * 64 * 64 + lane;
  if (half == 1 && kactive) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      xq[64 * r] = dq0[r];
      xq[64 * (16 + r)] = dq1[r];
      xk[64 * r] = dk0[r];
      xk[64 * (16 + r)] = dk1[r];
      xk[64 * (32 + r)] = dv0[r];
      xk[64 * (48 + r)] = dv1[r];
    }
  }
  __syncthreads();
  if (half == 1 || !kactive) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    dq0[r] += xq[64 * r];
    dq1[r] += xq[64 * (16 + r)];
    dk0[r] += xk[64 * r];
    dk1[r] += xk[64 * (16 + r)];
    dv0[r] += xk[64 * (32 + r)];
    dv1[r] += xk[64 * (48 + r)];
  }
  float* out = dqkv + ((int64_t)b * S + key) * ld + h * kXD;  // key == query index 32 g4 + li
  store_rows(out, dq0, dq1, hf, 0.125f);
  store_rows(out + H, dk0, dk1, hf, 1.f);
  store_rows(out + 2 * H, dv0, dv1, hf, 1.f);
}

// S > 128, kernel 1 of 2: dQ for 32 queries per wave (lane = query) over 128-key chunks of
// K / V staged fp32 in LDS; also writes D = rowsum(dO o O) for kernel 2.
//   sc[key][query] = K Q^T, dp = V dO^T (A = K / V rows from LDS, B = the lane's Q / dO row);
//   dQ^T += K^T dS^T (A gathered from the K rows, B = the dS registers).
__global__ void __launch_bounds__(256, 2)
    attn_bwd_dq_x6_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ mask,
                          const float* __restrict__ bqkv, const float* __restrict__ ctx,
                          const float* __restrict__ dctx, const float* __restrict__ lse, float* __restrict__ Dout,
                          float* __restrict__ dqkv, int S, int NH, float p, const uint32_t* __restrict__ dmask) {
  __shared__ __attribute__((aligned(16))) float Ks[128 * kBLD];
  __shared__ __attribute__((aligned(16))) float Vs[128 * kBLD];
  __shared__ float Ms[128];
  const int H = NH * kXD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int q0 = blockIdx.y * 128 + w * 32;
  const bool active = q0 < S;
  const float* rows = qkv + (int64_t)b * S * ld;
  const float dscale = drop_scale16(drop_thr16(p));

  float qr[4][8], dor[4][8];
  float dsum = 0.f, lq = 0.f;
  if (active) {
    const int64_t tok = (int64_t)b * S + q0 + li;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int d = 16 * s + 8 * hf;
      ld8(rows + (int64_t)(q0 + li) * ld + h * kXD + d, bofs(bqkv, h * kXD + d), 0.125f, qr[s]);
      ld8(dctx + tok * H + h * kXD + d, nullptr, 1.f, dor[s]);
      float o[8];
      ld8(ctx + tok * H + h * kXD + d, nullptr, 1.f, o);
#pragma unroll
      for (int j = 0; j < 8; ++j) dsum = fmaf(dor[s][j], o[j], dsum);
    }
    dsum += __shfl_xor(dsum, 32, 64);
    if (hf == 0) Dout[(int64_t)bh * S + q0 + li] = dsum;
    lq = lse[(int64_t)bh * S + q0 + li];
  }
  f32x16 dq0 = {}, dq1 = {};
  for (int c0 = 0; c0 < S; c0 += 128) {
    const int clen = min(128, S - c0);
    __syncthreads();
    stage_x6<256>(Ks, rows + H + h * kXD, ld, c0, clen, bofs(bqkv, H + h * kXD), 1.f);
    stage_x6<256>(Vs, rows + 2 * H + h * kXD, ld, c0, clen, bofs(bqkv, 2 * H + h * kXD), 1.f);
    for (int i = threadIdx.x; i < clen; i += blockDim.x) Ms[i] = (1.f - (float)mask[(int64_t)b * S + c0 + i]) * -10000.f;
    __syncthreads();
    if (!active) continue;
    for (int t = 0; t < clen; t += 32) {
      f32x16 sc = {}, dp = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bfx8 a[3], bb[3];
        lds_planes(Ks + (t + li) * kBLD + 16 * ks + 8 * hf, a);
        split8(qr[ks], bb[0], bb[1], bb[2]);
        sc = mma6(a, bb, sc);
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bfx8 a[3], bb[3];
        lds_planes(Vs + (t + li) * kBLD + 16 * ks + 8 * hf, a);
        split8(dor[ks], bb[0], bb[1], bb[2]);
        dp = mma6(a, bb, dp);
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
        const int kk = t + 16 * ks + 4 * hf;
        lds_col_planes(Ks, kk, li, a);
        dq0 = mma6(a, sb, dq0);
        lds_col_planes(Ks, kk, 32 + li, a);
        dq1 = mma6(a, sb, dq1);
      }
    }
  }
  if (!active) return;
  store_rows(dqkv + ((int64_t)b * S + q0 + li) * ld + h * kXD, dq0, dq1, hf, 0.125f);
}

// S > 128, kernel 2 of 2: dK / dV for 32 keys per wave (lane = key) over 128-query chunks of
// Q (biased, * 1/8) and dO staged fp32 in LDS (key_tile per 32-query tile).
__global__ void __launch_bounds__(256, 2)
    attn_bwd_dkv_x6_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ mask,
                           const float* __restrict__ bqkv, const float* __restrict__ dctx,
                           const float* __restrict__ lse, const float* __restrict__ Dd, float* __restrict__ dqkv, int S,
                           int NH, float p, const uint32_t* __restrict__ dmask) {
  __shared__ __attribute__((aligned(16))) float Qs[128 * kBLD];
  __shared__ __attribute__((aligned(16))) float Os[128 * kBLD];
  __shared__ float Ls[128];
  __shared__ float Ds[128];
  __shared__ uint32_t Wd[128][4];  // keep words of the chunk's queries for this block's 4 key words
  const int H = NH * kXD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hf = lane >> 5, li = lane & 31;
  const int k0 = blockIdx.y * 128 + w * 32;
  const bool active = k0 < S;
  const int key = k0 + li;
  const float* rows = qkv + (int64_t)b * S * ld;
  const float* drows = dctx + (int64_t)b * S * H;

  float kr[4][8], vr[4][8];
  float madd = 0.f;
  if (active) {
    row_frags(rows + (int64_t)key * ld + H + h * kXD, bofs(bqkv, H + h * kXD), hf, kr);
    row_frags(rows + (int64_t)key * ld + 2 * H + h * kXD, bofs(bqkv, 2 * H + h * kXD), hf, vr);
    madd = (1.f - (float)mask[(int64_t)b * S + key]) * -10000.f;
  }
  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  const KeyTile kt{Qs, Os, Ls, Ds, &Wd[0][w], 4, p, drop_scale16(drop_thr16(p))};
  for (int c0 = 0; c0 < S; c0 += 128) {
    const int clen = min(128, S - c0);
    __syncthreads();
    stage_x6<256>(Qs, rows + h * kXD, ld, c0, clen, bofs(bqkv, h * kXD), 0.125f);
    stage_x6<256>(Os, drows + h * kXD, H, c0, clen, nullptr, 1.f);
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
    for (int t = 0; t < clen; t += 32) key_tile(kt, t, kr, vr, madd, li, hf, dk0, dk1, dv0, dv1, nullptr, key);
  }
  if (!active) return;
  float* out = dqkv + ((int64_t)b * S + key) * ld + h * kXD;
  store_rows(out + H, dk0, dk1, hf, 1.f);
  store_rows(out + 2 * H, dv0, dv1, hf, 1.f);
}

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
// Key-block backward, S <= 128 ("k" kernel): ONE block of 8 waves per (batch, head) runs the five
// products of the flash backward (reference bert_modeling.py:361-376) once each -- the p pair above
// recomputes S and dP in both of its roles (7 products per tile) and needs a separate D pass.
//
//   * wave (g = w >> 2, wg = w & 3) owns keys 32 wg .. 32 wg + 31 (lane = key) and, per iteration,
//     query slice 2 it + g: S and dP with the key on the lane (A = Q / dO rows of the staged slice,
//     B = the lane's K row from the K image / its V row held split in registers), P and dS in
//     registers, dV^T += dO^T P and dK^T += Q^T dS with the registers as the B operand;
//   * dS crosses LDS once, as hi / mid / lo planes written by the lane that computed it, into a
//     [key][query] image; dQ of the slice = dS K then runs on v_mfma_f32_16x16x32_bf16 with both
//     operands read transposed (ds_read_b64_tr_b16) from the dS and K images, each wave one
//     16-wide d quarter over every key -- complete, so plain stores (no atomics, no partial slabs);
//   * D = rowsum(dO o O) is computed while dO is staged (no attn_bwd_dsum launch);
//   * the two wave groups' dK / dV accumulators are added in LDS in a fixed order (deterministic).
// LDS: K image 48 KB + Q / dO images of the iteration's 64 queries 2 x 24 KB + dS image 48 KB +
// lse / D / keep words = 145.5 KB: one block (2 waves per SIMD) per CU.
constexpr int kKRows = 128;                  // keys per block
constexpr int kKPlane = kKRows * kPRow;      // 16 KB: one plane of a 128-row image
constexpr int kKImg = 3 * kKPlane;           // 48 KB
constexpr int kKSmem = 2 * kKImg + 2 * kPImg + 64 * 4 * 2 + 4 * 64 * 4 + kXD * 4;

typedef float f32x4 __attribute__((ext_vector_type(4)));

HS_DEVICE f32x4 mma16(bfx8 a, bfx8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

HS_DEVICE f32x4 mma16_6(const bfx8 (&a)[3], const bfx8 (&b)[3], f32x4 acc) {
  acc = mma16(a[2], b[0], acc);
  acc = mma16(a[0], b[2], acc);
  acc = mma16(a[1], b[1], acc);
  acc = mma16(a[1], b[0], acc);
  acc = mma16(a[0], b[1], acc);
  return mma16(a[0], b[0], acc);
}

// row fragment of plane pl of an image with plane stride ps (bytes)
HS_DEVICE bfx8 prow_frag_s(const char* img, int ps, int pl, int row, int c) {
  return *reinterpret_cast<const bfx8*>(img + pl * ps + row * kPRow + 16 * (c ^ pswz(row)));
}

// 16x16x32 operand fragment, k along the image rows: lane (i = lane & 15, g = lane >> 4) gets
// column c0 + i of rows r0 + 8 g + (0..7) -- two ds_read_b64_tr_b16, each transposing the 4 x 16
// block its 16-lane group addresses (lane 4 qq + pp: row qq, columns 4 pp .. 4 pp + 3)
HS_DEVICE bfx8 ptr16_frag(const char* plb, int c0, int r0, int lane) {
  const int l16 = lane & 15, qq = l16 >> 2, pp = l16 & 3, g = lane >> 4;
  const int col = c0 + 4 * pp;
  ps4 v[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int row = r0 + 8 * g + 4 * jj + qq;
    const char* a = plb + row * kPRow + 16 * ((col >> 3) ^ pswz(row)) + 2 * (col & 7);
    v[jj] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) ps4*)(a));
  }
  const ps8 u = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
  return __builtin_bit_cast(bfx8, u);
}

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

// per-thread staging registers of one 64-query chunk: row t >> 3, 8-wide d chunk t & 7 of Q (raw),
// dO and O
struct StageRegs {
  float4 q[2], o[2], c[2];
};

HS_DEVICE void stage_load(StageRegs& r, const float* qrow, const float* orow, const float* crow, bool ok) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    r.q[i] = ok ? *reinterpret_cast<const float4*>(qrow + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
    r.o[i] = ok ? *reinterpret_cast<const float4*>(orow + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
    r.c[i] = ok ? *reinterpret_cast<const float4*>(crow + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

__global__ void __launch_bounds__(512, 1)
    attn_bwd_x6k_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ mask,
                        const float* __restrict__ bqkv, const float* __restrict__ ctx,
                        const float* __restrict__ dctx, const float* __restrict__ lse, float* __restrict__ dqkv, int S,
                        int NH, float p, const uint32_t* __restrict__ dmask, uint64_t* __restrict__ tbuf) {
  __shared__ __attribute__((aligned(16))) char smem[kKSmem];
  // diagnostic phase clock (tools/bench_attention.py --phases): shader-clock stamps of block 0..
  int tn = 0;
  auto stamp = [&]() {
    if (tbuf && threadIdx.x == 0) tbuf[blockIdx.x * 16 + tn] = __builtin_amdgcn_s_memtime();
    ++tn;
  };
  stamp();
  char* const Kimg = smem;                     // [key][d] planes, 128 rows
  char* const Qimg = Kimg + kKImg;             // [query of the chunk][d], 64 rows
  char* const Oimg = Qimg + kPImg;             // dO rows, same layout
  char* const Simg = Oimg + kPImg;             // dS planes [key][query of the chunk], 128 rows
  float* const Ls = reinterpret_cast<float*>(Simg + kKImg);
  float* const Ds = Ls + 64;
  uint32_t* const Wd = reinterpret_cast<uint32_t*>(Ds + 64);  // [key word][query]
  const int H = NH * kXD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w >> 2, wg = w & 3;
  const int nkw = S >> 5;  // 32-key words of a keep-mask row
  const bool kactive = 32 * wg < S;
  const float* rows = qkv + (int64_t)b * S * ld;
  const float dscale = drop_scale16(drop_thr16(p));
  // staging unit of this thread: chunk row sr, d = 8 sc8 .. 8 sc8 + 7
  const int sr = tid >> 3, sc8 = tid & 7;
  float* const Qb = reinterpret_cast<float*>(Wd + 4 * 64);  // the head's Q bias (64 floats)
  if (tid < kXD) Qb[tid] = bqkv ? bqkv[h * kXD + tid] : 0.f;
  auto stage_ptrs = [&](int c0, const float*& qr, const float*& orw, const float*& cr) {
    const int64_t tok = (int64_t)b * S + c0 + sr;
    qr = qkv + tok * ld + h * kXD + 8 * sc8;
    orw = dctx + tok * H + h * kXD + 8 * sc8;
    cr = ctx + tok * H + h * kXD + 8 * sc8;
  };

  // ---- prologue: chunk 0's Q / dO / O loads in flight with the K image and the lane's V row
  StageRegs st;
  {
    const float *qr, *orw, *cr;
    stage_ptrs(0, qr, orw, cr);
    stage_load(st, qr, orw, cr, sr < S);
  }
  {  // K image (biased): rows sr and sr + 64
    const float* bk = bofs(bqkv, H + h * kXD + 8 * sc8);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = sr + 64 * i;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // rows past S: zero (phase B sums all 128 keys)
      if (r < S) ld8(rows + (int64_t)r * ld + H + h * kXD + 8 * sc8, bk, 1.f, v);
      put_planes(Kimg, kKPlane, r, sc8, v);
    }
    if (32 * wg >= S) {  // keys past S: their dS rows stay zero
      const int row = 32 * wg + (lane >> 1);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<uint4*>(Simg + pl * kKPlane + row * kPRow + 16 * (4 * (lane & 1) + j)) = make_uint4(0, 0, 0, 0);
    }
  }
  bfx8 vb[4][3];
  float madd = 0.f;
  {
    const int li = lane & 31, hf = lane >> 5, key = 32 * wg + li;
    float vr[4][8];
    if (kactive) {
      row_frags(rows + (int64_t)key * ld + 2 * H + h * kXD, bofs(bqkv, 2 * H + h * kXD), hf, vr);
      madd = (1.f - (float)mask[(int64_t)b * S + key]) * -10000.f;
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) vr[s][j] = 0.f;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) split8(vr[s], vb[s][0], vb[s][1], vb[s][2]);
  }
  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  __syncthreads();  // Qb visible to the staging threads

  for (int c0 = 0; c0 < S; c0 += 64) {
    const int clen = min(64, S - c0);
    stamp();
    // ---- the chunk's staged registers -> Q (biased, * 1/8) / dO plane images, D, lse, keep words.
    // Nothing written here is read by the previous chunk's dQ phase: no barrier before it.
    {
      float v[8];
      const float* q = reinterpret_cast<const float*>(st.q);
      const float* o = reinterpret_cast<const float*>(st.o);
      const float* c = reinterpret_cast<const float*>(st.c);
      float dsum = 0.f;
      const float4 b0 = *reinterpret_cast<const float4*>(Qb + 8 * sc8), b1 = *reinterpret_cast<const float4*>(Qb + 8 * sc8 + 4);
      const float qb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] = (q[j] + qb[j]) * 0.125f;
        dsum = fmaf(o[j], c[j], dsum);
      }
      if (sr < clen) put_planes(Qimg, kPPlane, sr, sc8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = o[j];
      if (sr < clen) put_planes(Oimg, kPPlane, sr, sc8, v);
      dsum += __shfl_xor(dsum, 1, 64);
      dsum += __shfl_xor(dsum, 2, 64);
      dsum += __shfl_xor(dsum, 4, 64);
      if (sr < clen && sc8 == 0) Ds[sr] = dsum;
    }
    if (tid < clen) Ls[tid] = lse[(int64_t)bh * S + c0 + tid];
    if (p > 0.f && tid < 256) {
      const int q = tid & 63, kw = tid >> 6;
      if (q < clen && kw < nkw) Wd[kw * 64 + q] = dmask[((uint64_t)bh * S + c0 + q) * (uint64_t)nkw + kw];
    }
    __syncthreads();
    stamp();
    // the next chunk's loads fly under this chunk's MFMA phases
    if (c0 + 64 < S) {
      const float *qr, *orw, *cr;
      stage_ptrs(c0 + 64, qr, orw, cr);
      stage_load(st, qr, orw, cr, c0 + 64 + sr < S);
    }

    // ---- phase A: S, dP, P, dS, dV^T, dK^T for slice g (rows 32 g .. of the chunk's images)
    const bool has = c0 + 32 * g < S;
    if (has && kactive) {
      const int ln = opaque(lane), li = ln & 31, hf = ln >> 5, key = 32 * wg + li;
      const int qr = 32 * g;
      const int sw = pswz(li);  // = pswz(qr + li) = pswz(key): both rows share the chunk swizzle
      const char* qa = Qimg + (qr + li) * kPRow;
      const char* ka = Kimg + key * kPRow;
      f32x16 sc = {}, dp = {};
      // S then dP: 8 k-steps, each step's fragments read one step ahead of its MFMAs
      bfx8 fa[2][3], fk[2][3];
      auto frag_load = [&](int st, bfx8 (&a)[3], bfx8 (&k)[3]) {
        const int o = 16 * ((2 * (st & 3) + hf) ^ sw);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          a[pl] = *reinterpret_cast<const bfx8*>(qa + (st >> 2) * kPImg + pl * kPPlane + o);
          if (st < 4) k[pl] = *reinterpret_cast<const bfx8*>(ka + pl * kKPlane + o);
        }
      };
      __builtin_amdgcn_sched_barrier(0);
      frag_load(0, fa[0], fk[0]);
#pragma unroll
      for (int st = 0; st < 8; ++st) {
        if (st + 1 < 8) frag_load(st + 1, fa[(st + 1) & 1], fk[(st + 1) & 1]);
        if (st < 4)
          sc = mma6(fa[st & 1], fk[st & 1], sc);
        else
          dp = mma6(fa[st & 1], vb[st & 3], dp);
      }
      // pinned order: step st + 1's LDS reads issue before step st's six MFMAs
#define HS_RD(n) __builtin_amdgcn_sched_group_barrier(0x100, n, 0)
#define HS_MM() __builtin_amdgcn_sched_group_barrier(0x008, 6, 0)
      HS_RD(6); HS_RD(6); HS_MM(); HS_RD(6); HS_MM(); HS_RD(6); HS_MM(); HS_RD(3); HS_MM();
      HS_RD(3); HS_MM(); HS_RD(3); HS_MM(); HS_RD(3); HS_MM(); HS_MM();
#undef HS_RD
#undef HS_MM
      __builtin_amdgcn_sched_barrier(0);
      // P, dS (registers; split into planes), then dV^T / dK^T: 8 units (ks, product), each six
      // transposed-fragment reads + six MFMAs, reads pinned one unit ahead
      // P and dS of both k-steps (score registers 8 ks .. 8 ks + 7) split into planes; sc / dp die here
      bfx8 pb[2][3], sb[2][3];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float pd[8], ds[8];
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // runs of four consecutive queries: rows 8 (2 ks + i) + 4 hf + 0..3
          const int q0 = qr + 8 * (2 * ks + i) + 4 * hf;
          const float4 L4 = *reinterpret_cast<const float4*>(Ls + q0);
          const float4 D4 = *reinterpret_cast<const float4*>(Ds + q0);
          uint4 W4 = make_uint4(0u, 0u, 0u, 0u);
          if (p > 0.f) W4 = *reinterpret_cast<const uint4*>(Wd + wg * 64 + q0);
          const float Lv[4] = {L4.x, L4.y, L4.z, L4.w}, Dv[4] = {D4.x, D4.y, D4.z, D4.w};
          const uint32_t Wv[4] = {W4.x, W4.y, W4.z, W4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 8 * ks + 4 * i + e;
            const float pv = __expf(sc[r] + madd - Lv[e]);
            const float mk = p > 0.f ? (((Wv[e] >> li) & 1u) ? dscale : 0.f) : 1.f;
            pd[4 * i + e] = pv * mk;
            ds[4 * i + e] = pv * (dp[r] * mk - Dv[e]);
          }
        }
        split8(pd, pb[ks][0], pb[ks][1], pb[ks][2]);
        split8(ds, sb[ks][0], sb[ks][1], sb[ks][2]);
      }
      __builtin_amdgcn_sched_barrier(0);
      // dV^T / dK^T: 8 units (ks, product), each six transposed-fragment reads + six MFMAs, the
      // reads pinned one unit ahead
      bfx8 fu[2][3];
      const TrBase tb = tr_base(ln);
      auto unit_frag = [&](int u, bfx8 (&f)[3]) {  // u = 4 ks + {dO^T d 0-31, dO^T 32-63, Q^T 0-31, Q^T 32-63}
        const char* img = ((u & 2) ? Qimg : Oimg) + (qr + 16 * (u >> 2)) * kPRow;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) f[pl] = ptr_frag_b(img + pl * kPPlane, tb, u & 1);
      };
      unit_frag(0, fu[0]);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (u + 1 < 8) unit_frag(u + 1, fu[(u + 1) & 1]);
        const int ks = u >> 2;
        switch (u & 3) {
          case 0: dv0 = mma6(fu[u & 1], pb[ks], dv0); break;
          case 1: dv1 = mma6(fu[u & 1], pb[ks], dv1); break;
          case 2: dk0 = mma6(fu[u & 1], sb[ks], dk0); break;
          default: dk1 = mma6(fu[u & 1], sb[ks], dk1); break;
        }
      }
#define HS_RD() __builtin_amdgcn_sched_group_barrier(0x100, 6, 0)
#define HS_MM() __builtin_amdgcn_sched_group_barrier(0x008, 6, 0)
      HS_RD(); HS_RD(); HS_MM(); HS_RD(); HS_MM(); HS_RD(); HS_MM(); HS_RD(); HS_MM();
      HS_RD(); HS_MM(); HS_RD(); HS_MM(); HS_RD(); HS_MM(); HS_MM();
#undef HS_RD
#undef HS_MM
      __builtin_amdgcn_sched_barrier(0);
      // dS planes -> the [key][query] image: elements 0..3 of k-step ks are queries 16 ks + 4 hf + 0..3,
      // 4..7 are 16 ks + 8 + 4 hf + 0..3 (8-B runs of the image row `key`)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          const uint4 u = __builtin_bit_cast(uint4, sb[ks][pl]);
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int col = qr + 16 * ks + 8 * i + 4 * hf;
            *reinterpret_cast<uint2*>(Simg + pl * kKPlane + key * kPRow + 16 * ((col >> 3) ^ sw) + 2 * (col & 7)) =
                i == 0 ? make_uint2(u.x, u.y) : make_uint2(u.z, u.w);
          }
        }
    }
    __syncthreads();
    stamp();

    // ---- phase B: dQ of slice g = dS K (16 x 16 tiles: q halves x this wave's 16-wide d quarter)
    if (has) {
      const int ln = opaque(lane);
      f32x4 q0acc = {}, q1acc = {};
      // four 32-key k-steps (keys past S read as zero), each step's 18 transposed reads pinned
      // ahead of the previous step's 12 MFMAs
      bfx8 kf[2][3], a0[2][3], a1[2][3];
      auto qfrag = [&](int ks, bfx8 (&k)[3], bfx8 (&x0)[3], bfx8 (&x1)[3]) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          k[pl] = ptr16_frag(Kimg + pl * kKPlane, 16 * wg, 32 * ks, ln);
          x0[pl] = ptr16_frag(Simg + pl * kKPlane, 32 * g, 32 * ks, ln);
          x1[pl] = ptr16_frag(Simg + pl * kKPlane, 32 * g + 16, 32 * ks, ln);
        }
      };
      __builtin_amdgcn_sched_barrier(0);
      qfrag(0, kf[0], a0[0], a1[0]);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if (ks + 1 < 4) qfrag(ks + 1, kf[(ks + 1) & 1], a0[(ks + 1) & 1], a1[(ks + 1) & 1]);
        q0acc = mma16_6(a0[ks & 1], kf[ks & 1], q0acc);
        q1acc = mma16_6(a1[ks & 1], kf[ks & 1], q1acc);
      }
#define HS_RD() __builtin_amdgcn_sched_group_barrier(0x100, 18, 0)
#define HS_MM() __builtin_amdgcn_sched_group_barrier(0x008, 12, 0)
      HS_RD(); HS_RD(); HS_MM(); HS_RD(); HS_MM(); HS_RD(); HS_MM(); HS_MM();
#undef HS_RD
#undef HS_MM
      __builtin_amdgcn_sched_barrier(0);
      // C of a 16x16 tile: lane column = d, rows 4 (lane >> 4) + e = queries
      float* out = dqkv + ((int64_t)b * S + c0 + 32 * g + 4 * (ln >> 4)) * ld + h * kXD + 16 * wg + (ln & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        out[(int64_t)e * ld] = q0acc[e] * 0.125f;
        out[(int64_t)(16 + e) * ld] = q1acc[e] * 0.125f;
      }
    }
  }
  __syncthreads();  // every dQ phase is done with the images: reuse the LDS for the hand-off
  stamp();

  // ---- dK / dV: group 1 hands its partials to group 0 (fixed order), group 0 stores
  // the two groups swap halves: group 1 hands its dK partial to group 0, group 0 its dV partial to
  // group 1 ([register quad][lane] float4 images), each adds the other's half in the fixed order
  // (group 0 + group 1) and stores it
  float4* xk = reinterpret_cast<float4*>(smem) + (g * 4 + wg) * 8 * 64 + lane;  // written by group g
  if (kactive) {
    const f32x16& s0 = g ? dk0 : dv0;
    const f32x16& s1 = g ? dk1 : dv1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      xk[64 * r] = make_float4(s0[4 * r], s0[4 * r + 1], s0[4 * r + 2], s0[4 * r + 3]);
      xk[64 * (4 + r)] = make_float4(s1[4 * r], s1[4 * r + 1], s1[4 * r + 2], s1[4 * r + 3]);
    }
  }
  __syncthreads();
  if (!kactive) return;
  const float4* xo = reinterpret_cast<const float4*>(smem) + ((1 - g) * 4 + wg) * 8 * 64 + lane;  // the other group's
  f32x16& d0 = g ? dv0 : dk0;
  f32x16& d1 = g ? dv1 : dk1;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float4 u = xo[64 * r], v = xo[64 * (4 + r)];
    // group 0's partial first: d = g0 + g1 in both groups
    if (g == 0) {
      d0[4 * r] += u.x; d0[4 * r + 1] += u.y; d0[4 * r + 2] += u.z; d0[4 * r + 3] += u.w;
      d1[4 * r] += v.x; d1[4 * r + 1] += v.y; d1[4 * r + 2] += v.z; d1[4 * r + 3] += v.w;
    } else {
      d0[4 * r] = u.x + d0[4 * r]; d0[4 * r + 1] = u.y + d0[4 * r + 1];
      d0[4 * r + 2] = u.z + d0[4 * r + 2]; d0[4 * r + 3] = u.w + d0[4 * r + 3];
      d1[4 * r] = v.x + d1[4 * r]; d1[4 * r + 1] = v.y + d1[4 * r + 1];
      d1[4 * r + 2] = v.z + d1[4 * r + 2]; d1[4 * r + 3] = v.w + d1[4 * r + 3];
    }
  }
  const int li = lane & 31, hf = lane >> 5;
  float* out = dqkv + ((int64_t)b * S + 32 * wg + li) * ld + h * kXD + (g ? 2 * H : H);
  store_rows(out, d0, d1, hf, 1.f);
  stamp();
}

// ---------------------------------------------------------------------------
// Key-block backward in ONE 4-wave group ("c" kernel, HETSEQ_ATTN_BWD_X6=c): the key-block kernel's
// algorithm with 32-query chunks, so its LDS (97 KB: K image 48 KB, Q / dO images of 32 rows 24 KB, a
// 24 KB dS image that keeps keys 0-63 in columns 0-31 and keys 64-127 in columns 32-63 of a 64-row
// plane image) and its 4 x 256 VGPRs leave room on the CU for one GEMM block of the weight-gradient
// stream: the 8-wave kernel took whole CUs and lost in the step (profiles/r3_attention.md).
constexpr int kCPlane = 32 * kPRow;   // 4 KB: one plane of a 32-row image
constexpr int kCImg = 3 * kCPlane;    // 12 KB
constexpr int kCSmem = kKImg + 2 * kCImg + kPImg + 32 * 4 * 2 + 4 * 32 * 4 + kXD * 4;

__global__ void __launch_bounds__(256, 2)
    attn_bwd_x6c_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ mask,
                        const float* __restrict__ bqkv, const float* __restrict__ ctx,
                        const float* __restrict__ dctx, const float* __restrict__ lse, float* __restrict__ dqkv, int S,
                        int NH, float p, const uint32_t* __restrict__ dmask) {
  __shared__ __attribute__((aligned(16))) char smem[kCSmem];
  auto stamp = [] {};
  char* const Kimg = smem;                     // [key][d] planes, 128 rows
  char* const Qimg = Kimg + kKImg;             // [query of the chunk][d], 32 rows (plane stride kCPlane)
  char* const Oimg = Qimg + kCImg;             // dO rows, same layout
  char* const Simg = Oimg + kCImg;             // dS planes: row key & 63, columns 32 (key >> 6) + query
  float* const Ls = reinterpret_cast<float*>(Simg + kPImg);
  float* const Ds = Ls + 32;
  uint32_t* const Wd = reinterpret_cast<uint32_t*>(Ds + 32);  // [key word][query]
  const int H = NH * kXD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = 0, wg = w;
  const int nkw = S >> 5;  // 32-key words of a keep-mask row
  const bool kactive = 32 * wg < S;
  const float* rows = qkv + (int64_t)b * S * ld;
  const float dscale = drop_scale16(drop_thr16(p));
  // staging unit of this thread: chunk row sr, d = 8 sc8 .. 8 sc8 + 7
  const int sr = tid >> 3, sc8 = tid & 7;
  float* const Qb = reinterpret_cast<float*>(Wd + 4 * 32);  // the head's Q bias (64 floats)
  if (tid < kXD) Qb[tid] = bqkv ? bqkv[h * kXD + tid] : 0.f;
  auto stage_ptrs = [&](int c0, const float*& qr, const float*& orw, const float*& cr) {
    const int64_t tok = (int64_t)b * S + c0 + sr;
    qr = qkv + tok * ld + h * kXD + 8 * sc8;
    orw = dctx + tok * H + h * kXD + 8 * sc8;
    cr = ctx + tok * H + h * kXD + 8 * sc8;
  };

  // ---- prologue: chunk 0's Q / dO / O loads in flight with the K image and the lane's V row
  StageRegs st;
  {
    const float *qr, *orw, *cr;
    stage_ptrs(0, qr, orw, cr);
    stage_load(st, qr, orw, cr, sr < S);
  }
  {  // K image (biased): rows sr + 32 i (256 threads, 32 staging rows)
    const float* bk = bofs(bqkv, H + h * kXD + 8 * sc8);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = sr + 32 * i;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // rows past S: zero (phase B sums all 128 keys)
      if (r < S) ld8(rows + (int64_t)r * ld + H + h * kXD + 8 * sc8, bk, 1.f, v);
      put_planes(Kimg, kKPlane, r, sc8, v);
    }
    if (32 * wg >= S && lane < 32) {  // keys past S: their dS entries stay zero
      const int key = 32 * wg + lane, row = key & 63, h2 = key >> 6;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<uint4*>(Simg + pl * kPPlane + row * kPRow + 16 * ((4 * h2 + j) ^ pswz(row))) =
              make_uint4(0, 0, 0, 0);
    }
  }
  bfx8 vb[4][3];
  float madd = 0.f;
  {
    const int li = lane & 31, hf = lane >> 5, key = 32 * wg + li;
    float vr[4][8];
    if (kactive) {
      row_frags(rows + (int64_t)key * ld + 2 * H + h * kXD, bofs(bqkv, 2 * H + h * kXD), hf, vr);
      madd = (1.f - (float)mask[(int64_t)b * S + key]) * -10000.f;
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) vr[s][j] = 0.f;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) split8(vr[s], vb[s][0], vb[s][1], vb[s][2]);
  }
  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  __syncthreads();  // Qb visible to the staging threads

  for (int c0 = 0; c0 < S; c0 += 32) {
    const int clen = min(32, S - c0);
    stamp();
    // ---- the chunk's staged registers -> Q (biased, * 1/8) / dO plane images, D, lse, keep words.
    // Nothing written here is read by the previous chunk's dQ phase: no barrier before it.
    {
      float v[8];
      const float* q = reinterpret_cast<const float*>(st.q);
      const float* o = reinterpret_cast<const float*>(st.o);
      const float* c = reinterpret_cast<const float*>(st.c);
      float dsum = 0.f;
      const float4 b0 = *reinterpret_cast<const float4*>(Qb + 8 * sc8), b1 = *reinterpret_cast<const float4*>(Qb + 8 * sc8 + 4);
      const float qb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] = (q[j] + qb[j]) * 0.125f;
        dsum = fmaf(o[j], c[j], dsum);
      }
      if (sr < clen) put_planes(Qimg, kCPlane, sr, sc8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = o[j];
      if (sr < clen) put_planes(Oimg, kCPlane, sr, sc8, v);
      dsum += __shfl_xor(dsum, 1, 64);
      dsum += __shfl_xor(dsum, 2, 64);
      dsum += __shfl_xor(dsum, 4, 64);
      if (sr < clen && sc8 == 0) Ds[sr] = dsum;
    }
    if (tid < clen) Ls[tid] = lse[(int64_t)bh * S + c0 + tid];
    if (p > 0.f && tid < 128) {
      const int q = tid & 31, kw = tid >> 5;
      if (q < clen && kw < nkw) Wd[kw * 32 + q] = dmask[((uint64_t)bh * S + c0 + q) * (uint64_t)nkw + kw];
    }
    __syncthreads();
    stamp();
    // the next chunk's loads fly under this chunk's MFMA phases
    if (c0 + 32 < S) {
      const float *qr, *orw, *cr;
      stage_ptrs(c0 + 32, qr, orw, cr);
      stage_load(st, qr, orw, cr, c0 + 32 + sr < S);
    }

    // ---- phase A: S, dP, P, dS, dV^T, dK^T for slice g (rows 32 g .. of the chunk's images)
    const bool has = c0 + 32 * g < S;
    if (has && kactive) {
      const int ln = opaque(lane), li = ln & 31, hf = ln >> 5, key = 32 * wg + li;
      const int qr = 32 * g;
      const int sw = pswz(li);  // = pswz(qr + li) = pswz(key): both rows share the chunk swizzle
      const char* qa = Qimg + (qr + li) * kPRow;
      const char* ka = Kimg + key * kPRow;
      f32x16 sc = {}, dp = {};
      // S then dP: 8 k-steps, each step's fragments read one step ahead of its MFMAs
      bfx8 fa[2][3], fk[2][3];
      auto frag_load = [&](int st, bfx8 (&a)[3], bfx8 (&k)[3]) {
        const int o = 16 * ((2 * (st & 3) + hf) ^ sw);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          a[pl] = *reinterpret_cast<const bfx8*>(qa + (st >> 2) * kCImg + pl * kCPlane + o);
          if (st < 4) k[pl] = *reinterpret_cast<const bfx8*>(ka + pl * kKPlane + o);
        }
      };
      __builtin_amdgcn_sched_barrier(0);
      frag_load(0, fa[0], fk[0]);
#pragma unroll
      for (int st = 0; st < 8; ++st) {
        if (st + 1 < 8) frag_load(st + 1, fa[(st + 1) & 1], fk[(st + 1) & 1]);
        if (st < 4)
          sc = mma6(fa[st & 1], fk[st & 1], sc);
        else
          dp = mma6(fa[st & 1], vb[st & 3], dp);
      }
      // pinned order: step st + 1's LDS reads issue before step st's six MFMAs
#define HS_RD(n) __builtin_amdgcn_sched_group_barrier(0x100, n, 0)
#define HS_MM() __builtin_amdgcn_sched_group_barrier(0x008, 6, 0)
      HS_RD(6); HS_RD(6); HS_MM(); HS_RD(6); HS_MM(); HS_RD(6); HS_MM(); HS_RD(3); HS_MM();
      HS_RD(3); HS_MM(); HS_RD(3); HS_MM(); HS_RD(3); HS_MM(); HS_MM();
#undef HS_RD
#undef HS_MM
      __builtin_amdgcn_sched_barrier(0);
      // P, dS (registers; split into planes), then dV^T / dK^T: 8 units (ks, product), each six
      // transposed-fragment reads + six MFMAs, reads pinned one unit ahead
      // P and dS of both k-steps (score registers 8 ks .. 8 ks + 7) split into planes; sc / dp die here
      bfx8 pb[2][3], sb[2][3];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float pd[8], ds[8];
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // runs of four consecutive queries: rows 8 (2 ks + i) + 4 hf + 0..3
          const int q0 = qr + 8 * (2 * ks + i) + 4 * hf;
          const float4 L4 = *reinterpret_cast<const float4*>(Ls + q0);
          const float4 D4 = *reinterpret_cast<const float4*>(Ds + q0);
          uint4 W4 = make_uint4(0u, 0u, 0u, 0u);
          if (p > 0.f) W4 = *reinterpret_cast<const uint4*>(Wd + wg * 32 + q0);
          const float Lv[4] = {L4.x, L4.y, L4.z, L4.w}, Dv[4] = {D4.x, D4.y, D4.z, D4.w};
          const uint32_t Wv[4] = {W4.x, W4.y, W4.z, W4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 8 * ks + 4 * i + e;
            const float pv = __expf(sc[r] + madd - Lv[e]);
            const float mk = p > 0.f ? (((Wv[e] >> li) & 1u) ? dscale : 0.f) : 1.f;
            pd[4 * i + e] = pv * mk;
            ds[4 * i + e] = pv * (dp[r] * mk - Dv[e]);
          }
        }
        split8(pd, pb[ks][0], pb[ks][1], pb[ks][2]);
        split8(ds, sb[ks][0], sb[ks][1], sb[ks][2]);
      }
      __builtin_amdgcn_sched_barrier(0);
      // dV^T / dK^T: 8 units (ks, product), each six transposed-fragment reads + six MFMAs, the
      // reads pinned one unit ahead
      bfx8 fu[2][3];
      const TrBase tb = tr_base(ln);
      auto unit_frag = [&](int u, bfx8 (&f)[3]) {  // u = 4 ks + {dO^T d 0-31, dO^T 32-63, Q^T 0-31, Q^T 32-63}
        const char* img = ((u & 2) ? Qimg : Oimg) + (qr + 16 * (u >> 2)) * kPRow;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) f[pl] = ptr_frag_b(img + pl * kCPlane, tb, u & 1);
      };
      unit_frag(0, fu[0]);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (u + 1 < 8) unit_frag(u + 1, fu[(u + 1) & 1]);
        const int ks = u >> 2;
        switch (u & 3) {
          case 0: dv0 = mma6(fu[u & 1], pb[ks], dv0); break;
          case 1: dv1 = mma6(fu[u & 1], pb[ks], dv1); break;
          case 2: dk0 = mma6(fu[u & 1], sb[ks], dk0); break;
          default: dk1 = mma6(fu[u & 1], sb[ks], dk1); break;
        }
      }
#define HS_RD() __builtin_amdgcn_sched_group_barrier(0x100, 6, 0)
#define HS_MM() __builtin_amdgcn_sched_group_barrier(0x008, 6, 0)
      HS_RD(); HS_RD(); HS_MM(); HS_RD(); HS_MM(); HS_RD(); HS_MM(); HS_RD(); HS_MM();
      HS_RD(); HS_MM(); HS_RD(); HS_MM(); HS_RD(); HS_MM(); HS_MM();
#undef HS_RD
#undef HS_MM
      __builtin_amdgcn_sched_barrier(0);
      // dS planes -> the [key][query] image: elements 0..3 of k-step ks are queries 16 ks + 4 hf + 0..3,
      // 4..7 are 16 ks + 8 + 4 hf + 0..3 (8-B runs of the image row `key`)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          const uint4 u = __builtin_bit_cast(uint4, sb[ks][pl]);
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int col = 32 * (key >> 6) + 16 * ks + 8 * i + 4 * hf;  // row key & 63: its swizzle is sw
            *reinterpret_cast<uint2*>(Simg + pl * kPPlane + (key & 63) * kPRow + 16 * ((col >> 3) ^ sw) +
                                      2 * (col & 7)) = i == 0 ? make_uint2(u.x, u.y) : make_uint2(u.z, u.w);
          }
        }
    }
    __syncthreads();
    stamp();

    // ---- phase B: dQ of slice g = dS K (16 x 16 tiles: q halves x this wave's 16-wide d quarter)
    if (has) {
      const int ln = opaque(lane);
      f32x4 q0acc = {}, q1acc = {};
      // four 32-key k-steps (keys past S read as zero), each step's 18 transposed reads pinned
      // ahead of the previous step's 12 MFMAs
      bfx8 kf[2][3], a0[2][3], a1[2][3];
      auto qfrag = [&](int ks, bfx8 (&k)[3], bfx8 (&x0)[3], bfx8 (&x1)[3]) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          k[pl] = ptr16_frag(Kimg + pl * kKPlane, 16 * wg, 32 * ks, ln);
          x0[pl] = ptr16_frag(Simg + pl * kPPlane, 32 * (ks >> 1), 32 * (ks & 1), ln);
          x1[pl] = ptr16_frag(Simg + pl * kPPlane, 32 * (ks >> 1) + 16, 32 * (ks & 1), ln);
        }
      };
      __builtin_amdgcn_sched_barrier(0);
      qfrag(0, kf[0], a0[0], a1[0]);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if (ks + 1 < 4) qfrag(ks + 1, kf[(ks + 1) & 1], a0[(ks + 1) & 1], a1[(ks + 1) & 1]);
        q0acc = mma16_6(a0[ks & 1], kf[ks & 1], q0acc);
        q1acc = mma16_6(a1[ks & 1], kf[ks & 1], q1acc);
      }
#define HS_RD() __builtin_amdgcn_sched_group_barrier(0x100, 18, 0)
#define HS_MM() __builtin_amdgcn_sched_group_barrier(0x008, 12, 0)
      HS_RD(); HS_RD(); HS_MM(); HS_RD(); HS_MM(); HS_RD(); HS_MM(); HS_MM();
#undef HS_RD
#undef HS_MM
      __builtin_amdgcn_sched_barrier(0);
      // C of a 16x16 tile: lane column = d, rows 4 (lane >> 4) + e = queries
      float* out = dqkv + ((int64_t)b * S + c0 + 32 * g + 4 * (ln >> 4)) * ld + h * kXD + 16 * wg + (ln & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        out[(int64_t)e * ld] = q0acc[e] * 0.125f;
        out[(int64_t)(16 + e) * ld] = q1acc[e] * 0.125f;
      }
    }
  }
  // ---- dK / dV: every wave holds its keys' whole sums (one group): store them
  if (!kactive) return;
  const int li = lane & 31, hf = lane >> 5;
  float* out = dqkv + ((int64_t)b * S + 32 * wg + li) * ld + h * kXD;
  store_rows(out + H, dk0, dk1, hf, 1.f);
  store_rows(out + 2 * H, dv0, dv1, hf, 1.f);
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

// fp32 backward kernel family: HETSEQ_ATTN_BWD_X6=p (the plane-image dQ / dKV pair; default), k (key-block
// kernel for S <= 128, the pair above that) or g (fused S <= 128 / gather dQ / dKV pair).  The key-block
// kernel is 0.8x the pair's time alone on the chip but takes whole CUs (145 KB LDS, 512 VGPRs a block):
// beside the weight-gradient side stream the BERT-base step measured 15.65 ms with it vs 15.34 with the
// pair (bench.py --ab, profiles/r3_attention.md).
static int g_bwd_planes_env = [] {
  const char* e = std::getenv("HETSEQ_ATTN_BWD_X6");
  return e && e[0] == 'g' ? 0 : (e && e[0] == 'k' ? 2 : (e && e[0] == 'c' ? 4 : 1));
}();
static int g_bwd_planes = g_bwd_planes_env;
// dispatch order of the merged backward's roles: dK / dV blocks first (default) or dQ first
// (HETSEQ_ATTN_BWD_DKV_FIRST=0)
static const int g_bwd_dkv_first = [] {
  const char* e = std::getenv("HETSEQ_ATTN_BWD_DKV_FIRST");
  return e && e[0] == '0' ? 0 : 1;
}();
// fp32 forward: plane-image kernel (default) or the first x6 forward (HETSEQ_ATTN_FWD_X6=old)
static int g_fwd_planes = [] {
  const char* e = std::getenv("HETSEQ_ATTN_FWD_X6");
  return e && e[0] == 'o' ? 0 : 1;
}();
void set_attn_fwd_x6_planes(int on) { g_fwd_planes = on; }
// the plane pair computes D itself at S <= 128 (HETSEQ_ATTN_BWD_DSUM=1: the separate attn_bwd_dsum pass)
static int g_bwd_fused_d = [] {
  const char* e = std::getenv("HETSEQ_ATTN_BWD_DSUM");
  return e && e[0] == '1' ? 0 : 1;
}();
void set_attn_bwd_fused_d(int on) { g_bwd_fused_d = on; }
// diagnostic: per-block shader-clock stamps of the key-block backward (16 per block; nullptr = off)
static uint64_t* g_attn_tbuf = nullptr;
void set_attn_timing(uint64_t* buf) { g_attn_tbuf = buf; }
void set_attn_bwd_x6_planes(int on) { g_bwd_planes = on < 0 ? g_bwd_planes_env : on; }

// fused S <= 128 (grid B*NH x 512) or the dQ / dKV pair (grid (S/128, B*NH) x 256 each)
int launch_attn_bwd_x6(const float* qkv, const int64_t* mask, const float* bqkv, const float* ctx, const float* dctx,
                       const float* lse, float* Dbuf, float* dqkv, const uint32_t* dmask, int B, int S, int NH,
                       int D, float p, bool fused, hipStream_t st) {
  if (D != kXD || S % 32 != 0 || S <= 0 || (p > 0.f && dmask == nullptr)) return -1;
  if (g_bwd_planes == 4 && S <= kKRows) {  // one-group key-block kernel: one 4-wave block per (batch, head)
    hipLaunchKernelGGL(attn_bwd_x6c_kernel, dim3(B * NH), dim3(256), 0, st, qkv, mask, bqkv, ctx, dctx, lse, dqkv, S,
                       NH, p, dmask);
    return 0;
  }
  if (g_bwd_planes == 2 && S <= kKRows) {  // key-block kernel: one block per (batch, head)
    hipLaunchKernelGGL(attn_bwd_x6k_kernel, dim3(B * NH), dim3(512), 0, st, qkv, mask, bqkv, ctx, dctx, lse, dqkv, S,
                       NH, p, dmask, g_attn_tbuf);
    return 0;
  }
  if (g_bwd_planes) {  // plane-image kernels: D (in the roles for S <= 128), both roles in one launch
    const bool fused_d = g_bwd_fused_d && S <= 128;
    if (!fused_d) {
      const int64_t units = (int64_t)B * S * NH;
      hipLaunchKernelGGL(attn_bwd_dsum_kernel, dim3((unsigned)((units + 15) / 16)), dim3(256), 0, st, ctx, dctx, Dbuf,
                         B, S, NH);
    }
    dim3 grid(B * NH, 2 * ((S + 127) / 128));
    hipLaunchKernelGGL(attn_bwd_x6p_kernel, grid, dim3(256), 0, st, qkv, mask, bqkv, dctx, lse, Dbuf, dqkv, S, NH, p,
                       dmask, g_bwd_dkv_first, fused_d ? ctx : nullptr);
    return 0;
  }
  if (fused && S <= 128) {
    hipLaunchKernelGGL(attn_bwd_fused_x6_kernel, dim3(B * NH), dim3(512), 0, st, qkv, mask, bqkv, ctx, dctx, lse, dqkv,
                       S, NH, p, dmask);
    return 0;
  }
  dim3 grid(B * NH, (S + 127) / 128);  // head-major: a head's blocks share one XCD's L2
  hipLaunchKernelGGL(attn_bwd_dq_x6_kernel, grid, dim3(256), 0, st, qkv, mask, bqkv, ctx, dctx, lse, Dbuf, dqkv, S, NH,
                     p, dmask);
  hipLaunchKernelGGL(attn_bwd_dkv_x6_kernel, grid, dim3(256), 0, st, qkv, mask, bqkv, dctx, lse, Dbuf, dqkv, S, NH, p,
                     dmask);
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
  if (g_fwd_planes)
    hipLaunchKernelGGL(attn_fwd_x6p_kernel, grid, dim3(256), 0, st, qkv, mask, bqkv, ctx, lse, dmask, S, NH, p, seed,
                       off, g_seed_dev, bh0);
  else
    hipLaunchKernelGGL(attn_fwd_x6_kernel, grid, dim3(256), 0, st, qkv, mask, bqkv, ctx, lse, dmask, S, NH, p, seed,
                       off, g_seed_dev, bh0);
  return 0;
}
