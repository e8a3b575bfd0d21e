// fp32 attention as THREE split-fp16 products per fp32 product ("h3"; default fp32 attention engine).
//
// Same contract as the exact-fp32 kernels (attention.hip; reference bert_modeling.py:351-377), on the
// plane-image algorithm of the round-3 split-bf16 kernels (retired in round 6): Q/K/V read from the fused QKV projection
// output [B*S, 3H] with the projection bias folded into the loads, additive -10000 mask, Philox
// dropout with the 1-bit keep mask (identical bit stream and word layout), flash forward with the
// per-row log-sum-exp, and a backward of two roles in one launch (dK / dV blocks with the key on the
// lane, dQ blocks with the query on the lane).
//
// Products: the GEMM engine's h3 scheme (gemm.hip split4h): an operand scaled by a power of two s is
// split into fp16 hi + lo (22 significant bits) and a*b is accumulated from hi*hi + hi*lo + lo*hi on
// v_mfma_f32_32x32x16_f16 -- 3 MFMAs per product instead of a six-term bf16 split's 6, and 2 LDS planes per
// image instead of 3 (16 KB per 64-row chunk).  The scales are chosen IN the kernel, uniform along
// every product's contraction dimension, so no producer has to supply a |max|:
//   * the lane's own Q / K / V / dO row (contraction over d): its row |max| (the two lanes holding
//     one row agree through one shuffle);
//   * a staged 64-row chunk image (read by rows for d-contractions and transposed for the
//     contractions over rows): the chunk's |max| (one LDS exchange per chunk, under the barrier the
//     staging needs anyway); an accumulator that spans chunks is brought to the new chunk's scale by
//     an exact power-of-two multiply when the exponent changes;
//   * P (<= the dropout scale): a fixed scale;
//   * dS (magnitude known only once computed): a running per-lane exponent -- the accumulator is
//     rescaled (exactly) when a tile's |max| needs a smaller scale.
// Every scale maps the operand's largest |x| into [2^14, 2^15), so elements down to 2^-18 of it keep
// all 22 bits; the exact unscale multiplies the fp32 accumulator.  Error against fp64: within the
// exact-fp32 kernels' (tests/test_kernels_gpu.py::test_attention_h3_matches_fp64).
#include <cfloat>
#include <cstdlib>

#include "common.h"
#include "h3p.h"

namespace hs {

int launch_attn_bwd_dsum(const float* ctx, const float* dctx, float* Dout, int B, int S, int NH, hipStream_t st);

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 hx8 __attribute__((ext_vector_type(8)));
typedef _Float16 hx2 __attribute__((ext_vector_type(2)));
typedef float fx2 __attribute__((ext_vector_type(2)));
typedef short ps4 __attribute__((ext_vector_type(4)));
typedef short ps8 __attribute__((ext_vector_type(8)));

constexpr int kHD = 64;             // head dim
constexpr int kRowB = 128;          // bytes per image row (64 fp16)
constexpr int kPl = 64 * kRowB;     // one plane of a 64-row chunk: 8 KB
constexpr int kIm = 2 * kPl;        // hi + lo: 16 KB
constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;

HS_DEVICE f32x16 mma(hx8 a, hx8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0); }

// acc += a * b over the three split terms, smallest first (a, b: planes hi / lo)
HS_DEVICE f32x16 mma3(const hx8 (&a)[2], const hx8 (&b)[2], f32x16 acc) {
  acc = mma(a[1], b[0], acc);
  acc = mma(a[0], b[1], acc);
  return mma(a[0], b[0], acc);
}

// score register r of lane half hf -> row of the 32 x 32 tile
HS_DEVICE int xrow(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }

// power-of-two exponent for an operand whose |max| is m: s = 2^e puts m in [2^14, 2^15); zero / inf / NaN:
// unscaled (inf and NaN propagate through the split)
HS_DEVICE int h16e(float m) {
  if (!(m > 0.f) || !(m <= FLT_MAX)) return 0;
  return min(126, max(-126, 14 - ilogbf(m)));
}

// 8 fp32 * s (exact) -> fp16 hi / lo (round-to-nearest-even each; hi + lo = s*x to 2^-22)
HS_DEVICE void split8h(const float (&v)[8], float s, hx8& hi, hx8& lo) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const fx2 x = {v[2 * i] * s, v[2 * i + 1] * s};
    const hx2 h = __builtin_convertvector(x, hx2);
    const hx2 l = __builtin_convertvector(x - __builtin_convertvector(h, fx2), hx2);
    hi[2 * i] = h[0];
    hi[2 * i + 1] = h[1];
    lo[2 * i] = l[0];
    lo[2 * i + 1] = l[1];
  }
}

HS_DEVICE float amax8(const float (&v)[8], float m) {
#pragma unroll
  for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
  return m;
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

// Plane images of 64-row chunks: [row][64 d] fp16, 128-B rows, the 16-B chunk swizzle pswz (conflict-free
// b128 row reads and ds_read_b64_tr_b16 transposed reads; found by exhaustive search).
HS_DEVICE int pswz(int r) { return ((r >> 2) & 1) | (((r >> 3) & 1) << 1) | (((r >> 1) & 1) << 2); }

// 8 fp32 * s -> hi / lo planes at 16-B chunk c of row `row`
HS_DEVICE void put2(char* img, int row, int c, const float (&v)[8], float s) {
  hx8 hi, lo;
  split8h(v, s, hi, lo);
  const int off = row * kRowB + 16 * (c ^ pswz(row));
  *reinterpret_cast<hx8*>(img + off) = hi;
  *reinterpret_cast<hx8*>(img + kPl + off) = lo;
}

// row fragment of plane pl: row `row`, 16-B chunk c (= 2 k-step + lane half)
HS_DEVICE hx8 prow(const char* img, int pl, int row, int c) {
  return *reinterpret_cast<const hx8*>(img + pl * kPl + row * kRowB + 16 * (c ^ pswz(row)));
}

// Transposed fragments (rows = d, k = image rows in the score-register order) by two
// ds_read_b64_tr_b16; lane byte offsets per (d half, read) relative to a 16-row-aligned row q0
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
      t.o[dh][jj] = row * kRowB + 16 * ((col >> 3) ^ pswz(row)) + 2 * (col & 7);
    }
  return t;
}
// plb = plane base + q0 rows (q0 a multiple of 16: the swizzle depends on row bits 1..3 only)
HS_DEVICE hx8 ptr(const char* plb, const TrBase& t, int dh) {
  ps4 v[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj)
    v[jj] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) ps4*)(plb + t.o[dh][jj]));
  const ps8 u = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
  return __builtin_bit_cast(hx8, u);
}
HS_DEVICE void ptr2(const char* img, int q0, const TrBase& t, int dh, hx8 (&f)[2]) {
  f[0] = ptr(img + q0 * kRowB, t, dh);
  f[1] = ptr(img + kPl + q0 * kRowB, t, dh);
}

// 16 accumulator registers of two 32x32 C tiles (rows d, lane column) -> 64 fp32 of a token row; the
// |max| of the written values folds into cm (the h3 GEMMs' operand scale, written by the producer)
HS_DEVICE void store_rows(float* out, const f32x16& c0, const f32x16& c1, int hf, float scale, uint32_t& cm) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * hf;
    const float4 a = make_float4(c0[4 * g] * scale, c0[4 * g + 1] * scale, c0[4 * g + 2] * scale, c0[4 * g + 3] * scale);
    const float4 b = make_float4(c1[4 * g] * scale, c1[4 * g + 1] * scale, c1[4 * g + 2] * scale, c1[4 * g + 3] * scale);
    cm = amax_bits(amax_bits(amax_bits(amax_bits(cm, a.x), a.y), a.z), a.w);
    cm = amax_bits(amax_bits(amax_bits(amax_bits(cm, b.x), b.y), b.z), b.w);
    *reinterpret_cast<float4*>(out + d) = a;
    *reinterpret_cast<float4*>(out + 32 + d) = b;
  }
}

// Output also as h3p operand planes (h3p.h) of the next GEMM: `pl` plane 0 (plane 1 at + ps), `ex` the
// exponents; null pl = off.  A wave's 32 x 64 output tile is two exponent blocks.
struct AttnPl {
  uint16_t* pl;
  int64_t ps;
  int8_t* ex;
};

// the wave's tile (rows: the lanes, 32-aligned; columns 0-31 in c0, 32-63 in c1, * scale) into the
// blocked planes (h3p.h; row stride ld) at the lane's row `row`, the tile's first column col0 (a multiple
// of 32), and its two exponents at ex
HS_DEVICE void store_rows_h3p(const AttnPl& po, int64_t row, int64_t col0, int64_t ld, int8_t* ex, const f32x16& c0,
                              const f32x16& c1, int hf, float scale) {
  uint32_t m0 = 0u, m1 = 0u;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    m0 = amax_bits(m0, c0[r] * scale);
    m1 = amax_bits(m1, c1[r] * scale);
  }
  const int e0 = h3p_exp_bits(wave_umax(m0)), e1 = h3p_exp_bits(wave_umax(m1));
  const float s0 = h3p_scale(e0), s1 = h3p_scale(e1);
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d = 8 * g + 4 * hf;
    const float a[4] = {c0[4 * g] * scale, c0[4 * g + 1] * scale, c0[4 * g + 2] * scale, c0[4 * g + 3] * scale};
    const float b[4] = {c1[4 * g] * scale, c1[4 * g + 1] * scale, c1[4 * g + 2] * scale, c1[4 * g + 3] * scale};
    h3p_store4(po.pl, po.ps, h3p_index(row, col0 + d, ld, 1), a, s0);
    h3p_store4(po.pl, po.ps, h3p_index(row, col0 + 32 + d, ld, 1), b, s1);
  }
  if ((threadIdx.x & 63) == 0) {
    ex[0] = static_cast<int8_t>(e0);
    ex[1] = static_cast<int8_t>(e1);
  }
}

// The lane's row (dims 16 s + 8 hf + j, (x + bias) * scale) split with the row's exponent (both lane
// halves of the row agree); returns the exponent
HS_DEVICE int lane_row(const float* row, const float* bias, float scale, bool ok, int hf, hx8 (&f)[4][2]) {
  float v[4][8];
  float m = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (ok) {
      ld8(row + 16 * s + 8 * hf, bias ? bias + 16 * s + 8 * hf : nullptr, scale, v[s]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[s][j] = 0.f;
    }
    m = amax8(v[s], m);
  }
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  const int e = h16e(m);
  const float sc = ldexpf(1.f, e);
#pragma unroll
  for (int s = 0; s < 4; ++s) split8h(v[s], sc, f[s][0], f[s][1]);
  return e;
}

// Chunk staging: thread unit u = tid + 256 i (i = 0, 1) is row u >> 3, d = 8 (u & 7) .. + 7 of a
// 64-row chunk; two operands per chunk.
struct Chunk {
  float v[2][2][8];  // [operand][unit][8 d]
};

HS_DEVICE void chunk_load(Chunk& c, const float* base0, const float* base1, int64_t ld0, int64_t ld1, int r0, int n,
                          const float* bias0, const float* bias1, float scale0) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int u = threadIdx.x + 256 * i, r = u >> 3, c8 = 8 * (u & 7);
    if (r < n) {
      ld8(base0 + (int64_t)(r0 + r) * ld0 + c8, bias0 ? bias0 + c8 : nullptr, scale0, c.v[0][i]);
      ld8(base1 + (int64_t)(r0 + r) * ld1 + c8, bias1 ? bias1 + c8 : nullptr, 1.f, c.v[1][i]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) c.v[0][i][j] = c.v[1][i][j] = 0.f;
    }
  }
}

// the chunk's two |max| values into red[w][0..1] (wave maxima; read back after the next barrier)
HS_DEVICE void chunk_max(const Chunk& c, float* red) {
  float m0 = 0.f, m1 = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    m0 = amax8(c.v[0][i], m0);
    m1 = amax8(c.v[1][i], m1);
  }
  m0 = wave_max(m0);
  m1 = wave_max(m1);
  if ((threadIdx.x & 63) == 0) {
    red[2 * (threadIdx.x >> 6)] = m0;
    red[2 * (threadIdx.x >> 6) + 1] = m1;
  }
}

HS_DEVICE int red_exp(const float* red, int k) {
  return h16e(fmaxf(fmaxf(red[k], red[2 + k]), fmaxf(red[4 + k], red[6 + k])));
}

HS_DEVICE void chunk_put(const Chunk& c, char* img0, char* img1, int n, int e0, int e1) {
  const float s0 = ldexpf(1.f, e0), s1 = ldexpf(1.f, e1);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int u = threadIdx.x + 256 * i, r = u >> 3, c8 = u & 7;
    if (r < n) {
      put2(img0, r, c8, c.v[0][i], s0);
      put2(img1, r, c8, c.v[1][i], s1);
    }
  }
}

// fixed exponent of P (<= the dropout scale): its largest value below 2^14
HS_DEVICE int p_exp(float pmax) { return 13 - (pmax >= 2.f ? ilogbf(pmax) : 0); }

// running per-lane exponent of dS: a tile whose |max| needs a smaller scale rescales the accumulators
// of the lane's column (both lane halves agree) exactly; returns the scale for this tile
HS_DEVICE float ds_scale(const float (&ds)[2][8], int& es, f32x16& a0, f32x16& a1) {
  float m = 0.f;
#pragma unroll
  for (int k = 0; k < 2; ++k) m = amax8(ds[k], m);
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  const int et = (m > 0.f && m <= FLT_MAX) ? h16e(m) : es;
  const int en = min(es, et);
  if (__ballot(en != es)) {
    const float f = ldexpf(1.f, en - es);
    a0 *= f;
    a1 *= f;
    es = en;
  }
  return ldexpf(1.f, es);
}

// ---------------------------------------------------------------------------------------------------
// dK / dV for 32 keys per wave (lane = key) over 64-query chunks of Q (biased, * 1/8) and dO.
constexpr int kBwdLds = 2 * kIm + 64 * 4 * 2 + 64 * 4 * 4 + 2 * 8 * 4;

template <bool DS>
HS_DEVICE void dkv_body(char* __restrict__ smem, int bx, int bh, const float* __restrict__ qkv,
                        const int64_t* __restrict__ mask, const float* __restrict__ bqkv,
                        const float* __restrict__ dctx, const float* __restrict__ lse, const float* __restrict__ Dd,
                        float* __restrict__ dqkv, int S, int NH, float p, const uint32_t* __restrict__ dmask,
                        const float* __restrict__ ctx, float* __restrict__ amax, AttnPl po,
                        float* __restrict__ dsw) {
  char* const Qp = smem;
  char* const Op = smem + kIm;
  float* const Ls = reinterpret_cast<float*>(smem + 2 * kIm);
  float* const Ds = Ls + 64;
  uint32_t(*const Wd)[4] = reinterpret_cast<uint32_t(*)[4]>(Ds + 64);
  float* const red = reinterpret_cast<float*>(Wd + 64);  // [parity][wave][operand]
  const int H = NH * kHD;
  const int64_t ld = 3 * (int64_t)H;
  const int b = bh / NH, h = bh % NH;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5, li = lane & 31;
  const int k0 = bx * 128 + w * 32;
  const bool active = k0 < S;
  const int key = k0 + li;
  const float* rows = qkv + (int64_t)b * S * ld;
  const float* drows = dctx + (int64_t)b * S * H;
  const float* crows = ctx ? ctx + (int64_t)b * S * H : nullptr;
  const float dscale = drop_scale16(drop_thr16(p));
  const int ep = p_exp(p > 0.f ? dscale : 1.f);
  const float sp = ldexpf(1.f, ep);

  hx8 kb[4][2], vb[4][2];
  const int ek = lane_row(rows + (int64_t)key * ld + H + h * kHD, bofs(bqkv, H + h * kHD), 1.f, active, hf, kb);
  const int ev = lane_row(rows + (int64_t)key * ld + 2 * H + h * kHD, bofs(bqkv, 2 * H + h * kHD), 1.f, active, hf, vb);
  const float madd = active ? (1.f - (float)mask[(int64_t)b * S + key]) * (-10000.f * kLog2e) : 0.f;  // base 2

  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  int eq_run = 0, eo_run = 0, es = 126;
  Chunk cur;
  float dsum[2] = {0.f, 0.f};
  auto load = [&](int c0) {
    const int clen = min(64, S - c0);
    chunk_load(cur, rows + h * kHD, drows + h * kHD, ld, H, c0, clen, bofs(bqkv, h * kHD), nullptr, 0.125f);
    if (crows) {  // D = rowsum(dO o O) of the chunk's queries while dO is staged (S <= 128)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int u = tid + 256 * i, r = u >> 3, c8 = 8 * (u & 7);
        float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (r < clen) ld8(crows + (int64_t)(c0 + r) * H + h * kHD + c8, nullptr, 1.f, o);
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s = fmaf(cur.v[1][i][j], o[j], s);
        dsum[i] = s;
      }
    }
  };
  const TrBase tb = tr_base(lane);
  for (int c0 = 0, par = 0; c0 < S; c0 += 64, par ^= 1) {
    const int clen = min(64, S - c0);
    // loaded here: a register prefetch under the previous chunk spills, and an LDS-DMA prefetch
    // (round 4) measured no faster -- its extra barrier per chunk cost what the hidden latency saved
    load(c0);
    chunk_max(cur, red + 8 * par);
    __syncthreads();  // the previous chunk's images are free; the chunk's |max| partials visible
    const int eq = red_exp(red + 8 * par, 0), eo = red_exp(red + 8 * par, 1);
    chunk_put(cur, Qp, Op, clen, eq, eo);
    if (crows) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float s = dsum[i];
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        const int r = (tid + 256 * i) >> 3;
        if (r < clen && (tid & 7) == 0) Ds[r] = s;
      }
      for (int i = tid; i < clen; i += 256) Ls[i] = lse[(int64_t)bh * S + c0 + i] * kLog2e;
    } else {
      for (int i = tid; i < clen; i += 256) {
        Ls[i] = lse[(int64_t)bh * S + c0 + i] * kLog2e;
        Ds[i] = Dd[(int64_t)bh * S + c0 + i];
      }
    }
    if (p > 0.f)
      for (int i = tid; i < clen * 4; i += 256) {
        const int qi = i >> 2, kw = bx * 4 + (i & 3);
        Wd[qi][i & 3] = kw < (S >> 5) ? dmask[((uint64_t)bh * S + c0 + qi) * (uint64_t)(S >> 5) + kw] : 0u;
      }
    __syncthreads();  // the images are ready
    if (!active) continue;
    if (c0 > 0) {  // accumulators to this chunk's image scales (exact)
      const float fq = ldexpf(1.f, eq - eq_run), fo = ldexpf(1.f, eo - eo_run);
      dk0 *= fq;
      dk1 *= fq;
      dv0 *= fo;
      dv1 *= fo;
    }
    eq_run = eq;
    eo_run = eo;
    const float us = ldexpf(1.f, -(eq + ek)) * kLog2e, ud = ldexpf(1.f, -(eo + ev));
#pragma unroll 1
    for (int t = 0; t < clen; t += 32) {
      f32x16 sc = {}, dp = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const hx8 a[2] = {prow(Qp, 0, t + li, 2 * ks + hf), prow(Qp, 1, t + li, 2 * ks + hf)};
        sc = mma3(a, kb[ks], sc);
      }
      __builtin_amdgcn_sched_barrier(0);  // bound the live fragments (no spills at 256 VGPRs)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const hx8 a[2] = {prow(Op, 0, t + li, 2 * ks + hf), prow(Op, 1, t + li, 2 * ks + hf)};
        dp = mma3(a, vb[ks], dp);
      }
      __builtin_amdgcn_sched_barrier(0);
      // P in place of the scores; dV^T first, so the P-with-dropout copies die before dS exists
      // (the four accumulators and the lane's K / V fragments leave little register room)
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[r] = __builtin_amdgcn_exp2f(sc[r] * us + madd - Ls[t + xrow(r, hf)]);
      uint32_t kbits = 0xffffu;  // keep bit of score register r (one register, not 16 live multipliers)
      if (p > 0.f) {
        kbits = 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r) kbits |= ((Wd[t + xrow(r, hf)][w] >> li) & 1u) << r;
      }
      const float kscale = p > 0.f ? dscale : 1.f;
      auto keep = [&](int r) { return ((kbits >> r) & 1u) ? kscale : 0.f; };
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float pd[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) pd[j] = sc[8 * ks + j] * keep(8 * ks + j);
        hx8 pb[2], a[2];
        split8h(pd, sp, pb[0], pb[1]);
        ptr2(Op, t + 16 * ks, tb, 0, a);
        dv0 = mma3(a, pb, dv0);
        ptr2(Op, t + 16 * ks, tb, 1, a);
        dv1 = mma3(a, pb, dv1);
      }
      float ds[2][8];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int r = 8 * ks + j;
          ds[ks][j] = sc[r] * (dp[r] * ud * keep(r) - Ds[t + xrow(r, hf)]);
        }
      const float ss = ds_scale(ds, es, dk0, dk1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (DS) {  // dS [query][key] for the dQ kernel (attn_dq_ds_kernel): a row's 32 keys per store
          float* const tb_ = dsw + ((int64_t)bh * S + c0 + t + 16 * ks) * S;  // (uniform)
#pragma unroll
          for (int j = 0; j < 8; ++j) tb_[(4 * hf + (j & 3) + 8 * (j >> 2)) * S + key] = ds[ks][j];
        }
        hx8 sb[2], a[2];
        split8h(ds[ks], ss, sb[0], sb[1]);
        ptr2(Qp, t + 16 * ks, tb, 0, a);
        dk0 = mma3(a, sb, dk0);
        ptr2(Qp, t + 16 * ks, tb, 1, a);
        dk1 = mma3(a, sb, dk1);
      }
    }
  }
  if (!active) return;
  uint32_t cm = 0u;
  if (dqkv) {
    float* out = dqkv + ((int64_t)b * S + key) * ld + h * kHD;
    store_rows(out + H, dk0, dk1, hf, ldexpf(1.f, -(eq_run + es)), cm);
    store_rows(out + 2 * H, dv0, dv1, hf, ldexpf(1.f, -(eo_run + ep)), cm);
  }
  if (amax) amax_commit(amax, cm);
  if (po.pl) {  // dK, dV as h3p planes of dqkv [B*S][3H] (exponent row stride 3H / 32)
    const int64_t row = (int64_t)b * S + key;
    int8_t* ex = po.ex + ((int64_t)b * S + k0) / 32 * (ld / 32) + h * kHD / 32;
    store_rows_h3p(po, row, H + h * kHD, ld, ex + H / 32, dk0, dk1, hf, ldexpf(1.f, -(eq_run + es)));
    store_rows_h3p(po, row, 2 * H + h * kHD, ld, ex + 2 * H / 32, dv0, dv1, hf, ldexpf(1.f, -(eo_run + ep)));
  }
}

// dQ for 32 queries per wave (lane = query) over 64-key chunks of K / V (biased); D from Dd or, with ctx
// (S <= 128), rowsum(dO o O) computed here.
HS_DEVICE void dq_body(char* __restrict__ smem, int bx, int bh, const float* __restrict__ qkv,
                       const int64_t* __restrict__ mask, const float* __restrict__ bqkv,
                       const float* __restrict__ dctx, const float* __restrict__ lse, const float* __restrict__ Dd,
                       float* __restrict__ dqkv, int S, int NH, float p, const uint32_t* __restrict__ dmask,
                       const float* __restrict__ ctx, float* __restrict__ amax, AttnPl po) {
  char* const Kp = smem;
  char* const Vp = smem + kIm;
  float* const Ms = reinterpret_cast<float*>(smem + 2 * kIm);
  float* const red = Ms + 64 + 64 + 64 * 4;  // the dKV role's layout: [parity][wave][operand]
  const int H = NH * kHD;
  const int64_t ld = 3 * (int64_t)H;
  const int b = bh / NH, h = bh % NH;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5, li = lane & 31;
  const int q0 = bx * 128 + w * 32;
  const bool active = q0 < S;
  const int64_t tok = (int64_t)b * S + q0 + li;
  const float* rows = qkv + (int64_t)b * S * ld;
  const float dscale = drop_scale16(drop_thr16(p));

  hx8 qb[4][2], ob[4][2];
  const int eq = lane_row(rows + (int64_t)(q0 + li) * ld + h * kHD, bofs(bqkv, h * kHD), 0.125f, active, hf, qb);
  const int eo = lane_row(dctx + tok * H + h * kHD, nullptr, 1.f, active, hf, ob);
  float dsum = 0.f, lq = 0.f;
  if (active) {
    if (ctx) {  // D = rowsum(dO o O): this lane's half of the row, the other half from lane ^ 32
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        float o[8], dv[8];
        ld8(ctx + tok * H + h * kHD + 16 * s + 8 * hf, nullptr, 1.f, o);
        ld8(dctx + tok * H + h * kHD + 16 * s + 8 * hf, nullptr, 1.f, dv);
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum = fmaf(dv[j], o[j], dsum);
      }
    } else {
      dsum = Dd[(int64_t)bh * S + q0 + li];
    }
    lq = lse[(int64_t)bh * S + q0 + li] * kLog2e;  // base 2 (the forward's softmax)
  }
  if (ctx) dsum += __shfl_xor(dsum, 32, 64);

  f32x16 dq0 = {}, dq1 = {};
  int ek_run = 0, es = 126;
  Chunk cur;
  auto load = [&](int c0) {
    chunk_load(cur, rows + H + h * kHD, rows + 2 * H + h * kHD, ld, ld, c0, min(64, S - c0), bofs(bqkv, H + h * kHD),
               bofs(bqkv, 2 * H + h * kHD), 1.f);
  };
  const TrBase tb = tr_base(lane);
  for (int c0 = 0, par = 0; c0 < S; c0 += 64, par ^= 1) {
    const int clen = min(64, S - c0);
    load(c0);
    chunk_max(cur, red + 8 * par);
    __syncthreads();
    const int ek = red_exp(red + 8 * par, 0), ev = red_exp(red + 8 * par, 1);
    chunk_put(cur, Kp, Vp, clen, ek, ev);
    for (int i = tid; i < clen; i += 256) Ms[i] = (1.f - (float)mask[(int64_t)b * S + c0 + i]) * (-10000.f * kLog2e);
    __syncthreads();
    if (!active) continue;
    if (c0 > 0) {
      const float fk = ldexpf(1.f, ek - ek_run);
      dq0 *= fk;
      dq1 *= fk;
    }
    ek_run = ek;
    const float us = ldexpf(1.f, -(ek + eq)) * kLog2e, ud = ldexpf(1.f, -(ev + eo));
#pragma unroll 1
    for (int t = 0; t < clen; t += 32) {
      f32x16 sc = {}, dp = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const hx8 a[2] = {prow(Kp, 0, t + li, 2 * ks + hf), prow(Kp, 1, t + li, 2 * ks + hf)};
        sc = mma3(a, qb[ks], sc);
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const hx8 a[2] = {prow(Vp, 0, t + li, 2 * ks + hf), prow(Vp, 1, t + li, 2 * ks + hf)};
        dp = mma3(a, ob[ks], dp);
      }
      const uint32_t word = p > 0.f ? dmask[((uint64_t)bh * S + q0 + li) * (uint64_t)(S >> 5) + ((c0 + t) >> 5)] : 0u;
      float ds[2][8];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int r = 8 * ks + j, kj = xrow(r, hf);
          const float mk = p > 0.f ? (((word >> kj) & 1u) ? dscale : 0.f) : 1.f;
          const float pv = __builtin_amdgcn_exp2f(sc[r] * us + Ms[t + kj] - lq);
          ds[ks][j] = pv * (dp[r] * ud * mk - dsum);
        }
      const float ss = ds_scale(ds, es, dq0, dq1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        hx8 sb[2], a[2];
        split8h(ds[ks], ss, sb[0], sb[1]);
        ptr2(Kp, t + 16 * ks, tb, 0, a);
        dq0 = mma3(a, sb, dq0);
        ptr2(Kp, t + 16 * ks, tb, 1, a);
        dq1 = mma3(a, sb, dq1);
      }
    }
  }
  if (!active) return;
  uint32_t cm = 0u;
  if (dqkv) store_rows(dqkv + tok * ld + h * kHD, dq0, dq1, hf, 0.125f * ldexpf(1.f, -(ek_run + es)), cm);
  if (amax) amax_commit(amax, cm);
  if (po.pl)
    store_rows_h3p(po, tok, h * kHD, ld, po.ex + ((int64_t)b * S + q0) / 32 * (ld / 32) + h * kHD / 32, dq0, dq1, hf,
                   0.125f * ldexpf(1.f, -(ek_run + es)));
}

// D[bh][q] = rowsum(dO o O) over the head's 64 dims (the S > 128 backward reads it): 16 lanes per
// (token, head), float4 each.
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
    const int64_t o = tok * NH * kHD + h * kHD + 4 * l;
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

}  // namespace

int launch_attn_bwd_dsum(const float* ctx, const float* dctx, float* Dout, int B, int S, int NH, hipStream_t st) {
  const int64_t units = (int64_t)B * S * NH;
  hipLaunchKernelGGL(attn_bwd_dsum_kernel, dim3((unsigned)((units + 15) / 16)), dim3(256), 0, st, ctx, dctx, Dout, B, S,
                     NH);
  return 0;
}

// The backward's two roles in one launch (grid (B*NH, 2 * ceil(S/128)); dK / dV blocks first: the longer
// role goes out first and the dQ blocks fill the tail of the last round).  ctx != nullptr: D computed by
// the roles themselves (S <= 128).
__global__ void __launch_bounds__(256, 2)
    attn_bwd_h3_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ mask,
                       const float* __restrict__ bqkv, const float* __restrict__ dctx, const float* __restrict__ lse,
                       const float* __restrict__ Dd, float* __restrict__ dqkv, int S, int NH, float p,
                       const uint32_t* __restrict__ dmask, const float* __restrict__ ctx, float* __restrict__ amax,
                       AttnPl po, float* __restrict__ dsw) {
  __shared__ __attribute__((aligned(16))) char smem[kBwdLds];
  const int nq = (S + 127) / 128, bh = blockIdx.x, y = blockIdx.y;
  if (y < nq)
    dkv_body<false>(smem, y, bh, qkv, mask, bqkv, dctx, lse, Dd, dqkv, S, NH, p, dmask, ctx, amax, po, dsw);
  else
    dq_body(smem, y - nq, bh, qkv, mask, bqkv, dctx, lse, Dd, dqkv, S, NH, p, dmask, ctx, amax, po);
}

// the dK / dV blocks alone, writing dS for attn_dq_ds_kernel
__global__ void __launch_bounds__(256, 2)
    attn_bwd_h3_dkv_ds_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ mask,
                              const float* __restrict__ bqkv, const float* __restrict__ dctx,
                              const float* __restrict__ lse, const float* __restrict__ Dd, float* __restrict__ dqkv,
                              int S, int NH, float p, const uint32_t* __restrict__ dmask, const float* __restrict__ ctx,
                              float* __restrict__ amax, AttnPl po, float* __restrict__ dsw) {
  __shared__ __attribute__((aligned(16))) char smem[kBwdLds];
  dkv_body<true>(smem, blockIdx.y, blockIdx.x, qkv, mask, bqkv, dctx, lse, Dd, dqkv, S, NH, p, dmask, ctx, amax, po, dsw);
}

// diagnostic (set_attn_h3_variant bwd_roles 2): the dQ role's blocks alone
__global__ void __launch_bounds__(256, 2)
    attn_bwd_h3_dq_only_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ mask,
                               const float* __restrict__ bqkv, const float* __restrict__ dctx,
                               const float* __restrict__ lse, const float* __restrict__ Dd, float* __restrict__ dqkv,
                               int S, int NH, float p, const uint32_t* __restrict__ dmask, const float* __restrict__ ctx,
                               float* __restrict__ amax, AttnPl po) {
  __shared__ __attribute__((aligned(16))) char smem[kBwdLds];
  dq_body(smem, blockIdx.y, blockIdx.x, qkv, mask, bqkv, dctx, lse, Dd, dqkv, S, NH, p, dmask, ctx, amax, po);
}

// dQ from the dS the dK / dV blocks wrote ([query][key] fp32, attn_bwd_h3_kernel dsw): dQ = dS K / 8 per
// head, 32 queries per wave (lane = query) over 64-key chunks of K (biased), K split per chunk into plane
// images, dS split with the running per-lane exponent (ds_scale) -- the dQ role of the fused backward
// without recomputing the scores, P, dP and dS (round 6: that role was ~23 of the 58-us backward at
// B 32, S 128, tools/bench_attn.py).
__global__ void __launch_bounds__(256, 2)
    attn_dq_ds_kernel(const float* __restrict__ qkv, const float* __restrict__ bqkv, const float* __restrict__ dsw,
                      float* __restrict__ dqkv, int S, int NH, float* __restrict__ amax, AttnPl po) {
  __shared__ __attribute__((aligned(16))) char smem[kIm + 16 * 4];
  char* const Kp = smem;
  float* const red = reinterpret_cast<float*>(smem + kIm);  // [parity][wave]
  const int H = NH * kHD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5, li = lane & 31;
  const int q0 = blockIdx.y * 128 + w * 32;
  const bool active = q0 < S;
  const int64_t tok = (int64_t)b * S + q0 + li;
  const float* krows = qkv + (int64_t)b * S * ld + H + h * kHD;
  const float* kbias = bofs(bqkv, H + h * kHD);
  const float* dsrow = dsw + ((int64_t)bh * S + (active ? q0 + li : 0)) * S;  // this lane's query row of dS
  f32x16 dq0 = {}, dq1 = {};
  int ek_run = 0, es = 126;
  const TrBase tb = tr_base(lane);
  for (int c0 = 0, par = 0; c0 < S; c0 += 64, par ^= 1) {
    const int clen = min(64, S - c0);
    float kv[2][8];
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // thread unit u = tid + 256 i: key row u >> 3, dims 8 (u & 7) .. + 7
      const int u = tid + 256 * i, r = u >> 3, c8 = 8 * (u & 7);
      if (r < clen) {
        ld8(krows + (int64_t)(c0 + r) * ld + c8, kbias ? kbias + c8 : nullptr, 1.f, kv[i]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) kv[i][j] = 0.f;
      }
      m = amax8(kv[i], m);
    }
    // this chunk's dS rows, both 32-key tiles, in flight with the K rows (a 32-key tail chunk's second
    // tile re-reads the first: unconditional loads)
    float dsc[2][2][8];  // [tile][ks][j]: key c0 + 32 tile + xrow(8 ks + j, hf)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = min(32 * tt, clen - 32);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const float4 x = *reinterpret_cast<const float4*>(dsrow + c0 + t + 16 * ks + 4 * hf);
        const float4 y = *reinterpret_cast<const float4*>(dsrow + c0 + t + 16 * ks + 8 + 4 * hf);
        dsc[tt][ks][0] = x.x; dsc[tt][ks][1] = x.y; dsc[tt][ks][2] = x.z; dsc[tt][ks][3] = x.w;
        dsc[tt][ks][4] = y.x; dsc[tt][ks][5] = y.y; dsc[tt][ks][6] = y.z; dsc[tt][ks][7] = y.w;
      }
    }
    m = wave_max(m);
    if (lane == 0) red[8 * par + w] = m;
    __syncthreads();  // the previous chunk's image is free; the chunk's |max| partials visible
    const int ek = h16e(fmaxf(fmaxf(red[8 * par], red[8 * par + 1]), fmaxf(red[8 * par + 2], red[8 * par + 3])));
    const float sk = ldexpf(1.f, ek);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int u = tid + 256 * i, r = u >> 3;
      if (r < clen) put2(Kp, r, u & 7, kv[i], sk);
    }
    __syncthreads();  // the image is ready
    if (!active) continue;
    if (c0 > 0) {
      const float fk = ldexpf(1.f, ek - ek_run);
      dq0 *= fk;
      dq1 *= fk;
    }
    ek_run = ek;
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = 32 * tt;
      if (t >= clen) break;
      float (&ds)[2][8] = dsc[tt];  // ds[ks][j]: key t + xrow(8 ks + j, hf), the dQ role's register order
      const float ss = ds_scale(ds, es, dq0, dq1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        hx8 sb[2], a[2];
        split8h(ds[ks], ss, sb[0], sb[1]);
        ptr2(Kp, t + 16 * ks, tb, 0, a);
        dq0 = mma3(a, sb, dq0);
        ptr2(Kp, t + 16 * ks, tb, 1, a);
        dq1 = mma3(a, sb, dq1);
      }
    }
  }
  if (!active) return;
  uint32_t cm = 0u;
  if (dqkv) store_rows(dqkv + tok * ld + h * kHD, dq0, dq1, hf, 0.125f * ldexpf(1.f, -(ek_run + es)), cm);
  if (amax) amax_commit(amax, cm);
  if (po.pl)
    store_rows_h3p(po, tok, h * kHD, ld, po.ex + ((int64_t)b * S + q0) / 32 * (ld / 32) + h * kHD / 32, dq0, dq1, hf,
                   0.125f * ldexpf(1.f, -(ek_run + es)));
}

// Forward: a wave owns 32 queries (lane = query), S^T tiles with the key on the registers, online softmax;
// each 64-key chunk of K and V is split once into plane images with the chunk's exponents.  PAIR: a whole
// 64-key chunk's two score tiles at once (one workgroup per CU: its registers spill at two); else one
// 32-key tile at a time at two workgroups per CU (round 5).
template <bool PAIR>
__global__ void __launch_bounds__(256, PAIR ? 1 : 2)
    attn_fwd_h3_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ mask,
                       const float* __restrict__ bqkv, float* __restrict__ ctx, float* __restrict__ lse,
                       uint32_t* __restrict__ dmask, int S, int NH, float p, uint64_t seed, uint64_t off,
                       const uint64_t* __restrict__ seed_dev, int bh0, float* __restrict__ amax, AttnPl po) {
  seed = resolve_seed(seed, seed_dev);
  __shared__ __attribute__((aligned(16))) char smem[2 * kIm];
  __shared__ float Ms[64];
  __shared__ float red[2 * 8];
  char* const Kimg = smem;
  char* const Vimg = smem + kIm;
  const int H = NH * kHD;
  const int64_t ld = 3 * (int64_t)H;
  const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5, li = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q0 = blockIdx.y * 128 + w * 32;
  const bool active = q0 < S;
  const float* rows = qkv + (int64_t)b * S * ld;
  const uint32_t thr = drop_thr16(p);
  const float dscale = drop_scale16(thr);
  const int ep = p_exp(p > 0.f ? dscale : 1.f);
  const float sp = ldexpf(1.f, ep);

  // the softmax runs in base 2: scores, mask and running max carry log2(e), so every exponential is
  // one v_exp_f32 (no range fix-up around __expf); lse is written in natural units
  // the lane's Q row, biased, * 1/sqrt(64) (exact), split with its row exponent
  hx8 qf[4][2];
  const int eq = lane_row(rows + (int64_t)(q0 + li) * ld + h * kHD, bofs(bqkv, h * kHD), 0.125f, active, hf, qf);
  f32x16 o0 = {}, o1 = {};
  float m = -1e30f, l = 0.f;
  int ev_run = 0;
  const uint64_t erow = ((uint64_t)(bh0 + bh) * S + (q0 + li)) * (uint64_t)S;  // bh0: a batch slice's first head

  Chunk cur;
  auto load = [&](int c0) {
    chunk_load(cur, rows + H + h * kHD, rows + 2 * H + h * kHD, ld, ld, c0, min(64, S - c0), bofs(bqkv, H + h * kHD),
               bofs(bqkv, 2 * H + h * kHD), 1.f);
  };
  load(0);
  const TrBase tb = tr_base(lane);
  for (int c0 = 0, par = 0; c0 < S; c0 += 64, par ^= 1) {
    const int clen = min(64, S - c0);
    chunk_max(cur, red + 8 * par);
    __syncthreads();  // every wave done with the previous chunk's images; |max| partials visible
    const int ek = red_exp(red + 8 * par, 0), ev = red_exp(red + 8 * par, 1);
    chunk_put(cur, Kimg, Vimg, clen, ek, ev);
    for (int i = tid; i < clen; i += 256) Ms[i] = (1.f - (float)mask[(int64_t)b * S + c0 + i]) * (-10000.f * kLog2e);
    __syncthreads();
    if (c0 + 64 < S) load(c0 + 64);  // the next chunk's rows fly under this chunk's MFMAs
    if (!active) continue;
    if (c0 > 0) {
      const float fv = ldexpf(1.f, ev - ev_run);
      o0 *= fv;
      o1 *= fv;
    }
    ev_run = ev;
    const float us = ldexpf(1.f, -(ek + eq)) * kLog2e;
    if (PAIR && clen == 64) {
      // the chunk's two 32-key tiles together: two independent score accumulators (the 12-MFMA chains
      // interleave instead of running back to back), one softmax update and one rescale of the output
      // accumulators per chunk.  Same keep-bit stream and words as the per-tile path below.
      f32x16 s0 = {}, s1 = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const hx8 ka[2] = {prow(Kimg, 0, li, 2 * ks + hf), prow(Kimg, 1, li, 2 * ks + hf)};
        const hx8 kb[2] = {prow(Kimg, 0, 32 + li, 2 * ks + hf), prow(Kimg, 1, 32 + li, 2 * ks + hf)};
        s0 = mma3(ka, qf[ks], s0);
        s1 = mma3(kb, qf[ks], s1);
      }
      float mt = -1e30f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s0[r] = s0[r] * us + Ms[xrow(r, hf)];
        s1[r] = s1[r] * us + Ms[32 + xrow(r, hf)];
        mt = fmaxf(mt, fmaxf(s0[r], s1[r]));
      }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m, mt);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);
      m = mn;
      float ps = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {  // the scores' registers become P
        s0[r] = __builtin_amdgcn_exp2f(s0[r] - mn);
        s1[r] = __builtin_amdgcn_exp2f(s1[r] - mn);
        ps += s0[r] + s1[r];
      }
      ps += __shfl_xor(ps, 32, 64);
      l = l * alpha + ps;
      o0 *= alpha;
      o1 *= alpha;
      auto pv_tile = [&](f32x16& pr, const int tt) __attribute__((always_inline)) {
        if (p > 0.f) {
          const uint64_t e0 = (erow + c0 + 32 * tt) >> 3;
          const uint32_t mine =
              keep8_bits(seed, off, e0 + 2 * hf, thr) | (keep8_bits(seed, off, e0 + 2 * hf + 1, thr) << 8);
          const uint32_t other = static_cast<uint32_t>(__shfl_xor(static_cast<int>(mine), 32, 64));
          const uint32_t bits = hf == 0 ? (mine | (other << 16)) : (other | (mine << 16));
#pragma unroll
          for (int r = 0; r < 16; ++r) pr[r] = ((bits >> xrow(r, hf)) & 1u) ? pr[r] * dscale : 0.f;
          if (dmask && hf == 0) dmask[((uint64_t)bh * S + q0 + li) * (uint64_t)(S >> 5) + ((c0 + 32 * tt) >> 5)] = bits;
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          float pv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) pv[j] = pr[8 * ks + j];
          hx8 pf[2], a[2];
          split8h(pv, sp, pf[0], pf[1]);
          ptr2(Vimg, 32 * tt + 16 * ks, tb, 0, a);
          o0 = mma3(a, pf, o0);
          ptr2(Vimg, 32 * tt + 16 * ks, tb, 1, a);
          o1 = mma3(a, pf, o1);
        }
      };
      pv_tile(s0, 0);
      pv_tile(s1, 1);
      continue;
    }
#pragma unroll 1
    for (int t = 0; t < clen; t += 32) {
      f32x16 s = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const hx8 kf[2] = {prow(Kimg, 0, t + li, 2 * ks + hf), prow(Kimg, 1, t + li, 2 * ks + hf)};
        s = mma3(kf, qf[ks], s);
      }
      float mt = -1e30f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[r] = s[r] * us + Ms[t + xrow(r, hf)];
        mt = fmaxf(mt, s[r]);
      }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m, mt);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);
      m = mn;
      float pr[16];
      float ps = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        pr[r] = __builtin_amdgcn_exp2f(s[r] - mn);
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
        hx8 pf[2], a[2];
        split8h(pv, sp, pf[0], pf[1]);
        ptr2(Vimg, t + 16 * ks, tb, 0, a);
        o0 = mma3(a, pf, o0);
        ptr2(Vimg, t + 16 * ks, tb, 1, a);
        o1 = mma3(a, pf, o1);
      }
    }
  }
  if (!active) return;
  const float inv = ldexpf(1.f, -(ev_run + ep)) / l;
  uint32_t cm = 0u;
  store_rows(ctx + ((int64_t)b * S + q0 + li) * H + h * kHD, o0, o1, hf, inv, cm);
  if (amax) amax_commit(amax, cm);  // ctx's |max|: the output projection's operand scale
  if (po.pl)  // ctx as h3p planes of the output projection (exponent row stride H / 32)
    store_rows_h3p(po, (int64_t)b * S + q0 + li, h * kHD, H, po.ex + ((int64_t)b * S + q0) / 32 * (H / 32) + 2 * h, o0,
                   o1, hf, inv);
  if (hf == 0) lse[(int64_t)bh * S + q0 + li] = m * kLn2 + __logf(l);
}

}  // namespace hs

using namespace hs;

// The forward kernel per sequence length: the paired-tile one (one workgroup per CU) from S = 256 on,
// the per-tile one (two per CU) below -- measured in the step (bench.py --ab, round 6): phase 2
// (S 512) 11.98 vs 12.27 ms paired / per tile, phase 1 (S 128) 10.80 vs 10.68 ms.  The backward at
// one workgroup per CU (no spills, the score and dP chains interleaved) measured slower than at two
// (176 B of scratch) in both phases (10.98 vs 10.68 ms; 12.75 vs 12.27 ms) and was removed.
// set_attn_h3_variant: -1 = that choice, 0 / 1 = always per tile / paired (tests, A/B).
static int g_attn_fwd_pair = -1;
static int g_attn_bwd_roles = 3;  // diagnostic: 1 = only the dK / dV blocks, 2 = only the dQ blocks
void set_attn_h3_variant(int fwd_pair, int bwd_roles) {
  g_attn_fwd_pair = fwd_pair;
  g_attn_bwd_roles = bwd_roles > 0 ? bwd_roles : 3;
}

// amax (optional): a |max| slot (common.h) the kernels max |output| into (ctx forward, dqkv backward)
int launch_attn_fwd_h3(const float* qkv, const int64_t* mask, const float* bqkv, float* ctx, float* lse,
                       uint32_t* dmask, int B, int S, int NH, int D, float p, uint64_t seed, uint64_t off,
                       hipStream_t st, int bh0, float* amax, void* pl, int64_t ps, int8_t* ex) {
  if (D != kHD || S % 32 != 0 || S <= 0) return -1;
  const AttnPl po{static_cast<uint16_t*>(pl), ps, ex};
  // grid (B*NH, S/128): consecutive blocks are different heads, so every query block of a head lands on
  // the same XCD and its K / V come through one L2
  if (g_attn_fwd_pair > 0 || (g_attn_fwd_pair < 0 && S >= 256))
    hipLaunchKernelGGL(attn_fwd_h3_kernel<true>, dim3(B * NH, (S + 127) / 128), dim3(256), 0, st, qkv, mask, bqkv, ctx,
                       lse, dmask, S, NH, p, seed, off, g_seed_dev, bh0, amax, po);
  else
    hipLaunchKernelGGL(attn_fwd_h3_kernel<false>, dim3(B * NH, (S + 127) / 128), dim3(256), 0, st, qkv, mask, bqkv,
                       ctx, lse, dmask, S, NH, p, seed, off, g_seed_dev, bh0, amax, po);
  return 0;
}

// dsbuf (B * NH * S * S floats, or null): dQ from the dS the dK / dV blocks write there (attn_dq_ds_kernel)
// instead of the fused dQ role that recomputes it
int launch_attn_bwd_h3(const float* qkv, const int64_t* mask, const float* bqkv, const float* ctx, const float* dctx,
                       const float* lse, float* Dbuf, float* dqkv, const uint32_t* dmask, int B, int S, int NH, int D,
                       float p, hipStream_t st, float* amax, void* pl, int64_t ps, int8_t* ex, float* dsbuf) {
  if (D != kHD || S % 32 != 0 || S <= 0 || (p > 0.f && dmask == nullptr)) return -1;
  if (!dqkv && (!pl || amax)) return -1;  // dqkv may be written only as the planes
  const AttnPl po{static_cast<uint16_t*>(pl), ps, ex};
  const bool fused_d = S <= 128;  // each head's one dK / dV block stages every query once
  if (!fused_d) {
    if (Dbuf == nullptr) return -1;
    launch_attn_bwd_dsum(ctx, dctx, Dbuf, B, S, NH, st);
  }
  const int nq = (S + 127) / 128;
  if (dsbuf) {  // the dK / dV blocks (writing dS), then dQ from dS
    hipLaunchKernelGGL(attn_bwd_h3_dkv_ds_kernel, dim3(B * NH, nq), dim3(256), 0, st, qkv, mask, bqkv, dctx, lse, Dbuf,
                       dqkv, S, NH, p, dmask, fused_d ? ctx : nullptr, amax, po, dsbuf);
    hipLaunchKernelGGL(attn_dq_ds_kernel, dim3(B * NH, nq), dim3(256), 0, st, qkv, bqkv, (const float*)dsbuf, dqkv, S,
                       NH, amax, po);
    return 0;
  }
  const dim3 grid(B * NH, g_attn_bwd_roles == 3 ? 2 * nq : nq);
  if (g_attn_bwd_roles == 2) {  // (diagnostic: the dQ role alone -- its blocks' y index starts at nq)
    hipLaunchKernelGGL(attn_bwd_h3_dq_only_kernel, grid, dim3(256), 0, st, qkv, mask, bqkv, dctx, lse, Dbuf, dqkv, S, NH,
                       p, dmask, fused_d ? ctx : nullptr, amax, po);
    return 0;
  }
  hipLaunchKernelGGL(attn_bwd_h3_kernel, grid, dim3(256), 0, st, qkv, mask, bqkv, dctx, lse, Dbuf, dqkv, S, NH, p,
                     dmask, fused_d ? ctx : nullptr, amax, po, nullptr);
  return 0;
}
