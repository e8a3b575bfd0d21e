// Row LayerNorm family for BERT (K03, K05, K06, K10 of SURVEY §2.4).
//
// Reference math (bert_modeling.py:285-289): u = mean(x); s = mean((x-u)^2);
// y = w * (x-u)/sqrt(s+eps) + b with eps = 1e-12 and a BIASED variance.
// Reference call sites fused here:
//   * BertSelfOutput/BertOutput (bert_modeling.py:387-391, 423-427):
//       y = LN(dropout(dense_out + bias) + residual)        -> mode kBDR
//   * BertEmbeddings (bert_modeling.py:306-320):
//       y = dropout(LN(word[id] + pos[s] + type[tt]))         -> emb kernels
//   * BertPredictionHeadTransform LN (bert_modeling.py:525-528) -> mode kPlain
//
// Layout: one wave per row, lane l owns columns (k*64+l)*4 .. +3 for k < NV,
// so every global access is a coalesced 16-byte-per-lane vector (H = NV*256).
// Statistics are two-pass in registers (exactly the reference's formula).
// Backward kernels produce the row gradient and per-block column partials of
// dgamma/dbeta/dbias; `colpart_finalize` reduces the partials (no atomics,
// deterministic).  Dropout masks are regenerated from Philox (seed, offset).
#include <cstdlib>

#include "common.h"
#include "h3p.h"
#include "reduce.h"

namespace hs {

enum LnMode : int { kPlain = 0, kBDR = 1 };

template <int NV>
HS_DEVICE void row_stats(const float (&x)[NV][4], int H, float& mean, float& rstd, float eps) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) s += (x[k][0] + x[k][1]) + (x[k][2] + x[k][3]);
  mean = wave_sum(s) / H;
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d = x[k][j] - mean;
      v = fmaf(d, d, v);
    }
  v = wave_sum(v) / H;
  rstd = 1.0f / sqrtf(v + eps);
}

// NS > 0: the slab count at compile time -- every load of a row in flight at once, combined in the
// NS = 0 order (ln_fwd_h3p_coop_kernel); the bf16 step's calls are NS = 1.
template <int NV, typename T, int NS = 0>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const T* __restrict__ a, const float* __restrict__ bias,
                                                     const T* __restrict__ resid, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, T* __restrict__ y,
                                                     float* __restrict__ zsave, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, int rows, float eps, float p,
                                                     uint64_t seed, uint64_t off, int mode,
                                                     const uint64_t* __restrict__ seed_dev,
                                                     int nslab,
                                                     int64_t slab_stride, int row0, float* __restrict__ amax_y) {
  constexpr int H = NV * 256;
  const int lane = threadIdx.x & 63;
  const float scale = p < 1.f ? 1.0f / (1.0f - p) : 0.f;
  seed = resolve_seed(seed, seed_dev);
  uint32_t am = 0u;  // |max| of y as bits (amax_y: the next fp16-split GEMM's operand scale)
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += gridDim.x * 4) {
    const int64_t base = (int64_t)row * H;
    float x[NV][4];
    if constexpr (NS > 0) {
      float t[NS > 1 ? NS - 1 : 1][NV][4], bv[NV][4], rv[NV][4];
      const float* const bsrc = bias ? bias : gamma;
      const T* const rsrc = resid ? resid : a;
#pragma unroll
      for (int k = 0; k < NV; ++k) load4(a + base + (k * 64 + lane) * 4, x[k]);
#pragma unroll
      for (int sl = 1; sl < NS; ++sl)
#pragma unroll
        for (int k = 0; k < NV; ++k) load4(a + sl * slab_stride + base + (k * 64 + lane) * 4, t[sl - 1][k]);
#pragma unroll
      for (int k = 0; k < NV; ++k) load4(bsrc + (k * 64 + lane) * 4, bv[k]);
#pragma unroll
      for (int k = 0; k < NV; ++k) load4(rsrc + base + (k * 64 + lane) * 4, rv[k]);
      const bool hb = bias != nullptr, hr = resid != nullptr;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (k * 64 + lane) * 4;
#pragma unroll
        for (int sl = 1; sl < NS; ++sl)
#pragma unroll
          for (int j = 0; j < 4; ++j) x[k][j] += t[sl - 1][k][j];
#pragma unroll
        for (int j = 0; j < 4; ++j) x[k][j] = hb ? x[k][j] + bv[k][j] : x[k][j];
        if (mode == kBDR && p > 0.f) {
          float m[4];
          keep4(seed, off, (uint64_t)((int64_t)(row0 + row) * H + c) >> 2, p, scale, m);
#pragma unroll
          for (int j = 0; j < 4; ++j) x[k][j] *= m[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) x[k][j] = hr ? x[k][j] + rv[k][j] : x[k][j];
        if (zsave) store4(zsave + base + c, x[k]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (k * 64 + lane) * 4;
        load4(a + base + c, x[k]);
        for (int sl = 1; sl < nslab; ++sl) {  // split-K partials of the producing GEMM, summed in slice order
          float t[4];
          load4(a + sl * slab_stride + base + c, t);
#pragma unroll
          for (int j = 0; j < 4; ++j) x[k][j] += t[j];
        }
        if (bias) {
          float b[4];
          load4(bias + c, b);
#pragma unroll
          for (int j = 0; j < 4; ++j) x[k][j] += b[j];
        }
        if (mode == kBDR && p > 0.f) {  // counter of the element's row in the whole batch (row0: a row slice)
          float m[4];
          keep4(seed, off, (uint64_t)((int64_t)(row0 + row) * H + c) >> 2, p, scale, m);
#pragma unroll
          for (int j = 0; j < 4; ++j) x[k][j] *= m[j];
        }
        if (resid) {
          float r[4];
          load4(resid + base + c, r);
#pragma unroll
          for (int j = 0; j < 4; ++j) x[k][j] += r[j];
        }
        if (zsave) store4(zsave + base + c, x[k]);
      }
    }
    float mean, rstd;
    row_stats<NV>(x, H, mean, rstd, eps);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
      float gw[4], gb[4], o[4];
      load4(gamma + c, gw);
      load4(beta + c, gb);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = gw[j] * ((x[k][j] - mean) * rstd) + gb[j];
        am = amax_bits(am, o[j]);
      }
      store4(y + base + c, o);
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
  if (amax_y) amax_commit(amax_y, am);
}

// LayerNorm forward that also writes y as h3p operand planes (h3p.h): one block = 32 consecutive rows
// (the exponent block's height), 8 waves x 4 rows; after the rows, each 32-column group's |max| over
// the block's 32 rows (lanes, then waves through LDS) sets the block exponent, and every lane splits
// the y values it still holds.  Same per-row arithmetic as ln_fwd_kernel (bitwise the same y).
constexpr int kLnH3pWaves = 8;

template <int NV, typename T, int WV>
__global__ void __launch_bounds__(64 * WV) ln_fwd_h3p_kernel(
    const T* __restrict__ a, const float* __restrict__ bias, const T* __restrict__ resid,
    const float* __restrict__ gamma, const float* __restrict__ beta, T* __restrict__ y, float* __restrict__ zsave,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, float eps, float p, uint64_t seed, uint64_t off, int mode,
    const uint64_t* __restrict__ seed_dev, int nslab, int64_t slab_stride, int row0, float* __restrict__ amax_y,
    uint16_t* __restrict__ planes, int64_t ps, int8_t* __restrict__ exps) {
  constexpr int H = NV * 256, RPW = 32 / WV;
  __shared__ float red[WV][NV * 8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float scale = p < 1.f ? 1.0f / (1.0f - p) : 0.f;
  seed = resolve_seed(seed, seed_dev);
  uint32_t am = 0u;
  float o[RPW][NV][4];
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    const int row = blockIdx.x * 32 + w * RPW + j;
    const int64_t base = (int64_t)row * H;
    float x[NV][4];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
      load4(a + base + c, x[k]);
      for (int sl = 1; sl < nslab; ++sl) {
        float t[4];
        load4(a + sl * slab_stride + base + c, t);
#pragma unroll
        for (int e = 0; e < 4; ++e) x[k][e] += t[e];
      }
      if (bias) {
        float b[4];
        load4(bias + c, b);
#pragma unroll
        for (int e = 0; e < 4; ++e) x[k][e] += b[e];
      }
      if (mode == kBDR && p > 0.f) {
        float m[4];
        keep4(seed, off, (uint64_t)((int64_t)(row0 + row) * H + c) >> 2, p, scale, m);
#pragma unroll
        for (int e = 0; e < 4; ++e) x[k][e] *= m[e];
      }
      if (resid) {
        float r[4];
        load4(resid + base + c, r);
#pragma unroll
        for (int e = 0; e < 4; ++e) x[k][e] += r[e];
      }
      if (zsave) store4(zsave + base + c, x[k]);
    }
    float mean, rstd;
    row_stats<NV>(x, H, mean, rstd, eps);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
      float gw[4], gb[4];
      load4(gamma + c, gw);
      load4(beta + c, gb);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[j][k][e] = gw[e] * ((x[k][e] - mean) * rstd) + gb[e];
        am = amax_bits(am, o[j][k][e]);
      }
      store4(y + base + c, o[j][k]);
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
  if (amax_y) amax_commit(amax_y, am);
  // 32-column group k * 8 + lane / 8: the lane's |max| over its rows, its 8 lanes, then the 8 waves
  uint32_t gm[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    gm[k] = 0u;
#pragma unroll
    for (int j = 0; j < RPW; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) gm[k] = amax_bits(gm[k], o[j][k][e]);
#pragma unroll
    for (int sh = 1; sh < 8; sh <<= 1)
      gm[k] = max(gm[k], static_cast<uint32_t>(__shfl_xor(static_cast<int>(gm[k]), sh, 64)));
    if ((lane & 7) == 0) red[w][k * 8 + (lane >> 3)] = __uint_as_float(gm[k]);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    uint32_t m = 0u;
#pragma unroll
    for (int v = 0; v < WV; ++v) m = max(m, __float_as_uint(red[v][k * 8 + (lane >> 3)]));
    const int e = h3p_exp_bits(m);
    const float sc = h3p_scale(e);
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int row = blockIdx.x * 32 + w * RPW + j;
      h3p_store4(planes, ps, h3p_index(row, (k * 64 + lane) * 4, H, 1), o[j][k], sc);  // blocked planes
    }
    if (w == 0 && (lane & 7) == 0) exps[(int64_t)blockIdx.x * (H / 32) + k * 8 + (lane >> 3)] = static_cast<int8_t>(e);
  }
}

// The same LayerNorm forward on 4-wave workgroups of 4 RPW rows (8 with RPW 2: a 2048-row call is 256
// workgroups, one per CU, instead of 64 of 32 rows): the 32 / (4 RPW) workgroups of a 32-row panel
// combine their column-group |max| through the panel record (h3p.h psync_exchange) and each splits
// its own rows from registers.  Per-row arithmetic, y / z / planes / exponents bitwise those of
// ln_fwd_h3p_kernel.  `psync`: the records of panels panel0 + (rows of this call) / 32.
// NS > 0: the call's split-K slab count, fixed at compile time, so every load of a row -- the NS slabs,
// the bias and the residual -- is issued before the first is consumed (a runtime slab loop waited out
// each load in turn: 18 serialised round trips per row at two waves per SIMD); the sums keep the slice
// order, so the result is bitwise that of NS = 0 (runtime nslab, loads in turn).
template <int NV, int RPW, int NS = 0>
__global__ void __launch_bounds__(256) ln_fwd_h3p_coop_kernel(
    const float* __restrict__ a, const float* __restrict__ bias, const float* __restrict__ resid,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ y, float* __restrict__ zsave,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, float eps, float p, uint64_t seed, uint64_t off, int mode,
    const uint64_t* __restrict__ seed_dev, int nslab, int64_t slab_stride, int row0, float* __restrict__ amax_y,
    uint16_t* __restrict__ planes, int64_t ps, int8_t* __restrict__ exps, uint32_t* __restrict__ psync, int panel0) {
  constexpr int H = NV * 256, NG = H / 32, RB = 4 * RPW, NP = 32 / RB;
  __shared__ uint32_t red[4][NG];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int panel = blockIdx.x / NP;
  uint32_t* rec = psync + (int64_t)(panel0 + panel) * kPanelSyncWords;
  uint32_t gen = 0u;
  if (threadIdx.x == 0) gen = psync_gen(rec);  // in flight behind the row loads
  const float scale = p < 1.f ? 1.0f / (1.0f - p) : 0.f;
  seed = resolve_seed(seed, seed_dev);
  uint32_t am = 0u;
  float o[RPW][NV][4], gw[NV][4], gb[NV][4];  // (gamma / beta in flight with the first row's loads)
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    load4(gamma + (k * 64 + lane) * 4, gw[k]);
    load4(beta + (k * 64 + lane) * 4, gb[k]);
  }
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    const int row = blockIdx.x * RB + w * RPW + j;
    const int64_t base = (int64_t)row * H;
    float x[NV][4];
    if constexpr (NS > 0) {
      // every load first (absent bias / residual read stand-in rows -- gamma, the input -- and are
      // selected away), then the combination in the order of the NS = 0 path
      float t[NS > 1 ? NS - 1 : 1][NV][4], bv[NV][4], rv[NV][4];
      const float* const bsrc = bias ? bias : gamma;
      const float* const rsrc = resid ? resid : a;
#pragma unroll
      for (int k = 0; k < NV; ++k) load4(a + base + (k * 64 + lane) * 4, x[k]);
#pragma unroll
      for (int sl = 1; sl < NS; ++sl)
#pragma unroll
        for (int k = 0; k < NV; ++k) load4(a + sl * slab_stride + base + (k * 64 + lane) * 4, t[sl - 1][k]);
#pragma unroll
      for (int k = 0; k < NV; ++k) load4(bsrc + (k * 64 + lane) * 4, bv[k]);
#pragma unroll
      for (int k = 0; k < NV; ++k) load4(rsrc + base + (k * 64 + lane) * 4, rv[k]);
      const bool hb = bias != nullptr, hr = resid != nullptr;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (k * 64 + lane) * 4;
#pragma unroll
        for (int sl = 1; sl < NS; ++sl)
#pragma unroll
          for (int e = 0; e < 4; ++e) x[k][e] += t[sl - 1][k][e];
#pragma unroll
        for (int e = 0; e < 4; ++e) x[k][e] = hb ? x[k][e] + bv[k][e] : x[k][e];
        if (mode == kBDR && p > 0.f) {
          float m[4];
          keep4(seed, off, (uint64_t)((int64_t)(row0 + row) * H + c) >> 2, p, scale, m);
#pragma unroll
          for (int e = 0; e < 4; ++e) x[k][e] *= m[e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) x[k][e] = hr ? x[k][e] + rv[k][e] : x[k][e];
        if (zsave) store4(zsave + base + c, x[k]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = (k * 64 + lane) * 4;
        load4(a + base + c, x[k]);
        for (int sl = 1; sl < nslab; ++sl) {
          float t[4];
          load4(a + sl * slab_stride + base + c, t);
#pragma unroll
          for (int e = 0; e < 4; ++e) x[k][e] += t[e];
        }
        if (bias) {
          float b[4];
          load4(bias + c, b);
#pragma unroll
          for (int e = 0; e < 4; ++e) x[k][e] += b[e];
        }
        if (mode == kBDR && p > 0.f) {
          float m[4];
          keep4(seed, off, (uint64_t)((int64_t)(row0 + row) * H + c) >> 2, p, scale, m);
#pragma unroll
          for (int e = 0; e < 4; ++e) x[k][e] *= m[e];
        }
        if (resid) {
          float r[4];
          load4(resid + base + c, r);
#pragma unroll
          for (int e = 0; e < 4; ++e) x[k][e] += r[e];
        }
        if (zsave) store4(zsave + base + c, x[k]);
      }
    }
    float mean, rstd;
    row_stats<NV>(x, H, mean, rstd, eps);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[j][k][e] = gw[k][e] * ((x[k][e] - mean) * rstd) + gb[k][e];
        am = amax_bits(am, o[j][k][e]);
      }
      store4(y + base + c, o[j][k]);
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
  if (amax_y) amax_commit(amax_y, am);
  // column group k * 8 + lane / 8: the lane's |max| over its rows, its 8 lanes, the 4 waves, the panel
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    uint32_t gm = 0u;
#pragma unroll
    for (int j = 0; j < RPW; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) gm = amax_bits(gm, o[j][k][e]);
#pragma unroll
    for (int sh = 1; sh < 8; sh <<= 1) gm = max(gm, static_cast<uint32_t>(__shfl_xor(static_cast<int>(gm), sh, 64)));
    if ((lane & 7) == 0) red[w][k * 8 + (lane >> 3)] = gm;
  }
  __syncthreads();
  if (w == 0) {
    uint32_t m = 0u;
    if (lane < NG) m = max(max(red[0][lane], red[1][lane]), max(red[2][lane], red[3][lane]));
    const uint32_t g = static_cast<uint32_t>(__shfl(static_cast<int>(gen), 0, 64));
    m = psync_wait(rec, g, psync_arrive(rec, g, m, NG, NP), NG);
    if (lane < NG) red[0][lane] = m;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int e = h3p_exp_bits(red[0][k * 8 + (lane >> 3)]);
    const float sc = h3p_scale(e);
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int row = blockIdx.x * RB + w * RPW + j;
      h3p_store4(planes, ps, h3p_index(row, (k * 64 + lane) * 4, H, 1), o[j][k], sc);  // blocked planes
    }
    if (w == 0 && (lane & 7) == 0 && (blockIdx.x % NP) == 0)
      exps[(int64_t)panel * NG + k * 8 + (lane >> 3)] = static_cast<int8_t>(e);
  }
}

// Column partials are written as part[blockIdx.x][H] (one row per block); the WV waves'
// register partials are summed in a fixed pairwise order (deterministic).
template <int NV, int WV = 4>
HS_DEVICE void block_colpart_store(float (&acc)[NV][4], float* __restrict__ part, float* lds) {
  constexpr int H = NV * 256;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // lds: [WV][H]
#pragma unroll
  for (int k = 0; k < NV; ++k) store4(lds + w * H + (k * 64 + lane) * 4, acc[k]);
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += blockDim.x) {
    float v = (lds[c] + lds[H + c]) + (lds[2 * H + c] + lds[3 * H + c]);
    if (WV == 8) v += (lds[4 * H + c] + lds[5 * H + c]) + (lds[6 * H + c] + lds[7 * H + c]);
    part[(int64_t)blockIdx.x * H + c] = v;
  }
  __syncthreads();
}

// The same per-block column partials through a 3 KB LDS window instead of [WV][H]: waves 1-3 hand
// wave 0 one 256-column chunk at a time and wave 0 sums ((w0 + w1) + (w2 + w3)) -- the LN backward
// then needs 3 KB of LDS instead of 12 KB, so it still finds room on a CU whose LDS is taken by three
// 53 KB split-bf16 GEMM blocks of the other stream (160 KB - 3 x 53 KB = 4 KB left).
template <int NV>
HS_DEVICE void colpart_chunked_store(float (&acc)[NV][4], float* __restrict__ part, float* lds) {
  constexpr int H = NV * 256;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    if (w > 0) store4(lds + (w - 1) * 256 + lane * 4, acc[k]);
    __syncthreads();
    if (w == 0) {
      float a[4], b[4], c[4], o[4];
      load4(lds + lane * 4, a);
      load4(lds + 256 + lane * 4, b);
      load4(lds + 512 + lane * 4, c);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (acc[k][j] + a[j]) + (b[j] + c[j]);
      store4(part + (int64_t)blockIdx.x * H + (k * 64 + lane) * 4, o);
    }
    __syncthreads();
  }
}

// 0: [WV][H] LDS reduction (12 KB at H 768); 1: the 3 KB chunked one (default) -- set_ln_bwd_lds
static int g_lnbwd_chunked = 1;

// One row per wave at a time, with the NEXT row's dy / z / statistics loaded before this row's
// reductions (two rows of loads in flight per wave); gamma is loaded once per wave.  Small
// blocks (4 waves) so the kernel still finds room on CUs that run weight-gradient GEMM blocks of
// the side stream (an 8-wave, 156-VGPR variant waited for whole GEMM blocks to drain: 3x slower
// inside the training step).
constexpr int kLnBwdWaves = 4;

template <int NV, typename T, bool CHUNK = false>
__global__ void __launch_bounds__(64 * kLnBwdWaves) ln_bwd_kernel(
    const T* __restrict__ dy, const float* __restrict__ zsave, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const float* __restrict__ gamma, T* __restrict__ dz_out, T* __restrict__ da_out,
    float* __restrict__ part_gamma, float* __restrict__ part_beta, float* __restrict__ part_bias, int rows, float p,
    uint64_t seed, uint64_t off, int mode, const uint64_t* __restrict__ seed_dev,
    float* __restrict__ amax_out) {
  constexpr int H = NV * 256;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63;
  uint32_t am = 0u;  // |max| of da (mode kBDR) or dz (kPlain): the next fp16-split GEMM's operand scale
  const float scale = p < 1.f ? 1.0f / (1.0f - p) : 0.f;
  seed = resolve_seed(seed, seed_dev);
  float ag[NV][4], ab[NV][4], abias[NV][4], gw[NV][4];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    load4(gamma + (k * 64 + lane) * 4, gw[k]);
#pragma unroll
    for (int j = 0; j < 4; ++j) ag[k][j] = ab[k][j] = abias[k][j] = 0.f;
  }
  const int stride = gridDim.x * kLnBwdWaves;
  int row = blockIdx.x * kLnBwdWaves + (threadIdx.x >> 6);
  float d[NV][4], z[NV][4], mean = 0.f, rstd = 0.f;
  auto fetch = [&](int r, float (&dd)[NV][4], float (&zz)[NV][4], float& mu, float& rs) {
    const int64_t base = (int64_t)r * H;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      load4(dy + base + (k * 64 + lane) * 4, dd[k]);
      load4(zsave + base + (k * 64 + lane) * 4, zz[k]);
    }
    mu = mean_in[r];
    rs = rstd_in[r];
  };
  if (row < rows) fetch(row, d, z, mean, rstd);
  while (row < rows) {
    const int nxt = row + stride;
    float dn[NV][4], zn[NV][4], mn = 0.f, rn = 0.f;
    if (nxt < rows) fetch(nxt, dn, zn, mn, rn);
    const int64_t base = (int64_t)row * H;
    float xh[NV][4], g[NV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xh[k][j] = (z[k][j] - mean) * rstd;
        g[k][j] = d[k][j] * gw[k][j];
        ag[k][j] = fmaf(d[k][j], xh[k][j], ag[k][j]);
        ab[k][j] += d[k][j];
        s1 += g[k][j];
        s2 = fmaf(g[k][j], xh[k][j], s2);
      }
    s1 = wave_sum(s1) / H;
    s2 = wave_sum(s2) / H;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
      float dzv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) dzv[j] = rstd * (g[k][j] - s1 - xh[k][j] * s2);
      if (dz_out) store4(dz_out + base + c, dzv);
      if (mode != kBDR) {
#pragma unroll
        for (int j = 0; j < 4; ++j) am = amax_bits(am, dzv[j]);
      }
      if (mode == kBDR) {
        float m[4] = {1.f, 1.f, 1.f, 1.f};
        if (p > 0.f) keep4(seed, off, (uint64_t)(base + c) >> 2, p, scale, m);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          dzv[j] *= m[j];
          abias[k][j] += dzv[j];
          am = amax_bits(am, dzv[j]);
        }
        if (da_out) store4(da_out + base + c, dzv);
      }
    }
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        d[k][j] = dn[k][j];
        z[k][j] = zn[k][j];
      }
    mean = mn;
    rstd = rn;
    row = nxt;
  }
  if (amax_out) amax_commit(amax_out, am);
  if constexpr (CHUNK) {
    static_assert(kLnBwdWaves == 4, "chunked partials: 4 waves");
    __shared__ __attribute__((aligned(16))) float win[768];
    colpart_chunked_store<NV>(ag, part_gamma, win);
    colpart_chunked_store<NV>(ab, part_beta, win);
    if (mode == kBDR && part_bias) colpart_chunked_store<NV>(abias, part_bias, win);
  } else {
    block_colpart_store<NV, kLnBwdWaves>(ag, part_gamma, lds);
    block_colpart_store<NV, kLnBwdWaves>(ab, part_beta, lds);
    if (mode == kBDR && part_bias) block_colpart_store<NV, kLnBwdWaves>(abias, part_bias, lds);
  }
}

// Column partials of an 8-wave block through a 7 KB LDS window: waves 1-7 hand wave 0 one 256-column
// chunk at a time; wave 0 sums ((w0 + w1) + (w2 + w3)) + ((w4 + w5) + (w6 + w7)) (fixed order).
template <int NV>
HS_DEVICE void colpart8_store(float (&acc)[NV][4], float* __restrict__ part, float* lds) {
  constexpr int H = NV * 256;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    if (w > 0) store4(lds + (w - 1) * 256 + lane * 4, acc[k]);
    __syncthreads();
    if (w == 0) {
      float v[7][4], o[4];
#pragma unroll
      for (int u = 0; u < 7; ++u) load4(lds + u * 256 + lane * 4, v[u]);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = ((acc[k][e] + v[0][e]) + (v[1][e] + v[2][e])) + ((v[3][e] + v[4][e]) + (v[5][e] + v[6][e]));
      store4(part + (int64_t)blockIdx.x * H + (k * 64 + lane) * 4, o);
    }
    __syncthreads();
  }
}

// LayerNorm backward writing the residual-branch gradient da (mode kBDR) as h3p planes -- the next
// data- and weight-gradient GEMMs' operand -- instead of fp32: one block = 32 rows (8 waves x 4 rows),
// block exponents as in ln_fwd_h3p_kernel.  dz (fp32) and the per-block column partials of dgamma /
// dbeta / dbias as ln_bwd_kernel (same per-row arithmetic; partials over 32-row blocks).
template <int NV>
__global__ void __launch_bounds__(64 * kLnH3pWaves) ln_bwd_h3p_kernel(
    const float* __restrict__ dy, const float* __restrict__ zsave, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const float* __restrict__ gamma, float* __restrict__ dz_out,
    float* __restrict__ part_gamma, float* __restrict__ part_beta, float* __restrict__ part_bias, float p, uint64_t seed,
    uint64_t off, const uint64_t* __restrict__ seed_dev, uint16_t* __restrict__ planes, int64_t ps,
    int8_t* __restrict__ exps) {
  constexpr int H = NV * 256, RPW = 32 / kLnH3pWaves;
  __shared__ __attribute__((aligned(16))) float win[7 * 256];
  __shared__ float red[kLnH3pWaves][NV * 8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float scale = p < 1.f ? 1.0f / (1.0f - p) : 0.f;
  seed = resolve_seed(seed, seed_dev);
  float ag[NV][4], ab[NV][4], abias[NV][4], gw[NV][4], da[RPW][NV][4];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    load4(gamma + (k * 64 + lane) * 4, gw[k]);
#pragma unroll
    for (int e = 0; e < 4; ++e) ag[k][e] = ab[k][e] = abias[k][e] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    const int row = blockIdx.x * 32 + w * RPW + j;
    const int64_t base = (int64_t)row * H;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float d[NV][4], xh[NV][4], g[NV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      float z[4];
      load4(dy + base + (k * 64 + lane) * 4, d[k]);
      load4(zsave + base + (k * 64 + lane) * 4, z);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xh[k][e] = (z[e] - mean) * rstd;
        g[k][e] = d[k][e] * gw[k][e];
        ag[k][e] = fmaf(d[k][e], xh[k][e], ag[k][e]);
        ab[k][e] += d[k][e];
        s1 += g[k][e];
        s2 = fmaf(g[k][e], xh[k][e], s2);
      }
    }
    s1 = wave_sum(s1) / H;
    s2 = wave_sum(s2) / H;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
      float dzv[4], m[4] = {1.f, 1.f, 1.f, 1.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) dzv[e] = rstd * (g[k][e] - s1 - xh[k][e] * s2);
      store4(dz_out + base + c, dzv);
      if (p > 0.f) keep4(seed, off, (uint64_t)(base + c) >> 2, p, scale, m);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        da[j][k][e] = dzv[e] * m[e];
        abias[k][e] += da[j][k][e];
      }
    }
  }
  uint32_t gm[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    gm[k] = 0u;
#pragma unroll
    for (int j = 0; j < RPW; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) gm[k] = amax_bits(gm[k], da[j][k][e]);
#pragma unroll
    for (int sh = 1; sh < 8; sh <<= 1)
      gm[k] = max(gm[k], static_cast<uint32_t>(__shfl_xor(static_cast<int>(gm[k]), sh, 64)));
    if ((lane & 7) == 0) red[w][k * 8 + (lane >> 3)] = __uint_as_float(gm[k]);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    uint32_t m = 0u;
#pragma unroll
    for (int v = 0; v < kLnH3pWaves; ++v) m = max(m, __float_as_uint(red[v][k * 8 + (lane >> 3)]));
    const int e = h3p_exp_bits(m);
    const float sc = h3p_scale(e);
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int row = blockIdx.x * 32 + w * RPW + j;
      h3p_store4(planes, ps, h3p_index(row, (k * 64 + lane) * 4, H, 1), da[j][k], sc);  // blocked planes
    }
    if (w == 0 && (lane & 7) == 0) exps[(int64_t)blockIdx.x * (H / 32) + k * 8 + (lane >> 3)] = static_cast<int8_t>(e);
  }
  colpart8_store<NV>(ag, part_gamma, win);
  colpart8_store<NV>(ab, part_beta, win);
  colpart8_store<NV>(abias, part_bias, win);
}

// The same backward on 4-wave workgroups of 4 RPW rows (the forward's panel exchange for the da
// exponents): a 4096-row call is 512 workgroups instead of 128.  Column partials per WORKGROUP
// (part[rows / (4 RPW)][H], ln_bwd_h3p_part_rows) through the 3 KB chunked window.
template <int NV, int RPW>
__global__ void __launch_bounds__(256) ln_bwd_h3p_coop_kernel(
    const float* __restrict__ dy, const float* __restrict__ zsave, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const float* __restrict__ gamma, float* __restrict__ dz_out,
    float* __restrict__ part_gamma, float* __restrict__ part_beta, float* __restrict__ part_bias, float p, uint64_t seed,
    uint64_t off, const uint64_t* __restrict__ seed_dev, uint16_t* __restrict__ planes, int64_t ps,
    int8_t* __restrict__ exps, uint32_t* __restrict__ psync) {
  constexpr int H = NV * 256, NG = H / 32, RB = 4 * RPW, NP = 32 / RB;
  __shared__ __attribute__((aligned(16))) float win[3 * 256];
  __shared__ uint32_t red[4][NG];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int panel = blockIdx.x / NP;
  uint32_t* rec = psync + (int64_t)panel * kPanelSyncWords;
  uint32_t gen = 0u;
  if (threadIdx.x == 0) gen = psync_gen(rec);
  const float scale = p < 1.f ? 1.0f / (1.0f - p) : 0.f;
  seed = resolve_seed(seed, seed_dev);
  float ag[NV][4], ab[NV][4], abias[NV][4], gw[NV][4], da[RPW][NV][4];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    load4(gamma + (k * 64 + lane) * 4, gw[k]);
#pragma unroll
    for (int e = 0; e < 4; ++e) ag[k][e] = ab[k][e] = abias[k][e] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    const int row = blockIdx.x * RB + w * RPW + j;
    const int64_t base = (int64_t)row * H;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float d[NV][4], xh[NV][4], g[NV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      float z[4];
      load4(dy + base + (k * 64 + lane) * 4, d[k]);
      load4(zsave + base + (k * 64 + lane) * 4, z);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xh[k][e] = (z[e] - mean) * rstd;
        g[k][e] = d[k][e] * gw[k][e];
        ag[k][e] = fmaf(d[k][e], xh[k][e], ag[k][e]);
        ab[k][e] += d[k][e];
        s1 += g[k][e];
        s2 = fmaf(g[k][e], xh[k][e], s2);
      }
    }
    s1 = wave_sum(s1) / H;
    s2 = wave_sum(s2) / H;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
      float dzv[4], m[4] = {1.f, 1.f, 1.f, 1.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) dzv[e] = rstd * (g[k][e] - s1 - xh[k][e] * s2);
      store4(dz_out + base + c, dzv);
      if (p > 0.f) keep4(seed, off, (uint64_t)(base + c) >> 2, p, scale, m);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        da[j][k][e] = dzv[e] * m[e];
        abias[k][e] += da[j][k][e];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    uint32_t gm = 0u;
#pragma unroll
    for (int j = 0; j < RPW; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) gm = amax_bits(gm, da[j][k][e]);
#pragma unroll
    for (int sh = 1; sh < 8; sh <<= 1) gm = max(gm, static_cast<uint32_t>(__shfl_xor(static_cast<int>(gm), sh, 64)));
    if ((lane & 7) == 0) red[w][k * 8 + (lane >> 3)] = gm;
  }
  __syncthreads();
  bool last = false;
  const uint32_t g = static_cast<uint32_t>(__shfl(static_cast<int>(gen), 0, 64));
  if (w == 0) {
    uint32_t m = 0u;
    if (lane < NG) m = max(max(red[0][lane], red[1][lane]), max(red[2][lane], red[3][lane]));
    last = psync_arrive(rec, g, m, NG, NP);
  }
  // the column partials do not need the exponents: they cover the rest of the panel's arrivals
  colpart_chunked_store<NV>(ag, part_gamma, win);
  colpart_chunked_store<NV>(ab, part_beta, win);
  colpart_chunked_store<NV>(abias, part_bias, win);
  if (w == 0) {
    const uint32_t m = psync_wait(rec, g, last, NG);
    if (lane < NG) red[0][lane] = m;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int e = h3p_exp_bits(red[0][k * 8 + (lane >> 3)]);
    const float sc = h3p_scale(e);
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int row = blockIdx.x * RB + w * RPW + j;
      h3p_store4(planes, ps, h3p_index(row, (k * 64 + lane) * 4, H, 1), da[j][k], sc);  // blocked planes
    }
    if (w == 0 && (lane & 7) == 0 && (blockIdx.x % NP) == 0)
      exps[(int64_t)panel * NG + k * 8 + (lane >> 3)] = static_cast<int8_t>(e);
  }
}

// ------------------------------------------------------------ embeddings
template <int NV, typename T>
__global__ void __launch_bounds__(256) emb_fwd_kernel(const int64_t* __restrict__ ids, const int64_t* __restrict__ tt,
                                                      const float* __restrict__ wemb, const float* __restrict__ pemb,
                                                      const float* __restrict__ temb, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, T* __restrict__ y,
                                                      float* __restrict__ zsave, float* __restrict__ mean_out,
                                                      float* __restrict__ rstd_out, int rows, int S, int V, int TV,
                                                      float eps, float p, uint64_t seed, uint64_t off,
                                                      int* __restrict__ err, const uint64_t* __restrict__ seed_dev,
                                                      float* __restrict__ amax_y) {
  constexpr int H = NV * 256;
  const int lane = threadIdx.x & 63;
  const float scale = p < 1.f ? 1.0f / (1.0f - p) : 0.f;
  seed = resolve_seed(seed, seed_dev);
  uint32_t am = 0u;  // |max| of y (the first layer's fp16-split GEMM operand scale)
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += gridDim.x * 4) {
    const int64_t base = (int64_t)row * H;
    int64_t id = ids[row];
    int64_t t = tt ? tt[row] : 0;
    if (id < 0 || id >= V || t < 0 || t >= TV) {  // never read out of bounds; flag it
      if (lane == 0) atomicOr(err, 1);
      id = id < 0 ? 0 : (id >= V ? V - 1 : id);
      t = t < 0 ? 0 : (t >= TV ? TV - 1 : t);
    }
    const int s = row % S;
    float x[NV][4];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
      float w[4], q[4], r[4];
      load4(wemb + id * H + c, w);
      load4(pemb + (int64_t)s * H + c, q);
      load4(temb + t * H + c, r);
#pragma unroll
      for (int j = 0; j < 4; ++j) x[k][j] = (w[j] + q[j]) + r[j];
      store4(zsave + base + c, x[k]);
    }
    float mean, rstd;
    row_stats<NV>(x, H, mean, rstd, eps);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
      float gw[4], gb[4], o[4], m[4] = {1.f, 1.f, 1.f, 1.f};
      load4(gamma + c, gw);
      load4(beta + c, gb);
      if (p > 0.f) keep4(seed, off, (uint64_t)(base + c) >> 2, p, scale, m);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = (gw[j] * ((x[k][j] - mean) * rstd) + gb[j]) * m[j];
        am = amax_bits(am, o[j]);
      }
      store4(y + base + c, o);
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
  if (amax_y) amax_commit(amax_y, am);
}

// Embedding LayerNorm backward: writes dx = d(word + pos + type) per row (fp32)
// and the per-block dgamma/dbeta column partials.  The scatter of dx into the
// three embedding tables is done afterwards by the deterministic sorted-segment
// reduction (segsum_rows, elementwise.hip) -- no float atomics, so the
// embedding gradients are bitwise reproducible, and 4096 x 768 x 2 contended
// atomics (~180 us) become a sort plus ~3 streaming passes.
template <int NV, typename T>
__global__ void __launch_bounds__(256) emb_bwd_kernel(const T* __restrict__ dy, const float* __restrict__ zsave,
                                                      const float* __restrict__ mean_in,
                                                      const float* __restrict__ rstd_in,
                                                      const float* __restrict__ gamma, float* __restrict__ dx_out,
                                                      float* __restrict__ part_gamma, float* __restrict__ part_beta,
                                                      const int64_t* __restrict__ tt, float* __restrict__ part_type,
                                                      int rows, float p, uint64_t seed, uint64_t off,
                                                      const uint64_t* __restrict__ seed_dev) {
  constexpr int H = NV * 256;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63;
  const float scale = p < 1.f ? 1.0f / (1.0f - p) : 0.f;
  seed = resolve_seed(seed, seed_dev);
  float ag[NV][4], ab[NV][4], at0[NV][4], at1[NV][4];
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) ag[k][j] = ab[k][j] = at0[k][j] = at1[k][j] = 0.f;
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += gridDim.x * 4) {
    const int64_t base = (int64_t)row * H;
    const float mean = mean_in[row], rstd = rstd_in[row];
    const bool type1 = tt != nullptr && tt[row] == 1;
    float xh[NV][4], g[NV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
      float d[4], z[4], gw[4], m[4] = {1.f, 1.f, 1.f, 1.f};
      load4(dy + base + c, d);
      load4(zsave + base + c, z);
      load4(gamma + c, gw);
      if (p > 0.f) keep4(seed, off, (uint64_t)(base + c) >> 2, p, scale, m);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        d[j] *= m[j];
        xh[k][j] = (z[j] - mean) * rstd;
        g[k][j] = d[j] * gw[j];
        ag[k][j] = fmaf(d[j], xh[k][j], ag[k][j]);
        ab[k][j] += d[j];
        s1 += g[k][j];
        s2 = fmaf(g[k][j], xh[k][j], s2);
      }
    }
    s1 = wave_sum(s1) / H;
    s2 = wave_sum(s2) / H;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
      float dz[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dz[j] = rstd * (g[k][j] - s1 - xh[k][j] * s2);
        if (type1) at1[k][j] += dz[j]; else at0[k][j] += dz[j];
      }
      store4(dx_out + base + c, dz);
    }
  }
  block_colpart_store<NV>(ag, part_gamma, lds);
  block_colpart_store<NV>(ab, part_beta, lds);
  if (part_type) {  // token-type gradient (<= 2 types): per-block partials [2][grid][H]
    block_colpart_store<NV>(at0, part_type, lds);
    block_colpart_store<NV>(at1, part_type + (int64_t)gridDim.x * H, lds);
  }
}

// column-partial blocks of the LN / embedding backward: 256 (4 rows per wave; 512 / 1024 blocks
// measured 25.0 / 27.0 us isolated vs 25.3, and slower in the step)
static const int kLnBwdBlocks = 256;

// the LN forwards with the slab count fixed at compile time (1, 2, 4: every load of a row in flight
// at once) -- A/B hook set_ln_fwd_ns (0 = the runtime slab loop)
static int g_ln_fwd_ns = 1;

template <int NV, typename T>
void ln_fwd_launch(const void* a, const float* bias, const void* resid, const float* gamma, const float* beta, void* y,
                   float* zsave, float* mean, float* rstd, int rows, float eps, float p, uint64_t seed, uint64_t off,
                   int mode, int nslab, int64_t slab_stride, int row0, float* amax, hipStream_t st) {
  int grid = (rows + 3) / 4;
  if (grid > 4096) grid = 4096;
#define HS_LN_FWD(NS_)                                                                                           \
  hipLaunchKernelGGL((ln_fwd_kernel<NV, T, NS_>), dim3(grid), dim3(256), 0, st, (const T*)a, bias, (const T*)resid, \
                     gamma, beta, (T*)y, zsave, mean, rstd, rows, eps, p, seed, off, mode, g_seed_dev, nslab,         \
                     slab_stride, row0, amax)
  if (g_ln_fwd_ns && nslab == 1) HS_LN_FWD(1);
  else if (g_ln_fwd_ns && nslab == 2) HS_LN_FWD(2);
  else if (g_ln_fwd_ns && nslab == 4) HS_LN_FWD(4);
  else HS_LN_FWD(0);
#undef HS_LN_FWD
}

// h3p LN backward with the panel exchange (A/B hook, set_ln_bwd_coop): 1 = 8 rows per workgroup,
// 2 = 4 rows per workgroup, 0 = the 32-row-block kernel
static int g_ln_bwd_coop = 1;

// h3p LN forward kernel (A/B hook, set_ln_h3p_waves): 1 = panel exchange, 4 rows per workgroup (default:
// a 2048-row call is 512 workgroups); 0 = panel exchange, 8 rows per workgroup; 16 / 8 = one 32-row
// workgroup of 16 / 8 waves (round 5).  Measured (round 6, tools/bench_producers.py, 2048 rows, 2 slabs):
// 15.2 / 17.6 / 19.1 / 23.3 us alone; the BERT-base step 10.60 / 10.69 / 10.82 ms (bench.py --ab).
static int g_ln_h3p_waves = 1;

template <int NV, typename T>
void ln_fwd_h3p_launch(const void* a, const float* bias, const void* resid, const float* gamma, const float* beta,
                       void* y, float* zsave, float* mean, float* rstd, int rows, float eps, float p, uint64_t seed,
                       uint64_t off, int mode, int nslab, int64_t slab_stride, int row0, float* amax, uint16_t* planes,
                       int64_t ps, int8_t* exps, uint32_t* psync, int panel0, hipStream_t st) {
  if (psync && (g_ln_h3p_waves == 0 || g_ln_h3p_waves == 1)) {
    if (g_ln_h3p_waves == 0)
      hipLaunchKernelGGL((ln_fwd_h3p_coop_kernel<NV, 2>), dim3(rows / 8), dim3(256), 0, st, (const float*)a, bias,
                         (const float*)resid, gamma, beta, (float*)y, zsave, mean, rstd, eps, p, seed, off, mode,
                         g_seed_dev, nslab, slab_stride, row0, amax, planes, ps, exps, psync, panel0);
    else if (g_ln_fwd_ns && nslab == 1)
      hipLaunchKernelGGL((ln_fwd_h3p_coop_kernel<NV, 1, 1>), dim3(rows / 4), dim3(256), 0, st, (const float*)a, bias,
                         (const float*)resid, gamma, beta, (float*)y, zsave, mean, rstd, eps, p, seed, off, mode,
                         g_seed_dev, nslab, slab_stride, row0, amax, planes, ps, exps, psync, panel0);
    else if (g_ln_fwd_ns && nslab == 2)
      hipLaunchKernelGGL((ln_fwd_h3p_coop_kernel<NV, 1, 2>), dim3(rows / 4), dim3(256), 0, st, (const float*)a, bias,
                         (const float*)resid, gamma, beta, (float*)y, zsave, mean, rstd, eps, p, seed, off, mode,
                         g_seed_dev, nslab, slab_stride, row0, amax, planes, ps, exps, psync, panel0);
    else if (g_ln_fwd_ns && nslab == 4)
      hipLaunchKernelGGL((ln_fwd_h3p_coop_kernel<NV, 1, 4>), dim3(rows / 4), dim3(256), 0, st, (const float*)a, bias,
                         (const float*)resid, gamma, beta, (float*)y, zsave, mean, rstd, eps, p, seed, off, mode,
                         g_seed_dev, nslab, slab_stride, row0, amax, planes, ps, exps, psync, panel0);
    else
      hipLaunchKernelGGL((ln_fwd_h3p_coop_kernel<NV, 1>), dim3(rows / 4), dim3(256), 0, st, (const float*)a, bias,
                         (const float*)resid, gamma, beta, (float*)y, zsave, mean, rstd, eps, p, seed, off, mode,
                         g_seed_dev, nslab, slab_stride, row0, amax, planes, ps, exps, psync, panel0);
    return;
  }
  if (g_ln_h3p_waves != 8)
    hipLaunchKernelGGL((ln_fwd_h3p_kernel<NV, T, 16>), dim3(rows / 32), dim3(64 * 16), 0, st, (const T*)a, bias,
                       (const T*)resid, gamma, beta, (T*)y, zsave, mean, rstd, eps, p, seed, off, mode, g_seed_dev, nslab,
                       slab_stride, row0, amax, planes, ps, exps);
  else
    hipLaunchKernelGGL((ln_fwd_h3p_kernel<NV, T, 8>), dim3(rows / 32), dim3(64 * 8), 0, st, (const T*)a, bias,
                       (const T*)resid, gamma, beta, (T*)y, zsave, mean, rstd, eps, p, seed, off, mode, g_seed_dev, nslab,
                       slab_stride, row0, amax, planes, ps, exps);
}

template <int NV>
void ln_bwd_h3p_launch(const float* dy, const float* zsave, const float* mean, const float* rstd, const float* gamma,
                       float* dz, float* pg, float* pb, float* pbias, int rows, float p, uint64_t seed, uint64_t off,
                       uint16_t* planes, int64_t ps, int8_t* exps, uint32_t* psync, hipStream_t st) {
  if (psync && g_ln_bwd_coop == 1) {
    hipLaunchKernelGGL((ln_bwd_h3p_coop_kernel<NV, 2>), dim3(rows / 8), dim3(256), 0, st, dy, zsave, mean, rstd, gamma,
                       dz, pg, pb, pbias, p, seed, off, g_seed_dev, planes, ps, exps, psync);
    return;
  }
  if (psync && g_ln_bwd_coop == 2) {
    hipLaunchKernelGGL((ln_bwd_h3p_coop_kernel<NV, 1>), dim3(rows / 4), dim3(256), 0, st, dy, zsave, mean, rstd, gamma,
                       dz, pg, pb, pbias, p, seed, off, g_seed_dev, planes, ps, exps, psync);
    return;
  }
  hipLaunchKernelGGL((ln_bwd_h3p_kernel<NV>), dim3(rows / 32), dim3(64 * kLnH3pWaves), 0, st, dy, zsave, mean, rstd,
                     gamma, dz, pg, pb, pbias, p, seed, off, g_seed_dev, planes, ps, exps);
}

template <int NV, typename T>
void ln_bwd_launch(const void* dy, const float* zsave, const float* mean, const float* rstd, const float* gamma,
                   void* dz, void* da, float* pg, float* pb, float* pbias, int rows, float p, uint64_t seed,
                   uint64_t off, int mode, float* amax, hipStream_t st) {
  constexpr int H = NV * 256;
  if constexpr (NV <= 3) {
    if (g_lnbwd_chunked) {
      hipLaunchKernelGGL((ln_bwd_kernel<NV, T, true>), dim3(kLnBwdBlocks), dim3(64 * kLnBwdWaves), 0, st,
                         (const T*)dy, zsave, mean, rstd, gamma, (T*)dz, (T*)da, pg, pb, pbias, rows, p, seed, off, mode,
                         g_seed_dev, amax);
      return;
    }
  }
  hipLaunchKernelGGL((ln_bwd_kernel<NV, T>), dim3(kLnBwdBlocks), dim3(64 * kLnBwdWaves), kLnBwdWaves * H * sizeof(float), st, (const T*)dy,
                     zsave, mean, rstd, gamma, (T*)dz, (T*)da, pg, pb, pbias, rows, p, seed, off, mode, g_seed_dev,
                     amax);
}

template <int NV, typename T>
void emb_fwd_launch(const int64_t* ids, const int64_t* tt, const float* w, const float* pe, const float* te,
                    const float* gamma, const float* beta, void* y, float* zsave, float* mean, float* rstd, int rows,
                    int S, int V, int TV, float eps, float p, uint64_t seed, uint64_t off, int* err, float* amax,
                    hipStream_t st) {
  int grid = (rows + 3) / 4;
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL((emb_fwd_kernel<NV, T>), dim3(grid), dim3(256), 0, st, ids, tt, w, pe, te, gamma, beta, (T*)y,
                     zsave, mean, rstd, rows, S, V, TV, eps, p, seed, off, err, g_seed_dev, amax);
}

template <int NV, typename T>
void emb_bwd_launch(const void* dy, const float* zsave, const float* mean, const float* rstd, const float* gamma,
                    float* dx, float* pg, float* pb, const int64_t* tt, float* pt, int rows, float p, uint64_t seed,
                    uint64_t off, hipStream_t st) {
  constexpr int H = NV * 256;
  hipLaunchKernelGGL((emb_bwd_kernel<NV, T>), dim3(kLnBwdBlocks), dim3(256), 4 * H * sizeof(float), st,
                     (const T*)dy, zsave, mean, rstd, gamma, dx, pg, pb, tt, pt, rows, p, seed, off, g_seed_dev);
}

}  // namespace hs

using namespace hs;

#define HS_DISPATCH_H(H, ...)                              \
  switch (H) {                                             \
    case 256: { constexpr int NV = 1; __VA_ARGS__; break; } \
    case 512: { constexpr int NV = 2; __VA_ARGS__; break; } \
    case 768: { constexpr int NV = 3; __VA_ARGS__; break; } \
    case 1024: { constexpr int NV = 4; __VA_ARGS__; break; } \
    case 1536: { constexpr int NV = 6; __VA_ARGS__; break; } \
    case 2048: { constexpr int NV = 8; __VA_ARGS__; break; } \
    default: return -1;                                    \
  }

int ln_bwd_num_blocks() { return kLnBwdBlocks; }
void set_ln_bwd_lds(int chunked) { g_lnbwd_chunked = chunked; }

int launch_ln_fwd(int dtype, const void* a, const float* bias, const void* resid, const float* gamma,
                  const float* beta, void* y, float* zsave, float* mean, float* rstd, int rows, int H, float eps,
                  float p, uint64_t seed, uint64_t off, int mode, int nslab,
                  int64_t slab_stride, int row0, float* amax, hipStream_t st) {
  if (nslab < 1 || (nslab > 1 && (dtype != 0 || slab_stride < (int64_t)rows * H || slab_stride % 4))) return -1;
  if (dtype == 0) {
    HS_DISPATCH_H(H, (ln_fwd_launch<NV, float>(a, bias, resid, gamma, beta, y, zsave, mean, rstd, rows, eps, p, seed,
                                               off, mode, nslab, slab_stride, row0, amax, st)));
  } else {
    HS_DISPATCH_H(H, (ln_fwd_launch<NV, bf16_t>(a, bias, resid, gamma, beta, y, zsave, mean, rstd, rows, eps, p, seed,
                                                off, mode, 1, 0, row0, amax, st)));
  }
  return 0;
}

void set_ln_h3p_waves(int w) { hs::g_ln_h3p_waves = w; }
void set_ln_fwd_ns(int on) { hs::g_ln_fwd_ns = on ? 1 : 0; }

// LayerNorm forward writing y also as h3p planes (fp32 only; rows a multiple of 32)
int launch_ln_fwd_h3p(const void* a, const float* bias, const void* resid, const float* gamma, const float* beta,
                      void* y, float* zsave, float* mean, float* rstd, int rows, int H, float eps, float p,
                      uint64_t seed, uint64_t off, int mode, int nslab, int64_t slab_stride, int row0, float* amax,
                      void* planes, int64_t ps, int8_t* exps, uint32_t* psync, int panel0, hipStream_t st) {
  if (rows <= 0 || rows % 32 || !planes || !exps || ps % 4 || panel0 < 0) return -1;
  if (nslab < 1 || (nslab > 1 && (slab_stride < (int64_t)rows * H || slab_stride % 4))) return -1;
  HS_DISPATCH_H(H, (ln_fwd_h3p_launch<NV, float>(a, bias, resid, gamma, beta, y, zsave, mean, rstd, rows, eps, p, seed,
                                                 off, mode, nslab, slab_stride, row0, amax, (uint16_t*)planes, ps, exps,
                                                 psync, panel0, st)));
  return 0;
}

// rows per column-partial row of launch_ln_bwd_h3p with a panel record (32 without)
int ln_bwd_h3p_part_rows(int coop) { return !coop || !g_ln_bwd_coop ? 32 : g_ln_bwd_coop == 2 ? 4 : 8; }
void set_ln_bwd_coop(int on) { g_ln_bwd_coop = on; }

// LayerNorm backward (bias-dropout-residual mode, fp32) writing da as h3p planes; partials are
// [rows / ln_bwd_h3p_part_rows(psync != 0)][H].  psync: panel records of the call's rows / 32 panels
int launch_ln_bwd_h3p(const float* dy, const float* zsave, const float* mean, const float* rstd, const float* gamma,
                      float* dz, float* pg, float* pb, float* pbias, int rows, int H, float p, uint64_t seed,
                      uint64_t off, void* planes, int64_t ps, int8_t* exps, uint32_t* psync, hipStream_t st) {
  if (rows <= 0 || rows % 32 || !planes || !exps || !dz || ps % 4) return -1;
  HS_DISPATCH_H(H, (ln_bwd_h3p_launch<NV>(dy, zsave, mean, rstd, gamma, dz, pg, pb, pbias, rows, p, seed, off,
                                          (uint16_t*)planes, ps, exps, psync, st)));
  return 0;
}

int launch_ln_bwd(int dtype, const void* dy, const float* zsave, const float* mean, const float* rstd,
                  const float* gamma, void* dz, void* da, float* pg, float* pb, float* pbias, int rows, int H, float p,
                  uint64_t seed, uint64_t off, int mode, float* amax, hipStream_t st) {
  if (dtype == 0) {
    HS_DISPATCH_H(H, (ln_bwd_launch<NV, float>(dy, zsave, mean, rstd, gamma, dz, da, pg, pb, pbias, rows, p, seed, off,
                                               mode, amax, st)));
  } else {
    HS_DISPATCH_H(H, (ln_bwd_launch<NV, bf16_t>(dy, zsave, mean, rstd, gamma, dz, da, pg, pb, pbias, rows, p, seed,
                                                off, mode, amax, st)));
  }
  return 0;
}

int launch_emb_fwd(int dtype, const int64_t* ids, const int64_t* tt, const float* w, const float* pe, const float* te,
                   const float* gamma, const float* beta, void* y, float* zsave, float* mean, float* rstd, int rows,
                   int S, int H, int V, int TV, float eps, float p, uint64_t seed, uint64_t off, int* err,
                   float* amax, hipStream_t st) {
  if (dtype == 0) {
    HS_DISPATCH_H(H, (emb_fwd_launch<NV, float>(ids, tt, w, pe, te, gamma, beta, y, zsave, mean, rstd, rows, S, V, TV,
                                                eps, p, seed, off, err, amax, st)));
  } else {
    HS_DISPATCH_H(H, (emb_fwd_launch<NV, bf16_t>(ids, tt, w, pe, te, gamma, beta, y, zsave, mean, rstd, rows, S, V,
                                                 TV, eps, p, seed, off, err, amax, st)));
  }
  return 0;
}

int launch_emb_bwd(int dtype, const void* dy, const float* zsave, const float* mean, const float* rstd,
                   const float* gamma, float* dx, float* pg, float* pb, const int64_t* tt, float* pt, int rows, int H,
                   float p, uint64_t seed, uint64_t off, hipStream_t st) {
  if (dtype == 0) {
    HS_DISPATCH_H(H, (emb_bwd_launch<NV, float>(dy, zsave, mean, rstd, gamma, dx, pg, pb, tt, pt, rows, p, seed, off,
                                                st)));
  } else {
    HS_DISPATCH_H(H, (emb_bwd_launch<NV, bf16_t>(dy, zsave, mean, rstd, gamma, dx, pg, pb, tt, pt, rows, p, seed, off,
                                                 st)));
  }
  return 0;
}

void launch_colpart_finalize(const float* const* parts, float* const* outs, int n, int nparts, int H, int accumulate,
                             hipStream_t st) {
  launch_reduce_rows(parts, outs, n, nparts, H, accumulate, st);
}
