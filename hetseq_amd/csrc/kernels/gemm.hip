// LDS-tiled fp32 MFMA GEMM with fused BERT epilogues (K01/K03/K04 GEMM part).
//
//   C[M,N] = beta*C + op(A)[M,K] * op(B)[K,N]  (+ epilogue)
// row-major operands; op(A) = A (TA=0, A is [M,K]) or A^T (TA=1, A is [K,M]);
// op(B) = B (TB=0, B is [K,N]) or B^T (TB=1, B is [N,K]).  The three BERT
// Linear products are forward X*W^T (0,1), dgrad dY*W (0,0), wgrad dY^T*X (1,0).
//
// Epilogues (reference bert_modeling.py:104-111,166-172):
//   kEpiNone  : C = acc (+ beta*C)
//   kEpiBias  : C = acc + bias (+ beta*C)
//   kEpiGelu  : aux = acc ; C = gelu(acc + bias)        (FFN-in forward: the
//               pre-activation is kept for the backward, no separate GELU pass)
//   kEpiDGelu : C = acc * gelu'(aux + bias) ; per-block column sums of C
//               (FFN-out dgrad fused with the GELU backward and the FFN-in
//               bias gradient; partials finalised by reduce_rows)
//
// fp32 path (the reference trains in fp32): v_mfma_f32_32x32x2_f32, exact
// fp32 products.  256 threads = 2x2 waves, block tile BM x BN, BK = 32, each
// wave (BM/2)x(BN/2) = TM x TN MFMA tiles of 32x32.  Operand images in LDS:
//   * k-contiguous source (A for TA=0, B for TB=1): [mn][k], 36-float rows;
//     a lane's 4 k-values for 4 consecutive MFMAs are one conflict-free
//     ds_read_b128 (k order inside a k-group: k = 8g + 4*half + j, identical
//     for both operands, so the products pair up correctly);
//   * mn-contiguous source (TA=1 / TB=0): [k][mn], (BMN+32)-float rows, one
//     conflict-free ds_read_b32 per MFMA operand (no transpose on the way in).
// Global loads are 16-B and fully coalesced in both cases, prefetched into
// registers one K tile ahead (write-late into the other LDS buffer, one
// barrier per K tile).  Block ids are remapped so each XCD (private L2) gets a
// contiguous range of output tiles (bijective swizzle, any grid size).
//
// The launcher only serves shapes that tile exactly (M % BM, N % BN, K % 32,
// 16-B aligned operands); anything else returns -1 and the caller uses the
// library GEMM.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "reduce.h"

namespace hs {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

enum { kEpiNone = 0, kEpiBias = 1, kEpiGelu = 2, kEpiDGelu = 3 };
constexpr int GBK = 32;

// The two exact-fp32 MFMA shapes.  Lane l holds row (l % MF) of an operand
// tile and the k-slice q = l / MF; C register r sits at row Mf::row(r, q),
// column l % MF.
template <int MF>
struct Mf;
template <>
struct Mf<32> {  // v_mfma_f32_32x32x2_f32: 64-cycle issue, 16 accumulators
  using acc_t = f32x16;
  static constexpr int nreg = 16;
  HS_DEVICE static acc_t mma(float a, float b, acc_t c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0); }
  HS_DEVICE static int row(int r, int q) { return (r & 3) + 8 * (r >> 2) + 4 * q; }
};
template <>
struct Mf<16> {  // v_mfma_f32_16x16x4_f32: 32-cycle issue, 4 accumulators
  using acc_t = f32x4;
  static constexpr int nreg = 4;
  HS_DEVICE static acc_t mma(float a, float b, acc_t c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
  HS_DEVICE static int row(int r, int q) { return 4 * q + r; }
};

struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  float* aux;   // kEpiGelu: pre-activation out; kEpiDGelu: pre-activation in
  float* part;  // kEpiDGelu: [M/BM][N] column partial sums
  int64_t lda, ldb, ldc, ldaux;
  int M, N, K;
  float beta;
  int ksplit;   // >1: K is cut into ksplit slices, each writes a plain slab (no epilogue)
  float* slab;  // [ksplit][M][N] partial products (summed by splitk_reduce_kernel)
  // valid extents (EDGE launches only, else = M, N, K): the padded problem is M x N x K; operand
  // rows past them read as zeros, C rows past Mv are not written, bias past Nv reads as zero
  int Mv, Nv, Kv;
  int slice_major;  // split-K block order: 1 = all tiles of slice 0, then slice 1, ... (else tile-major)
  // fp16 two-term split (NT == 4): per-tensor |max| of op(A) / op(B) as na / nb adjacent slots each
  // (common.h kAmaxShards; e.g. one slot per half-batch producer); the kernel scales each operand by
  // a power of two from them
  const float* amax_a;
  const float* amax_b;
  int namax_a, namax_b;
  float* amax_c;  // GELU / dGELU epilogues: |max| of the written C (atomic max), the next product's operand
};

// LDS image geometry of one operand (rows = BM or BN).  The [k][mn] image is
// padded so the NQ = 64/MF lane groups (k rows 4 apart) hit disjoint banks.
template <int ROWS, bool KCONTIG, int MF>
struct Img {
  static constexpr int ld = KCONTIG ? GBK + 4 : ROWS + (MF == 32 ? 8 : 4);  // floats per LDS row
  static constexpr int size = KCONTIG ? ROWS * ld : GBK * ld;             // floats per buffer
  static constexpr int nld = ROWS * GBK / 4 / 256;                        // float4 loads per thread
};

// Global -> registers: the [ROWS x 32] (or [32 x ROWS]) tile at (r0, k0).
template <int ROWS, bool KCONTIG>
HS_DEVICE void g_load(const float* __restrict__ X, int64_t ldx, int r0, int k0, float4 (&r)[ROWS * GBK / 1024]) {
#pragma unroll
  for (int i = 0; i < ROWS * GBK / 1024; ++i) {
    const int u = threadIdx.x + 256 * i;
    if (KCONTIG) {  // X[row][k]: 8 lanes per 128-B row segment
      const int row = u >> 3, k4 = (u & 7) * 4;
      r[i] = *reinterpret_cast<const float4*>(X + (int64_t)(r0 + row) * ldx + k0 + k4);
    } else {  // X[k][row]
      const int k = u / (ROWS / 4), c4 = (u % (ROWS / 4)) * 4;
      r[i] = *reinterpret_cast<const float4*>(X + (int64_t)(k0 + k) * ldx + r0 + c4);
    }
  }
}

template <int ROWS, bool KCONTIG, int MF>
HS_DEVICE void s_store(float* __restrict__ S, const float4 (&r)[ROWS * GBK / 1024]) {
  using I = Img<ROWS, KCONTIG, MF>;
#pragma unroll
  for (int i = 0; i < I::nld; ++i) {
    const int u = threadIdx.x + 256 * i;
    if (KCONTIG) {
      const int row = u >> 3, k4 = (u & 7) * 4;
      *reinterpret_cast<float4*>(S + row * I::ld + k4) = r[i];
    } else {
      const int k = u / (ROWS / 4), c4 = (u % (ROWS / 4)) * 4;
      *reinterpret_cast<float4*>(S + k * I::ld + c4) = r[i];
    }
  }
}

// MFMA operand values of k-group g (KG = 4 * 64/MF k values) for the wave's MF-row
// tile starting at `row`: v[s] = X[row + lr][k = KG*g + 4*q + s], s = 0..3.  The
// same k map is used for both operands, so the products pair up correctly.
template <int ROWS, bool KCONTIG, int MF>
HS_DEVICE float4 frag(const float* __restrict__ S, int row, int g, int lr, int q) {
  using I = Img<ROWS, KCONTIG, MF>;
  constexpr int KG = 4 * (64 / MF);
  if (KCONTIG) return *reinterpret_cast<const float4*>(S + (row + lr) * I::ld + KG * g + 4 * q);
  const float* b = S + (KG * g + 4 * q) * I::ld + row + lr;
  return make_float4(b[0], b[I::ld], b[2 * I::ld], b[3 * I::ld]);
}

HS_DEVICE float comp(const float4& v, int s) { return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w; }

// ---------------------------------------------------------------------------
// fp32 products on the bf16 matrix cores.  CDNA4 runs v_mfma_f32_32x32x2_f32 at
// 1/16 of the bf16 rate (64 vs 1024 FLOP/clk/SIMD) and has no xf32, so an fp32
// operand x is split (round-to-nearest-even each time) into three bf16 terms
//   x = hi + mid + lo + r,   |r| <= 2^-27 |x|
// and a*b is summed from the 6 cross products of order <= 2^-16 (hi*hi, hi*mid,
// mid*hi, hi*lo, lo*hi, mid*mid; the dropped mid*lo, lo*mid, lo*lo are
// <= 2^-24 |a b|, the size of one fp32 rounding).  Every bf16 x bf16 product is
// exact in the fp32 accumulator, so the result carries fp32-level error
// (tests/test_kernels_gpu.py::test_gemm_x6_error_matches_fp32 measures it against fp64 next to the exact-fp32
// MFMA kernel) at 6/16 of the f32 MFMA's cycles.  (A two-term NT = 3 benchmarking variant, ~2^-16
// relative, was retired in round 6.)
typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bfx2 __attribute__((ext_vector_type(2)));
typedef float fx2 __attribute__((ext_vector_type(2)));

HS_DEVICE void split4(float4 x, uint2& hi, uint2& mi, uint2& lo) {
  const fx2 x0 = {x.x, x.y}, x1 = {x.z, x.w};
  const bfx2 h0 = __builtin_convertvector(x0, bfx2), h1 = __builtin_convertvector(x1, bfx2);
  const fx2 r0 = x0 - __builtin_convertvector(h0, fx2), r1 = x1 - __builtin_convertvector(h1, fx2);
  const bfx2 m0 = __builtin_convertvector(r0, bfx2), m1 = __builtin_convertvector(r1, bfx2);
  hi = make_uint2(__builtin_bit_cast(uint32_t, h0), __builtin_bit_cast(uint32_t, h1));
  mi = make_uint2(__builtin_bit_cast(uint32_t, m0), __builtin_bit_cast(uint32_t, m1));
  const bfx2 l0 = __builtin_convertvector(r0 - __builtin_convertvector(m0, fx2), bfx2);
  const bfx2 l1 = __builtin_convertvector(r1 - __builtin_convertvector(m1, fx2), bfx2);
  lo = make_uint2(__builtin_bit_cast(uint32_t, l0), __builtin_bit_cast(uint32_t, l1));
}

HS_DEVICE f32x16 mma_bf(bfx8 a, bfx8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0); }

// ---------------------------------------------------------------------------
// fp32 products as THREE fp16 products (NT == 4, "h3").  fp16 carries 11 significant bits against
// bf16's 8, so two terms hold 22 of fp32's 24:  s*x = hi + lo + r,  |r| <= 2^-22 |s*x|,  and
//   s_a s_b a*b = hi_a hi_b + hi_a lo_b + lo_a hi_b   (dropped: lo_a lo_b ~ 2^-22 |ab|)
// -- half the MFMA work of the six-term bf16 split (NT == 6).  fp16's range is what the per-tensor
// scale s (a power of two, exact) is for: s = 2^(14 - e) with 2^e <= amax < 2^(e+1) maps the
// operand's largest |x| into [2^14, 2^15) (no overflow; 65504 is fp16's largest) and keeps every
// element down to 2^-18 amax at the full 22 bits (below that lo is subnormal: absolute error
// <= 2^-25 / s = 2^-39 amax).  Per-element representation error is random in sign, so over a
// K-long dot product it grows as sqrt(K) x 2^-22 |a||b| -- under the fp32 accumulation's own
// rounding for K >= ~64 (tests/test_kernels_gpu.py::test_gemm_h3_error_matches_fp32 measures both
// against fp64).  Every fp16 x fp16 product is exact in the fp32 accumulator.
typedef _Float16 hx2 __attribute__((ext_vector_type(2)));
typedef _Float16 hx8 __attribute__((ext_vector_type(8)));

HS_DEVICE int h16_exp(const float* am, int nslots) {
  const float m = __uint_as_float(amax_read(am, nslots));  // (a NaN partial wins)
  if (!(m > 0.f) || !(m <= 3.4028235e38f)) return 0;  // zero, NaN or inf: unscaled (NaN / inf propagate)
  return min(126, max(-126, 14 - ilogbf(m)));
}

HS_DEVICE void split4h(float4 x, float s, uint2& hi, uint2& lo) {
  const fx2 x0 = {x.x * s, x.y * s}, x1 = {x.z * s, x.w * s};  // exact: s is a power of two
  const hx2 h0 = __builtin_convertvector(x0, hx2), h1 = __builtin_convertvector(x1, hx2);
  const fx2 r0 = x0 - __builtin_convertvector(h0, fx2), r1 = x1 - __builtin_convertvector(h1, fx2);  // exact
  const hx2 l0 = __builtin_convertvector(r0, hx2), l1 = __builtin_convertvector(r1, hx2);
  hi = make_uint2(__builtin_bit_cast(uint32_t, h0), __builtin_bit_cast(uint32_t, h1));
  lo = make_uint2(__builtin_bit_cast(uint32_t, l0), __builtin_bit_cast(uint32_t, l1));
}

// the split of one float4 for engine NT: bf16 hi / mid / lo (NT 6) or fp16 hi / lo (NT 4, planes 0, 1)
template <int NT>
HS_DEVICE void split_nt(float4 x, float s, uint2& p0, uint2& p1, uint2& p2) {
  if constexpr (NT == 4) split4h(x, s, p0, p1);
  else split4(x, p0, p1, p2);
}

template <int NT>
HS_DEVICE f32x16 mma_nt(bfx8 a, bfx8 b, f32x16 c) {
  if constexpr (NT == 4)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(hx8, a), __builtin_bit_cast(hx8, b), c, 0, 0, 0);
  else
    return mma_bf(a, b, c);
}

// (|max| of the values a lane wrote: amax_bits / amax_commit in common.h -- non-negative floats order as
// their bit patterns; NaN's pattern sorts above inf, so a NaN output reaches the consumer's scale as NaN)

// Shared GEMM epilogue (both kernels): split-K slab, or C = acc (+bias) (+beta*C) / GELU /
// dGELU + column partial sums.  acc[i][j] register r -> row m0+wm+MF*i+Mf::row(r,q), col n0+wn+MF*j+lr.
template <int BM, int BN, int MF, int EPI, bool EDGE = false>
HS_DEVICE void epilogue(const GemmArgs& p, typename Mf<MF>::acc_t (&acc)[BM / 2 / MF][BN / 2 / MF], float* smem, int m0,
                        int n0, int tm, int slice, int wm, int wn, int wr, int lr, int q) {
  using M_ = Mf<MF>;
  constexpr int TM = BM / 2 / MF, TN = BN / 2 / MF;
  if (p.ksplit > 1) {  // split-K: plain partial slab, bias / beta / sum in splitk_reduce_kernel
    float* sl = p.slab + (int64_t)slice * p.M * p.N;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < M_::nreg; ++r)
          sl[(int64_t)(m0 + wm + MF * i + M_::row(r, q)) * p.N + n0 + wn + MF * j + lr] = acc[i][j][r];
    return;
  }
  float csum[TN];
  uint32_t cmax = 0u;  // |max| of the written C as bits (GELU / dGELU epilogues, when p.amax_c is set)
  const bool use_beta = (EPI == kEpiNone || EPI == kEpiBias) && p.beta != 0.f;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    csum[j] = 0.f;
    const int n = n0 + wn + MF * j + lr;
    const float bv = (EPI != kEpiNone && (!EDGE || n < p.Nv)) ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int mb = m0 + wm + MF * i;
      if (EPI == kEpiGelu) {
#pragma unroll
        for (int r = 0; r < M_::nreg; ++r) {
          const int64_t m = mb + M_::row(r, q);
          p.aux[m * p.ldaux + n] = acc[i][j][r];
          const float y = gelu_f(acc[i][j][r] + bv);
          cmax = amax_bits(cmax, y);
          p.C[m * p.ldc + n] = y;
        }
      } else if (EPI == kEpiDGelu) {
        float pre[M_::nreg];
#pragma unroll
        for (int r = 0; r < M_::nreg; ++r) pre[r] = p.aux[(int64_t)(mb + M_::row(r, q)) * p.ldaux + n];
#pragma unroll
        for (int r = 0; r < M_::nreg; ++r) {
          const float v = acc[i][j][r] * gelu_grad_f(pre[r] + bv);
          csum[j] += v;
          cmax = amax_bits(cmax, v);
          p.C[(int64_t)(mb + M_::row(r, q)) * p.ldc + n] = v;
        }
      } else if (use_beta) {
        float old[M_::nreg];
#pragma unroll
        for (int r = 0; r < M_::nreg; ++r)
          old[r] = (!EDGE || mb + M_::row(r, q) < p.Mv) ? p.C[(int64_t)(mb + M_::row(r, q)) * p.ldc + n] : 0.f;
#pragma unroll
        for (int r = 0; r < M_::nreg; ++r)
          if (!EDGE || mb + M_::row(r, q) < p.Mv)
            p.C[(int64_t)(mb + M_::row(r, q)) * p.ldc + n] = acc[i][j][r] + bv + p.beta * old[r];
      } else {
#pragma unroll
        for (int r = 0; r < M_::nreg; ++r)
          if (!EDGE || mb + M_::row(r, q) < p.Mv) p.C[(int64_t)(mb + M_::row(r, q)) * p.ldc + n] = acc[i][j][r] + bv;
      }
    }
  }
  if ((EPI == kEpiGelu || EPI == kEpiDGelu) && p.amax_c) amax_commit(p.amax_c, cmax);
  if (EPI == kEpiDGelu && p.part) {  // (no part: the bias gradient is summed elsewhere)
    // column sums over the block's BM rows: lane groups, then the two wave rows via LDS
    float* red = smem;  // [BN] floats; the K loop ended with a barrier
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      csum[j] += __shfl_xor(csum[j], 32, 64);
      if (MF == 16) csum[j] += __shfl_xor(csum[j], 16, 64);
    }
    if (wr == 1 && q == 0)
#pragma unroll
      for (int j = 0; j < TN; ++j) red[wn + MF * j + lr] = csum[j];
    __syncthreads();
    if (wr == 0 && q == 0)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int c = wn + MF * j + lr;
        p.part[(int64_t)tm * p.N + n0 + c] = csum[j] + red[c];
      }
  }
}

template <int BM, int BN, int MF, bool TA, bool TB, int EPI>
__global__ void __launch_bounds__(256, 2) gemm_f32_kernel(GemmArgs p) {
  using IA = Img<BM, !TA, MF>;
  using IB = Img<BN, TB, MF>;
  using M_ = Mf<MF>;
  constexpr int TM = BM / 2 / MF, TN = BN / 2 / MF, NQ = 64 / MF, KG = 4 * NQ;
  __shared__ __attribute__((aligned(16))) float smem[2 * (IA::size + IB::size)];
  float* const As0 = smem;                 // A buffers at [0, 2*IA::size)
  float* const Bs0 = smem + 2 * IA::size;  // B buffers after them

  const int tiles_m = p.M / BM, tiles_n = p.N / BN, nwg = tiles_m * tiles_n * p.ksplit;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, qq = nwg / 8, rr = nwg % 8;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
  // the K slices of one tile sit next to each other (same XCD); M fastest: neighbours share the B panel
  const int slice = wg % p.ksplit, tile = wg / p.ksplit;
  const int tm = tile % tiles_m, tn = tile / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kofs = slice * (p.K / p.ksplit);

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int wm = wr * (BM / 2), wn = wc * (BN / 2);
  const int lr = lane % MF, q = lane / MF;

  typename M_::acc_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = typename M_::acc_t{};

  float4 ra[IA::nld], rb[IB::nld];
  const int KT = p.K / p.ksplit / GBK;
  g_load<BM, !TA>(p.A, p.lda, m0, kofs, ra);
  g_load<BN, TB>(p.B, p.ldb, n0, kofs, rb);
  s_store<BM, !TA, MF>(As0, ra);
  s_store<BN, TB, MF>(Bs0, rb);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    // prefetch the next K tile (the last iteration re-reads the final tile into the idle
    // buffer: keeps the staging registers unconditional, so they stay in VGPRs)
    const int kn = kofs + (kt + 1 < KT ? kt + 1 : kt) * GBK;
    g_load<BM, !TA>(p.A, p.lda, m0, kn, ra);
    g_load<BN, TB>(p.B, p.ldb, n0, kn, rb);
    const float* as = As0 + cur * IA::size;
    const float* bs = Bs0 + cur * IB::size;
#pragma unroll
    for (int g = 0; g < GBK / KG; ++g) {
      float4 av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = frag<BM, !TA, MF>(as, wm + MF * i, g, lr, q);
#pragma unroll
      for (int j = 0; j < TN; ++j) bv[j] = frag<BN, TB, MF>(bs, wn + MF * j, g, lr, q);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = M_::mma(comp(av[i], s), comp(bv[j], s), acc[i][j]);
    }
    // the other buffer was last read before the previous barrier
    s_store<BM, !TA, MF>(As0 + (cur ^ 1) * IA::size, ra);
    s_store<BN, TB, MF>(Bs0 + (cur ^ 1) * IB::size, rb);
    __syncthreads();
  }

  epilogue<BM, BN, MF, EPI>(p, acc, smem, m0, n0, tm, slice, wm, wn, wr, lr, q);
}

// ---------------------------------------------------------------------------
// Split-bf16 kernel: 128x128 block tile, 4 waves (2x2, 64x64 each = 2x2 MFMA
// tiles of 32x32x16), BK = 32.  The fp32 tile of each operand is split ONCE per
// block while it is staged: each thread loads a 4(mn) x 4(k) micro-block (16-B
// global loads, coalesced for either operand layout; the mn-contiguous case is
// transposed in registers), splits it and writes three 8-B bf16 quads per row
// into a k-contiguous LDS image
//   row r (208 B): [hi k0..31 | mid k0..31 | lo k0..31 | 16 B pad]
// so every MFMA fragment (8 consecutive k of one plane) is one ds_read_b128.
// The 16-B k-chunks of the images staged from mn-contiguous sources are
// XOR-swizzled by (r ^ r>>3) & 3: 2-way instead of 8-way bank conflicts on the
// transposing ds_write_b64 for 2-way on the reads; k-contiguous sources need no
// swizzle (conflict-free both ways; tools/lds_banks.py checks all four cases).
// One LDS buffer (53 KB) + a register prefetch of the next K tile: two barriers
// per K tile, two blocks per CU, so one block's staging overlaps the other's MFMAs.
constexpr int XROW = 208;  // bytes per LDS image row
// rows of the two-plane engines (NT 3, 4) drop the unused third plane: 144 B = 9 x 16 B, still an
// odd number of 16-B slots, so the fragment reads stay conflict-free (tools/lds_banks.py) and a
// block's two images take 36 KB instead of 53 KB
template <int NT>
constexpr int xrow() { return NT >= 6 ? XROW : 144; }

template <bool SWZ>
HS_DEVICE int xchunk(int r, int kc) { return SWZ ? kc ^ ((r ^ (r >> 3)) & 3) : kc; }

// per-thread byte offsets of the 4 rows (k-contiguous) / k rows (mn-contiguous) a thread stages;
// the K-tile base is a wave-uniform pointer, so the loads use the scalar-base addressing mode
template <bool KCONTIG>
HS_DEVICE void x_offsets(int64_t ldx, int r0, uint32_t (&o)[4], int t) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    o[i] = KCONTIG ? (uint32_t)(((int64_t)(r0 + 4 * (t >> 3) + i) * ldx + 4 * (t & 7)) * 4)
                   : (uint32_t)(((int64_t)(4 * (t >> 5) + i) * ldx + r0 + 4 * (t & 31)) * 4);
}

// lim (EDGE launches): rows of this operand tile that exist -- mn rows from the tile origin for
// k-contiguous sources, k rows from the K-tile origin for mn-contiguous ones; the rest read as 0
template <bool KCONTIG>
HS_DEVICE void x_load(const char* __restrict__ base, const uint32_t (&o)[4], float4 (&v)[4], int lim = 1 << 30) {
  const int t = threadIdx.x & 255;
  if (KCONTIG) {  // v[i] = k 4c..4c+3 of row 4g+i; 8 lanes per 128-B row segment
#pragma unroll
    for (int i = 0; i < 4; ++i)
      v[i] = 4 * (t >> 3) + i < lim ? *reinterpret_cast<const float4*>(base + o[i]) : make_float4(0.f, 0.f, 0.f, 0.f);
  } else {  // 32 lanes per 512-B k row, then a 4x4 register transpose
    float4 w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = 4 * (t >> 5) + j < lim ? *reinterpret_cast<const float4*>(base + o[j]) : make_float4(0.f, 0.f, 0.f, 0.f);
    v[0] = make_float4(w[0].x, w[1].x, w[2].x, w[3].x);
    v[1] = make_float4(w[0].y, w[1].y, w[2].y, w[3].y);
    v[2] = make_float4(w[0].z, w[1].z, w[2].z, w[3].z);
    v[3] = make_float4(w[0].w, w[1].w, w[2].w, w[3].w);
  }
}

template <bool KCONTIG, int NT>
HS_DEVICE void x_store(char* __restrict__ S, const float4 (&v)[4], int t, float sc = 1.f) {
  const int g = KCONTIG ? t >> 3 : t & 31, c = KCONTIG ? t & 7 : t >> 5;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 4 * g + i;
    uint2 h, m, l;
    split_nt<NT>(v[i], sc, h, m, l);
    char* row = S + r * xrow<NT>() + 16 * xchunk<!KCONTIG>(r, c >> 1) + 8 * (c & 1);
    *reinterpret_cast<uint2*>(row) = h;
    *reinterpret_cast<uint2*>(row + 64) = m;
    if (NT >= 6) *reinterpret_cast<uint2*>(row + 128) = l;
  }
}

// fragment of plane p (0 hi, 1 mid, 2 lo), k-slice ks, for the 32-row tile at `row`
template <bool SWZ, int NT = 6>
HS_DEVICE bfx8 x_frag(const char* __restrict__ S, int row, int p, int ks, int lr, int h) {
  const int r = row + lr;
  return *reinterpret_cast<const bfx8*>(S + r * xrow<NT>() + 64 * p + 16 * xchunk<SWZ>(r, 2 * ks + h));
}

// Transposed-read layout ("TR", mn-contiguous sources): instead of a register 4x4 transpose into
// the k-contiguous image, the split planes are stored as read -- [k row][128 mn] bf16, 256-B rows,
// 16-B chunks XOR-swizzled by 4 (r & 3) -- and each MFMA fragment (8 consecutive k of one mn) is
// gathered by two ds_read_b64_tr_b16.  The stores are row-contiguous (16 lanes = 128 B of one k
// row: conflict-free) and the transposed reads hit 4 different bank quarters per k-row quad.
constexpr int TROW = 256;                // bytes per k row of one plane
constexpr int TIMG = 3 * GBK * TROW;     // the three planes of one operand tile: 24 KB
template <int NT>
constexpr int timg() { return (NT >= 6 ? 3 : 2) * GBK * TROW; }  // two-plane engines: 16 KB
typedef short sx4 __attribute__((ext_vector_type(4)));
typedef short sx8 __attribute__((ext_vector_type(8)));

HS_DEVICE int tr_swz(int k) { return 4 * (k & 3); }

// v[j] = mn 4g..4g+3 of k row 4c + j (g = t & 31, c = t >> 5): 32 lanes per 512-B k row
HS_DEVICE void x_load_rows(const char* __restrict__ base, const uint32_t (&o)[4], float4 (&v)[4], int lim = 1 << 30) {
  const int t = threadIdx.x & 255;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    v[j] = 4 * (t >> 5) + j < lim ? *reinterpret_cast<const float4*>(base + o[j]) : make_float4(0.f, 0.f, 0.f, 0.f);
}

template <int NT>
HS_DEVICE void x_store_tr(char* __restrict__ S, const float4 (&v)[4], int t, float sc = 1.f) {
  const int g = t & 31, c = t >> 5;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = 4 * c + j;
    uint2 h, m, l;
    split_nt<NT>(v[j], sc, h, m, l);
    char* row = S + k * TROW + 16 * ((g >> 1) ^ tr_swz(k)) + 8 * (g & 1);
    *reinterpret_cast<uint2*>(row) = h;
    *reinterpret_cast<uint2*>(row + GBK * TROW) = m;
    if (NT >= 6) *reinterpret_cast<uint2*>(row + 2 * GBK * TROW) = l;
  }
}

// fragment of plane p, k-slice ks, for the 32-wide mn tile at rc: lane 4qq + pp of a 16-lane group
// addresses k row 16 ks + 8 (g >> 1) + 4 jj + qq, mn columns rc + 16 (g & 1) + 4 pp .. + 3
HS_DEVICE bfx8 x_frag_tr(const char* __restrict__ S, int rc, int p, int ks, int lane) {
  const int l16 = lane & 15, qq = l16 >> 2, pp = l16 & 3, g = lane >> 4;
  const int col = rc + 16 * (g & 1) + 4 * pp;
  const char* pl = S + p * GBK * TROW;
  sx4 v[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int k = 16 * ks + 8 * (g >> 1) + 4 * jj + qq;
    const char* a = pl + k * TROW + 16 * ((col >> 3) ^ tr_swz(k)) + 2 * (col & 7);
    v[jj] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sx4*)(a));
  }
  const sx8 u = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
  return __builtin_bit_cast(bfx8, u);
}

// 2x2 waves of 64x64; every thread stages 4x4 of A and of B into one set of LDS images while the next
// K tile is prefetched into registers under this tile's MFMAs.  (8-wave, double-buffered and
// two-deep-prefetch variants were measured slower in the step -- profiles/r2_gemm_experiments.md --
// and retired in round 6, as were the ablation builds.)
// TRL: mn-contiguous operands in the transposed-read layout (above) instead of the register
// transpose into k-contiguous images.
// OCC > 0: waves per SIMD the register allocation targets (3 = three blocks per CU, <= 168 VGPRs)
// instead of the default two blocks per CU
template <bool TA, bool TB, int EPI, int NT, bool EDGE = false, bool TRL = false, int OCC = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC ? OCC : 2, OCC ? OCC : 2))) gemm_x6s_kernel(GemmArgs p) {
  constexpr int BM = 128, BN = 128, TM = 2, TN = 2;
  static_assert(!EDGE || EPI <= kEpiBias, "edge-masked launches: plain / bias epilogue");
  constexpr bool TRA = TRL && TA, TRB = TRL && !TB;  // operands staged in the transposed-read layout
  constexpr int IA = TRA ? timg<NT>() : 128 * xrow<NT>(), IB = TRB ? timg<NT>() : 128 * xrow<NT>();
  __shared__ __attribute__((aligned(16))) char smem[IA + IB];
  char* const As = smem;
  char* const Bs = smem + IA;

  const int tiles_m = p.M / BM, tiles_n = p.N / BN, nwg = tiles_m * tiles_n * p.ksplit;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, qq = nwg / 8, rr = nwg % 8;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
  const int ntile = tiles_m * tiles_n;
  // slice-major: an XCD's contiguous range of blocks is (mostly) one K slice over a group of tiles,
  // so its L2 holds that slice's panels once instead of every slice of a few tiles
  const int slice = p.slice_major ? wg / ntile : wg % p.ksplit, tile = p.slice_major ? wg % ntile : wg / p.ksplit;
  // grouped order: 8 M-tiles x all N-tiles per group, N fastest inside it, so the 64 blocks an
  // XCD runs at a time cover an ~8x8 tile square (A and B panels each re-read 8x from its L2)
  const int gsz = 8 * tiles_n, grp = tile / gsz, gm = min(8, tiles_m - 8 * grp);
  const int tm = 8 * grp + (tile % gsz) % gm, tn = (tile % gsz) / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kofs = slice * (p.K / p.ksplit);

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int wm = wr * (BM / 2), wn = wc * (BN / 2);
  const int lr = lane & 31, q = lane >> 5;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  // staging: 32-bit per-thread offsets + a uniform K-tile base pointer (advanced per tile)
  const int st = threadIdx.x;
  uint32_t oa[4], ob[4];
  x_offsets<!TA>(p.lda, m0, oa, st);
  x_offsets<TB>(p.ldb, n0, ob, st);
  const int64_t sa = TA ? (int64_t)GBK * p.lda * 4 : GBK * 4, sb = TB ? GBK * 4 : (int64_t)GBK * p.ldb * 4;
  const char* ab = reinterpret_cast<const char*>(p.A) + (TA ? (int64_t)kofs * p.lda : kofs) * 4;
  const char* bb = reinterpret_cast<const char*>(p.B) + (TB ? kofs : (int64_t)kofs * p.ldb) * 4;
  float4 va[4], vb[4];
  int kld = kofs;  // absolute k of the tile ab / bb point at (edge guards of k-row operands)
  // per-operand staging: k-contiguous image (register transpose for mn-contiguous sources) or,
  // with TRL, the transposed-read layout
  auto ldA = [&](const char* base, float4(&v)[4], int lim = 1 << 30) {
    if (TRA) x_load_rows(base, oa, v, lim);
    else x_load<!TA>(base, oa, v, lim);
  };
  auto ldB = [&](const char* base, float4(&v)[4], int lim = 1 << 30) {
    if (TRB) x_load_rows(base, ob, v, lim);
    else x_load<TB>(base, ob, v, lim);
  };
  // fp16 split (NT == 4): power-of-two operand scales from the producers' |max| (h16_exp)
  int ea = 0, eb = 0;
  if constexpr (NT == 4) {
    ea = h16_exp(p.amax_a, p.namax_a);
    eb = h16_exp(p.amax_b, p.namax_b);
  }
  const float sca = ldexpf(1.f, ea), scb = ldexpf(1.f, eb);
  auto stoA = [&](char* S_, const float4(&v)[4]) {
    if (TRA) x_store_tr<NT>(S_, v, st, sca);
    else x_store<!TA, NT>(S_, v, st, sca);
  };
  auto stoB = [&](char* S_, const float4(&v)[4]) {
    if (TRB) x_store_tr<NT>(S_, v, st, scb);
    else x_store<TB, NT>(S_, v, st, scb);
  };
  auto load = [&]() {
    if (EDGE) {
      ldA(ab, va, TA ? p.Kv - kld : p.Mv - m0);
      ldB(bb, vb, TB ? p.Nv - n0 : p.Kv - kld);
    } else {
      ldA(ab, va);
      ldB(bb, vb);
    }
  };
  auto store = [&]() {
    stoA(As, va);
    stoB(Bs, vb);
  };
  // weight gradient with p.part (TA only, unmasked launches): the blocks of the first column tile also sum A over this slice's K -- the bias gradient
  // of the same product (QKV: db = sum over tokens of dqkv) -- from the registers they stage anyway.
  // Thread st holds columns m0 + 4 (st & 31) + e of k rows 4 (st >> 5) + 0..3 in both A layouts.
  const bool csum = TA && !EDGE && p.part != nullptr && tn == 0;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  auto acc_cols = [&]() {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a0 = TRA ? comp(va[0], e) : comp(va[e], 0), a1 = TRA ? comp(va[1], e) : comp(va[e], 1);
      const float a2 = TRA ? comp(va[2], e) : comp(va[e], 2), a3 = TRA ? comp(va[3], e) : comp(va[e], 3);
      cs[e] += (a0 + a1) + (a2 + a3);
    }
  };
  const int KT = p.K / p.ksplit / GBK;
  constexpr int NPL = NT >= 6 ? 3 : 2, NTERM = NT >= 6 ? 6 : 3;
  constexpr int PA[6] = {2, 0, 1, 1, 0, 0}, PB[6] = {0, 2, 1, 0, 1, 0};  // smallest terms first
  // one K tile of MFMA work from the LDS images: fragments of both k-slices first (one wait
  // each), then `between()` (the next global loads) so they fly under the MFMAs
  auto compute = [&](auto between, const char* Ab, const char* Bb) {
    bfx8 af[2][3][TM], bf[2][3][TN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[ks][pl][i] = TRA ? x_frag_tr(Ab, wm + 32 * i, pl, ks, lane) : x_frag<TA, NT>(Ab, wm + 32 * i, pl, ks, lr, q);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bf[ks][pl][j] = TRB ? x_frag_tr(Bb, wn + 32 * j, pl, ks, lane) : x_frag<!TB, NT>(Bb, wn + 32 * j, pl, ks, lr, q);
      }
    between();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int tt = 6 - NTERM; tt < 6; ++tt)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma_nt<NT>(af[ks][PA[tt]][i], bf[ks][PB[tt]][j], acc[i][j]);
  };
  {
    load();
    if (csum) acc_cols();
    store();
    __syncthreads();
    for (int kt = 0; kt < KT; ++kt) {
      // the last iteration re-reads its own tile: unconditional, so the registers stay static
      compute([&] {
        if (kt + 1 < KT) {
          ab += sa;
          bb += sb;
          kld += GBK;
        }
        load();
      }, As, Bs);
      __syncthreads();  // every wave is done reading this K tile
      if (csum && kt + 1 < KT) acc_cols();  // (not the re-read last tile)
      store();
      __syncthreads();
    }
    if (csum) {  // block-uniform: the 8 k-row groups' sums in a fixed order -> part[slice][m]
      float* red = reinterpret_cast<float*>(smem);
#pragma unroll
      for (int e = 0; e < 4; ++e) red[(st >> 5) * 128 + 4 * (st & 31) + e] = cs[e];
      __syncthreads();
      if (st < 128) {
        float v = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) v += red[c * 128 + st];
        p.part[(int64_t)slice * p.M + m0 + st] = v;
      }
      __syncthreads();
    }
  }
  if constexpr (NT == 4) {  // undo the operand scales (powers of two: exact unless subnormal)
    const float ia = ldexpf(1.f, -ea), ib = ldexpf(1.f, -eb);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = acc[i][j] * ia * ib;
  }
  // the epilogue's tile geometry: TM x TN 32x32 accumulators per wave, two wave rows
  epilogue<BM, 2 * 32 * TN, 32, EPI, EDGE>(p, acc, reinterpret_cast<float*>(smem), m0, n0, tm, slice, wm, wn, wr, lr,
                                           q);
}

// split-K block order of the split kernels: slice-major (BERT-base fp32 step 15.04 vs 15.13 ms
// tile-major, interleaved)
static const int g_slice_major = 1;
// mn-contiguous operands in the transposed-read layout: weight gradients 7-12 % and NN data gradients
// 3-10 % faster on the BERT shapes than the register transpose (profiles/r2_gemm_experiments.md).
// tile_override bit 8 forces it, bit 9 forces the register-transpose layout (tests).
static const int g_x6_tr_env = 1;
static int g_x6_tr = 0;
// h3 engine (NT 4) at three 4-wave blocks per CU (registers for 168 VGPRs; two planes need less LDS):
// tile_override bit 10 forces it.
// Bit mask of the product kinds (launch_occ3) that run at three blocks per CU.  Default 5 (forward and
// weight gradient): measured in the BERT-base fp32 step (interleaved A/B, 8 rounds) 12.13 ms against
// 12.35 with none; data gradients at 3 blocks lose (+0.5 ms: they share the CUs with the weight-gradient
// stream and the LN backward).  profiles/r4_h3_gemm.md.
static int g_h3_occ3_env = 5;
static int g_h3_occ3 = 0;

// split-K finish: C = sum_s slab[s] (+ bias) (+ beta * C), fixed slice order (deterministic).
// Blocks past `gmain` (weight gradient with fused column sums, wcol) finish the bias gradient in the
// same launch: colsum_out[m] (+)= sum_s part[s][m], slices in order -- no separate reduce_rows pass.
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ slab, int ksplit, int M, int N,
                                                            float* __restrict__ C, int64_t ldc,
                                                            const float* __restrict__ bias, float beta, int Mv, int Nv,
                                                            int gmain, const float* __restrict__ part,
                                                            float* __restrict__ colsum_out, int colsum_acc) {
  if ((int)blockIdx.x >= gmain) {
    const int m = ((int)blockIdx.x - gmain) * 256 + threadIdx.x;
    if (m < M) {
      float t = 0.f;
      for (int s = 0; s < ksplit; ++s) t += part[(int64_t)s * M + m];
      colsum_out[m] = colsum_acc ? colsum_out[m] + t : t;
    }
    return;
  }
  const int n4 = N / 4;
  const int64_t total = (int64_t)Mv * n4, plane = (int64_t)M * N;  // rows past Mv are padding: not written
  for (int64_t u = blockIdx.x * 256ll + threadIdx.x; u < total; u += (int64_t)gmain * 256) {
    const int m = (int)(u / n4), n = (int)(u % n4) * 4;
    const float* s0 = slab + (int64_t)m * N + n;
    float4 a = *reinterpret_cast<const float4*>(s0);
    for (int s = 1; s < ksplit; ++s) {
      const float4 b = *reinterpret_cast<const float4*>(s0 + s * plane);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    if (bias && n + 3 < Nv) {
      const float4 b = *reinterpret_cast<const float4*>(bias + n);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    } else if (bias) {  // the quad straddling the valid width (bias past Nv reads as zero)
      a.x += n < Nv ? bias[n] : 0.f;
      a.y += n + 1 < Nv ? bias[n + 1] : 0.f;
      a.z += n + 2 < Nv ? bias[n + 2] : 0.f;
      a.w += n + 3 < Nv ? bias[n + 3] : 0.f;
    }
    float4* c = reinterpret_cast<float4*>(C + (int64_t)m * ldc + n);
    if (beta != 0.f) {
      const float4 o = *c;
      a.x += beta * o.x; a.y += beta * o.y; a.z += beta * o.z; a.w += beta * o.w;
    }
    *c = a;
  }
}

// the h3 engine's three-blocks-per-CU variant (plain / bias epilogues only: the GELU epilogues spill
// 70-90 registers at 168)
template <bool TA, bool TB, int EPI, int NT>
bool launch_occ3(const GemmArgs& a, int blocks, hipStream_t st) {
  if constexpr (NT == 4 && EPI <= kEpiBias) {
    // g_h3_occ3 bit mask: 1 forward (x W^T), 2 data gradient (dY W), 4 weight gradient (dY^T X)
    if (!(g_h3_occ3 & (TA ? 4 : TB ? 1 : 2))) return false;
    if (g_x6_tr && (TA || !TB))
      hipLaunchKernelGGL((gemm_x6s_kernel<TA, TB, EPI, NT, false, true, 3>), dim3(blocks), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((gemm_x6s_kernel<TA, TB, EPI, NT, false, false, 3>), dim3(blocks), dim3(256), 0, st, a);
    return true;
  }
  return false;
}

template <int BM, int BN, int MF, bool TA, bool TB, int EPI, int NT>
void launch_cfg(const GemmArgs& a, hipStream_t st) {
  const int blocks = (a.M / BM) * (a.N / BN) * a.ksplit;
  const bool tr = g_x6_tr && (TA || !TB);
  if constexpr (NT > 0) {
    if (a.Mv != a.M || a.Nv != a.N || a.Kv != a.K) {  // padded problem (launch_gemm checked epi)
      if constexpr (EPI <= kEpiBias) {
        if (tr) hipLaunchKernelGGL((gemm_x6s_kernel<TA, TB, EPI, NT, true, true>), dim3(blocks), dim3(256), 0, st, a);
        else hipLaunchKernelGGL((gemm_x6s_kernel<TA, TB, EPI, NT, true>), dim3(blocks), dim3(256), 0, st, a);
      }
    } else if (launch_occ3<TA, TB, EPI, NT>(a, blocks, st)) {
    } else if (tr) {
      hipLaunchKernelGGL((gemm_x6s_kernel<TA, TB, EPI, NT, false, true>), dim3(blocks), dim3(256), 0, st, a);
    } else {
      hipLaunchKernelGGL((gemm_x6s_kernel<TA, TB, EPI, NT>), dim3(blocks), dim3(256), 0, st, a);
    }
  } else {
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, MF, TA, TB, EPI>), dim3(blocks), dim3(256), 0, st, a);
  }
}

template <int BM, int BN, int MF, int NT>
int launch_tile(int ta, int tb, int epi, const GemmArgs& a, hipStream_t st) {
  if (a.ksplit > 1) epi = kEpiNone;  // bias / beta are applied by the split-K reduction
  if (!ta && tb) {  // forward X * W^T
    if (epi == kEpiNone) launch_cfg<BM, BN, MF, false, true, kEpiNone, NT>(a, st);
    else if (epi == kEpiBias) launch_cfg<BM, BN, MF, false, true, kEpiBias, NT>(a, st);
    else if (epi == kEpiGelu) launch_cfg<BM, BN, MF, false, true, kEpiGelu, NT>(a, st);
    else return -1;
  } else if (!ta && !tb) {  // dgrad dY * W
    if (epi == kEpiNone) launch_cfg<BM, BN, MF, false, false, kEpiNone, NT>(a, st);
    else if (epi == kEpiDGelu) launch_cfg<BM, BN, MF, false, false, kEpiDGelu, NT>(a, st);
    else return -1;
  } else if (ta && !tb) {  // wgrad dY^T * X
    if (epi == kEpiNone) launch_cfg<BM, BN, MF, true, false, kEpiNone, NT>(a, st);
    else return -1;
  } else {
    return -1;
  }
  return 0;
}

template <int NT>
int launch_split(int tile, int ta, int tb, int epi, const GemmArgs& a, hipStream_t st) {
  if constexpr (NT > 0) return tile == 0 ? launch_tile<128, 128, 32, NT>(ta, tb, epi, a, st) : -1;
  else return tile == 0 ? launch_tile<128, 128, 32, 0>(ta, tb, epi, a, st)
         : tile == 1 ? launch_tile<128, 64, 32, 0>(ta, tb, epi, a, st)
                     : launch_tile<64, 64, 32, 0>(ta, tb, epi, a, st);
}

}  // namespace hs

using namespace hs;

static void launch_splitk_reduce_cols(const float* slab, int ksplit, int M, int N, float* C, int64_t ldc,
                                      const float* bias, float beta, int Mv, int Nv, hipStream_t st, const float* part,
                                      float* colsum_out, int colsum_acc) {
  if (g_hs_skip & kSkipSplitK) return;
  const int64_t n4 = (int64_t)Mv * (N / 4);
  const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
  const int gcol = colsum_out ? (M + 255) / 256 : 0;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid + gcol), dim3(256), 0, st, slab, ksplit, M, N, C, ldc, bias, beta,
                     Mv, Nv, grid, part, colsum_out, colsum_acc);
}
// (also called by gemm_planes.hip / gemm_h3p.hip)
void launch_splitk_reduce(const float* slab, int ksplit, int M, int N, float* C, int64_t ldc, const float* bias,
                          float beta, int Mv, int Nv, hipStream_t st) {
  launch_splitk_reduce_cols(slab, ksplit, M, N, C, ldc, bias, beta, Mv, Nv, st, nullptr, nullptr, 0);
}
// wcol's bias gradient folded into the split-K pass (set_wcol_fold(0): its own reduce_rows; tests)
static int g_wcol_fold = 1;
void set_wcol_fold(int on) { g_wcol_fold = on ? 1 : 0; }

// Tile choice: the largest tile that still gives >= 2 blocks per CU (256 CUs).
static int pick_tile(int M, int N) {
  if (M % 128 == 0 && N % 128 == 0 && (M / 128) * (N / 128) >= 512) return 0;
  if (M % 128 == 0 && N % 64 == 0 && (M / 128) * (N / 64) >= 384) return 1;
  if (M % 64 == 0 && N % 64 == 0) return 2;
  return -1;
}

// bf16-split products: 128x128 tiles (each wave 64x64: 4 accumulators share every split
// fragment) and K slices until the grid covers the 256 CUs about twice.
static int pick_tile_split(int M, int N, int K, int* ksplit) {
  if (M % 128 || N % 128) return -1;
  const int tile = 0, tiles = (M / 128) * (N / 128);
  int s = 1;
  while (tiles * s < 384 && s < 8 && K % (2 * s * GBK) == 0 && K / (2 * s) >= 256) s *= 2;
  *ksplit = s;
  return tile;
}

// dtype: 0 fp32 on the exact-fp32 MFMA; 2 fp32 as 6 bf16 split products (fp32-level
// error at any range, see split4); 4 fp32 as 3 fp16
// split products with per-tensor power-of-two scales (split4h; amax_a / amax_b required: na / nb
// partial |max| values each, up to 8).  amax_c: GELU / dGELU epilogues atomically max |C| into it.
// epi: 0 none, 1 +bias, 2 gelu(+bias) writing the pre-activation to aux,
// 3 dgelu (aux = pre-activation) with column sums of C written (or added,
// colsum_acc) to colsum_out.  part: scratch of (M/64)*N floats (epi 3 only).
// ksplit: 0 = automatic (split dtypes only), 1 = none, >1 forced (any dtype); slab: ksplit*M*N floats
// of scratch when the split is >1 (epi 0/1 only).  mv/nv/kv: valid extents of a padded problem.
// C == nullptr (no epilogue, split dtypes): the result stays in the slab -- ksplit partial
// [M][N] planes the consumer sums in slice order (gemm_last_ksplit() says how many), no reduce pass.
// Returns -1 when the request is not served (caller falls back to the library).
static thread_local int g_last_ks = 1;
int gemm_last_ksplit() { return g_last_ks; }
void set_h3_occ3(int mask) { g_h3_occ3_env = mask & 7; }

int launch_gemm(int dtype, int ta, int tb, int M, int N, int K, const void* A, int64_t lda, const void* B,
                int64_t ldb, void* C, int64_t ldc, const float* bias, int epi, float beta, float* aux, int64_t ldaux,
                float* part, float* colsum_out, int colsum_acc, int tile_override, hipStream_t st, int ksplit,
                float* slab, int64_t slab_floats, int mv, int nv, int kv, const float* amax_a, int namax_a,
                const float* amax_b, int namax_b, float* amax_c) {
  if ((dtype != 0 && dtype != 2 && dtype != 4) || M <= 0 || N <= 0 || K <= 0 || K % GBK != 0) return -1;
  if (dtype == 4 && (!amax_a || !amax_b || namax_a < 1 || namax_b < 1 || namax_a > 8 || namax_b > 8)) return -1;
  // (namax_*: adjacent |max| slots of kAmaxShards shards each, common.h)
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al16(A) || !al16(B) || lda % 4 || ldb % 4) return -1;
  if ((epi >= 1 && !bias) || (epi >= 2 && (!aux || beta != 0.f)) || (epi == 3 && (!part != !colsum_out)))
    return -1;
  const int nt = dtype == 2 ? 6 : dtype == 4 ? 4 : 0;
  int tile, ks = 1;
  if (nt) {
    tile = pick_tile_split(M, N, K, &ks);
    if (ksplit > 0) ks = ksplit;
    if (epi >= 2 || !slab) ks = 1;  // fused GELU epilogues need the whole K in one block
  } else {
    tile = pick_tile(M, N);
    if (ksplit > 1 && epi <= kEpiBias && slab) ks = ksplit;  // exact-fp32 engine: forced split only
  }
  g_x6_tr = tile_override >= 0 && (tile_override & 256) ? 1 : tile_override >= 0 && (tile_override & 512) ? 0
                                                              : g_x6_tr_env;
  g_h3_occ3 = tile_override >= 0 && (tile_override & 1024) ? 7 : g_h3_occ3_env;
  tile_override = tile_override >= 0 ? (tile_override & 3) : -1;
  if (tile_override >= 0) {  // benchmarking hook: force a tile shape (must divide the problem)
    const int bm = tile_override == 2 ? 64 : 128, bn = tile_override == 0 ? 128 : 64;
    tile = (M % bm == 0 && N % bn == 0) ? tile_override : -1;
  }
  if (tile < 0) return -1;
  const bool keep_slab = C == nullptr;
  if (keep_slab && (!nt || epi != kEpiNone || !slab || beta != 0.f)) return -1;  // no bias: the consumer adds it
  if (keep_slab && ks == 1) {  // one slice: the slab's plane 0 is C
    if ((int64_t)M * N > slab_floats) return -1;
    C = slab;
    ldc = N;
  }
  if (ks > 1 && (K % (ks * GBK) != 0 || (int64_t)ks * M * N > slab_floats || N % 4 || ldc % 4 || !al16(C)))
    return -1;
  // valid extents of a padded problem (0 = the whole dimension): split-bf16 engine, plain / bias
  // epilogue only; the caller guarantees the operand pads it does not guard are allocated
  mv = mv > 0 ? mv : M;
  nv = nv > 0 ? nv : N;
  kv = kv > 0 ? kv : K;
  if ((mv != M || nv != N || kv != K) && (!nt || epi > kEpiBias || mv > M || nv > N || kv > K)) return -1;
  // weight gradient + the column sums of A (its bias gradient) in the same launch: split
  // engines, unpadded; part = [ks][M] partials, summed into
  // colsum_out (added if colsum_acc) below
  const bool wcol = ta && epi == kEpiNone && part != nullptr;
  if (wcol && (!nt || !colsum_out || mv != M || nv != N || kv != K))
    return -1;
  GemmArgs a{static_cast<const float*>(A), static_cast<const float*>(B), static_cast<float*>(C), bias, aux, part,
             lda, ldb, ldc, ldaux, M, N, K, beta, ks, slab, mv, nv, kv, g_slice_major,
             amax_a, amax_b, namax_a, namax_b, amax_c};
  int rc;
  if (nt == 6)
    rc = launch_split<6>(tile, ta, tb, epi, a, st);
  else if (nt == 4)
    rc = launch_split<4>(tile, ta, tb, epi, a, st);
  else
    rc = launch_split<0>(tile, ta, tb, epi, a, st);
  if (rc != 0) return rc;
  g_last_ks = ks;
  const bool fold = wcol && ks > 1 && !keep_slab && g_wcol_fold;  // bias gradient in the split-K pass
  if (ks > 1 && !keep_slab)
    launch_splitk_reduce_cols(slab, ks, M, N, static_cast<float*>(C), ldc, epi >= 1 ? bias : nullptr, beta, a.Mv,
                              a.Nv, st, fold ? part : nullptr, fold ? colsum_out : nullptr, colsum_acc);
  if (epi == kEpiDGelu && part) {
    const int bm = tile == 2 ? 64 : 128;
    const float* parts[1] = {part};
    float* outs[1] = {colsum_out};
    launch_reduce_rows(parts, outs, 1, M / bm, N, colsum_acc, st);
  } else if (wcol && !fold) {
    const float* parts[1] = {part};
    float* outs[1] = {colsum_out};
    launch_reduce_rows(parts, outs, 1, ks, M, colsum_acc, st);
  }
  return 0;
}
