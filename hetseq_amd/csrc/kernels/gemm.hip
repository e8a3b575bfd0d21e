// LDS-tiled MFMA GEMM with fused epilogues (K01/K03/K04/K07 GEMM part).
//
//   C[M,N] = beta*C + op(A)[M,K] * op(B)[K,N]  (+ bias[N]) (-> GELU)
// row-major operands; op(A) = A (ta=0, A is [M,K]) or A^T (ta=1, A is [K,M]);
// op(B) = B (tb=0, B is [K,N]) or B^T (tb=1, B is [N,K]).  This covers the
// three BERT Linear products: forward X*W^T (ta=0,tb=1), dgrad dY*W (0,0) and
// wgrad dY^T*X (1,0).
//
// fp32 path (the reference trains in fp32): v_mfma_f32_32x32x2_f32, exact
// fp32 products.  Block tile 128x128, BK=16, 256 threads = 2x2 waves, each
// wave 64x64 = 2x2 MFMA tiles (64 accumulator VGPRs).  Both operands are
// staged k-major in LDS ([k][m] / [k][n], +4 padding) so the per-lane MFMA
// operand read (lane -> row l&31, k = l>>5) is a conflict-free ds_read_b32;
// the next K tile is prefetched into registers while the current one feeds
// the MFMAs (issue-early / write-late staging).  Tiles are remapped so that
// neighbouring output tiles share an XCD's L2 (bijective XCD swizzle).
#include "common.h"

namespace hs {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 16;
constexpr int LDA_S = BM + 4, LDB_S = BN + 4;

HS_DEVICE f32x16 mfma32x2(float a, float b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0); }

// Load a BK x 128 tile of op(X) (k-major image) into registers: 2048 floats,
// 8 per thread.  kmajor_src: source already [k][mn] (contiguous along mn).
template <bool kVec>
HS_DEVICE void load_tile(const float* __restrict__ X, int64_t ldx, bool kmajor_src, int mn0, int k0, int MN, int K,
                         float (&r)[8]) {
  const int t = threadIdx.x;
  if (kmajor_src) {
    // X is [K, MN]: element (k, mn) at X[k*ldx + mn]; thread covers k = t/32 (+8), mn = (t%32)*4
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = (t >> 5) + 8 * h;
      const int mn = (t & 31) * 4;
      const int gk = k0 + k, gm = mn0 + mn;
      if (kVec && gk < K && gm + 3 < MN) {
        const float4 v = *reinterpret_cast<const float4*>(X + (int64_t)gk * ldx + gm);
        r[4 * h] = v.x; r[4 * h + 1] = v.y; r[4 * h + 2] = v.z; r[4 * h + 3] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          r[4 * h + j] = (gk < K && gm + j < MN) ? X[(int64_t)gk * ldx + gm + j] : 0.f;
      }
    }
  } else {
    // X is [MN, K]: element (k, mn) at X[mn*ldx + k]; thread covers mn = t/4 (+64), k = (t%4)*4
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int mn = (t >> 2) + 64 * h;
      const int k = (t & 3) * 4;
      const int gk = k0 + k, gm = mn0 + mn;
      if (kVec && gm < MN && gk + 3 < K) {
        const float4 v = *reinterpret_cast<const float4*>(X + (int64_t)gm * ldx + gk);
        r[4 * h] = v.x; r[4 * h + 1] = v.y; r[4 * h + 2] = v.z; r[4 * h + 3] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          r[4 * h + j] = (gm < MN && gk + j < K) ? X[(int64_t)gm * ldx + gk + j] : 0.f;
      }
    }
  }
}

HS_DEVICE void store_tile(float* __restrict__ S, int lds_ld, bool kmajor_src, const float (&r)[8]) {
  const int t = threadIdx.x;
  if (kmajor_src) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = (t >> 5) + 8 * h;
      const int mn = (t & 31) * 4;
      *reinterpret_cast<float4*>(S + k * lds_ld + mn) = make_float4(r[4 * h], r[4 * h + 1], r[4 * h + 2], r[4 * h + 3]);
    }
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int mn = (t >> 2) + 64 * h;
      const int k = (t & 3) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) S[(k + j) * lds_ld + mn] = r[4 * h + j];
    }
  }
}

template <bool kVecA, bool kVecB>
__global__ void __launch_bounds__(256, 2)
    gemm_f32_kernel(int ta, int tb, int M, int N, int K, const float* __restrict__ A, int64_t lda,
                    const float* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc,
                    const float* __restrict__ bias, int epi, float beta) {
  __shared__ __attribute__((aligned(16))) float As[2][BK * LDA_S];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * LDB_S];
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  // bijective XCD swizzle: blocks b and b+8 share an XCD; give each XCD a contiguous tile range
  const int orig = blockIdx.x;
  const int xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  // tiles ordered along M within a column band of N (A tiles reused from L2)
  const int tm = wg % tiles_m, tn = wg / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const int li = lane & 31, hf = lane >> 5;

  // A image [k][m]: source k-major iff ta==1 ; B image [k][n]: source k-major iff tb==0
  const bool a_km = ta != 0, b_km = tb == 0;
  f32x16 acc[2][2] = {};
  float ra[8], rb[8];
  const int ktiles = (K + BK - 1) / BK;
  load_tile<kVecA>(A, lda, a_km, m0, 0, M, K, ra);
  load_tile<kVecB>(B, ldb, b_km, n0, 0, N, K, rb);
  store_tile(As[0], LDA_S, a_km, ra);
  store_tile(Bs[0], LDB_S, b_km, rb);
  __syncthreads();
  for (int kt = 0; kt < ktiles; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < ktiles) {
      load_tile<kVecA>(A, lda, a_km, m0, (kt + 1) * BK, M, K, ra);
      load_tile<kVecB>(B, ldb, b_km, n0, (kt + 1) * BK, N, K, rb);
    }
    const float* as = As[cur];
    const float* bs = Bs[cur];
#pragma unroll
    for (int ks = 0; ks < BK / 2; ++ks) {
      const int k = ks * 2 + hf;
      const float a0 = as[k * LDA_S + wm + li], a1 = as[k * LDA_S + wm + 32 + li];
      const float b0 = bs[k * LDB_S + wn + li], b1 = bs[k * LDB_S + wn + 32 + li];
      acc[0][0] = mfma32x2(a0, b0, acc[0][0]);
      acc[0][1] = mfma32x2(a0, b1, acc[0][1]);
      acc[1][0] = mfma32x2(a1, b0, acc[1][0]);
      acc[1][1] = mfma32x2(a1, b1, acc[1][1]);
    }
    if (kt + 1 < ktiles) {
      store_tile(As[cur ^ 1], LDA_S, a_km, ra);
      store_tile(Bs[cur ^ 1], LDB_S, b_km, rb);
    }
    __syncthreads();
  }
  // epilogue: acc[i][j] register r -> row m0+wm+32i+crow(r), col n0+wn+32j+li
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn + 32 * j + li;
    if (n >= N) continue;
    const float bv = (epi >= 1 && bias) ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hf;
        if (m >= M) continue;
        float v = acc[i][j][r] + bv;
        if (epi == 2) v = gelu_f(v);
        float* cp = C + (int64_t)m * ldc + n;
        if (beta != 0.f) v += beta * *cp;
        *cp = v;
      }
    }
  }
}

}  // namespace hs

using namespace hs;

// epi: 0 none, 1 +bias, 2 gelu(+bias). Returns -1 when the request is not
// served (caller falls back to the library GEMM).
int launch_gemm(int dtype, int ta, int tb, int M, int N, int K, const void* A, int64_t lda, const void* B,
                int64_t ldb, void* C, int64_t ldc, const float* bias, int epi, float beta, hipStream_t st) {
  if (dtype != 0 || M <= 0 || N <= 0 || K <= 0) return -1;
  const bool va = (lda % 4 == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  const bool vb = (ldb % 4 == 0) && ((reinterpret_cast<uintptr_t>(B) & 15) == 0);
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const float* a = static_cast<const float*>(A);
  const float* b = static_cast<const float*>(B);
  float* c = static_cast<float*>(C);
  if (va && vb)
    hipLaunchKernelGGL((gemm_f32_kernel<true, true>), dim3(tiles), dim3(256), 0, st, ta, tb, M, N, K, a, lda, b, ldb, c,
                       ldc, bias, epi, beta);
  else if (va)
    hipLaunchKernelGGL((gemm_f32_kernel<true, false>), dim3(tiles), dim3(256), 0, st, ta, tb, M, N, K, a, lda, b, ldb,
                       c, ldc, bias, epi, beta);
  else if (vb)
    hipLaunchKernelGGL((gemm_f32_kernel<false, true>), dim3(tiles), dim3(256), 0, st, ta, tb, M, N, K, a, lda, b, ldb,
                       c, ldc, bias, epi, beta);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<false, false>), dim3(tiles), dim3(256), 0, st, ta, tb, M, N, K, a, lda, b, ldb,
                       c, ldc, bias, epi, beta);
  return 0;
}
