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

template <int BM, int BN, int MF, bool TA, bool TB, int EPI, int ABL = 0>
__global__ void __launch_bounds__(256, 2) gemm_f32_kernel(GemmArgs p) {
  using IA = Img<BM, !TA, MF>;
  using IB = Img<BN, TB, MF>;
  using M_ = Mf<MF>;
  constexpr int TM = BM / 2 / MF, TN = BN / 2 / MF, NQ = 64 / MF, KG = 4 * NQ;
  __shared__ __attribute__((aligned(16))) float smem[2 * (IA::size + IB::size)];
  float* const As0 = smem;                 // A buffers at [0, 2*IA::size)
  float* const Bs0 = smem + 2 * IA::size;  // B buffers after them

  const int tiles_m = p.M / BM, tiles_n = p.N / BN, nwg = tiles_m * tiles_n;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, qq = nwg / 8, rr = nwg % 8;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
  const int tm = wg % tiles_m, tn = wg / tiles_m;  // M fastest: neighbours share the B panel
  const int m0 = tm * BM, n0 = tn * BN;

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
  const int KT = p.K / GBK;
  g_load<BM, !TA>(p.A, p.lda, m0, 0, ra);
  g_load<BN, TB>(p.B, p.ldb, n0, 0, rb);
  s_store<BM, !TA, MF>(As0, ra);
  s_store<BN, TB, MF>(Bs0, rb);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    // prefetch the next K tile (the last iteration re-reads the final tile into the idle
    // buffer: keeps the staging registers unconditional, so they stay in VGPRs)
    const int kn = (kt + 1 < KT ? kt + 1 : kt) * GBK;
    if (ABL == 0) {  // ABL: ablation builds for the microbenchmark (1: no global loads, 2: + no LDS writes/barrier)
      g_load<BM, !TA>(p.A, p.lda, m0, kn, ra);
      g_load<BN, TB>(p.B, p.ldb, n0, kn, rb);
    }
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
    if (ABL < 2) {
      s_store<BM, !TA, MF>(As0 + (cur ^ 1) * IA::size, ra);
      s_store<BN, TB, MF>(Bs0 + (cur ^ 1) * IB::size, rb);
    }
    if (ABL < 2) __syncthreads();
  }

  // epilogue: acc[i][j] register r -> row m0+wm+MF*i+Mf::row(r,q), col n0+wn+MF*j+lr
  float csum[TN];
  const bool use_beta = (EPI == kEpiNone || EPI == kEpiBias) && p.beta != 0.f;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    csum[j] = 0.f;
    const int n = n0 + wn + MF * j + lr;
    const float bv = (EPI != kEpiNone) ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int mb = m0 + wm + MF * i;
      if (EPI == kEpiGelu) {
#pragma unroll
        for (int r = 0; r < M_::nreg; ++r) {
          const int64_t m = mb + M_::row(r, q);
          p.aux[m * p.ldaux + n] = acc[i][j][r];
          p.C[m * p.ldc + n] = gelu_f(acc[i][j][r] + bv);
        }
      } else if (EPI == kEpiDGelu) {
        float pre[M_::nreg];
#pragma unroll
        for (int r = 0; r < M_::nreg; ++r) pre[r] = p.aux[(int64_t)(mb + M_::row(r, q)) * p.ldaux + n];
#pragma unroll
        for (int r = 0; r < M_::nreg; ++r) {
          const float v = acc[i][j][r] * gelu_grad_f(pre[r] + bv);
          csum[j] += v;
          p.C[(int64_t)(mb + M_::row(r, q)) * p.ldc + n] = v;
        }
      } else if (use_beta) {
        float old[M_::nreg];
#pragma unroll
        for (int r = 0; r < M_::nreg; ++r) old[r] = p.C[(int64_t)(mb + M_::row(r, q)) * p.ldc + n];
#pragma unroll
        for (int r = 0; r < M_::nreg; ++r)
          p.C[(int64_t)(mb + M_::row(r, q)) * p.ldc + n] = acc[i][j][r] + bv + p.beta * old[r];
      } else {
#pragma unroll
        for (int r = 0; r < M_::nreg; ++r) p.C[(int64_t)(mb + M_::row(r, q)) * p.ldc + n] = acc[i][j][r] + bv;
      }
    }
  }
  if (EPI == kEpiDGelu) {
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

static int g_ablation = 0;  // microbenchmark hook (tile_override bits 3-4)

template <int BM, int BN, int MF, bool TA, bool TB, int EPI>
void launch_cfg(const GemmArgs& a, hipStream_t st) {
  const int tiles = (a.M / BM) * (a.N / BN);
  if (EPI == kEpiNone && g_ablation == 1)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, MF, TA, TB, EPI, 1>), dim3(tiles), dim3(256), 0, st, a);
  else if (EPI == kEpiNone && g_ablation == 2)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, MF, TA, TB, EPI, 2>), dim3(tiles), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, MF, TA, TB, EPI>), dim3(tiles), dim3(256), 0, st, a);
}

template <int BM, int BN, int MF>
int launch_tile(int ta, int tb, int epi, const GemmArgs& a, hipStream_t st) {
  if (!ta && tb) {  // forward X * W^T
    if (epi == kEpiNone) launch_cfg<BM, BN, MF, false, true, kEpiNone>(a, st);
    else if (epi == kEpiBias) launch_cfg<BM, BN, MF, false, true, kEpiBias>(a, st);
    else if (epi == kEpiGelu) launch_cfg<BM, BN, MF, false, true, kEpiGelu>(a, st);
    else return -1;
  } else if (!ta && !tb) {  // dgrad dY * W
    if (epi == kEpiNone) launch_cfg<BM, BN, MF, false, false, kEpiNone>(a, st);
    else if (epi == kEpiDGelu) launch_cfg<BM, BN, MF, false, false, kEpiDGelu>(a, st);
    else return -1;
  } else if (ta && !tb) {  // wgrad dY^T * X
    if (epi == kEpiNone) launch_cfg<BM, BN, MF, true, false, kEpiNone>(a, st);
    else return -1;
  } else {
    return -1;
  }
  return 0;
}

}  // namespace hs

using namespace hs;

// Tile choice: the largest tile that still gives >= 2 blocks per CU (256 CUs).
static int pick_tile(int M, int N) {
  if (M % 128 == 0 && N % 128 == 0 && (M / 128) * (N / 128) >= 512) return 0;
  if (M % 128 == 0 && N % 64 == 0 && (M / 128) * (N / 64) >= 384) return 1;
  if (M % 64 == 0 && N % 64 == 0) return 2;
  return -1;
}

// epi: 0 none, 1 +bias, 2 gelu(+bias) writing the pre-activation to aux,
// 3 dgelu (aux = pre-activation) with column sums of C written (or added,
// colsum_acc) to colsum_out.  part: scratch of (M/64)*N floats (epi 3 only).
// Returns -1 when the request is not served (caller falls back to the library).
int launch_gemm(int dtype, int ta, int tb, int M, int N, int K, const void* A, int64_t lda, const void* B,
                int64_t ldb, void* C, int64_t ldc, const float* bias, int epi, float beta, float* aux, int64_t ldaux,
                float* part, float* colsum_out, int colsum_acc, int tile_override, hipStream_t st) {
  if (dtype != 0 || M <= 0 || N <= 0 || K <= 0 || K % GBK != 0) return -1;
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al16(A) || !al16(B) || lda % 4 || ldb % 4) return -1;
  if ((epi >= 1 && !bias) || (epi >= 2 && (!aux || beta != 0.f)) || (epi == 3 && (!part || !colsum_out)))
    return -1;
  int tile = pick_tile(M, N);
  const bool mfma16 = tile_override >= 0 && (tile_override & 4);  // benchmarking hook: 16x16x4 MFMA
  g_ablation = tile_override >= 0 ? (tile_override >> 3) & 3 : 0;
  tile_override = tile_override >= 0 ? (tile_override & 3) : -1;
  if (tile_override >= 0) {  // benchmarking hook: force a tile shape (must divide the problem)
    const int bm = tile_override == 2 ? 64 : 128, bn = tile_override == 0 ? 128 : 64;
    tile = (M % bm == 0 && N % bn == 0) ? tile_override : -1;
  }
  if (tile < 0) return -1;
  GemmArgs a{static_cast<const float*>(A), static_cast<const float*>(B), static_cast<float*>(C), bias, aux, part,
             lda, ldb, ldc, ldaux, M, N, K, beta};
  int rc;
  if (mfma16)
    rc = tile == 0 ? launch_tile<128, 128, 16>(ta, tb, epi, a, st)
         : tile == 1 ? launch_tile<128, 64, 16>(ta, tb, epi, a, st)
                     : launch_tile<64, 64, 16>(ta, tb, epi, a, st);
  else
    rc = tile == 0 ? launch_tile<128, 128, 32>(ta, tb, epi, a, st)
         : tile == 1 ? launch_tile<128, 64, 32>(ta, tb, epi, a, st)
                     : launch_tile<64, 64, 32>(ta, tb, epi, a, st);
  if (rc != 0) return rc;
  if (epi == kEpiDGelu) {
    const int bm = tile == 2 ? 64 : 128;
    const float* parts[1] = {part};
    float* outs[1] = {colsum_out};
    launch_reduce_rows(parts, outs, 1, M / bm, N, colsum_acc, st);
  }
  return 0;
}
