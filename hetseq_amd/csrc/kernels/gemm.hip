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

enum { kEpiNone = 0, kEpiBias = 1, kEpiGelu = 2, kEpiDGelu = 3 };
constexpr int GBK = 32;

HS_DEVICE f32x16 mfma_f32(float a, float b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0); }

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

// LDS image geometry of one operand (rows = BM or BN)
template <int ROWS, bool KCONTIG>
struct Img {
  static constexpr int ld = KCONTIG ? GBK + 4 : ROWS + 32;     // floats per LDS row
  static constexpr int size = KCONTIG ? ROWS * ld : GBK * ld;  // floats per buffer
  static constexpr int nld = ROWS * GBK / 4 / 256;             // float4 loads per thread
};

// Global -> registers: the [ROWS x 32] (or [32 x ROWS]) tile at (r0, k0).
template <int ROWS, bool KCONTIG>
HS_DEVICE void g_load(const float* __restrict__ X, int64_t ldx, int r0, int k0, float4 (&r)[Img<ROWS, KCONTIG>::nld]) {
#pragma unroll
  for (int i = 0; i < Img<ROWS, KCONTIG>::nld; ++i) {
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

template <int ROWS, bool KCONTIG>
HS_DEVICE void s_store(float* __restrict__ S, const float4 (&r)[Img<ROWS, KCONTIG>::nld]) {
  using I = Img<ROWS, KCONTIG>;
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

// MFMA operand values of k-group g for the wave's 32-row tile starting at `row`:
// v[j] = X[row + li][k = 8g + 4*hf + j], j = 0..3
template <int ROWS, bool KCONTIG>
HS_DEVICE void frag(const float* __restrict__ S, int row, int g, int li, int hf, float (&v)[4]) {
  using I = Img<ROWS, KCONTIG>;
  if (KCONTIG) {
    const float4 t = *reinterpret_cast<const float4*>(S + (row + li) * I::ld + 8 * g + 4 * hf);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = S[(8 * g + 4 * hf + j) * I::ld + row + li];
  }
}

template <int BM, int BN, bool TA, bool TB, int EPI>
__global__ void __launch_bounds__(256, 2) gemm_f32_kernel(GemmArgs p) {
  using IA = Img<BM, !TA>;
  using IB = Img<BN, TB>;
  constexpr int TM = BM / 64, TN = BN / 64;
  __shared__ __attribute__((aligned(16))) float smem[2 * (IA::size + IB::size)];
  float* const As0 = smem;                  // A buffers at [0, 2*IA::size)
  float* const Bs0 = smem + 2 * IA::size;   // B buffers after them

  const int tiles_m = p.M / BM, tiles_n = p.N / BN, nwg = tiles_m * tiles_n;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int tm = wg % tiles_m, tn = wg / tiles_m;  // M fastest: neighbours share the B panel
  const int m0 = tm * BM, n0 = tn * BN;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int wm = wr * (BM / 2), wn = wc * (BN / 2);
  const int li = lane & 31, hf = lane >> 5;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  float4 ra[IA::nld], rb[IB::nld];
  const int KT = p.K / GBK;
  // A tile origin: rows m0 (TA=0: A[m][k]) or columns m0 of A[k][m]
  g_load<BM, !TA>(p.A, p.lda, m0, 0, ra);
  g_load<BN, TB>(p.B, p.ldb, n0, 0, rb);
  s_store<BM, !TA>(As0, ra);
  s_store<BN, TB>(Bs0, rb);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) {
      g_load<BM, !TA>(p.A, p.lda, m0, (kt + 1) * GBK, ra);
      g_load<BN, TB>(p.B, p.ldb, n0, (kt + 1) * GBK, rb);
    }
    const float* as = As0 + cur * IA::size;
    const float* bs = Bs0 + cur * IB::size;
#pragma unroll
    for (int g = 0; g < GBK / 8; ++g) {
      float av[TM][4], bv[TN][4];
#pragma unroll
      for (int i = 0; i < TM; ++i) frag<BM, !TA>(as, wm + 32 * i, g, li, hf, av[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) frag<BN, TB>(bs, wn + 32 * j, g, li, hf, bv[j]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma_f32(av[i][s], bv[j][s], acc[i][j]);
    }
    if (kt + 1 < KT) {
      s_store<BM, !TA>(As0 + (cur ^ 1) * IA::size, ra);
      s_store<BN, TB>(Bs0 + (cur ^ 1) * IB::size, rb);
    }
    __syncthreads();
  }

  // epilogue: acc[i][j] register r -> row m0+wm+32i+(r&3)+8(r>>2)+4hf, col n0+wn+32j+li
  float csum[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    csum[j] = 0.f;
    const int n = n0 + wn + 32 * j + li;
    const float bv = (EPI != kEpiNone) ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hf;
        float* cp = p.C + (int64_t)m * p.ldc + n;
        float v = acc[i][j][r];
        if (EPI == kEpiGelu) {
          p.aux[(int64_t)m * p.ldaux + n] = v;
          v = gelu_f(v + bv);
        } else if (EPI == kEpiDGelu) {
          v *= gelu_grad_f(p.aux[(int64_t)m * p.ldaux + n] + bv);
          csum[j] += v;
        } else {
          v += bv;
          if (p.beta != 0.f) v += p.beta * *cp;
        }
        *cp = v;
      }
    }
  }
  if (EPI == kEpiDGelu) {
    // column sums over the block's BM rows: lane halves, then the two wave rows via LDS
    float* red = smem;  // [BN] floats; the K loop ended with a barrier
#pragma unroll
    for (int j = 0; j < TN; ++j) csum[j] += __shfl_xor(csum[j], 32, 64);
    if (wr == 1 && hf == 0)
#pragma unroll
      for (int j = 0; j < TN; ++j) red[wn + 32 * j + li] = csum[j];
    __syncthreads();
    if (wr == 0 && hf == 0)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int c = wn + 32 * j + li;
        p.part[(int64_t)tm * p.N + n0 + c] = csum[j] + red[c];
      }
  }
}

template <int BM, int BN, bool TA, bool TB, int EPI>
void launch_cfg(const GemmArgs& a, hipStream_t st) {
  const int tiles = (a.M / BM) * (a.N / BN);
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, TA, TB, EPI>), dim3(tiles), dim3(256), 0, st, a);
}

template <int BM, int BN>
int launch_tile(int ta, int tb, int epi, const GemmArgs& a, hipStream_t st) {
  if (!ta && tb) {  // forward X * W^T
    if (epi == kEpiNone) launch_cfg<BM, BN, false, true, kEpiNone>(a, st);
    else if (epi == kEpiBias) launch_cfg<BM, BN, false, true, kEpiBias>(a, st);
    else if (epi == kEpiGelu) launch_cfg<BM, BN, false, true, kEpiGelu>(a, st);
    else return -1;
  } else if (!ta && !tb) {  // dgrad dY * W
    if (epi == kEpiNone) launch_cfg<BM, BN, false, false, kEpiNone>(a, st);
    else if (epi == kEpiDGelu) launch_cfg<BM, BN, false, false, kEpiDGelu>(a, st);
    else return -1;
  } else if (ta && !tb) {  // wgrad dY^T * X
    if (epi == kEpiNone) launch_cfg<BM, BN, true, false, kEpiNone>(a, st);
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
                float* part, float* colsum_out, int colsum_acc, hipStream_t st) {
  if (dtype != 0 || M <= 0 || N <= 0 || K <= 0 || K % GBK != 0) return -1;
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al16(A) || !al16(B) || lda % 4 || ldb % 4) return -1;
  if ((epi >= 1 && !bias) || (epi >= 2 && (!aux || beta != 0.f)) || (epi == 3 && (!part || !colsum_out)))
    return -1;
  const int tile = pick_tile(M, N);
  if (tile < 0) return -1;
  GemmArgs a{static_cast<const float*>(A), static_cast<const float*>(B), static_cast<float*>(C), bias, aux, part,
             lda, ldb, ldc, ldaux, M, N, K, beta};
  int rc = tile == 0 ? launch_tile<128, 128>(ta, tb, epi, a, st)
           : tile == 1 ? launch_tile<128, 64>(ta, tb, epi, a, st)
                       : launch_tile<64, 64>(ta, tb, epi, a, st);
  if (rc != 0) return rc;
  if (epi == kEpiDGelu) {
    const int bm = tile == 2 ? 64 : 128;
    const float* parts[1] = {part};
    float* outs[1] = {colsum_out};
    launch_reduce_rows(parts, outs, 1, M / bm, N, colsum_acc, st);
  }
  return 0;
}
