// fp32 GEMM as three fp16 MFMA products over pre-split, block-scaled operand planes ("h3p"; the
// operand format is described in h3p.h).  K01/K03/K04 GEMM parts of the BERT layer, reference
// bert_modeling.py:352-354 (the attention projections), 166-172 (LinearActivation), 423-427
// (BertOutput) and their autograd backward, which the reference runs as plain fp32 GEMMs.
//
//   C[M,N] = beta*C + op(A)[M,K] * op(B)[K,N]  (+ bias / GELU / dGELU epilogue)
// op(A) = A (TA=0, A stored [M][K]) or A^T (TA=1, stored [K][M]); op(B) = B (TB=0, stored [K][N])
// or B^T (TB=1, stored [N][K]).  The three Linear products: forward X W^T (0,1), data gradient
// dY W (0,0), weight gradient dY^T X (1,0).
//
// Why this structure (gfx950):
//  * the operand split (fp32 -> fp16 hi + lo) happens ONCE, in the kernel that produces the
//    tensor, not in every GEMM block that stages it: the K loop is LDS-DMA + MFMA only.  The
//    in-kernel-split engine (gemm.hip, gemm_x6s_kernel NT=4) spends as many issue cycles on the
//    split VALU and the transposing ds_writes as on its MFMAs (profiles/r4_fp32_pmc.md);
//  * the producers write the planes BLOCKED (h3p.h: 32 x 32 blocks of 2 KB): a 32-deep K tile of a
//    128-wide operand is four whole blocks in either orientation, so every LDS-DMA wave-instruction
//    reads full 128-B lines (row-major planes gave the k-contiguous operands 64- or 32-B pieces of
//    each row: 2-4x the L2 requests and TA time, profiles/r5_fp32_pmc.md);
//  * 128 x 128 tile, 4 waves (2 x 2, 64 x 64 each = 2 x 2 v_mfma_f32_32x32x16_f16 tiles), 16-deep K
//    steps in a four-step LDS ring (64 KB + 4 KB of block factors: two workgroups per CU, so the
//    backward's weight-gradient stream shares the CUs), each step's DMA issued three steps ahead;
//  * the LDS image is written lane-linearly by the DMA, so the bank swizzle is in each lane's SOURCE
//    address: k-contiguous operands as [128 rows][16 k] (32-B rows, 16-B chunks XOR (r>>3)&1,
//    ds_read_b128 fragments), mn-contiguous ones (the data gradient's weight, both weight-gradient
//    operands) as [16 k][128] (256-B rows, chunks XOR 4(r&3), fragments by ds_read_b64_tr_b16 -- the
//    gfx950 transposing read): no transpose pass anywhere;
//  * block scales: each 32-deep K tile's MFMAs accumulate into a fresh register tile (first MFMA with
//    an inline-zero C), which is added to the fp32 accumulator with the tile's factor 2^-(e_a + e_b)
//    by one v_pk_fma per register pair.  The accumulator therefore holds TRUE fp32 values (no running
//    exponent, no overflow the fp32 result would not have), and each operand block keeps its own
//    2^18 window.  The factors of the block's K range are tabulated in LDS once (4 KB);
//  * XCD-contiguous, grouped block order (bijective for any grid): an XCD's resident blocks share
//    operand panels in its private L2.
// Epilogues: fp32 C (+ bias) (+ beta C); split-K fp32 slabs (summed by splitk_reduce_kernel, or by
// the consumer); GELU (pre-activation kept in aux) and dGELU (column partials of the bias
// gradient), each optionally writing its output as blocked h3p planes for the next GEMM.
// (Round 5 measured and removed two alternatives, tools/bench_h3p.py / profiles/r5_fp32_pmc.md: a
// two-stage 32-deep loop -- one vmcnt(0) + barrier per tile -- 14 % slower over the BERT layer's
// twelve products; three workgroups per CU -- a three-step ring, one fragment register set read at
// each step's start, factors per step, 168 VGPRs -- 14 % slower: the exposed fragment reads and the
// per-step FMAs cost more than the third resident tile saves on the 576- / 768-tile grids.)
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "h3p.h"
#include "reduce.h"

namespace hs {
namespace {

typedef _Float16 qh8 __attribute__((ext_vector_type(8)));
typedef short qs4 __attribute__((ext_vector_type(4)));
typedef short qs8 __attribute__((ext_vector_type(8)));
typedef float qf16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void q_lds_t;
typedef __attribute__((address_space(1))) const void q_gbl_t;

constexpr int QT = 128, QBK = 32;  // tile edge; K tile (exponent block) depth
constexpr int QMAXKT = 128;         // K tiles per block (K / ksplit <= 4096)

enum { kQNone = 0, kQBias = 1, kQGelu = 2, kQDGelu = 3 };

struct QArgs {
  const uint16_t* A;
  const int8_t* ea;
  const uint16_t* B;
  const int8_t* eb;
  int64_t lda, a_ps, lde_a, ldb, b_ps, lde_b;
  float* C;
  int64_t ldc;
  const float* bias;
  float* aux;  // GELU: pre-activation out; dGELU: pre-activation in
  int64_t ldaux;
  float* part;  // dGELU: [M/128][N] column partials
  uint16_t* cp;  // plane output of the epilogue's result (GELU / dGELU)
  int8_t* ec;
  int64_t ldcp, cp_ps, lde_c;
  float* slab;  // split-K: [ksplit][M][N]
  int M, N, K, ksplit;
  float beta;
  int ablk, bblk;  // operand plane layout: 0 row-major, 1 blocked (h3p.h: 32 x 32 blocks of 2 KB per plane)
  // valid extents of a padded problem (the tied decoder's vocabulary padded to 512): C rows from Mv on
  // are not written (they are the NEXT tensor of the flat gradient store), bias entries from Nv on
  // read as zero (the padded columns of C stay exactly the zero the padded operand rows give)
  int Mv, Nv;
};

HS_DEVICE qf16 q_mma(qh8 a, qh8 b, qf16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0); }
// x of lane l ^ 1 (one DPP quad permutation [1, 0, 3, 2])
HS_DEVICE float q_swap1(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
}
HS_DEVICE int q_row(int r, int q) { return (r & 3) + 8 * (r >> 2) + 4 * q; }

// Shared epilogue: register r of acc[i][j] -> row m0+wm+32i+q_row(r,q), col n0+wn+32j+lr.  `smem`: the
// kernel's LDS (free: the K loop ended with a barrier), used for the dGELU column sums.
// dGELU: the pre-activation of a 32 x 32 tile as this lane's eight float2 (row 4 q + odd + row offset of
// register pair r / 2, columns cp2, cp2 + 1; the pairing of the epilogue below)
HS_DEVICE void q_aux_load(const QArgs& p, float2 (&v)[8], int mb, int nb, int lane) {
  const int lr = lane & 31, q = lane >> 5, odd = lane & 1;
  const float* auxb = p.aux + (int64_t)(mb + 4 * q + odd) * p.ldaux + (nb + (lr & ~1));
#pragma unroll
  for (int r = 0; r < 16; r += 2)
    v[r / 2] = *reinterpret_cast<const float2*>(auxb + (int64_t)((r & 3) + 8 * (r >> 2)) * p.ldaux);
}

template <int EPI, int NPF>
HS_DEVICE void q_epilogue(const QArgs& p, qf16 (&acc)[2][2], char* smem, int m0, int n0, int tm, int slice, int wm,
                          int wn, int wr, int lane, const float2 (&pf)[NPF][8]) {
  const int lr = lane & 31, q = lane >> 5;
  if (p.ksplit > 1) {  // fp32 partial slab; bias / beta / the sum in splitk_reduce_kernel (or the consumer)
    float* sl = p.slab + (int64_t)slice * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          sl[(int64_t)(m0 + wm + 32 * i + q_row(r, q)) * p.N + n0 + wn + 32 * j + lr] = acc[i][j][r];
    return;
  }
  float csum[2] = {0.f, 0.f};
  if (EPI <= kQBias && m0 + 128 > p.Mv) {  // a tile reaching past the valid rows (padded problems only)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn + 32 * j + lr;
      const float bv = EPI != kQNone && n < p.Nv ? p.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t m = m0 + wm + 32 * i + q_row(r, q);
          if (m < p.Mv)
            p.C[m * p.ldc + n] = acc[i][j][r] + bv + (p.beta != 0.f ? p.beta * p.C[m * p.ldc + n] : 0.f);
        }
    }
    return;
  }
  if constexpr (EPI == kQGelu || EPI == kQDGelu) {
    // Lanes l and l ^ 1 hold adjacent columns of the same rows: one DPP swap per register pair gives
    // each lane two adjacent columns of ONE row (the even lane row R, the odd lane row R + 1 of the
    // pair), so the pre-activation moves as 8-byte accesses at constant offsets from one base per tile.
    // The GELU math runs on the pair (acc[r], acc[r + 1]) -- one column, two rows -- as packed fp32.
    // The epilogue runs when the tile's MFMAs are done and is VALU-bound (round 6, tools/bench_h3p_epi.py
    // with each part skipped in turn: at M 4096 the erff-based GELU math cost 18 us of a 92-us FFN-in
    // product, the plane stores 9, the pre-activation store 3; the dGELU's pre-activation loads 18).
    const int odd = lane & 1, cp2 = lr & ~1;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn + 32 * j + lr;
      const float bv = n < p.Nv ? p.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int mb = m0 + wm + 32 * i;
        float* const auxb = p.aux + (int64_t)(mb + 4 * q + odd) * p.ldaux + (n0 + wn + 32 * j + cp2);
        // the pre-activation moves first, then the math of the tile's eight pairs as one block (eight
        // independent dependency chains for the scheduler to interleave)
        hs_f2 pre[8];
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const int64_t ro = (int64_t)((r & 3) + 8 * (r >> 2)) * p.ldaux;  // row q_row(r, q) - 4 q
          if (EPI == kQGelu) {
            pre[r / 2] = hs_f2{acc[i][j][r], acc[i][j][r + 1]};
            const float recv = q_swap1(odd ? acc[i][j][r] : acc[i][j][r + 1]);
            *reinterpret_cast<float2*>(auxb + ro) =
                odd ? make_float2(recv, acc[i][j][r + 1]) : make_float2(acc[i][j][r], recv);
          } else {
            const float2 ld = 2 * i + j < NPF ? pf[(2 * i + j) % NPF][r / 2]
                                              : *reinterpret_cast<const float2*>(auxb + ro);
            const float recv = q_swap1(odd ? ld.x : ld.y);
            pre[r / 2] = hs_f2{odd ? recv : ld.x, odd ? ld.y : recv};
          }
        }
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          hs_f2 res;
          if (EPI == kQGelu) {
            res = gelu_v(pre[r / 2] + bv);
          } else {
            res = hs_f2{acc[i][j][r], acc[i][j][r + 1]} * gelu_grad_v(pre[r / 2] + bv);
          }
          acc[i][j][r] = res.x;
          acc[i][j][r + 1] = res.y;
        }
        if (EPI == kQDGelu)
#pragma unroll
          for (int r = 0; r < 16; ++r) csum[j] += acc[i][j][r];
        if (p.C)
#pragma unroll
          for (int r = 0; r < 16; ++r) p.C[(int64_t)(mb + q_row(r, q)) * p.ldc + n] = acc[i][j][r];
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn + 32 * j + lr;
      const float bv = EPI != kQNone && n < p.Nv ? p.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int mb = m0 + wm + 32 * i;
        if (p.beta != 0.f) {
          float old[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) old[r] = p.C[(int64_t)(mb + q_row(r, q)) * p.ldc + n];
#pragma unroll
          for (int r = 0; r < 16; ++r)
            p.C[(int64_t)(mb + q_row(r, q)) * p.ldc + n] = acc[i][j][r] + bv + p.beta * old[r];
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) p.C[(int64_t)(mb + q_row(r, q)) * p.ldc + n] = acc[i][j][r] + bv;
        }
      }
    }
  }
  if ((EPI == kQGelu || EPI == kQDGelu) && p.cp) {
    // the result as h3p planes: one exponent per 32 x 32 accumulator tile (= one exponent block, 2 KB
    // per plane, 64-B rows); the same pairing as above makes every plane access 4 bytes wide
    const int odd = lane & 1, cp2 = lr & ~1;
    const uint32_t sel_send = odd ? 0x05040100u : 0x07060302u;
    const uint32_t sel_hi = odd ? 0x03020504u : 0x05040100u, sel_lo = odd ? 0x03020706u : 0x07060100u;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        uint32_t mb = 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r) mb = amax_bits(mb, acc[i][j][r]);
        const int e = h3p_exp_bits(wave_umax(mb));
        const float sc = h3p_scale(e);
        const int rb = (m0 + wm) / 32 + i, cb = (n0 + wn) / 32 + j;
        if (lane == 0) p.ec[(int64_t)rb * p.lde_c + cb] = static_cast<int8_t>(e);
        uint16_t* const blk = p.cp + (int64_t)rb * 32 * p.ldcp + (int64_t)cb * 1024 + (4 * q + odd) * 32 + cp2;
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          uint32_t h, l;  // rows r, r + 1 of this lane's column: (hi_r | hi_r+1 << 16), (lo_r | lo_r+1 << 16)
          h3p_split2(acc[i][j][r], acc[i][j][r + 1], sc, h, l);
          // the even lane keeps row r and sends row r + 1 (hi | lo << 16); the odd lane the reverse
          // (byte selectors per lane parity: v_perm_b32 picks bytes 0-3 from its second operand)
          const uint32_t send = __builtin_amdgcn_perm(l, h, sel_send);
          const uint32_t recv = __builtin_bit_cast(uint32_t, q_swap1(__builtin_bit_cast(float, send)));
          const uint32_t hi = __builtin_amdgcn_perm(recv, h, sel_hi);
          const uint32_t lo = __builtin_amdgcn_perm(recv, l, sel_lo);
          const int ro = ((r & 3) + 8 * (r >> 2)) * 32;
          *reinterpret_cast<uint32_t*>(blk + ro) = hi;
          *reinterpret_cast<uint32_t*>(blk + p.cp_ps + ro) = lo;
        }
      }
  }
  if (EPI == kQDGelu && p.part) {  // column sums over the block's 128 rows: lane halves, then wave rows
    float* red = reinterpret_cast<float*>(smem);  // the K loop ended with a barrier
#pragma unroll
    for (int j = 0; j < 2; ++j) csum[j] += __shfl_xor(csum[j], 32, 64);
    if (wr == 1 && q == 0)
#pragma unroll
      for (int j = 0; j < 2; ++j) red[wn + 32 * j + lr] = csum[j];
    __syncthreads();
    if (wr == 0 && q == 0)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = wn + 32 * j + lr;
        p.part[(int64_t)tm * p.N + n0 + c] = csum[j] + red[c];
      }
  }
}

// ---------------------------------------------------------------- the K loop: 16-deep steps, 4-deep ring
//   step s: this wave's share of step s+1 landed (counted vmcnt: step s+2 stays in flight) ->
//   barrier (step s+1 visible to every wave; every wave's reads of step s-1 done, its stage free) ->
//   step s's 12 MFMAs (fragments in registers, read during step s-1), with the DMA of step s+3 into
//   the freed stage and the fragment reads of step s+1 interleaved between them in pinned order.
// The DMA pieces are asm statements: hipcc would otherwise drain vmcnt(0) before every LDS read it
// cannot prove disjoint from a pending DMA.  Block factors apply per 32-deep K tile (every second
// step).
constexpr int RBK = 16;
constexpr int RPLANE = QT * RBK * 2;  // one plane of one operand step: 4 KB
constexpr int ROPND = 2 * RPLANE;     // 8 KB
constexpr int RSTAGE = 2 * ROPND;     // A and B: 16 KB
constexpr int RNS = 4;
constexpr int RSMEM = RNS * RSTAGE + 2 * QMAXKT * 4 * 4;

template <bool KC>
struct RImg {
  static constexpr int row_bytes = KC ? RBK * 2 : QT * 2;  // 32 ([mn][k]) or 256 ([k][mn])
  // k-contiguous: rows 8 apart share banks -> chunk ^ ((r >> 3) & 1) spreads a b128 lane group over
  // both chunk columns (conflict-free); [k][mn]: the transposed read's four k rows in four quarters
  HS_DEVICE static int swz(int r) { return KC ? ((r >> 3) & 1) : 4 * (r & 3); }
};

// byte offsets (plane 0, k = 0 of the block's range) of this wave's two pieces of one operand:
// piece j (0, 1) fills bytes [1024 (4 j + w), +1024) of the operand's 8 KB step image
template <bool KC>
HS_DEVICE void r_offsets(uint32_t (&off)[2], int64_t ld, int64_t ps, int mn0, int w, int lane, int blk) {
  using I = RImg<KC>;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int byte = 1024 * (4 * j + w) + 16 * lane;
    const int plane = byte / RPLANE, ib = byte % RPLANE;
    const int row = ib / I::row_bytes, cl = (ib % I::row_bytes) / 16;
    const int gc = cl ^ I::swz(row);
    const int64_t e = KC ? h3p_index(mn0 + row, 8 * gc, ld, blk) : h3p_index(row, mn0 + 8 * gc, ld, blk);
    off[j] = static_cast<uint32_t>(2 * (e + plane * ps));
  }
}

// one LDS-DMA piece (1 KB per wave), hidden from hipcc's wait insertion (see above); M0 is written and
// restored inside the statement
HS_DEVICE void r_dma(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst));
}

// vmcnt(N) through the builtin (gfx9 encoding), lgkmcnt / expcnt untouched
template <int N_>
HS_DEVICE void r_wait_vm() {
  static_assert(N_ >= 0 && N_ < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N_ & 15) | ((N_ >> 4) << 14) | 0x70 | 0xF00);
}

HS_DEVICE void r_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's fragment reads are back
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <bool KC>
HS_DEVICE qh8 r_frag(const char* img, int p, int rc, int lane) {
  using I = RImg<KC>;
  const char* pl = img + p * RPLANE;
  if (KC) {
    const int r = rc + (lane & 31), c = lane >> 5;
    return *reinterpret_cast<const qh8*>(pl + r * I::row_bytes + 16 * (c ^ I::swz(r)));
  } else {
    const int l16 = lane & 15, q = l16 >> 2, pp = l16 & 3, g = lane >> 4;
    const int col = rc + 16 * (g & 1) + 4 * pp;
    qs4 v[2];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int row = 8 * (g >> 1) + 4 * jj + q;
      const char* a = pl + row * I::row_bytes + 16 * ((col >> 3) ^ I::swz(row)) + 2 * (col & 7);
      v[jj] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) qs4*)(a));
    }
    const qs8 u = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
    return __builtin_bit_cast(qh8, u);
  }
}

// The DMA lead is four steps: step s refills its OWN stage -- free once the barrier opening step s has
// passed (every wave read step s's fragments into registers during step s - 1) -- so three steps stay
// in flight in the four stages (round 5 refilled the stage of step s - 1: two in flight; the step
// measured the same: 10.79 vs 10.80 ms, bench.py --ab, round 6).
// Issue order inside a step: the eight fragment reads of step s + 1 between the step's first eight
// MFMAs, the four DMA pieces after the last four, so the reads complete under the step's last MFMAs
// instead of in front of the closing lgkmcnt(0) + barrier (round 5 issued the DMA first: the layer's
// twelve products 643.6 -> 634.1 us alone, the step 10.81 -> 10.73 ms, tools/bench_h3p.py and
// bench.py --ab, round 6).
#ifndef HS_QAUX_PREFETCH
#define HS_QAUX_PREFETCH 2
#endif
constexpr int kQAuxPrefetch = HS_QAUX_PREFETCH;

template <bool TA, bool TB, int EPI>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) gemm_h3p_kernel(QArgs p) {
  constexpr int LEAD = 4;
  constexpr bool AK = !TA, BKc = TB;
  __shared__ __attribute__((aligned(1024))) char smem[RSMEM];
  float* const fA = reinterpret_cast<float*>(smem + RNS * RSTAGE);
  float* const fB = fA + QMAXKT * 4;

  const int tiles_m = p.M / QT, tiles_n = p.N / QT, ntile = tiles_m * tiles_n, nwg = ntile * p.ksplit;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, qq = nwg / 8, rr = nwg % 8;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
  const int slice = wg / ntile, tile = wg % ntile;
  const int gsz = 8 * tiles_n, grp = tile / gsz, gm = min(8, tiles_m - 8 * grp);
  const int tm = 8 * grp + (tile % gsz) % gm, tn = (tile % gsz) / gm;
  const int m0 = tm * QT, n0 = tn * QT;
  const int kofs = slice * (p.K / p.ksplit);
  const int KT = p.K / p.ksplit / QBK;  // 32-deep K tiles (exponent blocks)
  const int NSTEP = 2 * KT;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1, wm = 64 * wr, wn = 64 * wc;

  for (int u = threadIdx.x; u < 4 * KT; u += 256) {
    const int t = u >> 2, g = u & 3, kb = kofs / QBK + t;
    const int64_t ia = AK ? (int64_t)(m0 / 32 + g) * p.lde_a + kb : (int64_t)kb * p.lde_a + m0 / 32 + g;
    const int64_t ib = BKc ? (int64_t)(n0 / 32 + g) * p.lde_b + kb : (int64_t)kb * p.lde_b + n0 / 32 + g;
    fA[u] = __builtin_ldexpf(1.f, -(int)p.ea[ia]);
    fB[u] = __builtin_ldexpf(1.f, -(int)p.eb[ib]);
  }

  uint32_t offA[2], offB[2];
  r_offsets<AK>(offA, p.lda, p.a_ps, m0, w, lane, p.ablk);
  r_offsets<BKc>(offB, p.ldb, p.b_ps, n0, w, lane, p.bblk);
  // byte offset of 16-deep step s: k-contiguous = columns 16 s.., else rows 16 s.. (h3p_index is
  // linear in whole blocks, so a step is its 32-deep tile plus the half-tile's offset)
  const int64_t tileA = 2 * (AK ? h3p_index(0, QBK, p.lda, p.ablk) : h3p_index(QBK, 0, p.lda, p.ablk));
  const int64_t tileB = 2 * (BKc ? h3p_index(0, QBK, p.ldb, p.bblk) : h3p_index(QBK, 0, p.ldb, p.bblk));
  const int64_t halfA = 2 * (AK ? h3p_index(0, RBK, p.lda, p.ablk) : h3p_index(RBK, 0, p.lda, p.ablk));
  const int64_t halfB = 2 * (BKc ? h3p_index(0, RBK, p.ldb, p.bblk) : h3p_index(RBK, 0, p.ldb, p.bblk));
  const char* ga = reinterpret_cast<const char*>(p.A) + (kofs / QBK) * tileA;
  const char* gb = reinterpret_cast<const char*>(p.B) + (kofs / QBK) * tileB;
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((q_lds_t*)smem));
  // DMA piece j of step s (clamped: past the last step a stage nobody reads again gets the last step's
  // bytes again, so every step issues the same four pieces and the counted waits stay exact)
  auto dma = [&](int j, int s, int stage) __attribute__((always_inline)) {
    const int64_t ss = min(s, NSTEP - 1);
    const char* src = j < 2 ? ga + (ss >> 1) * tileA + (ss & 1) * halfA + offA[j]
                            : gb + (ss >> 1) * tileB + (ss & 1) * halfB + offB[j - 2];
    r_dma(src, __builtin_amdgcn_readfirstlane(lds0 + stage * RSTAGE + (j < 2 ? 0 : ROPND) + 1024 * (4 * (j & 1) + w)));
  };

  qf16 acc[2][2], tmp[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = qf16{};
  struct Frags {
    qh8 a[2][2], b[2][2];  // [plane][tile]
  };
  // fragment reads of one step as 8 pieces: A (plane, tile), then B (plane, tile)
  auto read_piece = [&](Frags& f, int stage, int r) __attribute__((always_inline)) {
    const char* img = smem + stage * RSTAGE;
    if (r < 4) f.a[r >> 1][r & 1] = r_frag<AK>(img, r >> 1, wm + 32 * (r & 1), lane);
    else f.b[(r - 4) >> 1][r & 1] = r_frag<BKc>(img + ROPND, (r - 4) >> 1, wn + 32 * (r & 1), lane);
  };
  // 12 MFMAs (terms smallest first: lo_a hi_b, hi_a lo_b, hi_a hi_b; 4 tiles each); between them, in
  // source order pinned by sched_barrier: the four DMA pieces of step s+3, then the 8 fragment reads
  // of step s+1
  auto body = [&](const Frags& f, Frags& nf, int s, int st_free, int st_next, bool first, bool read_next)
      __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < 12; ++c) {
      const int term = c >> 2, i = (c >> 1) & 1, j = c & 1;
      const qh8 a = term == 0 ? f.a[1][i] : f.a[0][i];
      const qh8 b = term == 1 ? f.b[1][j] : f.b[0][j];
      tmp[i][j] = q_mma(a, b, (first && term == 0) ? qf16{} : tmp[i][j]);
      if (c < 8) {
        if (read_next) read_piece(nf, st_next, c);
      } else {
        dma(c - 8, s + LEAD, st_free);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // dGELU: the pre-activation of the first kQAuxPrefetch tiles is loaded before the K loop (the
  // epilogue's loads were 17 us of a 99-us FFN-out data gradient, issued when the MFMAs are done;
  // the prologue's first counted wait covers them too)
  constexpr int NPF = EPI == kQDGelu ? kQAuxPrefetch : 1;
  float2 pf[NPF][8];
  if constexpr (EPI == kQDGelu) {
#pragma unroll
    for (int t = 0; t < NPF; ++t) q_aux_load(p, pf[t], m0 + wm + 32 * (t >> 1), n0 + wn + 32 * (t & 1), lane);
  }
  // prologue: LEAD steps in flight, wait for the first
#pragma unroll
  for (int j = 0; j < 4; ++j) dma(j, 0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j) dma(j, 1, 1);
#pragma unroll
  for (int j = 0; j < 4; ++j) dma(j, 2, 2);
#pragma unroll
  for (int j = 0; j < 4; ++j) dma(j, 3, 3);
  r_wait_vm<12>();
  __syncthreads();  // step 0 and the factor tables visible to every wave
  Frags F[2];
#pragma unroll
  for (int r = 0; r < 8; ++r) read_piece(F[0], 0, r);
  // K tile t = steps 2t (F[0], stage 2t % 4) and 2t+1 (F[1]); stage of step s is s % 4
  for (int t = 0; t < KT; ++t) {
    const int s0 = 2 * t, st0 = s0 & 3;
    r_wait_vm<4 * (LEAD - 2)>();  // step s0+1 landed (this wave's pieces); the later ones in flight
    r_barrier();
    body(F[0], F[1], s0, (st0 + LEAD) & 3, (st0 + 1) & 3, true, true);
    r_wait_vm<4 * (LEAD - 2)>();
    r_barrier();
    const float2 fa = *reinterpret_cast<const float2*>(fA + 4 * t + 2 * wr);
    const float2 fb = *reinterpret_cast<const float2*>(fB + 4 * t + 2 * wc);
    // (the last tile's reads of "step s0+2" fetch a stage holding a duplicate DMA: harmless, unused)
    body(F[1], F[0], s0 + 1, (st0 + 1 + LEAD) & 3, (st0 + 2) & 3, false, true);
    const float fac[2][2] = {{fa.x * fb.x, fa.x * fb.y}, {fa.y * fb.x, fa.y * fb.y}};
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] += tmp[i][j] * fac[i][j];
  }
  r_wait_vm<0>();  // the trailing duplicate DMAs land before the LDS is reused
  __syncthreads();
  q_epilogue<EPI, NPF>(p, acc, smem, m0, n0, tm, slice, wm, wn, wr, lane, pf);
}

// ---------------------------------------------------------------- fp32 -> h3p planes
// Column partials of a blocked h3p operand: part[r / 32][c] = sum over the 32 rows of panel r / 32 of the
// value the planes hold, (hi + lo) 2^-e (exact in fp32: 22 bits), rows in order (deterministic).  The
// QKV bias gradient of the fused layer comes from dqkv's planes this way: the attention backward then
// writes dqkv only as planes (no fp32 copy: 38 MB of writes and reads less per BERT-base layer).
__global__ void __launch_bounds__(128) h3p_colpart_kernel(const uint16_t* __restrict__ pl, int64_t ld, int64_t ps,
                                                         const int8_t* __restrict__ ex, int64_t lde, int cols,
                                                         float* __restrict__ part) {
  const int panel = blockIdx.y, c = (blockIdx.x * 128 + threadIdx.x) * 2;
  if (c >= cols) return;
  const int cb = c >> 5;
  const uint16_t* base = pl + (int64_t)panel * 32 * ld + (int64_t)cb * 1024 + (c & 31);
  uint32_t hv[32], lv[32];
#pragma unroll
  for (int r = 0; r < 32; ++r) {
    hv[r] = *reinterpret_cast<const uint32_t*>(base + r * 32);
    lv[r] = *reinterpret_cast<const uint32_t*>(base + ps + r * 32);
  }
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int r = 0; r < 32; ++r) {
    const h3p_h2 h = __builtin_bit_cast(h3p_h2, hv[r]), l = __builtin_bit_cast(h3p_h2, lv[r]);
    s0 += static_cast<float>(h[0]) + static_cast<float>(l[0]);
    s1 += static_cast<float>(h[1]) + static_cast<float>(l[1]);
  }
  const float sc = h3p_scale(-ex[(int64_t)panel * lde + cb]);
  *reinterpret_cast<float2*>(part + (int64_t)panel * cols + c) = make_float2(s0 * sc, s1 * sc);
}

struct QSplitSeg {
  const float* src;
  uint16_t* dst;
  int8_t* ex;
  int64_t lds, ldd, ps, lde;
  int rows, cols, blk0;  // blk0: index of the segment's first 32 x 32 block in the launch
  int blocked;           // destination layout (h3p_index)
  int vrows;             // source rows that exist (rows past them split as zeros: a padded vocabulary)
  int pad_;
};

// one wave per 32 x 32 block: lane l loads row (l >> 3) + 8 q, columns 4 (l & 7) .. +3 (q = 0..3),
// the block |max| by a wave reduction, then both planes and the exponent
__global__ void __launch_bounds__(256) h3p_split_kernel(QSplitSeg one, const QSplitSeg* __restrict__ many, int nseg,
                                                        int total) {
  const int b = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  if (b >= total) return;  // wave-uniform
  QSplitSeg s = one;
  if (many) {
    int i = 0;
    while (i + 1 < nseg && many[i + 1].blk0 <= b) ++i;
    s = many[i];
  }
  const int lb = b - s.blk0, nbc = s.cols / 32;
  const int br = lb / nbc, bc = lb % nbc;
  const int lane = threadIdx.x & 63;
  const int r0 = br * 32 + (lane >> 3), c = bc * 32 + 4 * (lane & 7);
  float v[4][4];
  uint32_t m = 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (r0 + 8 * k < s.vrows) {
      load4(s.src + (int64_t)(r0 + 8 * k) * s.lds + c, v[k]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[k][e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) m = amax_bits(m, v[k][e]);
  }
  const int e = h3p_exp_bits(wave_umax(m));
  const float sc = h3p_scale(e);
#pragma unroll
  for (int k = 0; k < 4; ++k) h3p_store4(s.dst, s.ps, h3p_index(r0 + 8 * k, c, s.ldd, s.blocked), v[k], sc);
  if (lane == 0) s.ex[(int64_t)br * s.lde + bc] = static_cast<int8_t>(e);
}

template <bool TA, bool TB, int EPI>
void q_launch(const QArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((gemm_h3p_kernel<TA, TB, EPI>), dim3((a.M / QT) * (a.N / QT) * a.ksplit), dim3(256), 0, st, a);
}

template <bool TA, bool TB>
int q_launch_epi(int epi, const QArgs& a, hipStream_t st) {
  if (epi == kQNone) q_launch<TA, TB, kQNone>(a, st);
  else if (epi == kQBias) q_launch<TA, TB, kQBias>(a, st);
  else if (epi == kQGelu && !TA && TB) q_launch<false, true, kQGelu>(a, st);
  else if (epi == kQDGelu && !TA && !TB) q_launch<false, false, kQDGelu>(a, st);
  else return -1;
  return 0;
}

}  // namespace
}  // namespace hs

using namespace hs;

// gemm.hip: C = sum of the ksplit fp32 slabs (fixed order) (+ bias) (+ beta * C)
void launch_splitk_reduce(const float* slab, int ksplit, int M, int N, float* C, int64_t ldc, const float* bias,
                          float beta, int Mv, int Nv, hipStream_t st);

// Returns -1 (nothing launched) for a request the kernel does not serve.  Strides and plane strides
// in elements; lde_*: row stride of the exponent arrays.  C == nullptr with ksplit > 1: the partial
// slabs are left for the consumer (no reduce pass).  cp / ec (GELU, dGELU): the result's planes.
// Mv / Nv (0: M / N): valid extents of a padded problem -- C rows from Mv on are left untouched,
// bias entries from Nv on read as zero (plain and bias epilogues).
int launch_gemm_h3p_v(int ta, int tb, int M, int N, int K, const void* A, int64_t lda, int64_t a_ps, const int8_t* ea,
                      int64_t lde_a, const void* B, int64_t ldb, int64_t b_ps, const int8_t* eb, int64_t lde_b,
                      float* C, int64_t ldc, const float* bias, int epi, float beta, float* aux, int64_t ldaux,
                      float* part, float* colsum, int colsum_acc, void* cp, int64_t ldcp, int64_t cp_ps, int8_t* ec,
                      int64_t lde_c, int ksplit, float* slab, int64_t slab_floats, int ablk, int bblk, int Mv, int Nv,
                      hipStream_t st) {
  ksplit = std::max(1, ksplit);
  Mv = Mv > 0 ? Mv : M;
  Nv = Nv > 0 ? Nv : N;
  if (Mv > M || Nv > N || (Mv < M && (epi > 1 || !C))) return -1;  // (valid rows: plain / bias products into C)
  if ((ablk && lda % 32) || (bblk && ldb % 32)) return -1;
  if (M <= 0 || N <= 0 || K <= 0 || M % QT || N % QT || K % (QBK * ksplit) || K / ksplit / QBK > QMAXKT) return -1;
  if (ta && tb) return -1;
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!A || !B || !ea || !eb || !al16(A) || !al16(B) || lda % 8 || ldb % 8 || a_ps % 8 || b_ps % 8) return -1;
  if (epi < 0 || epi > 3 || (epi >= 1 && !bias) || (epi >= 2 && (!aux || beta != 0.f || ksplit > 1))) return -1;
  if (epi == 3 && colsum && !part) return -1;  // (part without colsum: the caller reduces the partials)
  if (cp && (epi < 2 || !ec || ldcp % 32)) return -1;  // (the result's planes are written blocked)
  if (epi < 2 && !C && ksplit == 1) return -1;
  if (epi >= 2 && !C && !cp) return -1;
  if (ksplit > 1 && (!slab || (int64_t)ksplit * M * N > slab_floats || (C && (N % 4 || ldc % 4 || !al16(C)))))
    return -1;
  // 32-bit per-lane DMA offsets: each operand's span (both planes) below 4 GiB
  const int64_t spanA = 2 * (a_ps + (int64_t)(ta ? K : M) * lda), spanB = 2 * (b_ps + (int64_t)(tb ? N : K) * ldb);
  if (spanA >= (1ll << 32) || spanB >= (1ll << 32)) return -1;
  QArgs a{static_cast<const uint16_t*>(A), ea, static_cast<const uint16_t*>(B), eb, lda, a_ps, lde_a, ldb, b_ps,
          lde_b, C, ldc, bias, aux, ldaux, part, static_cast<uint16_t*>(cp), ec, ldcp, cp_ps, lde_c, slab, M, N, K,
          ksplit, beta, ablk, bblk, Mv, Nv};
  const int rc = !ta && tb ? q_launch_epi<false, true>(ksplit > 1 ? 0 : epi, a, st)
                 : !ta   ? q_launch_epi<false, false>(ksplit > 1 ? 0 : epi, a, st)
                         : q_launch_epi<true, false>(ksplit > 1 ? 0 : epi, a, st);
  if (rc) return rc;
  if (ksplit > 1 && C) launch_splitk_reduce(slab, ksplit, M, N, C, ldc, epi == 1 ? bias : nullptr, beta, Mv, Nv, st);
  if (epi == kQDGelu && part && colsum) {
    const float* parts[1] = {part};
    float* outs[1] = {colsum};
    launch_reduce_rows(parts, outs, 1, M / QT, N, colsum_acc, st);
  }
  return 0;
}

int launch_gemm_h3p(int ta, int tb, int M, int N, int K, const void* A, int64_t lda, int64_t a_ps, const int8_t* ea,
                    int64_t lde_a, const void* B, int64_t ldb, int64_t b_ps, const int8_t* eb, int64_t lde_b, float* C,
                    int64_t ldc, const float* bias, int epi, float beta, float* aux, int64_t ldaux, float* part,
                    float* colsum, int colsum_acc, void* cp, int64_t ldcp, int64_t cp_ps, int8_t* ec, int64_t lde_c,
                    int ksplit, float* slab, int64_t slab_floats, int ablk, int bblk, hipStream_t st) {
  return launch_gemm_h3p_v(ta, tb, M, N, K, A, lda, a_ps, ea, lde_a, B, ldb, b_ps, eb, lde_b, C, ldc, bias, epi, beta,
                           aux, ldaux, part, colsum, colsum_acc, cp, ldcp, cp_ps, ec, lde_c, ksplit, slab, slab_floats,
                           ablk, bblk, 0, 0, st);
}

int launch_h3p_colpart(const void* pl, int64_t ld, int64_t ps, const int8_t* ex, int64_t lde, int rows, int cols,
                       float* part, hipStream_t st) {
  if (rows <= 0 || rows % 32 || cols <= 0 || cols % 32 || ld % 32 || ps % 2) return -1;
  hipLaunchKernelGGL(h3p_colpart_kernel, dim3((cols + 255) / 256, rows / 32), dim3(128), 0, st,
                     static_cast<const uint16_t*>(pl), ld, ps, ex, lde, cols, part);
  return 0;
}

// fp32 [rows][cols] (row stride lds) -> h3p planes (row stride ldd, plane stride ps) + exponents; source
// rows from vrows on (0: rows) are not read and split as zeros
int launch_h3p_split(const float* src, int64_t lds, int rows, int cols, void* dst, int64_t ldd, int64_t ps, int8_t* ex,
                     int64_t lde, int blocked, int vrows, hipStream_t st) {
  vrows = vrows > 0 ? vrows : rows;
  if (rows <= 0 || cols <= 0 || rows % 32 || cols % 32 || lds % 4 || ldd % 4 || ps % 4 || vrows > rows) return -1;
  if (blocked && ldd % 32) return -1;
  if ((reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 7)) return -1;
  QSplitSeg s{src, static_cast<uint16_t*>(dst), ex, lds, ldd, ps, lde, rows, cols, 0, blocked, vrows, 0};
  const int total = (rows / 32) * (cols / 32);
  hipLaunchKernelGGL(h3p_split_kernel, dim3((total + 3) / 4), dim3(256), 0, st, s, nullptr, 1, total);
  return 0;
}

// several tensors in one launch: `table` = nseg QSplitSeg records in device memory (blk0 ascending,
// built by the caller with h3p_split_seg_bytes / the Python packer), `total` = all their blocks
int h3p_split_seg_bytes() { return static_cast<int>(sizeof(QSplitSeg)); }
void launch_h3p_split_multi(const void* table, int nseg, int total, hipStream_t st) {
  QSplitSeg none{};
  hipLaunchKernelGGL(h3p_split_kernel, dim3((total + 3) / 4), dim3(256), 0, st, none,
                     static_cast<const QSplitSeg*>(table), nseg, total);
}
