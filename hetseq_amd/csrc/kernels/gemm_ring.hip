// fp32 GEMM on pre-split bf16 planes, LDS-DMA ring pipeline (K01/K03/K04 GEMM parts).
//
//   C[M,N] = beta*C + op(A)[M,K] * op(B)[K,N]  (+ bias / GELU / dGELU epilogue)
//
// Operands are three bf16 planes x = hi + mid + lo (|x - sum| <= 2^-27 |x|, see
// gemm_planes.hip) and every fp32 product is the six cross terms of order <= 2^-16,
// accumulated in fp32 -- fp32-level error on the bf16 matrix cores.
//
// Why a second plane kernel.  gemm_planes_kernel (and the in-kernel-split gemm_x6s_kernel)
// use 128x128 tiles, one LDS-DMA stage in flight and a vmcnt(0) + barrier per K tile: the
// "2-barrier" structure whose ceiling the CDNA guide puts near 900 TF/s, and 128x128 tiles
// that quantise badly on 256 CUs for BERT's M = 4096 products (4096 x 768: 192 tiles;
// 4096 x 2304: 576 = 2.25 rounds).  This kernel is built around the MI355X instead:
//
//  * tile 128 x BN with BN = 96 or 128 chosen per shape (launcher): 4096 x 768 -> 256 tiles
//    (one per CU), 4096 x 2304 -> 768 (three rounds), 4096 x 3072 -> 768 of 128 x 128;
//  * a THREE-stage LDS ring (P = 3 planes x (128 + BN) x 32 bf16 = 42 / 48 KB per stage,
//    126 / 144 KB in all; one workgroup per CU): the DMA of tile t+3 is issued as soon as
//    tile t's fragments are in registers, so two tiles are always in flight;
//  * counted `s_waitcnt vmcnt(NJ)` (never 0 inside the loop) and ONE raw `s_barrier` per K
//    tile, all LDS in one __shared__ array, no ordinary global loads in the loop (the three
//    compiler traps of the guide's projection-GEMM notes);
//  * fragments of tile t+1 are read (ds_read_b128 / ds_read_b64_tr_b16) while tile t's 6 x
//    4 x (BN/32) MFMAs run; v_mfma_f32_16x16x32_bf16 (the shape that holds the higher clock
//    under load on gfx950);
//  * LDS images written lane-linearly by global_load_lds_dwordx4, swizzled through the
//    per-lane SOURCE address: k-contiguous [rows][32] images XOR their 16-B chunk with
//    (-(row >> 2)) & 3 (conflict-free for the 16x16x32 operand's ds_read_b128 lane groups);
//    mn-contiguous [32 k][R] images (dgrad weight, both weight-gradient operands) are read
//    with the transposing ds_read_b64_tr_b16 and XOR their 32-B column blocks so the two
//    16-lane groups of a half (k rows 8 apart) hit different banks;
//  * block ids remapped XCD-contiguously (bijective), grouped 4 M-tiles x all N-tiles;
//  * split-K into fp32 slabs (splitk_reduce_kernel, fixed order) for the weight gradients.
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "reduce.h"

namespace hs {
namespace ring {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef short s8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

enum { kNone = 0, kBias = 1, kGelu = 2, kDGelu = 3 };
constexpr int BM = 128, BK = 32, P = 3, NS = 3, NT = 256;

struct Args {
  const uint16_t* A;  // plane 0 of op(A)'s storage; plane p at A + p * a_ps (elements)
  const uint16_t* B;
  float* C;
  const float* bias;
  float* aux;      // kGelu: pre-activation out; kDGelu: pre-activation in
  float* part;     // kDGelu: [M/128][N] column partial sums
  float* slab;     // split-K: [ksplit][M][N] fp32 partial products
  uint16_t* outp;  // optional: C written again as three bf16 planes (plane stride o_ps, row stride ldc)
  int64_t lda, ldb, ldc, ldaux, a_ps, b_ps, o_ps;
  int M, N, K, ksplit;
  float beta;
};

// LDS image of one operand plane: R rows of op(X) (m or n) x BK of k.
template <int R, bool KC>
struct Img {
  static constexpr int bytes = R * BK * 2;
  static constexpr int row_bytes = KC ? BK * 2 : R * 2;  // [R][32] or [32][R]
  // stored 16-B chunk position of logical chunk c in LDS row `row` (an involution)
  HS_DEVICE static int pos(int row, int c) {
    if (KC) return c ^ ((-(row >> 2)) & 3);
    if (R == 128) return c ^ (2 * ((row & 3) | (((row >> 3) & 1) << 2)));
    return c ^ (2 * ((row >> 3) & 1));  // R = 96: 192-B rows already spread 4 rows over the banks
  }
};

HS_DEVICE f4 mma(bf8 a, bf8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

// One LDS read of a fragment piece.  Fragment of plane `pl` for the 16 rows (of op(X)) starting at
// `rc`: lane l holds row rc + (l & 15), k = 8 (l >> 4) .. + 7 -- the 16x16x32 A and B operand map
// (identical for both operands).  A k-contiguous image gives the whole fragment in one
// ds_read_b128 (both halves); an mn-contiguous one takes two transposing ds_read_b64_tr_b16
// (half jj: k rows 8g + 4jj + q of 16-lane group g; lane 4q+p' addresses columns rc + 4p'..+3).
template <int R, bool KC>
HS_DEVICE void frag_piece(s4 (&dst)[2], const char* img, int pl, int rc, int jj, int lane) {
  using I = Img<R, KC>;
  const char* base = img + pl * I::bytes;
  if (KC) {
    const int r = rc + (lane & 15), c = lane >> 4;
    const s8 v = *reinterpret_cast<const s8*>(base + r * I::row_bytes + 16 * I::pos(r, c));
    dst[0] = s4{v[0], v[1], v[2], v[3]};
    dst[1] = s4{v[4], v[5], v[6], v[7]};
    return;
  }
  const int l16 = lane & 15, q = l16 >> 2, pp = l16 & 3, g = lane >> 4;
  const int col = rc + 4 * pp;
  const int row = 8 * g + 4 * jj + q;
  const char* a = base + row * I::row_bytes + 16 * I::pos(row, col >> 3) + 2 * (col & 7);
  dst[jj] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a));
}

HS_DEVICE bf8 as_frag(const s4 (&h)[2]) {
  const s8 u = {h[0].x, h[0].y, h[0].z, h[0].w, h[1].x, h[1].y, h[1].z, h[1].w};
  return __builtin_bit_cast(bf8, u);
}

// One LDS-DMA piece (1 KB per wave) as an asm statement: M0 = the wave-uniform LDS destination,
// written and restored inside the statement (M0 is compiler-reserved).  Hidden from hipcc on
// purpose: hipcc tracks builtin LDS-DMA writes and, unable to prove that a transposing LDS read
// does not alias them, drains vmcnt(0) before the first ds_read_b64_tr_b16 after every DMA issue --
// the whole ring in flight, every K tile.  The counts are ours (wait_vm), the ordering against the
// stage's readers is the workgroup barrier's.
HS_DEVICE void dma_piece(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst));
}

// Per-lane source offsets (bytes, from the operand's plane-0 base at the tile's k origin) of this
// wave's LDS-DMA pieces.  The first JA pieces of every wave are A's, the last JB B's (a compile-time
// split: no per-piece operand select).  A-piece j of wave w fills A-image KB min(4 j + w, NKA - 1),
// likewise for B: past an image's last KB a wave repeats the last one (identical bytes to the
// identical place: a benign duplicate that keeps every wave's piece count, hence its vmcnt, equal).
template <int BN, bool AK, bool BKc>
struct Dma {
  using IA = Img<BM, AK>;
  using IB = Img<BN, BKc>;
  static constexpr int SA = P * IA::bytes, NKA = SA / 1024, NKB = P * IB::bytes / 1024;
  static constexpr int JA = (NKA + 3) / 4, JB = (NKB + 3) / 4, NJ = JA + JB;
  HS_DEVICE static void offsets(uint32_t (&off)[NJ], int (&dst)[NJ], const Args& p, int m0, int n0, int w, int lane) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const bool b = j >= JA;
      const int gi = b ? min(4 * (j - JA) + w, NKB - 1) : min(4 * j + w, NKA - 1);
      dst[j] = (b ? SA : 0) + 1024 * gi;
      const int ob = 1024 * gi + 16 * lane;  // byte inside the operand's planes
      const int pbytes = b ? IB::bytes : IA::bytes, rbytes = b ? IB::row_bytes : IA::row_bytes;
      const bool kc = b ? BKc : AK;
      const int plane = ob / pbytes, ib = ob % pbytes;
      const int row = ib / rbytes, cpos = (ib % rbytes) / 16;
      const int c = b ? IB::pos(row, cpos) : IA::pos(row, cpos);  // pos is an involution
      const int64_t ld = b ? p.ldb : p.lda, ps = b ? p.b_ps : p.a_ps;
      const int mn0 = b ? n0 : m0;
      const int64_t e = kc ? (int64_t)(mn0 + row) * ld + 8 * c : (int64_t)row * ld + mn0 + 8 * c;
      off[j] = static_cast<uint32_t>(2 * (e + plane * ps));
    }
  }
};

// Waits go through __builtin_amdgcn_s_waitcnt (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] |
// lgkmcnt[11:8] | vmcnt_hi[15:14]) rather than inline asm: the compiler's own wait insertion then
// knows which loads have completed.  Had it not known that a barrier's lgkmcnt(0) retired the
// current fragments, it would wait for the NEXT tile's fragment reads (issued after the barrier)
// before the first MFMA, serialising the read / MFMA overlap.
template <int N_>
HS_DEVICE void wait_vm() {
  static_assert(N_ >= 0 && N_ < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N_ & 15) | ((N_ >> 4) << 14) | 0x70 | 0xF00);
}

HS_DEVICE void barrier_lds() {
  // this wave's fragment reads are back, then the workgroup barrier.  The sched_barriers keep the
  // machine scheduler from moving MFMAs or LDS reads across it; the asm statement's memory clobber
  // does the same for the IR passes.
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), vmcnt / expcnt untouched
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int BN, bool TA, bool TB, int EPI>
__global__ void __launch_bounds__(NT, 1) gemm_ring_kernel(Args p) {
  constexpr bool AK = !TA, BKc = TB;  // k-contiguous storage?
  using IA = Img<BM, AK>;
  using IB = Img<BN, BKc>;
  constexpr int SA = P * IA::bytes, STAGE = SA + P * IB::bytes;
  using D = Dma<BN, AK, BKc>;
  constexpr int NJ = D::NJ;  // DMA pieces per wave per tile
  constexpr int TM = 4, TN = BN / 32;         // 16x16 accumulator tiles per wave (wave tile 64 x BN/2)
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];

  // ---- block -> (tile, K slice): XCD-contiguous, groups of 4 M-tiles x all N-tiles, slice-major
  const int tiles_m = p.M / BM, tiles_n = p.N / BN, ntile = tiles_m * tiles_n, nwg = ntile * p.ksplit;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, qq = nwg / 8, rr = nwg % 8;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
  const int slice = wg / ntile, tile = wg % ntile;
  const int gsz = 4 * tiles_n, grp = tile / gsz, gm = min(4, tiles_m - 4 * grp);
  const int tm = 4 * grp + (tile % gsz) % gm, tn = (tile % gsz) / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kofs = slice * (p.K / p.ksplit);
  const int KT = p.K / p.ksplit / BK;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1, wm = 64 * wr, wn = (BN / 2) * wc;

  uint32_t off[NJ];
  int dst[NJ];
  D::offsets(off, dst, p, m0, n0, w, lane);
  const int64_t stepA = AK ? 2 * BK : 2 * (int64_t)BK * p.lda, stepB = BKc ? 2 * BK : 2 * (int64_t)BK * p.ldb;
  const char* ga = reinterpret_cast<const char*>(p.A) + (AK ? 2 * (int64_t)kofs : 2 * (int64_t)kofs * p.lda);
  const char* gb = reinterpret_cast<const char*>(p.B) + (BKc ? 2 * (int64_t)kofs : 2 * (int64_t)kofs * p.ldb);

  // tile t -> stage; past the last tile the DMA re-reads the last one (a stage nobody reads again),
  // so every step issues the same NJ pieces and the loop body is one basic block: the waits are
  // compile-time counts and the sched_barriers hold the source order below
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)smem));
  auto dma = [&](int j, int t, int stage) __attribute__((always_inline)) {
    const int tt = min(t, KT - 1);
    const char* src = (j >= D::JA ? gb + (int64_t)tt * stepB : ga + (int64_t)tt * stepA) + off[j];
    dma_piece(src, __builtin_amdgcn_readfirstlane(lds0 + stage * STAGE + dst[j]));
  };

  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  struct Frags {
    s4 a[P][TM][2], b[P][TN][2];
  };
  // fragment reads of a tile as a flat list of pieces: A (plane, i, half) then B (plane, j, half)
  constexpr int RA = AK ? 1 : 2, RB = BKc ? 1 : 2;
  constexpr int NRA = P * TM * RA, NRD = NRA + P * TN * RB;
  auto read_piece = [&](Frags& f, int stage, int r) __attribute__((always_inline)) {
    const char* img = smem + stage * STAGE;
    if (r < NRA) {
      const int pl = r / (TM * RA), i = (r / RA) % TM, jj = r % RA;
      frag_piece<BM, AK>(f.a[pl][i], img, pl, wm + 16 * i, jj, lane);
    } else {
      const int q = r - NRA, pl = q / (TN * RB), j = (q / RB) % TN, jj = q % RB;
      frag_piece<BN, BKc>(f.b[pl][j], img + SA, pl, wn + 16 * j, jj, lane);
    }
  };
  // the six cross terms, smallest first: lo*hi, hi*lo, mid*mid, mid*hi, hi*mid, hi*hi
  constexpr int PA[6] = {2, 0, 1, 1, 0, 0}, PB[6] = {0, 2, 1, 0, 1, 0};
  // 12 chunks of MFMAs (term tt = c / 2, accumulator rows i of half c % 2, all columns); between
  // them, in source order pinned by sched_barrier: one DMA piece per chunk, then the next tile's
  // fragment reads spread evenly -- the memory instructions issue under the matrix pipe
  constexpr int NCH = 12;
  static_assert(NJ <= NCH, "one DMA piece per chunk");
  auto step_body = [&](const Frags& f, Frags& nf, int t, int st_free, int st_next) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int tt = c >> 1, h = c & 1;
#pragma unroll
      for (int ii = 0; ii < TM / 2; ++ii) {
        const int i = 2 * h + ii;
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mma(as_frag(f.a[PA[tt]][i]), as_frag(f.b[PB[tt]][j]), acc[i][j]);
      }
      if (c < NJ) dma(c, t + 3, st_free);
#pragma unroll
      for (int r = 0; r < NRD; ++r)
        if (r >= c * NRD / NCH && r < (c + 1) * NRD / NCH) read_piece(nf, st_next, r);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- prologue: three tiles in flight, wait for the first
#pragma unroll
  for (int j = 0; j < NJ; ++j) dma(j, 0, 0);
#pragma unroll
  for (int j = 0; j < NJ; ++j) dma(j, 1, 1);
#pragma unroll
  for (int j = 0; j < NJ; ++j) dma(j, 2, 2);
  wait_vm<2 * NJ>();
  barrier_lds();
  Frags F[2];
#pragma unroll
  for (int r = 0; r < NRD; ++r) read_piece(F[0], 0, r);

  // ---- main loop, unrolled by two so the fragment sets keep static registers.  Step t: tile t+1
  // landed (this wave's part; t+2 stays in flight) -> barrier (tile t+1 visible to all, every
  // wave's reads of tile t done, so its stage is free) -> tile t's MFMAs with the DMA of tile t+3
  // into the freed stage and the reads of tile t+1's fragments interleaved
  int st0 = 0;  // stage of tile t
  auto step = [&](int t, auto par) __attribute__((always_inline)) {
    constexpr int cur = decltype(par)::value;
    const int st1 = st0 == 2 ? 0 : st0 + 1;
    wait_vm<NJ>();
    barrier_lds();
    step_body(F[cur], F[cur ^ 1], t, st0, st1);
    st0 = st1;
  };
  int t = 0;
  for (; t + 1 < KT; t += 2) {
    step(t, std::integral_constant<int, 0>{});
    step(t + 1, std::integral_constant<int, 1>{});
  }
  if (t < KT) step(t, std::integral_constant<int, 0>{});
  wait_vm<0>();  // the trailing re-read DMAs land before LDS is reused or released
  barrier_lds();

  // ---- epilogue.  The accumulators are staged through LDS (the ring's stages, free now) as the fp32
  // tile T[128][BN], then finished row-contiguously: each thread owns 8 consecutive columns of a
  // row, so every global access -- C, the pre-activation, the split-K slab, the three output planes
  // -- is a 16-B (or 3 x 16-B) vector instead of a 4-B (2-B for planes) access per MFMA register.
  // acc[i][j][r] is row wm + 16 i + 4 (lane >> 4) + r, column wn + 16 j + (lane & 15) of the tile.
  constexpr int LDT = BN + 4;  // padded rows: the four 16-lane groups' rows 4 apart hit disjoint banks
  static_assert(BM * LDT * 4 <= NS * STAGE, "epilogue tile fits the ring");
  float* T = reinterpret_cast<float*>(smem);
  {
    const int lr = lane & 15, lq = lane >> 4;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) T[(wm + 16 * i + 4 * lq + r) * LDT + wn + 16 * j + lr] = acc[i][j][r];
  }
  barrier_lds();
  constexpr int NG = BN / 8;  // 8-column groups per row
  typedef float f8 __attribute__((ext_vector_type(8)));
  auto ld8 = [](const float* q) __attribute__((always_inline)) {
    const f4 x = *reinterpret_cast<const f4*>(q), y = *reinterpret_cast<const f4*>(q + 4);
    return f8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  };
  auto st8 = [](float* q, f8 v) __attribute__((always_inline)) {
    *reinterpret_cast<f4*>(q) = f4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f4*>(q + 4) = f4{v[4], v[5], v[6], v[7]};
  };
  if (p.ksplit > 1) {  // plain fp32 partial slab; bias / beta / the sum in splitk_reduce_kernel
    float* sl = p.slab + (int64_t)slice * p.M * p.N;
    for (int u = threadIdx.x; u < BM * NG; u += NT) {
      const int row = u / NG, c = (u % NG) * 8;
      st8(sl + (int64_t)(m0 + row) * p.N + n0 + c, ld8(T + row * LDT + c));
    }
    return;
  }
  // the runtime options (beta-accumulate, plane output, fp32 output) become template flags: a
  // per-element branch around a load makes hipcc wait vmcnt(0) for every element
  auto finish = [&](auto use_beta, auto use_planes, auto write_c) __attribute__((always_inline)) {
    constexpr bool UB = decltype(use_beta)::value, UP = decltype(use_planes)::value, WC = decltype(write_c)::value;
    for (int u = threadIdx.x; u < BM * NG; u += NT) {
      const int row = u / NG, c = (u % NG) * 8;
      const int64_t m = m0 + row;
      const int n = n0 + c;
      const f8 a = ld8(T + row * LDT + c);
      const f8 bv = EPI != kNone ? ld8(p.bias + n) : f8{};
      f8 v;
      if (EPI == kGelu) {
        st8(p.aux + m * p.ldaux + n, a);  // the un-biased pre-activation, for the backward
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = gelu_f(a[k] + bv[k]);
      } else if (EPI == kDGelu) {
        const f8 pre = ld8(p.aux + m * p.ldaux + n);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = a[k] * gelu_grad_f(pre[k] + bv[k]);
        st8(T + row * LDT + c, v);  // kept for the bias-gradient column sums below
      } else {
        v = a + bv;
        if (UB) v += p.beta * ld8(p.C + m * p.ldc + n);
      }
      if (WC) st8(p.C + m * p.ldc + n, v);
      if (UP) {  // the value again as planes, for the GEMMs that consume it
        const float lo4[4] = {v[0], v[1], v[2], v[3]}, hi4[4] = {v[4], v[5], v[6], v[7]};
        store4_planes(p.outp, p.o_ps, m * p.ldc + n, lo4);
        store4_planes(p.outp, p.o_ps, m * p.ldc + n + 4, hi4);
      }
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (EPI >= kGelu) {  // fused-activation outputs: planes only when the fp32 copy has no reader (C null)
    if (p.outp && p.C) finish(F_{}, T_{}, T_{});
    else if (p.outp) finish(F_{}, T_{}, F_{});
    else finish(F_{}, F_{}, T_{});
  } else if (p.beta != 0.f) {
    finish(T_{}, F_{}, T_{});
  } else {
    finish(F_{}, F_{}, T_{});
  }
  if (EPI == kDGelu) {  // column sums of the block's 128 rows, fixed order (deterministic)
    barrier_lds();
    for (int c = threadIdx.x; c < BN; c += NT) {
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
      for (int row = 0; row < BM; row += 4) {
        s0 += T[row * LDT + c];
        s1 += T[(row + 1) * LDT + c];
        s2 += T[(row + 2) * LDT + c];
        s3 += T[(row + 3) * LDT + c];
      }
      p.part[(int64_t)tm * p.N + n0 + c] = (s0 + s1) + (s2 + s3);
    }
  }
}

// BN for an M x N problem: the smaller work per CU over the rounds a 256-CU chip needs
// (ceil(tiles / 256) * BN columns of 128-row tiles), the wider tile on a tie
inline int pick_bn(int M, int N) {
  const bool ok96 = N % 96 == 0, ok128 = N % 128 == 0;
  if (!ok96 && !ok128) return 0;
  if (!ok96) return 128;
  if (!ok128) return 96;
  const long t96 = (long)(M / BM) * (N / 96), t128 = (long)(M / BM) * (N / 128);
  const long w96 = (t96 + 255) / 256 * 96, w128 = (t128 + 255) / 256 * 128;
  return w128 <= w96 ? 128 : 96;
}

template <int BN>
int launch_bn(int ta, int tb, int epi, const Args& a, hipStream_t st) {
  const dim3 grid((a.M / BM) * (a.N / BN) * a.ksplit), blk(NT);
#define HS_RING(TA_, TB_, E_) hipLaunchKernelGGL((gemm_ring_kernel<BN, TA_, TB_, E_>), grid, blk, 0, st, a)
  if (!ta && tb) {  // forward X W^T
    if (epi == kNone) HS_RING(false, true, kNone);
    else if (epi == kBias) HS_RING(false, true, kBias);
    else if (epi == kGelu) HS_RING(false, true, kGelu);
    else return -1;
  } else if (!ta && !tb) {  // dgrad dY W
    if (epi == kNone) HS_RING(false, false, kNone);
    else if (epi == kDGelu) HS_RING(false, false, kDGelu);
    else return -1;
  } else if (ta && !tb) {  // wgrad dY^T X
    if (epi == kNone) HS_RING(true, false, kNone);
    else return -1;
  } else {
    return -1;
  }
#undef HS_RING
  return 0;
}

}  // namespace ring
}  // namespace hs

void launch_splitk_reduce(const float* slab, int ksplit, int M, int N, float* C, int64_t ldc, const float* bias,
                          float beta, int Mv, int Nv, hipStream_t st);

// Returns -1 (nothing launched) when the shape is not served: M % 128, N % 96 and N % 128, K % (32 ksplit),
// 16-B aligned plane rows, fused epilogues with a K split.  bn: 0 = pick, else 96 / 128.
int launch_gemm_ring(int ta, int tb, int M, int N, int K, const void* A, int64_t lda, int64_t a_ps, const void* B,
                     int64_t ldb, int64_t b_ps, float* C, int64_t ldc, const float* bias, int epi, float beta,
                     float* aux, int64_t ldaux, float* part, float* colsum_out, int colsum_acc, int ksplit,
                     float* slab, int64_t slab_floats, void* outp, int64_t o_ps, int bn, hipStream_t st) {
  using namespace hs::ring;
  ksplit = std::max(1, ksplit);
  if (bn == 0) bn = pick_bn(M, N);
  if (bn == 128 && ta && N % 96 == 0) bn = 96;  // the 128-wide weight-gradient build spills
  if ((bn != 96 && bn != 128) || M <= 0 || N <= 0 || K <= 0 || M % BM || N % bn || K % (BK * ksplit)) return -1;
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al16(A) || !al16(B) || lda % 8 || ldb % 8 || a_ps % 8 || b_ps % 8) return -1;
  if ((epi >= 1 && !bias) || (epi >= 2 && (!aux || beta != 0.f)) || (epi == 3 && (!part || !colsum_out))) return -1;
  if (ksplit > 1 && (epi > 1 || outp || !slab || (int64_t)ksplit * M * N > slab_floats || N % 4 || ldc % 4))
    return -1;
  if (outp && (epi < 2 || o_ps <= 0)) return -1;  // plane outputs: the GELU / dGELU epilogues only
  if (!C && !outp) return -1;
  // the row-contiguous epilogue moves 8 columns per thread as 16-B vectors (planes: 8-B pieces)
  if ((C && (!al16(C) || ldc % 4)) || (aux && (!al16(aux) || ldaux % 4)) || (bias && !al16(bias)) ||
      (outp && ((reinterpret_cast<uintptr_t>(outp) & 7) || o_ps % 4 || ldc % 4)) || (slab && !al16(slab)))
    return -1;
  // 32-bit per-lane DMA offsets: the operand span (all planes) must stay below 4 GiB
  const int64_t spanA = 2 * (2 * a_ps + (int64_t)(ta ? K : M) * lda);
  const int64_t spanB = 2 * (2 * b_ps + (int64_t)(tb ? N : K) * ldb);
  if (spanA >= (1ll << 32) || spanB >= (1ll << 32)) return -1;
  Args a{static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), C, bias, aux, part, slab,
         static_cast<uint16_t*>(outp), lda, ldb, ldc, ldaux, a_ps, b_ps, o_ps, M, N, K, ksplit, beta};
  const int rc = bn == 96 ? launch_bn<96>(ta, tb, epi, a, st) : launch_bn<128>(ta, tb, epi, a, st);
  if (rc) return rc;
  if (ksplit > 1) launch_splitk_reduce(slab, ksplit, M, N, C, ldc, epi == 1 ? bias : nullptr, beta, M, N, st);
  if (epi == kDGelu) {
    const float* parts[1] = {part};
    float* outs[1] = {colsum_out};
    hs::launch_reduce_rows(parts, outs, 1, M / BM, N, colsum_acc, st);
  }
  return 0;
}
