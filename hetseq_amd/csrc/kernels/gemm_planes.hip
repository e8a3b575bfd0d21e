// bf16 MFMA GEMM on "plane" operands (the --dtype bf16 step's hand-written GEMMs).
//
//   C[M,N] = beta*C + op(A)[M,K] * op(B)[K,N]  (+ bias / GELU / dGELU epilogue)
//
// Operands are bf16 matrices (P = 1: the bf16 activation / weight shadow itself).
// The kernel template keeps a plane count P, but only P = 1 is instantiated: the
// split-bf16 fp32 engine (P = 3, six cross products) was retired in round 5 for the
// three-product fp16 block-scaled engine (gemm_h3p.hip), which reads half the bytes.
// The K loop is pure data movement + MFMA:
//
//  * tiles of 128x128, 4 waves (2x2, 64x64 each = 2x2 v_mfma_f32_32x32x16_bf16
//    accumulators), BK = 32 (P = 3) or 64 (P = 1);
//  * both operand layouts are served from LDS without any transpose pass:
//      k-contiguous source (A for TA=0, B for TB=1): image [128 rows][BK] read with
//        ds_read_b128, 16-B chunks XOR-swizzled by row (conflict-free for the
//        32x32x16 operand map);
//      mn-contiguous source (TA=1 / TB=0: the dgrad weight and both weight-gradient
//        operands): image [BK rows][128] read with ds_read_b64_tr_b16 (the gfx950
//        transposing LDS read: 4 k-rows of 16 columns per 16-lane group), chunks
//        XOR-swizzled by 4*(row & 3) (conflict-free per 32-lane half);
//  * staging is global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip): the LDS image
//    is written lane-linearly, so the swizzle lives in each lane's SOURCE address;
//    two LDS stages, the next K tile in flight under the current tile's MFMAs, one
//    vmcnt(0) + barrier per K tile, all LDS in one __shared__ array;
//  * block ids are remapped XCD-contiguously (bijective for any grid) and grouped
//    8 M-tiles x all N-tiles so an XCD's resident blocks share operand panels in
//    its private L2;
//  * optional split-K into fp32 slabs (summed in fixed order by splitk_reduce_kernel
//    in gemm.hip) for the K = 4096 weight gradients whose tile grids are small.
// Epilogue (shared by both P): C in fp32 or bf16, + bias, beta-accumulate, GELU
// (pre-activation kept in aux), dGELU with per-block column partials of the bias
// gradient (finalised by reduce_rows).
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "reduce.h"

namespace hs {

typedef __bf16 pbf8 __attribute__((ext_vector_type(8)));
typedef short ps4 __attribute__((ext_vector_type(4)));
typedef float pf16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

enum { kPEpiNone = 0, kPEpiBias = 1, kPEpiGelu = 2, kPEpiDGelu = 3 };
constexpr int kPB = 128;  // block tile (rows and columns)

struct PlanesArgs {
  const uint16_t* A;  // plane 0 of op(A)'s storage; plane p at A + p * a_ps
  const uint16_t* B;
  void* C;
  const float* bias;
  void* aux;    // kEpiGelu: pre-activation out; kEpiDGelu: pre-activation in (same dtype as C)
  float* part;  // kEpiDGelu: [M/128][N] column partial sums
  float* slab;  // split-K: [ksplit][M][N] fp32 partial products
  int64_t lda, ldb, ldc, ldaux, a_ps, b_ps;
  int M, N, K, ksplit;
  float beta;
  int slice_major;  // split-K block order (see gemm.hip): 1 = slice-major
  int Mv;           // valid rows of a padded problem (fp32 C, plain / bias epilogue): rows from Mv on are not written
};

// LDS image geometry of one operand plane (128 x BK bf16 elements either way).
template <int BK, bool KCONTIG>
struct PImg {
  static constexpr int bytes = kPB * BK * 2;
  static constexpr int row_bytes = KCONTIG ? BK * 2 : kPB * 2;  // 64 / 128 or 256
  static constexpr int chunks = row_bytes / 16;                 // 16-B chunks per row
  // chunk swizzle of row r: k-contiguous rows spread the b128 row reads of 16 lanes over
  // all 16 bank quads; mn-contiguous (256-B) rows put the 4 k-rows of a transposed read
  // into 4 different quarters of the bank row
  HS_DEVICE static int swz(int r) {
    if (KCONTIG) return (r >> (row_bytes == 32 ? 3 : row_bytes == 64 ? 2 : 1)) & (chunks - 1);
    return 4 * (r & 3);
  }
};

// Per-lane source byte offsets (from the plane-0 base at k = 0) of this wave's LDS-DMA
// instructions for one operand: instruction j writes image bytes [1024 * (4 j + w), +1024)
// of the operand's P planes.
template <int BK, bool KCONTIG, int NJ, int WV>
HS_DEVICE void dma_offsets(uint32_t* off, int64_t ld, int64_t ps, int mn0, int w, int lane) {
  using I = PImg<BK, KCONTIG>;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int byte = 1024 * (WV * j + w) + 16 * lane;
    const int plane = byte / I::bytes, ib = byte % I::bytes;
    const int row = ib / I::row_bytes, cl = (ib % I::row_bytes) / 16;
    const int gc = cl ^ I::swz(row);  // the chunk this LDS position holds
    const int64_t e = KCONTIG ? (int64_t)(mn0 + row) * ld + 8 * gc   // [mn][k]: row = mn, chunk = 8 k
                              : (int64_t)row * ld + mn0 + 8 * gc;    // [k][mn]: row = k, chunk = 8 mn
    off[j] = static_cast<uint32_t>(2 * (e + plane * ps));
  }
}

template <int NJ, int WV>
HS_DEVICE void dma_issue(const char* base, const uint32_t* off, char* img, int w) {
#pragma unroll
  for (int j = 0; j < NJ; ++j)
    __builtin_amdgcn_global_load_lds((gbl_void_t*)(base + off[j]), (lds_void_t*)(img + 1024 * (WV * j + w)), 16, 0, 0);
}

// MFMA operand (8 consecutive k of one row / column) of plane p for the 32-wide tile at
// `rc` (row of op(A) or column of op(B)), k-slice ks of the stage.
template <int BK, bool KCONTIG>
HS_DEVICE pbf8 frag(const char* img, int p, int rc, int ks, int lane) {
  using I = PImg<BK, KCONTIG>;
  const char* pl = img + p * I::bytes;
  if (KCONTIG) {
    const int r = rc + (lane & 31), c = 2 * ks + (lane >> 5);
    return *reinterpret_cast<const pbf8*>(pl + r * I::row_bytes + 16 * (c ^ I::swz(r)));
  } else {
    // transposed read: lane 4q+p' of a 16-lane group addresses k-row k0+q, columns c0+4p'..+3
    const int l16 = lane & 15, q = l16 >> 2, pp = l16 & 3, g = lane >> 4;
    const int col = rc + 16 * (g & 1) + 4 * pp;
    ps4 v[2];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int row = 16 * ks + 8 * (g >> 1) + 4 * jj + q;
      const char* a = pl + row * I::row_bytes + 16 * ((col >> 3) ^ I::swz(row)) + 2 * (col & 7);
      v[jj] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) ps4*)(a));
    }
    typedef short ps8 __attribute__((ext_vector_type(8)));
    const ps8 u = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
    return __builtin_bit_cast(pbf8, u);
  }
}

HS_DEVICE pf16 mma16(pbf8 a, pbf8 b, pf16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0); }
HS_DEVICE int acc_row(int r, int q) { return (r & 3) + 8 * (r >> 2) + 4 * q; }

HS_DEVICE void store_c(float* p, float v) { *p = v; }
HS_DEVICE void store_c(bf16_t* p, float v) { *p = from_f<bf16_t>(v); }
HS_DEVICE float load_c(const float* p) { return *p; }
HS_DEVICE float load_c(const bf16_t* p) { return to_f(*p); }
template <typename TC>
HS_DEVICE float round_c(float v) { return to_f(from_f<TC>(v)); }

// waves per SIMD the block may count on: the blocks per CU its LDS image allows, capped so the
// register budget stays >= 128 VGPRs (4 waves: 3 blocks, 8 waves: 2 blocks); WV / 4 waves per SIMD
// per block
template <int P, int BK, int STAGES, int WV>
constexpr int planes_waves_per_simd() {
  constexpr int by_lds = (160 * 1024) / (STAGES * P * 2 * kPB * BK * 2);
  constexpr int cap = WV == 8 ? 2 : 3;
  return (by_lds < cap ? by_lds : cap) * (WV / 4);
}

// WV = 4: 2x2 waves of 64x64 (2x2 accumulators each, one wave per SIMD per block);
// WV = 8: 2x4 waves of 64x32 (2x1 accumulators, two waves per SIMD: one wave's LDS-DMA issue
//         overlaps its partner's MFMAs)
template <int P, int BK, int STAGES, int WV, bool TA, bool TB, int EPI, typename TC>
__global__ void __launch_bounds__(64 * WV, (planes_waves_per_simd<P, BK, STAGES, WV>()))
    gemm_planes_kernel(PlanesArgs p) {
  constexpr bool AK = !TA, BKc = TB;  // k-contiguous storage?
  using IA = PImg<BK, AK>;
  using IB = PImg<BK, BKc>;
  constexpr int STAGE = P * (IA::bytes + IB::bytes);
  constexpr int NA = P * IA::bytes / (1024 * WV), NB = P * IB::bytes / (1024 * WV);
  constexpr int WC = WV / 2, TN = 2 / (WV / 4);  // wave columns, 32-wide accumulator columns per wave
  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE];

  const int tiles_m = p.M / kPB, tiles_n = p.N / kPB, nwg = tiles_m * tiles_n * p.ksplit;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, qq = nwg / 8, rr = nwg % 8;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + orig / 8;
  const int ntile = tiles_m * tiles_n;
  const int slice = p.slice_major ? wg / ntile : wg % p.ksplit, tile = p.slice_major ? wg % ntile : wg / p.ksplit;
  const int gsz = 8 * tiles_n, grp = tile / gsz, gm = min(8, tiles_m - 8 * grp);
  const int tm = 8 * grp + (tile % gsz) % gm, tn = (tile % gsz) / gm;
  const int m0 = tm * kPB, n0 = tn * kPB;
  const int kofs = slice * (p.K / p.ksplit);
  const int KT = p.K / p.ksplit / BK;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w / WC, wc = w % WC, wm = 64 * wr, wn = (kPB / WC) * wc;

  uint32_t offA[NA], offB[NB];
  dma_offsets<BK, AK, NA, WV>(offA, p.lda, p.a_ps, m0, w, lane);
  dma_offsets<BK, BKc, NB, WV>(offB, p.ldb, p.b_ps, n0, w, lane);
  // K-tile advance of the (wave-uniform) source bases, in bytes
  const int64_t stepA = AK ? 2 * BK : 2 * (int64_t)BK * p.lda, stepB = BKc ? 2 * BK : 2 * (int64_t)BK * p.ldb;
  const char* ga = reinterpret_cast<const char*>(p.A) + (AK ? 2 * (int64_t)kofs : 2 * (int64_t)kofs * p.lda);
  const char* gb = reinterpret_cast<const char*>(p.B) + (BKc ? 2 * (int64_t)kofs : 2 * (int64_t)kofs * p.ldb);

  pf16 acc[2][TN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = pf16{};

  // product terms (plane of A, plane of B), smallest first
  constexpr int NTERM = P == 3 ? 6 : 1;
  constexpr int TA_[6] = {2, 0, 1, 1, 0, 0}, TB_[6] = {0, 2, 1, 0, 1, 0};
  constexpr int T0 = P == 3 ? 0 : 5;

  // One wave per SIMD (the x6 image needs 96 KB of LDS): the fragment reads of k-slice ks+1 are
  // issued before the MFMAs of slice ks, and the next tile's first slice right after the
  // barrier that publishes its DMA, so LDS latency hides under MFMAs.
  constexpr int NKS = BK / 16;
  struct Frags {
    pbf8 a[P][2], b[P][TN];
  };
  auto read = [&](Frags& f, const char* stage, int ks) {
#pragma unroll
    for (int pl = 0; pl < P; ++pl)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        f.a[pl][i] = frag<BK, AK>(stage, pl, wm + 32 * i, ks, lane);
        if (i < TN) f.b[pl][i] = frag<BK, BKc>(stage + P * IA::bytes, pl, wn + 32 * i, ks, lane);
      }
  };
  auto mma = [&](const Frags& f) {
#pragma unroll
    for (int tt = T0; tt < T0 + NTERM; ++tt)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mma16(f.a[TA_[tt]][i], f.b[TB_[tt]][j], acc[i][j]);
  };

  Frags f[2];
  if constexpr (STAGES == 1) {
    // one LDS image: DMA, wait, compute, and a barrier before the next DMA overwrites it; the
    // other blocks resident on the CU (LDS allows 3) fill the MFMA pipe meanwhile
    for (int t = 0; t < KT; ++t) {
      dma_issue<NA, WV>(ga + t * stepA, offA, smem, w);
      dma_issue<NB, WV>(gb + t * stepB, offB, smem + P * IA::bytes, w);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      read(f[0], smem, 0);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        if (ks + 1 < NKS) read(f[(ks + 1) & 1], smem, ks + 1);
        mma(f[ks & 1]);
      }
      __syncthreads();
    }
  } else {
  dma_issue<NA, WV>(ga, offA, smem, w);
  dma_issue<NB, WV>(gb, offB, smem + P * IA::bytes, w);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  read(f[0], smem, 0);
  // one K tile; the fragment set a slice uses alternates, so with an odd slice count the parity
  // flips per tile: PAR (the tile's parity, compile-time) keeps every index static
  auto tile = [&](int t, auto par) {
    constexpr int F0 = decltype(par)::value * NKS;
    const char* cur = smem + (t & 1) * STAGE;
    char* nxt = smem + ((t + 1) & 1) * STAGE;
    if (t + 1 < KT) {  // the other stage was last read before the previous barrier
      dma_issue<NA, WV>(ga + (t + 1) * stepA, offA, nxt, w);
      dma_issue<NB, WV>(gb + (t + 1) * stepB, offB, nxt + P * IA::bytes, w);
    }
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (ks + 1 < NKS) {
        read(f[(F0 + ks + 1) & 1], cur, ks + 1);
        mma(f[(F0 + ks) & 1]);
      } else {
        // keep the previous slice's MFMAs ahead of the barrier (the scheduler would sink them
        // past it, exposing the last slice's LDS reads to the barrier's lgkmcnt(0))
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // tile t+1 landed in every wave's share; nobody reads tile t any more
        if (t + 1 < KT) read(f[(F0 + ks + 1) & 1], nxt, 0);
        mma(f[(F0 + ks) & 1]);
      }
    }
  };
  for (int t = 0; t < KT; t += 2) {
    tile(t, std::integral_constant<int, 0>{});
    if (t + 1 < KT) tile(t + 1, std::integral_constant<int, 1>{});
  }
  }  // STAGES == 2

  // ---------------- epilogue: register r of acc[i][j] -> row m0+wm+32i+acc_row(r,q), col n0+wn+32j+lr
  const int lr = lane & 31, q = lane >> 5;
  if (p.ksplit > 1) {  // plain fp32 partial slab; bias / beta / sum in splitk_reduce_kernel
    float* sl = p.slab + (int64_t)slice * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          sl[(int64_t)(m0 + wm + 32 * i + acc_row(r, q)) * p.N + n0 + wn + 32 * j + lr] = acc[i][j][r];
    return;
  }
  TC* C = static_cast<TC*>(p.C);
  TC* aux = static_cast<TC*>(p.aux);
  if constexpr (sizeof(TC) == 2) {
    // bf16 C: stage the fp32 tile through LDS in two 64-row halves (32 KB, the smallest stage of
    // any variant) and finish it row-contiguously: 8 columns per thread, one 16-B load of the
    // bias / pre-activation / old C and one 16-B store per 8 outputs instead of per-register
    // 2-B accesses.  dGELU column sums: per-thread partials over its rows, then a fixed-order
    // LDS reduction (deterministic).
    static_assert(STAGES * STAGE >= 64 * kPB * 4, "epilogue staging fits the operand buffers");
    float* T = reinterpret_cast<float*>(smem);
    constexpr int NT = 64 * WV, GRP = NT / 16;  // threads; threads sharing a column group
    const int cg = (threadIdx.x & 15) * 8;
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (EPI != kPEpiNone) {
      const float4 b0 = *reinterpret_cast<const float4*>(p.bias + n0 + cg);
      const float4 b1 = *reinterpret_cast<const float4*>(p.bias + n0 + cg + 4);
      bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w; bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
    }
    auto unpack = [](uint4 u, float (&v)[8]) {
      const uint32_t x[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[2 * k] = __uint_as_float(x[k] << 16);
        v[2 * k + 1] = __uint_as_float(x[k] & 0xffff0000u);
      }
    };
    auto pack = [](const float (&v)[8]) {
      uint32_t x[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        x[k] = (uint32_t)from_f<bf16_t>(v[2 * k]).x | ((uint32_t)from_f<bf16_t>(v[2 * k + 1]).x << 16);
      return make_uint4(x[0], x[1], x[2], x[3]);
    };
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      __syncthreads();  // operand buffers (or the previous half) no longer read
      if (wr == hh)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) T[(32 * i + acc_row(r, q)) * kPB + wn + 32 * j + lr] = acc[i][j][r];
      __syncthreads();
      for (int row = threadIdx.x >> 4; row < 64; row += GRP) {
        const int64_t m = m0 + 64 * hh + row;
        const float4 a0 = *reinterpret_cast<const float4*>(T + row * kPB + cg);
        const float4 a1 = *reinterpret_cast<const float4*>(T + row * kPB + cg + 4);
        const float a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        float o[8];
        uint4* cp = reinterpret_cast<uint4*>(C + m * p.ldc + n0 + cg);
        if (EPI == kPEpiGelu) {  // GELU of the STORED (rounded) pre-activation, as the backward sees it
          const uint4 pre = pack(a);
          *reinterpret_cast<uint4*>(aux + m * p.ldaux + n0 + cg) = pre;
          float ar[8];
          unpack(pre, ar);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = gelu_f(ar[k] + bv[k]);
        } else if (EPI == kPEpiDGelu) {
          float pre[8];
          unpack(*reinterpret_cast<const uint4*>(aux + m * p.ldaux + n0 + cg), pre);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            o[k] = a[k] * gelu_grad_f(pre[k] + bv[k]);
            cs[k] += o[k];
          }
        } else if (p.beta != 0.f) {
          float old[8];
          unpack(*cp, old);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = a[k] + bv[k] + p.beta * old[k];
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = a[k] + bv[k];
        }
        *cp = pack(o);
      }
    }
    if (EPI == kPEpiDGelu) {  // column partials of the block's 128 rows: GRP thread partials per column
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 8; ++k) T[(threadIdx.x >> 4) * kPB + cg + k] = cs[k];
      __syncthreads();
      if (threadIdx.x < kPB) {
        float t = 0.f;
        for (int g = 0; g < GRP; ++g) t += T[g * kPB + threadIdx.x];  // fixed order
        p.part[(int64_t)tm * p.N + n0 + threadIdx.x] = t;
      }
    }
    return;
  }
  if (EPI <= kPEpiBias && m0 + kPB > p.Mv) {  // a tile reaching past the valid rows (padded problems only)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn + 32 * j + lr;
      const float bv = EPI != kPEpiNone ? p.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t m = m0 + wm + 32 * i + acc_row(r, q);
          if (m < p.Mv)
            store_c(C + m * p.ldc + n, acc[i][j][r] + bv + (p.beta != 0.f ? p.beta * load_c(C + m * p.ldc + n) : 0.f));
        }
    }
    return;
  }
  float csum[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) csum[j] = 0.f;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn + 32 * j + lr;
    const float bv = EPI != kPEpiNone ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + 32 * i + acc_row(r, q);
        const float a = acc[i][j][r];
        if (EPI == kPEpiGelu) {  // GELU of the STORED pre-activation (what the backward will see)
          store_c(aux + m * p.ldaux + n, a);
          store_c(C + m * p.ldc + n, gelu_f(round_c<TC>(a) + bv));
        } else if (EPI == kPEpiDGelu) {
          const float v = a * gelu_grad_f(load_c(aux + m * p.ldaux + n) + bv);
          csum[j] += v;
          store_c(C + m * p.ldc + n, v);
        } else if (p.beta != 0.f) {
          store_c(C + m * p.ldc + n, a + bv + p.beta * load_c(C + m * p.ldc + n));
        } else {
          store_c(C + m * p.ldc + n, a + bv);
        }
      }
    }
  }
  if (EPI == kPEpiDGelu) {  // column sums over the block's 128 rows: lane halves, then wave rows via LDS
    float* red = reinterpret_cast<float*>(smem);  // the K loop ended with a barrier
#pragma unroll
    for (int j = 0; j < TN; ++j) csum[j] += __shfl_xor(csum[j], 32, 64);
    if (wr == 1 && q == 0)
#pragma unroll
      for (int j = 0; j < TN; ++j) red[wn + 32 * j + lr] = csum[j];
    __syncthreads();
    if (wr == 0 && q == 0)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int c = wn + 32 * j + lr;
        p.part[(int64_t)tm * p.N + n0 + c] = csum[j] + red[c];
      }
  }
}

// split-K finish for a bf16 C: C = bf16(sum_s slab[s] (+ bias) (+ beta * C)), slices in fixed
// order (deterministic); 8 columns per thread (16-B bf16 stores)
__global__ void __launch_bounds__(256) splitk_reduce_bf16_kernel(const float* __restrict__ slab, int ksplit, int M,
                                                                 int N, bf16_t* __restrict__ C, int64_t ldc,
                                                                 const float* __restrict__ bias, float beta) {
  const int n8 = N / 8;
  const int64_t total = (int64_t)M * n8, plane = (int64_t)M * N;
  for (int64_t u = blockIdx.x * 256ll + threadIdx.x; u < total; u += (int64_t)gridDim.x * 256) {
    const int m = (int)(u / n8), n = (int)(u % n8) * 8;
    const float* s0 = slab + (int64_t)m * N + n;
    float a[8];
    {
      const float4 x = *reinterpret_cast<const float4*>(s0), y = *reinterpret_cast<const float4*>(s0 + 4);
      a[0] = x.x; a[1] = x.y; a[2] = x.z; a[3] = x.w; a[4] = y.x; a[5] = y.y; a[6] = y.z; a[7] = y.w;
    }
    for (int sl = 1; sl < ksplit; ++sl) {
      const float4 x = *reinterpret_cast<const float4*>(s0 + sl * plane);
      const float4 y = *reinterpret_cast<const float4*>(s0 + sl * plane + 4);
      a[0] += x.x; a[1] += x.y; a[2] += x.z; a[3] += x.w; a[4] += y.x; a[5] += y.y; a[6] += y.z; a[7] += y.w;
    }
    if (bias)
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += bias[n + k];
    uint4* c = reinterpret_cast<uint4*>(C + (int64_t)m * ldc + n);
    if (beta != 0.f) {
      const uint4 o = *c;
      const uint32_t w[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[2 * k] += beta * __uint_as_float(w[k] << 16);
        a[2 * k + 1] += beta * __uint_as_float(w[k] & 0xffff0000u);
      }
    }
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      w[k] = (uint32_t)from_f<bf16_t>(a[2 * k]).x | ((uint32_t)from_f<bf16_t>(a[2 * k + 1]).x << 16);
    *c = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

template <int P, int BK, int STAGES, int WV, typename TC>
int launch_planes_cfg(int ta, int tb, int epi, const PlanesArgs& a, hipStream_t st) {
  const dim3 grid((a.M / kPB) * (a.N / kPB) * a.ksplit), blk(64 * WV);
#define HS_PL(TA_, TB_, E_) \
  hipLaunchKernelGGL((gemm_planes_kernel<P, BK, STAGES, WV, TA_, TB_, E_, TC>), grid, blk, 0, st, a)
  if (!ta && tb) {  // forward X W^T
    if (epi == kPEpiNone) HS_PL(false, true, kPEpiNone);
    else if (epi == kPEpiBias) HS_PL(false, true, kPEpiBias);
    else if (epi == kPEpiGelu) HS_PL(false, true, kPEpiGelu);
    else return -1;
  } else if (!ta && !tb) {  // dgrad dY W
    if (epi == kPEpiNone) HS_PL(false, false, kPEpiNone);
    else if (epi == kPEpiDGelu) HS_PL(false, false, kPEpiDGelu);
    else return -1;
  } else if (ta && !tb) {  // wgrad dY^T X
    if (epi == kPEpiNone) HS_PL(true, false, kPEpiNone);
    else return -1;
  } else {
    return -1;
  }
#undef HS_PL
  return 0;
}

}  // namespace hs

// gemm.hip: C = sum of the ksplit fp32 slabs (fixed order) (+ bias) (+ beta * C)
void launch_splitk_reduce(const float* slab, int ksplit, int M, int N, float* C, int64_t ldc, const float* bias,
                          float beta, int Mv, int Nv, hipStream_t st);

using namespace hs;

static int g_planes_variant = 0;  // microbenchmark / tuning hook
void set_planes_variant(int v) { g_planes_variant = v; }

// planes: 1 (bf16) or 3 (split fp32); c_dtype: 0 fp32 C, 1 bf16 C.  Operand strides / plane
// strides in elements.  Returns -1 (nothing launched) for shapes it does not serve: M, N
// split-K block order: tile-major
static const int g_planes_slice_major = 0;

// multiples of 128, K a multiple of BK * ksplit, 16-B aligned rows.
int launch_gemm_planes(int planes, int c_dtype, int ta, int tb, int M, int N, int K, const void* A, int64_t lda,
                       int64_t a_ps, const void* B, int64_t ldb, int64_t b_ps, void* C, int64_t ldc,
                       const float* bias, int epi, float beta, void* aux, int64_t ldaux, float* part,
                       float* colsum_out, int colsum_acc, int ksplit, float* slab, int64_t slab_floats,
                       int variant, hipStream_t st, int Mv) {
  if (planes != 1) return -1;
  // Mv (0: M): valid rows of a padded problem -- fp32 C, plain / bias epilogue; C rows from Mv on are
  // neither read nor written (the tied decoder's weight gradient over the padded vocabulary)
  Mv = Mv > 0 ? Mv : M;
  if (Mv > M || (Mv < M && (c_dtype || epi > 1))) return -1;  // (the split-fp32 P = 3 engine was retired for h3p, gemm_h3p.hip)
  // variant (tile K depth, LDS stages, waves): 0 = two stages, 4 waves; 1 = one stage; 2 = half
  // depth; 3 = 8 waves; 4 = 8 waves + one stage.  < 0: the process default (set_planes_variant)
  if (variant < 0) variant = g_planes_variant;
  const int BK = planes == 3 ? (variant == 2 ? 16 : 32) : (variant == 2 ? 32 : 64);
  ksplit = std::max(1, ksplit);
  if (M <= 0 || N <= 0 || K <= 0 || M % kPB || N % kPB || K % (BK * ksplit)) return -1;
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al16(A) || !al16(B) || lda % 8 || ldb % 8 || (planes == 3 && (a_ps % 8 || b_ps % 8))) return -1;
  if ((epi >= 1 && !bias) || (epi >= 2 && (!aux || beta != 0.f)) || (epi == 3 && (!part || !colsum_out))) return -1;
  // split-K: fp32 slabs, then a fixed-order reduction applying bias / beta (fp32 or bf16 C)
  if (ksplit > 1 && (epi > 1 || !slab || (int64_t)ksplit * M * N > slab_floats || ldc % 8 || N % 8 ||
                     (c_dtype && !al16(C))))
    return -1;
  // bf16 C: the epilogue moves 8 columns per 16-B access (C, pre-activation, old C)
  if (c_dtype && ksplit == 1 && (!al16(C) || ldc % 8 || (epi >= 2 && (!al16(aux) || ldaux % 8)) ||
                                 (epi >= 1 && !al16(bias))))
    return -1;
  // 32-bit per-lane DMA offsets: the operand span (all planes) must stay below 4 GiB
  const int64_t spanA = 2 * ((planes - 1) * a_ps + (int64_t)(ta ? K : M) * lda);
  const int64_t spanB = 2 * ((planes - 1) * b_ps + (int64_t)(tb ? N : K) * ldb);
  if (spanA >= (1ll << 32) || spanB >= (1ll << 32)) return -1;
  PlanesArgs a{static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), C, bias, aux, part, slab,
               lda, ldb, ldc, ldaux, a_ps, b_ps, M, N, K, ksplit, beta, g_planes_slice_major, Mv};
  int rc;
#define HS_CFG(P_, BK_, S_, W_)                                                        \
  (c_dtype ? launch_planes_cfg<P_, BK_, S_, W_, bf16_t>(ta, tb, epi, a, st) \
           : launch_planes_cfg<P_, BK_, S_, W_, float>(ta, tb, epi, a, st))
  rc = variant == 1 ? HS_CFG(1, 64, 1, 4) : variant == 2 ? HS_CFG(1, 32, 2, 4) : variant == 3 ? HS_CFG(1, 64, 2, 8)
       : variant == 4 ? HS_CFG(1, 64, 1, 8) : HS_CFG(1, 64, 2, 4);
#undef HS_CFG
  if (rc) return rc;
  if (ksplit > 1 && c_dtype) {
    const int64_t units = (int64_t)M * (N / 8);
    hipLaunchKernelGGL(splitk_reduce_bf16_kernel, dim3((int)std::min<int64_t>((units + 255) / 256, 2048)), dim3(256),
                       0, st, slab, ksplit, M, N, static_cast<bf16_t*>(C), ldc, epi == 1 ? bias : nullptr, beta);
  } else if (ksplit > 1) {
    launch_splitk_reduce(slab, ksplit, M, N, static_cast<float*>(C), ldc, epi == 1 ? bias : nullptr, beta, Mv, N, st);
  }
  if (epi == kPEpiDGelu) {
    const float* parts[1] = {part};
    float* outs[1] = {colsum_out};
    launch_reduce_rows(parts, outs, 1, M / kPB, N, colsum_acc, st);
  }
  return 0;
}
