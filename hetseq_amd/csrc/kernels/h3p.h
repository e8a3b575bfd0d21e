// Block-scaled split-fp16 operand format ("h3p") shared by the h3p GEMM (gemm_h3p.hip) and the
// kernels that produce its operands (split pass, LayerNorm forward / backward, attention, the GEMM's
// own GELU / dGELU epilogues).
//
// An fp32 matrix X [R][C] (R, C multiples of 32) is stored as
//   * two fp16 planes, hi and lo, each [R][ld] (plane 1 at plane 0 + ps elements), and
//   * one exponent e per 32 x 32 block, int8 [R/32][C/32]:
//       x * 2^e = hi + lo + r,  hi = fp16(x * 2^e),  lo = fp16(x * 2^e - hi),  |r| <= 2^-22 |x * 2^e|
//     with e = 14 - floor(log2 |max of the block|), so the block's largest element lands in
//     [2^14, 2^15) (fp16's largest finite value is 65504) and every element down to 2^-18 of the
//     BLOCK's maximum keeps 22 significant bits (the window is per 32 x 32 block, not per tensor).
// Plane layout (per tensor): row-major ([R][ld], element (r, c) at r ld + c) or BLOCKED: the same
// 32-row panels, each stored as ld / 32 consecutive 32 x 32 blocks of 2 KB (row-major 64-B rows
// inside), element (r, c) at (r / 32) 32 ld + (c / 32) 1024 + (r % 32) 32 + c % 32.  A blocked 32-deep
// K tile of a 128-wide GEMM operand is four whole 2-KB blocks in EITHER orientation, so the GEMM's
// LDS-DMA reads full 128-B lines for k-contiguous operands too (row-major: 64 B of each row).
// A product a * b is then hi_a hi_b + hi_a lo_b + lo_a hi_b (the dropped lo_a lo_b is ~2^-22 |ab|),
// each fp16 x fp16 product exact in the fp32 accumulator: three fp16 MFMAs per fp32 product, with
// the block factor 2^-(e_a + e_b) applied once per 32-deep K tile (gemm_h3p.hip).
#pragma once
#include "common.h"

namespace hs {

constexpr int kH3pBlk = 32;  // exponent block edge (rows and columns)

// exponent of a block whose |max| is m (0 for zero / NaN / inf blocks: NaN and inf propagate)
HS_DEVICE int h3p_exp(float m) {
  if (!(m > 0.f) || !(m <= 3.4028235e38f)) return 0;
  return min(100, max(-100, 14 - ilogbf(m)));
}
// ... from |max| kept as bits (amax_bits)
HS_DEVICE int h3p_exp_bits(uint32_t mb) { return h3p_exp(__uint_as_float(mb)); }

typedef _Float16 h3p_h2 __attribute__((ext_vector_type(2)));
typedef float h3p_f2 __attribute__((ext_vector_type(2)));

// hi / lo fp16 pairs of two values scaled by s = 2^e (packed: element 0 in the low half)
HS_DEVICE void h3p_split2(float x0, float x1, float s, uint32_t& hi, uint32_t& lo) {
#pragma clang fp contract(off)  // the residual of the scaled value exactly as rounded, never an fma
  const h3p_f2 v = {x0 * s, x1 * s};  // exact: s is a power of two
  const h3p_h2 h = __builtin_convertvector(v, h3p_h2);
  const h3p_f2 r = v - __builtin_convertvector(h, h3p_f2);  // exact
  const h3p_h2 l = __builtin_convertvector(r, h3p_h2);
  hi = __builtin_bit_cast(uint32_t, h);
  lo = __builtin_bit_cast(uint32_t, l);
}

// four consecutive values of a row -> 8 B of each plane at element index i (plane 1 at + ps)
HS_DEVICE void h3p_store4(uint16_t* __restrict__ pl, int64_t ps, int64_t i, const float v[4], float s) {
  uint32_t h0, l0, h1, l1;
  h3p_split2(v[0], v[1], s, h0, l0);
  h3p_split2(v[2], v[3], s, h1, l1);
  *reinterpret_cast<uint2*>(pl + i) = make_uint2(h0, h1);
  *reinterpret_cast<uint2*>(pl + i + ps) = make_uint2(l0, l1);
}

HS_DEVICE float h3p_scale(int e) { return __builtin_ldexpf(1.f, e); }

// element index of (r, c) in a plane (layout above; ld a multiple of 32 when blocked)
HS_DEVICE int64_t h3p_index(int64_t r, int64_t c, int64_t ld, int blocked) {
  return blocked ? (r >> 5) * 32 * ld + (c >> 5) * 1024 + (r & 31) * 32 + (c & 31) : r * ld + c;
}

// ---------------------------------------------------------------- panel exchange
// Block exponents from producers whose workgroups hold fewer than the 32 rows of an exponent block:
// the np workgroups of one 32-row PANEL combine their per-32-column-group |max| through a record of
// kPanelSyncWords uint32 in device memory (zero-initialised once by the owner, ops/bert_ops.py
// panel_sync), and every workgroup then splits its own rows, still in registers, with the panel's
// exponents.  A 32-row workgroup puts a 2048-row call on 64 of the 256 CUs (round-5 LayerNorm
// forward: 40 us in the step for ~25 MB); 8-row workgroups spread it over all of them.
//   word 0: generation (one increment per completed exchange), word 16: arrival count,
//   words 64 + 64 (g & 1) ..: the |max| buffer of generation g (<= 64 groups: H <= 2048).
// Every access is an agent-scope atomic, so no XCD's L2 or CU's L1 can hold a stale copy.  Protocol:
// a workgroup reads g before it arrives (g cannot move before the last of the np arrivals), maxes its
// values into buffer g & 1, waits for those atomics to return, then adds 1 to the count.  The last
// arriver clears the count and the OTHER parity's buffer (the next call's; the previous call that
// used it has ended: same stream), then increments the generation; the others poll the generation.
// All then read buffer g & 1 (every max into it was performed before its writer's arrival).  Calls
// that may run concurrently (the forward's two half-batch streams) use disjoint panels; the np
// workgroups of a panel need not be co-resident at launch (a polling workgroup holds a slot only
// until the rest of its panel, which nothing else waits on, is dispatched), and the poll is bounded
// (word 32 records a timeout).
constexpr int kPanelSyncWords = 256;

HS_DEVICE uint32_t psync_gen(uint32_t* rec) {
  return __hip_atomic_fetch_add(rec, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// psync_arrive: called by ALL 64 lanes of ONE wave of the workgroup; lane c < ng holds the
// workgroup's |max| bits of column group c in `m`, g = psync_gen() read before this workgroup
// arrived.  Returns true in the last arriver (which has already published the generation).
// psync_wait: the same wave, later (work independent of the exponents may run in between);
// returns the panel's |max| of group c in lane c.
HS_DEVICE bool psync_arrive(uint32_t* rec, uint32_t g, uint32_t m, int ng, int np) {
  const int lane = threadIdx.x & 63;
  uint32_t* cur = rec + 64 + 64 * (g & 1u);
  if (lane < ng) (void)__hip_atomic_fetch_max(cur + lane, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the maxima are performed before the arrival
  uint32_t arrived = 0u;
  if (lane == 0) arrived = __hip_atomic_fetch_add(rec + 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool last = __shfl(static_cast<int>(arrived), 0, 64) == np - 1;
  if (last) {  // every arrival (and so every max) is in: reset for the next call, then publish
    uint32_t* nxt = rec + 64 + 64 * ((g + 1u) & 1u);
    if (lane == 0) (void)__hip_atomic_exchange(rec + 16, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane < ng) (void)__hip_atomic_exchange(nxt + lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) (void)__hip_atomic_fetch_add(rec, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return last;
}

HS_DEVICE uint32_t psync_wait(uint32_t* rec, uint32_t g, bool last, int ng) {
  const int lane = threadIdx.x & 63;
  if (!last && lane == 0) {
    int spins = 0;
    while (psync_gen(rec) == g) {
      if (++spins > (1 << 22)) {
        (void)__hip_atomic_exchange(rec + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  asm volatile("" ::: "memory");  // the reads below stay behind the poll
  uint32_t r = 0u;
  if (lane < ng)
    r = __hip_atomic_fetch_or(rec + 64 + 64 * (g & 1u) + lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return r;
}

}  // namespace hs
