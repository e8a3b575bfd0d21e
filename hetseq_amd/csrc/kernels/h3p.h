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

}  // namespace hs
