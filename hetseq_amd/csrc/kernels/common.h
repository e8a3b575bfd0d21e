// Shared device helpers for the gfx950 (CDNA4) kernel library.
//
// Conventions used by every kernel in this directory:
//  * wave64 everywhere: lane = threadIdx.x & 63, reductions use __shfl_xor over
//    64 lanes; blocks are multiples of 64 threads.
//  * storage types are `float` and `bf16_t` (raw uint16 bits); all math is
//    fp32.  bf16 conversion is round-to-nearest-even with NaN kept NaN.
//  * randomness is counter-based Philox4x32-10 keyed by (seed, offset), so a
//    dropout mask is regenerated bit-identically in the backward kernel and no
//    mask tensor is ever stored.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HS_DEVICE __device__ __forceinline__

namespace hs {

struct bf16_t {
  uint16_t x;
};

HS_DEVICE float to_f(float v) { return v; }
HS_DEVICE float to_f(bf16_t v) { return __uint_as_float(static_cast<uint32_t>(v.x) << 16); }

template <typename T>
HS_DEVICE T from_f(float v);
template <>
HS_DEVICE float from_f<float>(float v) { return v; }
template <>
HS_DEVICE bf16_t from_f<bf16_t>(float v) {
  uint32_t u = __float_as_uint(v);
  bf16_t r;
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) {
    r.x = static_cast<uint16_t>((u >> 16) | 0x40);  // quiet NaN stays NaN
  } else {
    u += 0x7fffu + ((u >> 16) & 1u);
    r.x = static_cast<uint16_t>(u >> 16);
  }
  return r;
}

// ---------------------------------------------------------------- reductions
HS_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
HS_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
HS_DEVICE uint32_t wave_umax(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), o, 64)));
  return v;
}
// |max| of a lane's values, kept as bits of |x| (integer max = float max, NaN above inf): amax_bits
// folds one value in; a wave's result goes out with one atomic max (amax_commit).
HS_DEVICE uint32_t amax_bits(uint32_t m, float x) { return max(m, __float_as_uint(x) & 0x7fffffffu); }
// A |max| SLOT (the h3 GEMM engine's operand scale source, ops/gemm.py AmaxPool) is kAmaxShards
// partial maxima one 64-B line apart: writers spread their atomics over the shards by wave index, so
// a thousand blocks finishing together do not serialise on one address (one address took ~11 ns per
// atomic: 82 us for a 4096-wave kernel's tail); readers max over the shards (amax_read).
constexpr int kAmaxShards = 32;
constexpr int kAmaxStride = 16;  // floats between shards
HS_DEVICE void amax_put(float* slot, uint32_t m, int who) {
  atomicMax(reinterpret_cast<unsigned int*>(slot + (who % kAmaxShards) * kAmaxStride), m);
}
// the wave's |max| into its shard (all 64 lanes call it; lane 0 issues the atomic)
HS_DEVICE void amax_commit(float* slot, uint32_t m) {
  m = wave_umax(m);
  if ((threadIdx.x & 63) == 0) amax_put(slot, m, (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
}
// |max| over `nslots` adjacent slots as |x| bits, read cooperatively by the whole wave (every lane
// gets the result; all 64 lanes must call it)
HS_DEVICE uint32_t amax_read(const float* slot, int nslots) {
  uint32_t b = 0u;
  for (int i = threadIdx.x & 63; i < nslots * kAmaxShards; i += 64)
    b = max(b, __float_as_uint(slot[i * kAmaxStride]) & 0x7fffffffu);
  return wave_umax(b);
}
HS_DEVICE double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------- Philox
struct Philox {
  // Philox4x32-10 (Salmon et al., SC'11).  One call yields 4 uint32.
  HS_DEVICE static uint4 gen(uint64_t seed, uint64_t counter_hi, uint32_t counter_lo) {
    uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
    uint32_t c0 = counter_lo, c1 = 0u, c2 = static_cast<uint32_t>(counter_hi),
             c3 = static_cast<uint32_t>(counter_hi >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      // one 32x32->64 multiply each (v_mad_u64_u32) instead of separate mul_hi / mul_lo
      const uint64_t p0 = static_cast<uint64_t>(0xD2511F53u) * c0, p1 = static_cast<uint64_t>(0xCD9E8D57u) * c2;
      const uint32_t hi0 = static_cast<uint32_t>(p0 >> 32), lo0 = static_cast<uint32_t>(p0);
      const uint32_t hi1 = static_cast<uint32_t>(p1 >> 32), lo1 = static_cast<uint32_t>(p1);
      c0 = hi1 ^ c1 ^ k0;
      c1 = lo1;
      c2 = hi0 ^ c3 ^ k1;
      c3 = lo0;
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
  }
};

// Keep-decision for element `idx` of a dropout site: uniform in [0,1) from 24
// random bits, keep if u >= p.  4 consecutive elements share one Philox call.
HS_DEVICE float u01(uint32_t r) { return static_cast<float>(r >> 8) * (1.0f / 16777216.0f); }

HS_DEVICE uint4 philox_at(uint64_t seed, uint64_t offset, uint64_t q) {
  // counter = (offset + high bits of q, low 32 bits of q)
  return Philox::gen(seed, offset + (q >> 32), static_cast<uint32_t>(q));
}

HS_DEVICE void keep4(uint64_t seed, uint64_t offset, uint64_t q, float p, float scale, float m[4]) {
  const uint4 r = philox_at(seed, offset, q);
  m[0] = u01(r.x) >= p ? scale : 0.f;
  m[1] = u01(r.y) >= p ? scale : 0.f;
  m[2] = u01(r.z) >= p ? scale : 0.f;
  m[3] = u01(r.w) >= p ? scale : 0.f;
}

// Dropout seed source.  Normally the per-update seed is a kernel argument; in
// HIP-graph mode (runtime/graphs.py) the captured launches must not bake it in,
// so launchers pass g_seed_dev -- a device word the host refreshes before every
// replay -- and kernels read it instead.  Set through the `set_seed_ptr` binding.
extern const uint64_t* g_seed_dev;

// Diagnostic ablation (set_skip_launches; bench.py --ab skip_*): launches of the classes whose bit is
// set return without launching -- kSkipSplitK the split-K finishing passes, kSkipReduceRows the
// column-partial reductions.  Results are then meaningless; every buffer and address stays the same.
enum : int { kSkipSplitK = 1, kSkipReduceRows = 2 };
extern int g_hs_skip;
HS_DEVICE uint64_t resolve_seed(uint64_t seed, const uint64_t* seed_dev) { return seed_dev ? *seed_dev : seed; }

// 16-bit dropout decisions: one Philox call -> 8 keep bits (bit e: element e of the
// group), keep iff the 16-bit uniform >= thr16 = round(p * 65536).  Halves the RNG
// cost of keep4 where a kernel needs bits rather than 24-bit uniforms.
HS_DEVICE uint32_t drop_thr16(float p) { return min(65536u, static_cast<uint32_t>(p * 65536.f + 0.5f)); }
HS_DEVICE float drop_scale16(uint32_t thr) { return thr >= 65536u ? 0.f : 65536.f / static_cast<float>(65536u - thr); }
HS_DEVICE uint32_t keep8_bits(uint64_t seed, uint64_t offset, uint64_t q, uint32_t thr) {
  const uint4 r = philox_at(seed, offset, q);
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
  uint32_t bits = 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    bits |= ((w[i] & 0xffffu) >= thr ? 1u : 0u) << (2 * i);
    bits |= ((w[i] >> 16) >= thr ? 1u : 0u) << (2 * i + 1);
  }
  return bits;
}

// vector load/store helpers for 4 consecutive elements
HS_DEVICE void load4(const float* p, float v[4]) {
  const float4 t = *reinterpret_cast<const float4*>(p);
  v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
}
HS_DEVICE void load4(const bf16_t* p, float v[4]) {
  const uint2 t = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(t.x << 16);
  v[1] = __uint_as_float(t.x & 0xffff0000u);
  v[2] = __uint_as_float(t.y << 16);
  v[3] = __uint_as_float(t.y & 0xffff0000u);
}
HS_DEVICE void store4(float* p, const float v[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
HS_DEVICE void store4(bf16_t* p, const float v[4]) {
  const bf16_t a = from_f<bf16_t>(v[0]), b = from_f<bf16_t>(v[1]), c = from_f<bf16_t>(v[2]),
               d = from_f<bf16_t>(v[3]);
  uint2 t;
  t.x = static_cast<uint32_t>(a.x) | (static_cast<uint32_t>(b.x) << 16);
  t.y = static_cast<uint32_t>(c.x) | (static_cast<uint32_t>(d.x) << 16);
  *reinterpret_cast<uint2*>(p) = t;
}

// GELU with the reference's constant c = 1.41421 (bert_modeling.py:104-111): x/2 (1 + erf(x/c)).
// 1 + erf(z) is evaluated as erfc(-z) from one branch-free rational form, erfc(a) = t exp(-a^2 + P(t)),
// t = 1 / (1 + a/2), a = |z| (Numerical Recipes' erfcc, fractional error < 1.2e-7 on [0, inf)): about
// 15 VALU operations and one exp.  The library erff takes a different polynomial per |z| range, so a
// wave holding both ranges ran both: in the GEMM epilogues, which run when the tile's MFMAs are done,
// the GELU math alone took 18 us of a 92-us FFN-in product (tools/bench_h3p_epi.py, round 6).  The
// form is also accurate in relative terms on the negative tail, where 1 + erff(z) cancels (measured in
// fp32 against fp64 over [-10, 10]: max abs error 3.8e-7, as the erff form's 4.4e-7).
typedef float hs_f2 __attribute__((ext_vector_type(2)));
HS_DEVICE hs_f2 hs_f2s(float v) { return hs_f2{v, v}; }
HS_DEVICE hs_f2 hs_exp2v(hs_f2 x) { return hs_f2{__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)}; }
// 1 + erf(z) on two values at once (packed fp32 FMAs: half the VALU issue of two scalar evaluations),
// the exponential as exp2 of a log2(e)-scaled argument (the coefficients carry the factor: no range
// fix-up around the exp)
HS_DEVICE hs_f2 gelu_phi2v(hs_f2 z) {
  constexpr float L = 1.4426950408889634f;  // log2(e)
  const hs_f2 a = __builtin_elementwise_abs(z);
  const hs_f2 d = __builtin_elementwise_fma(hs_f2s(0.5f), a, hs_f2s(1.f));
  const hs_f2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  hs_f2 p = hs_f2s(0.17087277f * L);
  p = __builtin_elementwise_fma(p, t, hs_f2s(-0.82215223f * L));
  p = __builtin_elementwise_fma(p, t, hs_f2s(1.48851587f * L));
  p = __builtin_elementwise_fma(p, t, hs_f2s(-1.13520398f * L));
  p = __builtin_elementwise_fma(p, t, hs_f2s(0.27886807f * L));
  p = __builtin_elementwise_fma(p, t, hs_f2s(-0.18628806f * L));
  p = __builtin_elementwise_fma(p, t, hs_f2s(0.09678418f * L));
  p = __builtin_elementwise_fma(p, t, hs_f2s(0.37409196f * L));
  p = __builtin_elementwise_fma(p, t, hs_f2s(1.00002368f * L));
  p = __builtin_elementwise_fma(p, t, hs_f2s(-1.26551223f * L));
  const hs_f2 e = t * hs_exp2v(__builtin_elementwise_fma(-a, a * L, p));  // erfc(|z|)
  return hs_f2{z.x < 0.f ? e.x : 2.f - e.x, z.y < 0.f ? e.y : 2.f - e.y};
}
// GELU and its derivative on two values (the GEMM epilogues: register pairs r, r + 1 are the two rows a
// lane holds in one column)
HS_DEVICE hs_f2 gelu_v(hs_f2 x) { return x * 0.5f * gelu_phi2v(x * (1.f / 1.41421f)); }
HS_DEVICE hs_f2 gelu_grad_v(hs_f2 x) {
  // d/dx [x/2 (1+erf(x/c))] = 1/2 (1+erf(x/c)) + x/(c*sqrt(pi)) exp(-(x/c)^2)
  constexpr float L = 1.4426950408889634f;
  const hs_f2 z = x * (1.f / 1.41421f);
  const hs_f2 g = hs_exp2v(-z * (z * L));  // exp(-z^2)
  return __builtin_elementwise_fma(x * (0.5641895835477563f / 1.41421f), g, 0.5f * gelu_phi2v(z));
}
// one value: the same arithmetic in lane x of the pair
HS_DEVICE float gelu_f(float x) { return gelu_v(hs_f2{x, 0.f}).x; }
HS_DEVICE float gelu_grad_f(float x) { return gelu_grad_v(hs_f2{x, 0.f}).x; }

inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

}  // namespace hs
