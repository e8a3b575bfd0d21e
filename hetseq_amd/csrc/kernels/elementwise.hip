// Elementwise / reduction kernels for the BERT hot path.
//
//  * bias_gelu_fwd: y = gelu(x + b) with the reference's erf(x/1.41421) GELU
//    (reference: bert_modeling.py:108-111, LinearActivation :166-172)  [K04]
//  * gelu_bwd_colsum: dx = dy * gelu'(x + b) fused with the column sum of dx
//    (the bias gradient) as per-block partials                         [K04]
//  * colsum_partial: column partial sums of a [rows, N] matrix (bias grads)
//  * mlm_compact: device-side compaction of the masked-LM rows (label != -1)
//    into a fixed-capacity index list -- the decoder then runs on only those
//    rows, exactly (rows with label -1 contribute neither loss nor gradient;
//    reference runs the decoder on every token, bert_modeling.py:547) [K07]
//  * gather_rows / scatter_rows: move hidden rows in and out of that list.
//
// Rows are processed as tiles: a block of 256 threads covers 1024 columns
// (4 per thread, 16-byte vectors) and a chunk of rows, keeping per-column
// partial sums in registers -> one partial row per block, no atomics.
#include <algorithm>

#include "common.h"
#include "reduce.h"

namespace hs {

template <typename T>
__global__ void __launch_bounds__(256) bias_gelu_fwd_kernel(const T* __restrict__ x, const float* __restrict__ b,
                                                            T* __restrict__ y, int64_t rows, int N) {
  const int64_t total4 = rows * N / 4;
  const int n4 = N / 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total4; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % n4) * 4;
    float v[4], bb[4];
    load4(x + 4 * i, v);
    load4(b + c, bb);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = gelu_f(v[j] + bb[j]);
    store4(y + 4 * i, v);
  }
}

// grid = (ceil(N/1024), row_chunks); part is [row_chunks, N]
template <typename T, bool kGelu>
__global__ void __launch_bounds__(256) colsum_tile_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const float* __restrict__ b, T* __restrict__ dx,
                                                          float* __restrict__ part, int64_t rows, int N,
                                                          int rows_per_chunk, float* __restrict__ amax) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 4;
  uint32_t mb = 0u;  // |max| of the written dx (kGelu with amax: the next product's h3 operand scale)
  if (c < N) {
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  int64_t r1 = r0 + rows_per_chunk;
  if (r1 > rows) r1 = rows;
  float bb[4] = {0.f, 0.f, 0.f, 0.f};
  if (kGelu) load4(b + c, bb);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  int64_t r = r0;
  // 4 rows per step with every load issued first: the strip walk is latency-bound otherwise
  for (; r + 4 <= r1; r += 4) {
    float d[4][4], v[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      load4(dy + (r + u) * N + c, d[u]);
      if (kGelu) load4(x + (r + u) * N + c, v[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (kGelu) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          d[u][j] *= gelu_grad_f(v[u][j] + bb[j]);
          mb = amax_bits(mb, d[u][j]);
        }
        store4(dx + (r + u) * N + c, d[u]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += d[u][j];
    }
  }
  for (; r < r1; ++r) {
    const int64_t o = r * N + c;
    float d[4];
    load4(dy + o, d);
    if (kGelu) {
      float v[4];
      load4(x + o, v);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        d[j] *= gelu_grad_f(v[j] + bb[j]);
        mb = amax_bits(mb, d[j]);
      }
      store4(dx + o, d);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] += d[j];
  }
  store4(part + (int64_t)blockIdx.y * N + c, acc);
  }
  if (kGelu && amax) amax_commit(amax, mb);  // (every lane reaches it: no early return above)
}

// column partial sums for N not a multiple of 4 (e.g. the 30522-wide vocab)
template <typename T>
__global__ void __launch_bounds__(256) colsum_scalar_kernel(const T* __restrict__ x, float* __restrict__ part,
                                                            int64_t rows, int N, int rows_per_chunk) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= N) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  int64_t r1 = r0 + rows_per_chunk;
  if (r1 > rows) r1 = rows;
  float acc = 0.f;
  for (int64_t r = r0; r < r1; ++r) acc += to_f(x[r * N + c]);
  part[(int64_t)blockIdx.y * N + c] = acc;
}

// Single-block exclusive scan over `rows` labels; writes idx[cap] (padded
// with -1), count[0] = number of valid rows, overflow flag if count > cap.
__global__ void __launch_bounds__(1024) mlm_compact_kernel(const int64_t* __restrict__ labels, int rows,
                                                           int ignore_index, int cap, int32_t* __restrict__ idx,
                                                           int64_t* __restrict__ lab_out, int32_t* __restrict__ count,
                                                           int* __restrict__ err) {
  __shared__ int wsum[16];
  __shared__ int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int base = 0; base < rows; base += 1024) {
    const int r = base + threadIdx.x;
    const int64_t lab = r < rows ? labels[r] : ignore_index;
    const int flag = lab != ignore_index ? 1 : 0;
    // wave inclusive scan via ballot popcount
    const unsigned long long bal = __ballot(flag);
    const unsigned long long below = lane == 0 ? 0ull : (bal & ((~0ull) >> (64 - lane)));
    const int wpre = __popcll(below);
    if (lane == 63) wsum[w] = wpre + flag;
    __syncthreads();
    int off = carry;
    for (int i = 0; i < w; ++i) off += wsum[i];
    const int pos = off + wpre;
    if (flag && pos < cap) {
      idx[pos] = r;
      lab_out[pos] = lab;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int i = 0; i < 16; ++i) t += wsum[i];
      carry += t;
    }
    __syncthreads();
  }
  const int total = carry;
  for (int i = threadIdx.x; i < cap; i += 1024)
    if (i >= total) {
      idx[i] = -1;
      lab_out[i] = ignore_index;
    }
  if (threadIdx.x == 0) {
    count[0] = total < cap ? total : cap;
    if (total > cap) atomicOr(err, 2);
  }
}

// out[i] = src[idx[i]] (zero row for idx < 0); H multiple of 4
template <typename T>
__global__ void gather_rows_kernel(const T* __restrict__ src, const int32_t* __restrict__ idx, T* __restrict__ out,
                                   int n, int H) {
  const int i = blockIdx.x;
  const int r = idx[i];
  for (int c = threadIdx.x * 4; c < H; c += blockDim.x * 4) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (r >= 0) load4(src + (int64_t)r * H + c, v);
    store4(out + (int64_t)i * H + c, v);
  }
}

// dst[idx[i]] += src[i] (rows unique by construction, so no atomics needed)
template <typename T>
__global__ void scatter_add_rows_kernel(const T* __restrict__ src, const int32_t* __restrict__ idx,
                                        T* __restrict__ dst, int n, int H) {
  const int i = blockIdx.x;
  const int r = idx[i];
  if (r < 0) return;
  for (int c = threadIdx.x * 4; c < H; c += blockDim.x * 4) {
    float a[4], b[4];
    load4(src + (int64_t)i * H + c, a);
    load4(dst + (int64_t)r * H + c, b);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] += a[j];
    store4(dst + (int64_t)r * H + c, b);
  }
}

static int ew_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

// Deterministic scatter-add of rows by key, dst[key] += sum of src rows with that
// key, for keys sorted ascending (order = the stable sort permutation of the rows).
// Two levels, both in fixed order (bitwise reproducible, no atomics, no host sync
// for the number of distinct keys), and parallel even for very long runs
// ([PAD] / [MASK] tokens repeat thousands of times in a batch):
//   1. seg_partial: block b walks sorted rows [32b, 32b+32) and writes the sum of
//      every run piece inside its chunk to P[piece start];
//   2. seg_combine: the block at each run start adds the run's pieces (one per
//      32-row chunk the run touches) into dst[key].
constexpr int kSegChunk = 32;

__global__ void __launch_bounds__(256) seg_partial_kernel(const float* __restrict__ src,
                                                           const int64_t* __restrict__ order,
                                                           const int64_t* __restrict__ keys, float* __restrict__ P,
                                                           int n, int H) {
  const int r0 = blockIdx.x * kSegChunk, r1 = min(n, r0 + kSegChunk);
  for (int c = threadIdx.x * 4; c < H; c += blockDim.x * 4) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int start = r0;
    for (int j = r0; j < r1; ++j) {
      float v[4];
      load4(src + order[j] * H + c, v);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] += v[q];
      if (j + 1 == r1 || keys[j + 1] != keys[j]) {  // end of a run piece
        store4(P + (int64_t)start * H + c, acc);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = 0.f;
        start = j + 1;
      }
    }
  }
}

__global__ void __launch_bounds__(256) seg_combine_kernel(const float* __restrict__ P, const int64_t* __restrict__ keys,
                                                           float* __restrict__ dst, int n, int H, int K) {
  const int i = blockIdx.x;
  const int64_t key = keys[i];
  if ((i > 0 && keys[i - 1] == key) || key < 0 || key >= K) return;
  // keys are sorted: binary-search the run end instead of walking it (runs like [PAD] span thousands of rows)
  int lo = i + 1, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (keys[mid] == key) lo = mid + 1; else hi = mid;
  }
  const int end = lo;
  for (int c = threadIdx.x * 4; c < H; c += blockDim.x * 4) {
    // pieces: the run's first chunk, then one per further chunk; 4 independent
    // accumulators keep 4 loads in flight for long runs (fixed combine order)
    float acc[4][4];
    load4(P + (int64_t)i * H + c, acc[0]);
#pragma unroll
    for (int u = 1; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[u][q] = 0.f;
    int j = (i / kSegChunk + 1) * kSegChunk;
    for (; j + 3 * kSegChunk < end; j += 4 * kSegChunk)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float v[4];
        load4(P + (int64_t)(j + u * kSegChunk) * H + c, v);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[u][q] += v[q];
      }
    for (; j < end; j += kSegChunk) {
      float v[4];
      load4(P + (int64_t)j * H + c, v);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[0][q] += v[q];
    }
    float d[4];
    load4(dst + key * H + c, d);
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] += (acc[0][q] + acc[1][q]) + (acc[2][q] + acc[3][q]);
    store4(dst + key * H + c, d);
  }
}

// Position-embedding gradient: dpos[s] += sum_b dx[b*S + s] (fixed order, 8 rows in flight).
__global__ void __launch_bounds__(256) pos_grad_kernel(const float* __restrict__ dx, float* __restrict__ dpos, int B,
                                                       int S, int H) {
  const int s = blockIdx.x;
  for (int c = threadIdx.x * 4; c < H; c += blockDim.x * 4) {
    float acc[8][4];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[u][q] = 0.f;
    int b = 0;
    for (; b + 8 <= B; b += 8)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float v[4];
        load4(dx + ((int64_t)(b + u) * S + s) * H + c, v);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[u][q] += v[q];
      }
    for (; b < B; ++b) {
      float v[4];
      load4(dx + ((int64_t)b * S + s) * H + c, v);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[0][q] += v[q];
    }
    float d[4];
    load4(dpos + (int64_t)s * H + c, d);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      d[q] += ((acc[0][q] + acc[1][q]) + (acc[2][q] + acc[3][q])) + ((acc[4][q] + acc[5][q]) + (acc[6][q] + acc[7][q]));
    store4(dpos + (int64_t)s * H + c, d);
  }
}

}  // namespace hs

using namespace hs;

int launch_segsum_rows(const float* src, const int64_t* order, const int64_t* keys, float* scratch, float* dst, int n,
                       int H, int K, hipStream_t st) {
  if (H % 4 != 0 || n < 0) return -1;
  if (n == 0) return 0;
  const int threads = std::min(256, ((H / 4 + 63) / 64) * 64);
  hipLaunchKernelGGL(seg_partial_kernel, dim3((n + kSegChunk - 1) / kSegChunk), dim3(threads), 0, st, src, order, keys,
                     scratch, n, H);
  hipLaunchKernelGGL(seg_combine_kernel, dim3(n), dim3(threads), 0, st, scratch, keys, dst, n, H, K);
  return 0;
}

// Stable key sort for the embedding backward's sorted-run gradient sums (replaces torch.sort).
// Every element's output slot is its rank: the number of composite words (key << ib) | index
// (ib = bits of n - 1; unique, so the order is total and stable) smaller than its own.  A block
// ranks 64 elements; its 4 waves each count over a quarter of all n words (broadcast LDS reads)
// and the quarter counts are summed (integers: exact in any order).  O(n^2) compares, but n is
// a batch's token count: 4096 -> 64 blocks of 1024 compares per thread, a few microseconds.
// n <= 16384 and key bits + index bits <= 32; other sizes return -1 (library sort fallback).
constexpr int kSortMax = 16384;

__global__ void __launch_bounds__(256) sort_keys_kernel(const int64_t* __restrict__ keys, int n, int ib,
                                                        int64_t bound, int64_t* __restrict__ out_keys,
                                                        int64_t* __restrict__ out_order, int* __restrict__ err) {
  __shared__ uint32_t s[kSortMax];
  __shared__ int part[4][64];
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    int64_t k = keys[i];
    if (k < 0 || k >= bound) {  // would wrap inside the packed word: flag it, sort it clamped
      if (err && blockIdx.x == 0) atomicOr(err, 4);
      k = k < 0 ? 0 : bound - 1;
    }
    s[i] = (static_cast<uint32_t>(k) << ib) | static_cast<uint32_t>(i);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  const uint32_t me = i < n ? s[i] : 0u;
  const int q = (n + 3) / 4, j0 = w * q, j1 = min(n, j0 + q);
  int cnt = 0;
  for (int j = j0; j < j1; ++j) cnt += s[j] < me ? 1 : 0;
  part[w][lane] = cnt;
  __syncthreads();
  if (w == 0 && i < n) {
    const int r = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
    out_keys[r] = static_cast<int64_t>(me >> ib);
    out_order[r] = static_cast<int64_t>(i);
  }
}

int launch_sort_keys(const int64_t* keys, int n, int64_t key_bound, int64_t* out_keys, int64_t* out_order, int* err,
                     hipStream_t st) {
  if (n <= 0 || n > kSortMax || key_bound <= 0) return -1;
  int ib = 0, kb = 0;
  while ((1 << ib) < n) ++ib;
  while ((int64_t(1) << kb) < key_bound) ++kb;
  if (ib + kb > 32) return -1;
  hipLaunchKernelGGL(sort_keys_kernel, dim3((n + 63) / 64), dim3(256), 0, st, keys, n, ib, key_bound, out_keys,
                     out_order, err);
  return 0;
}

int launch_pos_grad(const float* dx, float* dpos, int B, int S, int H, hipStream_t st) {
  if (H % 4 != 0) return -1;
  hipLaunchKernelGGL(pos_grad_kernel, dim3(S), dim3(std::min(256, ((H / 4 + 63) / 64) * 64)), 0, st, dx, dpos, B, S,
                     H);
  return 0;
}

void launch_bias_gelu_fwd(int dtype, const void* x, const float* b, void* y, int64_t rows, int N, hipStream_t st) {
  const int g = ew_grid(rows * N / 4);
  if (dtype == 0)
    hipLaunchKernelGGL(bias_gelu_fwd_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)x, b, (float*)y, rows, N);
  else
    hipLaunchKernelGGL(bias_gelu_fwd_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)x, b, (bf16_t*)y, rows,
                       N);
}

int colsum_row_chunks(int64_t rows) {
  int chunks = (int)((rows + 15) / 16);  // >= 2 blocks per CU for the 3072-wide FFN strip
  if (chunks > 512) chunks = 512;
  if (chunks < 1) chunks = 1;
  return chunks;
}

// gelu backward fused with bias-grad partials; if x == nullptr plain column sum of dy.
void launch_colsum(int dtype, const void* dy, const void* x, const float* b, void* dx, float* part, float* out,
                   int64_t rows, int N, int accumulate, hipStream_t st, float* amax) {
  const int chunks = colsum_row_chunks(rows);
  const int rpc = (int)((rows + chunks - 1) / chunks);
  dim3 grid((N / 4 + 255) / 256, chunks);
  if (N % 4 != 0) {  // plain column sum only (callers guarantee x == nullptr)
    dim3 g2((N + 255) / 256, chunks);
    if (dtype == 0)
      hipLaunchKernelGGL(colsum_scalar_kernel<float>, g2, dim3(256), 0, st, (const float*)dy, part, rows, N, rpc);
    else
      hipLaunchKernelGGL(colsum_scalar_kernel<bf16_t>, g2, dim3(256), 0, st, (const bf16_t*)dy, part, rows, N, rpc);
  } else if (dtype == 0) {
    if (x)
      hipLaunchKernelGGL((colsum_tile_kernel<float, true>), grid, dim3(256), 0, st, (const float*)dy, (const float*)x,
                         b, (float*)dx, part, rows, N, rpc, amax);
    else
      hipLaunchKernelGGL((colsum_tile_kernel<float, false>), grid, dim3(256), 0, st, (const float*)dy, nullptr, b,
                         nullptr, part, rows, N, rpc, nullptr);
  } else {
    if (x)
      hipLaunchKernelGGL((colsum_tile_kernel<bf16_t, true>), grid, dim3(256), 0, st, (const bf16_t*)dy,
                         (const bf16_t*)x, b, (bf16_t*)dx, part, rows, N, rpc, amax);
    else
      hipLaunchKernelGGL((colsum_tile_kernel<bf16_t, false>), grid, dim3(256), 0, st, (const bf16_t*)dy, nullptr, b,
                         nullptr, part, rows, N, rpc, nullptr);
  }
  const float* pp[1] = {part};
  float* oo[1] = {out};
  launch_reduce_rows(pp, oo, 1, chunks, N, accumulate, st);
}

void launch_mlm_compact(const int64_t* labels, int rows, int ignore_index, int cap, int32_t* idx, int64_t* lab_out,
                        int32_t* count, int* err, hipStream_t st) {
  hipLaunchKernelGGL(mlm_compact_kernel, dim3(1), dim3(1024), 0, st, labels, rows, ignore_index, cap, idx, lab_out,
                     count, err);
}

void launch_gather_rows(int dtype, const void* src, const int32_t* idx, void* out, int n, int H, hipStream_t st) {
  if (n <= 0) return;
  if (dtype == 0)
    hipLaunchKernelGGL(gather_rows_kernel<float>, dim3(n), dim3(64), 0, st, (const float*)src, idx, (float*)out, n, H);
  else
    hipLaunchKernelGGL(gather_rows_kernel<bf16_t>, dim3(n), dim3(64), 0, st, (const bf16_t*)src, idx, (bf16_t*)out, n,
                       H);
}

void launch_scatter_add_rows(int dtype, const void* src, const int32_t* idx, void* dst, int n, int H,
                             hipStream_t st) {
  if (n <= 0) return;
  if (dtype == 0)
    hipLaunchKernelGGL(scatter_add_rows_kernel<float>, dim3(n), dim3(64), 0, st, (const float*)src, idx, (float*)dst,
                       n, H);
  else
    hipLaunchKernelGGL(scatter_add_rows_kernel<bf16_t>, dim3(n), dim3(64), 0, st, (const bf16_t*)src, idx,
                       (bf16_t*)dst, n, H);
}

// ---------------------------------------------------------------------------
// Per-tensor |max| for the fp16-split GEMM engine (gemm.hip split4h): the operand scale is a power
// of two from it.  Producers that write an operand fold this reduction into their own epilogue
// (one atomic max per wave); these kernels serve the rest -- the weights once per update, and
// operands no fused producer wrote.  Non-negative floats order as their bit patterns, so an
// unsigned atomic max is exact and order-independent (deterministic); NaN sorts above inf.
namespace hs {

// |x| as bits: integer max over them is the float max of |x|, with any NaN above inf
HS_DEVICE uint32_t absbits4(uint4 v) {
  return max(max(v.x & 0x7fffffffu, v.y & 0x7fffffffu), max(v.z & 0x7fffffffu, v.w & 0x7fffffffu));
}

// 4 independent 16-B loads per lane per iteration; the wave maxima of a block are combined in LDS and
// the block issues ONE atomic, into its shard of the slot
__global__ void __launch_bounds__(256) amax_kernel(const float* __restrict__ x, int64_t n4, float* __restrict__ out) {
  const uint4* v = reinterpret_cast<const uint4*>(x);
  const int64_t stride = (int64_t)gridDim.x * 256;
  uint32_t m = 0u;
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride)
    m = max(max(m, max(absbits4(v[i]), absbits4(v[i + stride]))), max(absbits4(v[i + 2 * stride]),
                                                                       absbits4(v[i + 3 * stride])));
  for (; i < n4; i += stride) m = max(m, absbits4(v[i]));
  m = wave_umax(m);
  __shared__ uint32_t red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) amax_put(out, max(max(red[0], red[1]), max(red[2], red[3])), blockIdx.x);
}

// block b reduces float4 range [tab[3b+1], tab[3b+2]) of the flat buffer into slot tab[3b] of out
__global__ void __launch_bounds__(256) amax_seg_kernel(const float* __restrict__ base, const int64_t* __restrict__ tab,
                                                       float* __restrict__ out) {
  const int64_t seg = tab[3 * blockIdx.x], lo = tab[3 * blockIdx.x + 1], hi = tab[3 * blockIdx.x + 2];
  const uint4* v = reinterpret_cast<const uint4*>(base);
  uint32_t m = 0u;
  int64_t i = lo + threadIdx.x;
  for (; i + 768 < hi; i += 1024)
    m = max(max(m, max(absbits4(v[i]), absbits4(v[i + 256]))), max(absbits4(v[i + 512]), absbits4(v[i + 768])));
  for (; i < hi; i += 256) m = max(m, absbits4(v[i]));
  m = wave_umax(m);
  __shared__ uint32_t red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    amax_put(out + seg * kAmaxShards * kAmaxStride, max(max(red[0], red[1]), max(red[2], red[3])), blockIdx.x);
}

// zero float4 ranges: block b clears [tab[2 b], tab[2 b + 1]) (float4 indices from base) -- the part of the
// flat gradient buffer a lazy zero_grad clears (runtime/flat.py: the regions the backward overwrites stay)
__global__ void __launch_bounds__(256) zero_segs_kernel(float* __restrict__ base, const int64_t* __restrict__ tab) {
  const int64_t lo = tab[2 * blockIdx.x], hi = tab[2 * blockIdx.x + 1];
  float4* v = reinterpret_cast<float4*>(base);
  for (int64_t i = lo + threadIdx.x; i < hi; i += 256) v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

}  // namespace hs

// |max| of x[0, n) (n % 4 == 0, 16-B aligned) into the slot `out` (common.h: kAmaxShards shards);
// zero_first: the slot is cleared on the stream first
int launch_amax(const float* x, int64_t n, float* out, int zero_first, hipStream_t st) {
  if (n % 4 || (reinterpret_cast<uintptr_t>(x) & 15)) return -1;
  if (zero_first && hipMemsetAsync(out, 0, sizeof(float) * kAmaxShards * kAmaxStride, st) != hipSuccess) return -1;
  if (n == 0) return 0;
  const int64_t n4 = n / 4;
  const int grid = (int)std::min<int64_t>((n4 + 1023) / 1024, 1024);
  hipLaunchKernelGGL(amax_kernel, dim3(grid), dim3(256), 0, st, x, n4, out);
  return 0;
}

// per-segment |max| over a flat buffer into slots (segment i -> slot i of `out`): tab = [nblk][3] int64
// (segment, first float4, end float4)
void launch_amax_seg(const float* base, const int64_t* tab, int nblk, float* out, hipStream_t st) {
  if (nblk > 0) hipLaunchKernelGGL(amax_seg_kernel, dim3(nblk), dim3(256), 0, st, base, tab, out);
}

void launch_zero_segs(float* base, const int64_t* tab, int nblk, hipStream_t st) {
  if (nblk > 0) hipLaunchKernelGGL(zero_segs_kernel, dim3(nblk), dim3(256), 0, st, base, tab);
}
