// fp32 / bf16 MFMA issue-rate microbenchmark (no memory traffic): what the
// chip sustains under a dense MFMA stream, to calibrate GEMM efficiency claims.
// build: hipcc --offload-arch=gfx950 -O3 mfma_peak.hip -o mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

template <int NACC>
__global__ void __launch_bounds__(256) f32_32x32(float* out, int iters, float a0) {
  f32x16 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f32x16{};
  float a = a0 + threadIdx.x, b = a0 * 2.f;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ void __launch_bounds__(256) f32_16x16(float* out, int iters, float a0) {
  f32x4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f32x4{};
  float a = a0 + threadIdx.x, b = a0 * 2.f;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ void __launch_bounds__(256) bf16_32x32(float* out, int iters, float a0) {
  f32x16 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f32x16{};
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (short)(0x3f80 + threadIdx.x + j);
    b[j] = (short)(0x3f00 + j);
  }
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i], 0, 0, 0);
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
double run(K kernel, int blocks, int iters, double flop_per_iter_per_wave) {
  float* out;
  hipMalloc(&out, blocks * 256 * sizeof(float));
  hipLaunchKernelGGL(kernel, dim3(blocks), dim3(256), 0, 0, out, 10, 1.0f);
  hipDeviceSynchronize();
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  hipEventRecord(s);
  hipLaunchKernelGGL(kernel, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms;
  hipEventElapsedTime(&ms, s, e);
  hipFree(out);
  return flop_per_iter_per_wave * iters * blocks * 4 / (ms * 1e-3) / 1e12;
}

int main() {
  const int cus = 256;
  for (int wps : {1, 2}) {  // waves per SIMD = blocks per CU (4 waves per block)
    const int blocks = cus * wps;
    printf("waves/SIMD=%d  f32 32x32x2 acc4: %.1f TF  acc8: %.1f TF | f32 16x16x4 acc4: %.1f TF  acc8: %.1f TF | "
           "bf16 32x32x16 acc4: %.1f TF\n",
           wps, run(f32_32x32<4>, blocks, 20000, 4 * 32 * 32 * 2 * 2.0),
           run(f32_32x32<8>, blocks, 10000, 8 * 32 * 32 * 2 * 2.0),
           run(f32_16x16<4>, blocks, 40000, 4 * 16 * 16 * 4 * 2.0),
           run(f32_16x16<8>, blocks, 20000, 8 * 16 * 16 * 4 * 2.0),
           run(bf16_32x32<4>, blocks, 20000, 4 * 32 * 32 * 16 * 2.0));
  }
  return 0;
}
