// Stand-in for a data-parallel collective on a one-GPU box (bench.py --emulate-world W).
//
// The pool this framework is developed on has one MI355X per job, so RCCL never runs with more
// than one rank there; what the W-rank step would look like is PREDICTED by replacing each
// gradient collective of a 1-rank run with this kernel, enqueued exactly where the collective
// would be (the native engine's greatest-priority comm stream, behind the producer events):
//   * `channels` workgroups, like RCCL's one workgroup per channel -- they take CU slots beside
//     the backward's GEMM blocks for the collective's whole duration (the footprint a 1-rank
//     run, whose all-reduce is a no-op, never shows);
//   * together they stream `traffic` bytes: read from the bucket (wrapping), written to a scratch
//     buffer -- the HBM bytes a ring collective moves on each rank (what it receives and stores);
//   * every workgroup then stays resident until `hold_ns` after it started: the analytic transfer
//     time of the collective over xGMI (parallel/comm.py EmulatedComm picks it from the bytes each
//     rank receives and a bus bandwidth).
// The bucket itself is never modified (a 1-rank all-reduce is the identity), so the trained
// numbers are the 1-rank run's; only the timing is the W-rank prediction.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace hs {

__global__ void __launch_bounds__(256) comm_emul_kernel(const uint4* __restrict__ src, int64_t src16,
                                                        uint4* __restrict__ scratch, int64_t scr16, int64_t traffic16,
                                                        uint64_t hold_ticks) {
  const uint64_t t0 = wall_clock64();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  uint32_t sink = 0u;
  // four 16-B loads in flight per thread, as RCCL's unrolled copy/reduce primitives keep: with one,
  // the 32 workgroups are load-latency bound under a busy chip and stretch the collective well past
  // its link time (a layer's 28 MB reduce-scatter: 210 us against 74)
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < traffic16; i += 4 * stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = src[(i + u * stride) % src16];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      scratch[(i + u * stride) % scr16] = v[u];
      sink ^= v[u].x;
    }
  }
  for (; i < traffic16; i += stride) {
    const uint4 v = src[i % src16];
    scratch[i % scr16] = v;
    sink ^= v.x;
  }
  // hold the slot for the rest of the collective's analytic time (wall_clock64: constant-rate
  // counter, 100 MHz on gfx950); s_sleep keeps the resident waves off the issue ports
  while (wall_clock64() - t0 < hold_ticks) __builtin_amdgcn_s_sleep(8);
  if (sink == 0x9e3779b9u && threadIdx.x == 1023) scratch[0] = uint4{sink, 0u, 0u, 0u};  // keep the reads live
}

}  // namespace hs

// C signature the native comm engine (csrc/comm/comm.cpp) calls through a function pointer
extern "C" void hetseq_comm_emulation(const void* src, int64_t src_bytes, void* scratch, int64_t scratch_bytes,
                                      int64_t traffic_bytes, int channels, int64_t hold_ns, hipStream_t st) {
  // whole 16-B lines inside the bucket only: a bucket slice of the flat gradient or the stats vector
  // need not be 16-B aligned, and one shorter than a line is read from the (aligned) scratch instead
  const uintptr_t s0 = reinterpret_cast<uintptr_t>(src), s1 = s0 + (uintptr_t)std::max<int64_t>(src_bytes, 0);
  const uintptr_t a0 = (s0 + 15) & ~(uintptr_t)15;
  int64_t src16 = a0 < s1 ? (int64_t)((s1 - a0) / 16) : 0;
  const int64_t scr16 = std::max<int64_t>(scratch_bytes / 16, 1);
  if (src16 < 1) {
    src = scratch;
    src16 = scr16;
  } else {
    src = reinterpret_cast<const void*>(a0);
  }
  const int64_t traffic16 = std::max<int64_t>(traffic_bytes / 16, 0);
  int freq_khz = 100000;  // the wall clock's rate (hipDeviceAttributeWallClockRate, kHz)
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) {
    int f = 0;
    if (hipDeviceGetAttribute(&f, hipDeviceAttributeWallClockRate, dev) == hipSuccess && f > 0) freq_khz = f;
  }
  const uint64_t ticks = (uint64_t)((double)std::max<int64_t>(hold_ns, 0) * freq_khz / 1e6);
  hipLaunchKernelGGL(hs::comm_emul_kernel, dim3(std::max(channels, 1)), dim3(256), 0, st,
                     reinterpret_cast<const uint4*>(src), src16, reinterpret_cast<uint4*>(scratch), scr16, traffic16,
                     ticks);
}
