// pybind11 entry points for the gfx950 kernel library.
//
// Every entry takes raw device addresses (Python passes tensor.data_ptr())
// and the HIP stream handle (torch.cuda.current_stream().cuda_stream).  Shape
// and dtype validation happens in Python (hetseq_amd/ops/_C.py) BEFORE the
// launch, so a kernel never sees a shape its grid does not assume.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>
#include <pybind11/stl.h>

namespace py = pybind11;
using u64 = uint64_t;
using i64 = int64_t;

#define P(T, x) reinterpret_cast<T>(static_cast<uintptr_t>(x))
#define ST(x) reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(x))

// optim.hip
void launch_grad_norm(const float*, int64_t, double*, const float*, float, float*, hipStream_t);
int sumsq_blocks();
void launch_sumsq_segs(const float*, const int64_t*, int, int, double*, hipStream_t);
void launch_sum_partials(const double*, int, double*, hipStream_t);
void launch_norm_finalize(const double*, int, const float*, float, float*, hipStream_t);
void launch_stats_accum(double*, const float*, const float*, double, double, double, hipStream_t);
void launch_stats_finalize(double*, double, double, float*, hipStream_t);
void launch_adam_flat(float*, const float*, float*, float*, void*, int64_t, const float*, float, float, float, float,
                      float, float, float, float, const float*, hipStream_t);
void set_adam_config(int grid_cap, int unroll, int nt);
void launch_adadelta_flat(float*, const float*, float*, float*, void*, int64_t, const float*, float, float, float,
                          float, float, hipStream_t);
void launch_lamb_flat(float*, const float*, float*, float*, float*, void*, const int64_t*, int, float*, const float*,
                      float, float, float, float, float, float, float, float, float, hipStream_t);
void launch_cast_f32_bf16(const float*, void*, int64_t, hipStream_t);
// layernorm.hip
int ln_bwd_num_blocks();
int launch_ln_fwd(int, const void*, const float*, const void*, const float*, const float*, void*, float*, float*,
                  float*, int, int, float, float, u64, u64, int, int, int64_t, int, float*, hipStream_t);
int launch_ln_bwd(int, const void*, const float*, const float*, const float*, const float*, void*, void*, float*,
                  float*, float*, int, int, float, u64, u64, int, float*, hipStream_t);
int launch_emb_fwd(int, const int64_t*, const int64_t*, const float*, const float*, const float*, const float*,
                   const float*, void*, float*, float*, float*, int, int, int, int, int, float, float, u64, u64, int*,
                   float*, hipStream_t);
int launch_emb_bwd(int, const void*, const float*, const float*, const float*, const float*, float*, float*, float*,
                   const int64_t*, float*, int, int, float, u64, u64, hipStream_t);
void set_ln_h3p_waves(int w);
void set_ln_fwd_ns(int on);
int launch_ln_fwd_h3p(const void*, const float*, const void*, const float*, const float*, void*, float*, float*, float*,
                      int, int, float, float, u64, u64, int, int, int64_t, int, float*, void*, int64_t, int8_t*,
                      uint32_t*, int, hipStream_t);
int launch_ln_bwd_h3p(const float*, const float*, const float*, const float*, const float*, float*, float*, float*,
                      float*, int, int, float, u64, u64, void*, int64_t, int8_t*, uint32_t*, hipStream_t);
int ln_bwd_h3p_part_rows(int coop);
void set_ln_bwd_coop(int on);
void set_attn_h3_variant(int fwd_pair, int bwd_occ);
int launch_attn_fwd_h3(const float*, const int64_t*, const float*, float*, float*, uint32_t*, int, int, int, int, float,
                       uint64_t, uint64_t, hipStream_t, int, float*, void*, int64_t, int8_t*);
int launch_attn_bwd_h3(const float*, const int64_t*, const float*, const float*, const float*, const float*, float*,
                       float*, const uint32_t*, int, int, int, int, float, hipStream_t, float*, void*, int64_t,
                       int8_t*, float*);
void launch_colpart_finalize(const float* const*, float* const*, int, int, int, int, hipStream_t);
int launch_segsum_rows(const float*, const int64_t*, const int64_t*, float*, float*, int, int, int, hipStream_t);
int launch_sort_keys(const int64_t*, int, int64_t, int64_t*, int64_t*, int*, hipStream_t);
int launch_pos_grad(const float*, float*, int, int, int, hipStream_t);
// elementwise.hip
void launch_bias_gelu_fwd(int, const void*, const float*, void*, int64_t, int, hipStream_t);
int colsum_row_chunks(int64_t);
void launch_colsum(int, const void*, const void*, const float*, void*, float*, float*, int64_t, int, int, hipStream_t,
                   float*);
void launch_mlm_compact(const int64_t*, int, int, int, int32_t*, int64_t*, int32_t*, int*, hipStream_t);
void launch_gather_rows(int, const void*, const int32_t*, void*, int, int, hipStream_t);
void launch_scatter_add_rows(int, const void*, const int32_t*, void*, int, int, hipStream_t);
int launch_amax(const float*, int64_t, float*, int, hipStream_t);
void launch_amax_seg(const float*, const int64_t*, int, float*, hipStream_t);
void launch_zero_segs(float*, const int64_t*, int, hipStream_t);
// pool_nsp.hip
int launch_pool_nsp_fwd(int, const void*, int, int, int, const float*, const float*, const float*, const float*,
                        const int64_t*, const float*, float*, float*, float*, float*, float*, hipStream_t);
int launch_pool_nsp_bwd(int, const float*, const void*, void*, int, int, int, const float*, const float*,
                        const int64_t*, const float*, const float*, const float*, const float*, float*, float*,
                        float*, float*, float*, float*, float*, int, hipStream_t, int);
void launch_pool_nsp_wgrad(int, const void*, const float*, const float*, const float*, int, int, int, float*, float*,
                           float*, float*, int, hipStream_t);
// attention.hip
void set_attn_fp32_mode(int mode);
void set_ln_bwd_lds(int chunked);
int attn_fp32_mode();
int launch_attn_fwd(int, const void*, const int64_t*, const float*, void*, float*, uint32_t*, int, int, int, int, float,
                    u64, u64, hipStream_t, int, float*, int*);
int launch_attn_bwd(int, const void*, const int64_t*, const float*, const void*, const void*, const float*, float*,
                    void*, const uint32_t*, int, int, int, int, float, hipStream_t, float*, int*);
// xent.hip
void launch_xent_fwd(int, const void*, const int64_t*, int, int, int64_t, int, float*, float*, float*, hipStream_t);
void launch_xent_bwd(int, void*, const int64_t*, const float*, int, int, int64_t, int, const float*, const float*,
                     hipStream_t, float*);
// gemm.hip
int gemm_last_ksplit();
void set_h3_occ3(int on);
int launch_gemm(int dtype, int ta, int tb, int M, int N, int K, const void* A, int64_t lda, const void* B,
                int64_t ldb, void* C, int64_t ldc, const float* bias, int epi, float beta, float* aux, int64_t ldaux,
                float* part, float* colsum_out, int colsum_acc, int tile_override, hipStream_t st, int ksplit,
                float* slab, int64_t slab_floats, int mv, int nv, int kv, const float* amax_a, int namax_a,
                const float* amax_b, int namax_b, float* amax_c);
void set_wcol_fold(int on);

// gemm_planes.hip
int launch_gemm_planes(int planes, int c_dtype, int ta, int tb, int M, int N, int K, const void* A, int64_t lda,
                       int64_t a_ps, const void* B, int64_t ldb, int64_t b_ps, void* C, int64_t ldc,
                       const float* bias, int epi, float beta, void* aux, int64_t ldaux, float* part,
                       float* colsum_out, int colsum_acc, int ksplit, float* slab, int64_t slab_floats,
                       int variant, hipStream_t st, int Mv);
void set_planes_variant(int v);

// gemm_h3p.hip
int launch_gemm_h3p_v(int ta, int tb, int M, int N, int K, const void* A, int64_t lda, int64_t a_ps, const int8_t* ea,
                      int64_t lde_a, const void* B, int64_t ldb, int64_t b_ps, const int8_t* eb, int64_t lde_b,
                      float* C, int64_t ldc, const float* bias, int epi, float beta, float* aux, int64_t ldaux,
                      float* part, float* colsum, int colsum_acc, void* cp, int64_t ldcp, int64_t cp_ps, int8_t* ec,
                      int64_t lde_c, int ksplit, float* slab, int64_t slab_floats, int ablk, int bblk, int Mv, int Nv,
                      hipStream_t st);
int launch_gemm_h3p(int ta, int tb, int M, int N, int K, const void* A, int64_t lda, int64_t a_ps, const int8_t* ea,
                    int64_t lde_a, const void* B, int64_t ldb, int64_t b_ps, const int8_t* eb, int64_t lde_b, float* C,
                    int64_t ldc, const float* bias, int epi, float beta, float* aux, int64_t ldaux, float* part,
                    float* colsum, int colsum_acc, void* cp, int64_t ldcp, int64_t cp_ps, int8_t* ec, int64_t lde_c,
                    int ksplit, float* slab, int64_t slab_floats, int ablk, int bblk, hipStream_t st);
int launch_h3p_split(const float* src, int64_t lds, int rows, int cols, void* dst, int64_t ldd, int64_t ps, int8_t* ex,
                     int64_t lde, int blocked, int vrows, hipStream_t st);
int h3p_split_seg_bytes();
int launch_h3p_colpart(const void*, int64_t, int64_t, const int8_t*, int64_t, int, int, float*, hipStream_t);
void launch_h3p_split_multi(const void* table, int nseg, int total, hipStream_t st);

// mnist.hip
void launch_mnist_conv1_fwd(const float*, const float*, const float*, float*, int, hipStream_t);
void launch_mnist_im2col(const float*, float*, int, int, hipStream_t);
void launch_mnist_perm(const float*, float*, int, int, hipStream_t);
void launch_mnist_pool_fwd(const float*, float*, uint8_t*, int, int, float, uint64_t, uint64_t, hipStream_t);
void launch_mnist_pool_bwd(const float*, const uint8_t*, float*, int, int, float, hipStream_t);
void launch_mnist_head_fwd(const float*, const float*, const float*, const int64_t*, float*, float*, float*, int, float,
                           uint64_t, uint64_t, hipStream_t);
void launch_mnist_loss(const float*, const float*, const int64_t*, int, int, float*, float*, float*, hipStream_t);
void launch_mnist_head_bwd(const float*, const float*, const float*, const int64_t*, const float*, const float*,
                           const float*, float*, float*, int, int, int, float, hipStream_t);
void launch_mnist_fc2_wgrad(const float*, const float*, float*, float*, float*, int, hipStream_t);
void launch_mnist_col2im(const float*, const float*, float*, int, hipStream_t);
void launch_mnist_conv1_wgrad(const float*, const float*, float*, float*, float*, int, hipStream_t);

// comm_emul.hip (called by the native comm engine through its address)
extern "C" void hetseq_comm_emulation(const void*, int64_t, void*, int64_t, int64_t, int, int64_t, hipStream_t);

// HIP-graph mode: device word holding the dropout seed (see common.h resolve_seed)
namespace hs {
const uint64_t* g_seed_dev = nullptr;
int g_hs_skip = 0;
}

static void check(int rc, const char* what) {
  if (rc != 0) throw std::invalid_argument(std::string(what) + ": unsupported shape for the HIP kernel");
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
static void check_launch(const char* what) { check(0, what); }
// An error left pending by an EARLIER HIP call (torch's or ours) is raised here, named against the
// op about to launch, instead of being cleared and lost.  Only the status codes torch's own
// queries and P2P probes leave behind are benign and cleared: hipErrorNotReady (event / stream
// queries), peer access already enabled / not enabled.
static void pre_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess || e == hipErrorNotReady || e == hipErrorPeerAccessAlreadyEnabled ||
      e == hipErrorPeerAccessNotEnabled)
    return;
  throw std::runtime_error(std::string("HIP error pending before ") + what + " (left by an earlier call): " +
                           hipGetErrorString(e));
}

// Stream fork/join for the weight-gradient side stream (runtime/streams.py): record an event on
// `signal`, make `waiter` wait for it.  A ring of timing-free events, created once; an event is
// re-recorded only after 64 later forks, long after the wait that used it was enqueued (a wait
// captures the event's state at enqueue time).
// Cross-stream ordering point: `waiter` runs nothing enqueued after this until `signal` has
// finished everything enqueued so far.  Events from a ring of 64, created with
// g_wait_flags (hipEventDisableTiming by default; tools/probes/fork_gap.py measures the flag
// choices, set_stream_wait_flags switches them).
static unsigned g_wait_flags = hipEventDisableTiming;
void hs_stream_wait(hipStream_t waiter, hipStream_t signal) {
  static hipEvent_t ring[64];
  static int n = 0;
  static unsigned made = ~0u;
  if (made != g_wait_flags) {
    if (made != ~0u) {
      if (hipDeviceSynchronize() != hipSuccess) throw std::runtime_error("stream_wait: hipDeviceSynchronize");
      for (auto& e : ring) (void)hipEventDestroy(e);
    }
    for (auto& e : ring)
      if (hipEventCreateWithFlags(&e, g_wait_flags) != hipSuccess) throw std::runtime_error("hipEventCreate");
    made = g_wait_flags;
  }
  hipEvent_t e = ring[n++ & 63];
  if (hipEventRecord(e, signal) != hipSuccess || hipStreamWaitEvent(waiter, e, 0) != hipSuccess)
    throw std::runtime_error("stream_wait: hipEventRecord/hipStreamWaitEvent failed");
}

static void stream_wait(hipStream_t waiter, hipStream_t signal) { hs_stream_wait(waiter, signal); }

// layer_prog.cpp
std::vector<std::string> layer_plan_fields();
void layer_fwd_h3p(int64_t, int64_t, int64_t, int64_t, int64_t, uint64_t, uint64_t, uint64_t, uint64_t, uint64_t,
                   uint64_t, float, float, float, int64_t, int64_t, int64_t, int64_t, int);
void layer_bwd_h3p(int64_t, int64_t, int64_t, int64_t, int64_t, uint64_t, uint64_t, uint64_t, uint64_t, float, float,
                   int, int64_t, int64_t, int64_t);

PYBIND11_MODULE(_hip, m) {
  m.doc() = "hetseq_amd CDNA4 (gfx950) kernels";
  m.attr("arch") = "gfx950";
  m.def("pci_bus_id", [](int dev) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) throw std::runtime_error("hipDeviceGetPCIBusId");
    return std::string(bus);
  }, "PCI bus id of HIP device `dev` (bench.py: one rank per distinct device)");

  m.def("layer_plan_fields", &layer_plan_fields, "field names of a layer program's int64 plan (layer_prog.cpp)");
  m.def("layer_fwd_h3p", [](i64 plan, i64 x, i64 xp, i64 xe, i64 mask, u64 sa, u64 oa, u64 s1, u64 o1, u64 s2, u64 o2,
                            float eps, float p_h, float p_a, i64 st0, i64 st1, i64 amax0, i64 amax1, int stagger) {
    pre_launch("layer_fwd_h3p");
    layer_fwd_h3p(plan, x, xp, xe, mask, sa, oa, s1, o1, s2, o2, eps, p_h, p_a, st0, st1, amax0, amax1, stagger);
    check_launch("layer_fwd_h3p");
  }, "one fused encoder-layer forward on the h3p engine from its plan (ops/layer_prog.py); stagger: the second "
     "chain starts after the first chain's QKV product (1), attention (2) or first LayerNorm (3)",
     py::arg("plan"), py::arg("x"), py::arg("xp"), py::arg("xe"), py::arg("mask"), py::arg("sa"), py::arg("oa"),
     py::arg("s1"), py::arg("o1"), py::arg("s2"), py::arg("o2"), py::arg("eps"), py::arg("p_h"), py::arg("p_a"),
     py::arg("st0"), py::arg("st1"), py::arg("amax0"), py::arg("amax1"), py::arg("stagger") = 0);
  m.def("layer_bwd_h3p", [](i64 plan, i64 dh2, i64 xp, i64 xe, i64 mask, u64 s1, u64 o1, u64 s2, u64 o2, float p_h,
                            float p_a, int wacc, i64 st0, i64 st1, i64 events) {
    pre_launch("layer_bwd_h3p");
    layer_bwd_h3p(plan, dh2, xp, xe, mask, s1, o1, s2, o2, p_h, p_a, wacc, st0, st1, events);
    check_launch("layer_bwd_h3p");
  }, "one fused encoder-layer backward on the h3p engine from its plan (ops/layer_prog.py); events: 0 or the "
     "address of 4 hipEvent_t recorded as each parameter-gradient group completes", py::arg("plan"), py::arg("dh2"),
     py::arg("xp"), py::arg("xe"), py::arg("mask"), py::arg("s1"), py::arg("o1"), py::arg("s2"), py::arg("o2"),
     py::arg("p_h"), py::arg("p_a"), py::arg("wacc"), py::arg("st0"), py::arg("st1"), py::arg("events") = 0);
  m.def("event_create", []() {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) throw std::runtime_error("hipEventCreate");
    return (i64) reinterpret_cast<uintptr_t>(e);
  }, "a raw timing-free hipEvent_t (process lifetime; layer-program readiness events)");
  m.def("sumsq_blocks", &sumsq_blocks);
  m.def("sumsq_segs", [](i64 g, i64 segs, int nseg, int nblk, i64 partial, i64 st) {
    pre_launch("sumsq_segs");
    if (nseg < 1 || nblk < nseg) throw std::invalid_argument("sumsq_segs: >= 1 range, >= 1 block per range");
    launch_sumsq_segs(P(const float*, g), P(const int64_t*, segs), nseg, nblk, P(double*, partial), ST(st));
    check_launch("sumsq_segs");
  }, "sums of squares of the ranges segs[3i:3i+2] of g into nblk fp64 partials (range i from block segs[3i+2]; "
     "a sharded gradient's owned ranges, one launch)");
  m.def("sum_partials", [](i64 partial, int n, i64 out, i64 st) {
    pre_launch("sum_partials");
    launch_sum_partials(P(const double*, partial), n, P(double*, out), ST(st));
    check_launch("sum_partials");
  });
  m.def("norm_finalize", [](i64 partial, int n, i64 scale, float max_norm, i64 out, i64 st) {
    pre_launch("norm_finalize");
    launch_norm_finalize(P(const double*, partial), n, P(const float*, scale), max_norm, P(float*, out), ST(st));
    check_launch("norm_finalize");
  }, "total norm / combined multiplier / clip coefficient from fp64 partial sums of squares");
  m.def("grad_norm", [](i64 g, i64 n, i64 partial, i64 scale, float max_norm, i64 out, i64 st) {
    pre_launch("grad_norm");
    launch_grad_norm(P(const float*, g), n, P(double*, partial), P(const float*, scale), max_norm, P(float*, out), ST(st));
    check_launch("grad_norm");
  });
  m.def("stats_accum", [](i64 st, i64 loss, i64 nll, double ss, double ns, double nt, i64 stream) {
    pre_launch("stats_accum");
    launch_stats_accum(P(double*, st), P(const float*, loss), P(const float*, nll), ss, ns, nt, ST(stream));
    check_launch("stats_accum");
  });
  m.def("stats_finalize", [](i64 st, double ln2, double w, i64 scale, i64 stream) {
    pre_launch("stats_finalize");
    launch_stats_finalize(P(double*, st), ln2, w, P(float*, scale), ST(stream));
    check_launch("stats_finalize");
  });
  // betas / rho arrive as Python doubles: 1 - beta is formed in double and rounded once (see optim.hip)
  m.def("adam_flat", [](i64 p, i64 g, i64 mm, i64 v, i64 shadow, i64 n, i64 gmul, float lr, double b1, double b2,
                        float eps, float wd, float step_size, i64 st, i64 hyper) {
    pre_launch("adam_flat");
    launch_adam_flat(P(float*, p), P(const float*, g), P(float*, mm), P(float*, v), P(void*, shadow), n,
                     P(const float*, gmul), lr, (float)b1, (float)b2, (float)(1.0 - b1), (float)(1.0 - b2), eps, wd,
                     step_size, P(const float*, hyper), ST(st));
    check_launch("adam_flat");
  }, pybind11::arg("p"), pybind11::arg("g"), pybind11::arg("m"), pybind11::arg("v"), pybind11::arg("shadow"),
     pybind11::arg("n"), pybind11::arg("gmul"), pybind11::arg("lr"), pybind11::arg("b1"), pybind11::arg("b2"),
     pybind11::arg("eps"), pybind11::arg("wd"), pybind11::arg("step_size"), pybind11::arg("st"),
     pybind11::arg("hyper") = 0);
  m.def("set_adam_config", &set_adam_config, "fp32 Adam pass launch shape: grid cap, float4 groups per thread per "
        "iteration (1 / 2 / 4), streaming accesses (benchmarking)");
  m.def("adadelta_flat", [](i64 p, i64 g, i64 sq, i64 acc, i64 shadow, i64 n, i64 gmul, float lr, double rho,
                            float eps, float wd, i64 st) {
    pre_launch("adadelta_flat");
    launch_adadelta_flat(P(float*, p), P(const float*, g), P(float*, sq), P(float*, acc), P(void*, shadow), n,
                         P(const float*, gmul), lr, (float)rho, (float)(1.0 - rho), eps, wd, ST(st));
    check_launch("adadelta_flat");
  });
  m.def("lamb_flat", [](i64 p, i64 g, i64 mm, i64 v, i64 upd, i64 shadow, i64 seg_off, int nseg, i64 seg_norms, i64 gmul,
                        float lr, double b1, double b2, float eps, float wd, float bc1, float bc2, i64 st) {
    pre_launch("lamb_flat");
    launch_lamb_flat(P(float*, p), P(const float*, g), P(float*, mm), P(float*, v), P(float*, upd), P(void*, shadow),
                     P(const int64_t*, seg_off), nseg, P(float*, seg_norms), P(const float*, gmul), lr, (float)b1,
                     (float)b2, (float)(1.0 - b1), (float)(1.0 - b2), eps, wd, bc1, bc2, ST(st));
    check_launch("lamb_flat");
  });
  m.def("cast_f32_bf16", [](i64 x, i64 y, i64 n, i64 st) {
    pre_launch("cast_f32_bf16");
    launch_cast_f32_bf16(P(const float*, x), P(void*, y), n, ST(st));
    check_launch("cast_f32_bf16");
  });

  m.def("ln_bwd_num_blocks", &ln_bwd_num_blocks);
  m.def("ln_fwd", [](int dt, i64 a, i64 bias, i64 resid, i64 gamma, i64 beta, i64 y, i64 zsave, i64 mean, i64 rstd,
                     int rows, int H, float eps, float p, u64 seed, u64 off, int mode, i64 st,
                     int nslab, i64 slab_stride, int row0, i64 amax) {
    pre_launch("ln_fwd");
    check(launch_ln_fwd(dt, P(const void*, a), P(const float*, bias), P(const void*, resid), P(const float*, gamma),
                        P(const float*, beta), P(void*, y), P(float*, zsave), P(float*, mean), P(float*, rstd), rows, H,
                        eps, p, seed, off, mode, nslab, slab_stride, row0, P(float*, amax), ST(st)),
          "ln_fwd");
  }, py::arg("dt"), py::arg("a"), py::arg("bias"), py::arg("resid"), py::arg("gamma"), py::arg("beta"), py::arg("y"),
     py::arg("zsave"), py::arg("mean"), py::arg("rstd"), py::arg("rows"), py::arg("H"), py::arg("eps"), py::arg("p"),
     py::arg("seed"), py::arg("off"), py::arg("mode"), py::arg("st"),
     py::arg("nslab") = 1, py::arg("slab_stride") = 0, py::arg("row0") = 0, py::arg("amax") = 0);
  m.def("ln_bwd", [](int dt, i64 dy, i64 zsave, i64 mean, i64 rstd, i64 gamma, i64 dz, i64 da, i64 pg, i64 pb, i64 pbias,
                     int rows, int H, float p, u64 seed, u64 off, int mode, i64 st, i64 amax) {
    pre_launch("ln_bwd");
    check(launch_ln_bwd(dt, P(const void*, dy), P(const float*, zsave), P(const float*, mean), P(const float*, rstd),
                        P(const float*, gamma), P(void*, dz), P(void*, da), P(float*, pg), P(float*, pb),
                        P(float*, pbias), rows, H, p, seed, off, mode, P(float*, amax), ST(st)),
          "ln_bwd");
  }, py::arg("dt"), py::arg("dy"), py::arg("zsave"), py::arg("mean"), py::arg("rstd"), py::arg("gamma"), py::arg("dz"),
     py::arg("da"), py::arg("pg"), py::arg("pb"), py::arg("pbias"), py::arg("rows"), py::arg("H"), py::arg("p"),
     py::arg("seed"), py::arg("off"), py::arg("mode"), py::arg("st"),
     py::arg("amax") = 0);
  m.def("emb_fwd", [](int dt, i64 ids, i64 tt, i64 w, i64 pe, i64 te, i64 gamma, i64 beta, i64 y, i64 zsave, i64 mean,
                      i64 rstd, int rows, int S, int H, int V, int TV, float eps, float p, u64 seed, u64 off, i64 err,
                      i64 st, i64 amax) {
    pre_launch("emb_fwd");
    check(launch_emb_fwd(dt, P(const int64_t*, ids), P(const int64_t*, tt), P(const float*, w), P(const float*, pe),
                         P(const float*, te), P(const float*, gamma), P(const float*, beta), P(void*, y),
                         P(float*, zsave), P(float*, mean), P(float*, rstd), rows, S, H, V, TV, eps, p, seed, off,
                         P(int*, err), P(float*, amax), ST(st)),
          "emb_fwd");
  }, py::arg("dt"), py::arg("ids"), py::arg("tt"), py::arg("w"), py::arg("pe"), py::arg("te"), py::arg("gamma"),
     py::arg("beta"), py::arg("y"), py::arg("zsave"), py::arg("mean"), py::arg("rstd"), py::arg("rows"), py::arg("S"),
     py::arg("H"), py::arg("V"), py::arg("TV"), py::arg("eps"), py::arg("p"), py::arg("seed"), py::arg("off"),
     py::arg("err"), py::arg("st"), py::arg("amax") = 0);
  m.def("emb_bwd", [](int dt, i64 dy, i64 zsave, i64 mean, i64 rstd, i64 gamma, i64 dx, i64 pg, i64 pb, i64 tt, i64 pt,
                      int rows, int H, float p, u64 seed, u64 off, i64 st) {
    pre_launch("emb_bwd");
    check(launch_emb_bwd(dt, P(const void*, dy), P(const float*, zsave), P(const float*, mean), P(const float*, rstd),
                         P(const float*, gamma), P(float*, dx), P(float*, pg), P(float*, pb), P(const int64_t*, tt),
                         P(float*, pt), rows, H, p, seed, off, ST(st)),
          "emb_bwd");
  });
  m.def("sort_keys", [](i64 keys, int n, i64 bound, i64 out_keys, i64 out_order, i64 err, i64 st) {
    pre_launch("sort_keys");
    const int rc = launch_sort_keys(P(const int64_t*, keys), n, bound, P(int64_t*, out_keys), P(int64_t*, out_order),
                                    P(int*, err), ST(st));
    if (rc == 0) check_launch("sort_keys");  // a failed launch must not leave out_keys / out_order unwritten
    return rc;
  }, "stable sort of n int64 keys in [0, bound): sorted keys + source indices; -1 = unsupported size; a key "
     "outside [0, bound) sets bit 2 of *err and sorts as clamped");
  // ---- MNISTNet (mnist.hip); every entry raw pointers + batch size + stream
  m.def("mnist_conv1_fwd", [](i64 x, i64 w, i64 b, i64 y, int B, i64 st) {
    pre_launch("mnist_conv1_fwd");
    launch_mnist_conv1_fwd(P(const float*, x), P(const float*, w), P(const float*, b), P(float*, y), B, ST(st));
    check_launch("mnist_conv1_fwd");
  });
  m.def("mnist_im2col", [](i64 h1, i64 col, int B, int R, i64 st) {
    pre_launch("mnist_im2col");
    check(R >= B * 576 ? 0 : -1, "mnist_im2col");
    launch_mnist_im2col(P(const float*, h1), P(float*, col), B, R, ST(st));
    check_launch("mnist_im2col");
  });
  m.def("mnist_perm", [](i64 src, i64 dst, int rows, int mode, i64 st) {
    pre_launch("mnist_perm");
    check(mode >= 0 && mode <= 3 ? 0 : -1, "mnist_perm");
    launch_mnist_perm(P(const float*, src), P(float*, dst), rows, mode, ST(st));
    check_launch("mnist_perm");
  });
  m.def("mnist_pool_fwd", [](i64 c2, i64 pooled, i64 arg, int B, int Bp, float p, u64 seed, u64 off, i64 st) {
    pre_launch("mnist_pool_fwd");
    launch_mnist_pool_fwd(P(const float*, c2), P(float*, pooled), P(uint8_t*, arg), B, Bp, p, seed, off, ST(st));
    check_launch("mnist_pool_fwd");
  });
  m.def("mnist_pool_bwd", [](i64 dpooled, i64 arg, i64 dc2, int B, int R, float p, i64 st) {
    pre_launch("mnist_pool_bwd");
    check(R >= B * 576 ? 0 : -1, "mnist_pool_bwd");
    launch_mnist_pool_bwd(P(const float*, dpooled), P(const uint8_t*, arg), P(float*, dc2), B, R, p, ST(st));
    check_launch("mnist_pool_bwd");
  });
  m.def("mnist_head_fwd", [](i64 pre, i64 w2, i64 b2, i64 target, i64 h, i64 logp, i64 nll, int B, float p, u64 seed,
                             u64 off, i64 st) {
    pre_launch("mnist_head_fwd");
    launch_mnist_head_fwd(P(const float*, pre), P(const float*, w2), P(const float*, b2), P(const int64_t*, target),
                          P(float*, h), P(float*, logp), P(float*, nll), B, p, seed, off, ST(st));
    check_launch("mnist_head_fwd");
  });
  m.def("mnist_loss", [](i64 nll, i64 logp, i64 target, int B, int mean, i64 loss, i64 correct, i64 count, i64 st) {
    pre_launch("mnist_loss");
    launch_mnist_loss(P(const float*, nll), P(const float*, logp), P(const int64_t*, target), B, mean, P(float*, loss),
                      P(float*, correct), P(float*, count), ST(st));
    check_launch("mnist_loss");
  });
  m.def("mnist_head_bwd", [](i64 dloss, i64 count, i64 logp, i64 target, i64 pre, i64 h, i64 w2, i64 dlogits,
                             i64 dpre, int B, int Bp, int mean, float p, i64 st) {
    pre_launch("mnist_head_bwd");
    launch_mnist_head_bwd(P(const float*, dloss), P(const float*, count), P(const float*, logp),
                          P(const int64_t*, target), P(const float*, pre), P(const float*, h), P(const float*, w2),
                          P(float*, dlogits), P(float*, dpre), B, Bp, mean, p, ST(st));
    check_launch("mnist_head_bwd");
  });
  m.def("mnist_fc2_wgrad", [](i64 dlogits, i64 h, i64 part, i64 dw2, i64 db2, int B, i64 st) {
    pre_launch("mnist_fc2_wgrad");
    launch_mnist_fc2_wgrad(P(const float*, dlogits), P(const float*, h), P(float*, part), P(float*, dw2),
                           P(float*, db2), B, ST(st));
    check_launch("mnist_fc2_wgrad");
  });
  m.def("mnist_col2im", [](i64 dcol, i64 h1, i64 dh1, int B, i64 st) {
    pre_launch("mnist_col2im");
    launch_mnist_col2im(P(const float*, dcol), P(const float*, h1), P(float*, dh1), B, ST(st));
    check_launch("mnist_col2im");
  });
  m.def("mnist_conv1_wgrad", [](i64 dh1, i64 x, i64 part, i64 dw1, i64 db1, int B, i64 st) {
    pre_launch("mnist_conv1_wgrad");
    launch_mnist_conv1_wgrad(P(const float*, dh1), P(const float*, x), P(float*, part), P(float*, dw1),
                             P(float*, db1), B, ST(st));
    check_launch("mnist_conv1_wgrad");
  });
  m.def("segsum_rows", [](i64 src, i64 order, i64 keys, i64 scratch, i64 dst, int n, int H, int K, i64 st) {
    pre_launch("segsum_rows");
    check(launch_segsum_rows(P(const float*, src), P(const int64_t*, order), P(const int64_t*, keys),
                             P(float*, scratch), P(float*, dst), n, H, K, ST(st)),
          "segsum_rows");
  });
  m.def("pos_grad", [](i64 dx, i64 dpos, int B, int S, int H, i64 st) {
    pre_launch("pos_grad");
    check(launch_pos_grad(P(const float*, dx), P(float*, dpos), B, S, H, ST(st)), "pos_grad");
  });
  m.def("colpart_finalize", [](py::list parts, py::list outs, int nparts, int H, int accumulate, i64 st) {
    pre_launch("colpart_finalize");
    const int n = static_cast<int>(parts.size());
    if (n < 1 || n > 3 || outs.size() != parts.size()) throw std::invalid_argument("colpart_finalize: 1..3 pairs");
    const float* pp[3];
    float* oo[3];
    for (int i = 0; i < n; ++i) {
      pp[i] = P(const float*, parts[i].cast<i64>());
      oo[i] = P(float*, outs[i].cast<i64>());
    }
    launch_colpart_finalize(pp, oo, n, nparts, H, accumulate, ST(st));
    check_launch("colpart_finalize");
  });

  m.def("bias_gelu_fwd", [](int dt, i64 x, i64 b, i64 y, i64 rows, int N, i64 st) {
    pre_launch("bias_gelu_fwd");
    launch_bias_gelu_fwd(dt, P(const void*, x), P(const float*, b), P(void*, y), rows, N, ST(st));
    check_launch("bias_gelu_fwd");
  });
  m.def("gemm_h3p", [](int ta, int tb, int M, int N, int K, i64 A, i64 lda, i64 a_ps, i64 ea, i64 lde_a, i64 B,
                       i64 ldb, i64 b_ps, i64 eb, i64 lde_b, i64 C, i64 ldc, i64 bias, int epi, float beta, i64 aux,
                       i64 ldaux, i64 part, i64 colsum, int colsum_acc, i64 cp, i64 ldcp, i64 cp_ps, i64 ec, i64 lde_c,
                       int ksplit, i64 slab, i64 slab_floats, i64 st, int ablk, int bblk, int mv, int nv) {
    pre_launch("gemm_h3p");
    const int rc = launch_gemm_h3p_v(ta, tb, M, N, K, P(const void*, A), lda, a_ps, P(const int8_t*, ea), lde_a,
                                     P(const void*, B), ldb, b_ps, P(const int8_t*, eb), lde_b, P(float*, C), ldc,
                                     P(const float*, bias), epi, beta, P(float*, aux), ldaux, P(float*, part),
                                     P(float*, colsum), colsum_acc, P(void*, cp), ldcp, cp_ps, P(int8_t*, ec), lde_c,
                                     ksplit, P(float*, slab), slab_floats, ablk, bblk, mv, nv, ST(st));
    if (rc == 0) check_launch("gemm_h3p");
    return rc;
  }, "fp32 GEMM as three fp16 products over block-scaled h3p planes (gemm_h3p.hip); -1 = not served",
     py::arg("ta"), py::arg("tb"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("A"), py::arg("lda"),
     py::arg("a_ps"), py::arg("ea"), py::arg("lde_a"), py::arg("B"), py::arg("ldb"), py::arg("b_ps"), py::arg("eb"),
     py::arg("lde_b"), py::arg("C"), py::arg("ldc"), py::arg("bias"), py::arg("epi"), py::arg("beta"), py::arg("aux"),
     py::arg("ldaux"), py::arg("part"), py::arg("colsum"), py::arg("colsum_acc"), py::arg("cp"), py::arg("ldcp"),
     py::arg("cp_ps"), py::arg("ec"), py::arg("lde_c"), py::arg("ksplit"), py::arg("slab"), py::arg("slab_floats"),
     py::arg("st"), py::arg("ablk") = 0, py::arg("bblk") = 0, py::arg("mv") = 0, py::arg("nv") = 0);
  m.def("h3p_colpart", [](i64 pl, i64 ld, i64 ps, i64 ex, i64 lde, int rows, int cols, i64 part, i64 st) {
    pre_launch("h3p_colpart");
    check(launch_h3p_colpart(P(const void*, pl), ld, ps, P(const int8_t*, ex), lde, rows, cols, P(float*, part), ST(st)),
          "h3p_colpart");
  }, "column partials per 32-row panel of a blocked h3p operand: part[r / 32][c] (fp32 [rows / 32, cols])");
  m.def("h3p_split", [](i64 src, i64 lds, int rows, int cols, i64 dst, i64 ldd, i64 ps, i64 ex, i64 lde, i64 st,
                        int blocked, int vrows) {
    pre_launch("h3p_split");
    check(launch_h3p_split(P(const float*, src), lds, rows, cols, P(void*, dst), ldd, ps, P(int8_t*, ex), lde, blocked,
                           vrows, ST(st)),
          "h3p_split");
  }, py::arg("src"), py::arg("lds"), py::arg("rows"), py::arg("cols"), py::arg("dst"), py::arg("ldd"), py::arg("ps"),
     py::arg("ex"), py::arg("lde"), py::arg("st"), py::arg("blocked") = 0, py::arg("vrows") = 0);
  m.def("h3p_split_seg_bytes", &h3p_split_seg_bytes);
  m.def("attn_fwd_h3p", [](i64 qkv, i64 mask, i64 bqkv, i64 ctx, i64 lse, i64 dmask, int B, int S, int NH, float p,
                           u64 seed, u64 off, int bh0, i64 pl, i64 ps, i64 ex, i64 st) {
    pre_launch("attn_fwd_h3p");
    check(launch_attn_fwd_h3(P(const float*, qkv), P(const int64_t*, mask), P(const float*, bqkv), P(float*, ctx),
                             P(float*, lse), P(uint32_t*, dmask), B, S, NH, 64, p, seed, off, ST(st), bh0, nullptr,
                             P(void*, pl), ps, P(int8_t*, ex)),
          "attn_fwd_h3p");
  }, "h3 attention forward also writing ctx as h3p planes");
  m.def("attn_bwd_h3p", [](i64 qkv, i64 mask, i64 bqkv, i64 ctx, i64 dctx, i64 lse, i64 dbuf, i64 dqkv, i64 dmask,
                           int B, int S, int NH, float p, i64 pl, i64 ps, i64 ex, i64 st, i64 dsbuf) {
    pre_launch("attn_bwd_h3p");
    check(launch_attn_bwd_h3(P(const float*, qkv), P(const int64_t*, mask), P(const float*, bqkv),
                             P(const float*, ctx), P(const float*, dctx), P(const float*, lse), P(float*, dbuf),
                             P(float*, dqkv), P(const uint32_t*, dmask), B, S, NH, 64, p, ST(st), nullptr,
                             P(void*, pl), ps, P(int8_t*, ex), P(float*, dsbuf)),
          "attn_bwd_h3p");
  }, "h3 attention backward also writing dqkv as h3p planes (dqkv 0: only as the planes; dsbuf: B*NH*S*S floats, "
     "dQ from the stored dS)", py::arg("qkv"), py::arg("mask"), py::arg("bqkv"), py::arg("ctx"), py::arg("dctx"),
     py::arg("lse"), py::arg("dbuf"), py::arg("dqkv"), py::arg("dmask"), py::arg("B"), py::arg("S"), py::arg("NH"),
     py::arg("p"), py::arg("pl"), py::arg("ps"), py::arg("ex"), py::arg("st"), py::arg("dsbuf") = 0);
  m.def("set_ln_fwd_ns", &set_ln_fwd_ns, "h3p LN forward: slab count at compile time (1) / runtime loop (0)");
  m.def("set_ln_h3p_waves", &set_ln_h3p_waves,
        "h3p LayerNorm forward kernel: 0 / 1 panel exchange at 8 / 4 rows per workgroup, 16 / 8 one 32-row block");
  m.def("ln_bwd_h3p_part_rows", &ln_bwd_h3p_part_rows, "rows per column-partial row of ln_bwd_h3p (coop: psync given)");
  m.def("set_ln_bwd_coop", &set_ln_bwd_coop, "h3p LayerNorm backward: 1 / 2 panel exchange (8 / 4 rows per workgroup), 0 32-row blocks");
  m.def("set_attn_h3_variant", &set_attn_h3_variant,
        "h3 attention forward: -1 by sequence length (paired 64-key tiles from S = 256), 1 paired, 0 per tile");
  m.def("panel_sync_words", []() { return 256; }, "uint32 words of one 32-row panel record (h3p.h kPanelSyncWords)");
  m.def("ln_fwd_h3p", [](i64 a, i64 bias, i64 resid, i64 gamma, i64 beta, i64 y, i64 z, i64 mean, i64 rstd, int rows,
                         int H, float eps, float p, u64 seed, u64 off, int mode, int nslab, i64 slab_stride, int row0,
                         i64 amax, i64 planes, i64 ps, i64 exps, i64 psync, int panel0, i64 st) {
    pre_launch("ln_fwd_h3p");
    check(launch_ln_fwd_h3p(P(const void*, a), P(const float*, bias), P(const void*, resid), P(const float*, gamma),
                            P(const float*, beta), P(void*, y), P(float*, z), P(float*, mean), P(float*, rstd), rows, H,
                            eps, p, seed, off, mode, nslab, slab_stride, row0, P(float*, amax), P(void*, planes), ps,
                            P(int8_t*, exps), P(uint32_t*, psync), panel0, ST(st)),
          "ln_fwd_h3p");
  });
  m.def("ln_bwd_h3p", [](i64 dy, i64 z, i64 mean, i64 rstd, i64 gamma, i64 dz, i64 pg, i64 pb, i64 pbias, int rows,
                         int H, float p, u64 seed, u64 off, i64 planes, i64 ps, i64 exps, i64 psync, i64 st) {
    pre_launch("ln_bwd_h3p");
    check(launch_ln_bwd_h3p(P(const float*, dy), P(const float*, z), P(const float*, mean), P(const float*, rstd),
                            P(const float*, gamma), P(float*, dz), P(float*, pg), P(float*, pb), P(float*, pbias), rows,
                            H, p, seed, off, P(void*, planes), ps, P(int8_t*, exps), P(uint32_t*, psync), ST(st)),
          "ln_bwd_h3p");
  });
  m.def("h3p_split_multi", [](i64 table, int nseg, int total, i64 st) {
    pre_launch("h3p_split_multi");
    launch_h3p_split_multi(P(const void*, table), nseg, total, ST(st));
    check_launch("h3p_split_multi");
  });
  m.def("gemm_planes", [](int planes, int c_dtype, int ta, int tb, int M, int N, int K, i64 A, i64 lda, i64 a_ps,
                          i64 B, i64 ldb, i64 b_ps, i64 C, i64 ldc, i64 bias, int epi, float beta, i64 aux,
                          i64 ldaux, i64 part, i64 colsum, int colsum_acc, int ksplit, i64 slab, i64 slab_floats,
                          int variant, i64 st, int mv) {
    pre_launch("gemm_planes");
    const int rc = launch_gemm_planes(planes, c_dtype, ta, tb, M, N, K, P(const void*, A), lda, a_ps,
                                      P(const void*, B), ldb, b_ps, P(void*, C), ldc, P(const float*, bias), epi,
                                      beta, P(void*, aux), ldaux, P(float*, part), P(float*, colsum), colsum_acc,
                                      ksplit, P(float*, slab), slab_floats, variant, ST(st), mv);
    if (rc == 0) check_launch("gemm_planes");
    return rc;
  }, py::arg("planes"), py::arg("c_dtype"), py::arg("ta"), py::arg("tb"), py::arg("M"), py::arg("N"), py::arg("K"),
     py::arg("A"), py::arg("lda"), py::arg("a_ps"), py::arg("B"), py::arg("ldb"), py::arg("b_ps"), py::arg("C"),
     py::arg("ldc"), py::arg("bias"), py::arg("epi"), py::arg("beta"), py::arg("aux"), py::arg("ldaux"),
     py::arg("part"), py::arg("colsum"), py::arg("colsum_acc"), py::arg("ksplit"), py::arg("slab"),
     py::arg("slab_floats"), py::arg("variant"), py::arg("st"), py::arg("mv") = 0);
  m.def("set_planes_variant", &set_planes_variant, "plane GEMM variant: 0 default, 1 one LDS stage, 2 half K depth");
  m.def("pool_nsp_fwd", [](int dt, i64 seq, int B, int S, int H, i64 Wp, i64 bp, i64 Wn, i64 bn, i64 label,
                           i64 mlm_loss, i64 pooled, i64 logits, i64 lse, i64 stats, i64 total, i64 st) {
    pre_launch("pool_nsp_fwd");
    check(launch_pool_nsp_fwd(dt, P(const void*, seq), B, S, H, P(const float*, Wp), P(const float*, bp),
                              P(const float*, Wn), P(const float*, bn), P(const int64_t*, label),
                              P(const float*, mlm_loss), P(float*, pooled), P(float*, logits), P(float*, lse),
                              P(float*, stats), P(float*, total), ST(st)),
          "pool_nsp_fwd");
  });
  m.def("pool_nsp_bwd", [](int dt, i64 dloss, i64 seq, i64 dseq, int B, int S, int H, i64 Wp, i64 Wn, i64 label,
                           i64 pooled, i64 logits, i64 lse, i64 stats, i64 dlogits, i64 dpre, i64 part, i64 dWp,
                           i64 dbp, i64 dWn, i64 dbn, int accumulate, i64 st, int with_wgrad) {
    pre_launch("pool_nsp_bwd");
    check(launch_pool_nsp_bwd(dt, P(const float*, dloss), P(const void*, seq), P(void*, dseq), B, S, H,
                              P(const float*, Wp), P(const float*, Wn), P(const int64_t*, label),
                              P(const float*, pooled), P(const float*, logits), P(const float*, lse),
                              P(const float*, stats), P(float*, dlogits), P(float*, dpre), P(float*, part),
                              P(float*, dWp),
                              P(float*, dbp), P(float*, dWn), P(float*, dbn), accumulate, ST(st), with_wgrad),
          "pool_nsp_bwd");
  }, pybind11::arg("dt"), pybind11::arg("dloss"), pybind11::arg("seq"), pybind11::arg("dseq"), pybind11::arg("B"),
     pybind11::arg("S"), pybind11::arg("H"), pybind11::arg("Wp"), pybind11::arg("Wn"), pybind11::arg("label"),
     pybind11::arg("pooled"), pybind11::arg("logits"), pybind11::arg("lse"), pybind11::arg("stats"),
     pybind11::arg("dlogits"), pybind11::arg("dpre"), pybind11::arg("part"), pybind11::arg("dWp"), pybind11::arg("dbp"),
     pybind11::arg("dWn"), pybind11::arg("dbn"), pybind11::arg("accumulate"), pybind11::arg("st"),
     pybind11::arg("with_wgrad") = 1);
  m.def("pool_nsp_wgrad", [](int dt, i64 seq, i64 dpre, i64 dlogits, i64 pooled, int B, int S, int H, i64 dWp, i64 dbp,
                             i64 dWn, i64 dbn, int accumulate, i64 st) {
    pre_launch("pool_nsp_wgrad");
    launch_pool_nsp_wgrad(dt, P(const void*, seq), P(const float*, dpre), P(const float*, dlogits),
                          P(const float*, pooled), B, S, H, P(float*, dWp), P(float*, dbp), P(float*, dWn),
                          P(float*, dbn), accumulate, ST(st));
    check_launch("pool_nsp_wgrad");
  });
  m.def("colsum_row_chunks", &colsum_row_chunks);
  m.def("colsum", [](int dt, i64 dy, i64 x, i64 b, i64 dx, i64 part, i64 out, i64 rows, int N, int accumulate, i64 st,
                     i64 amax) {
    pre_launch("colsum");
    launch_colsum(dt, P(const void*, dy), P(const void*, x), P(const float*, b), P(void*, dx), P(float*, part),
                  P(float*, out), rows, N, accumulate, ST(st), P(float*, amax));
    check_launch("colsum");
  }, pybind11::arg("dt"), pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("b"), pybind11::arg("dx"),
     pybind11::arg("part"), pybind11::arg("out"), pybind11::arg("rows"), pybind11::arg("N"),
     pybind11::arg("accumulate"), pybind11::arg("st"), pybind11::arg("amax") = 0);
  m.def("mlm_compact", [](i64 labels, int rows, int ignore, int cap, i64 idx, i64 lab_out, i64 count, i64 err, i64 st) {
    pre_launch("mlm_compact");
    launch_mlm_compact(P(const int64_t*, labels), rows, ignore, cap, P(int32_t*, idx), P(int64_t*, lab_out),
                       P(int32_t*, count), P(int*, err), ST(st));
    check_launch("mlm_compact");
  });
  m.def("gather_rows", [](int dt, i64 src, i64 idx, i64 out, int n, int H, i64 st) {
    pre_launch("gather_rows");
    launch_gather_rows(dt, P(const void*, src), P(const int32_t*, idx), P(void*, out), n, H, ST(st));
    check_launch("gather_rows");
  });
  m.def("scatter_add_rows", [](int dt, i64 src, i64 idx, i64 dst, int n, int H, i64 st) {
    pre_launch("scatter_add_rows");
    launch_scatter_add_rows(dt, P(const void*, src), P(const int32_t*, idx), P(void*, dst), n, H, ST(st));
    check_launch("scatter_add_rows");
  });

  m.def("comm_emulation_fn", []() { return reinterpret_cast<i64>(&hetseq_comm_emulation); },
        "address of the collective stand-in launcher (bench.py --emulate-world; csrc/comm/comm.cpp set_emulation)");
  m.def("comm_emulation", [](i64 src, i64 src_bytes, i64 scratch, i64 scratch_bytes, i64 traffic, int channels,
                             i64 hold_ns, i64 st) {
    pre_launch("comm_emulation");
    hetseq_comm_emulation(P(const void*, src), src_bytes, P(void*, scratch), scratch_bytes, traffic, channels, hold_ns,
                          ST(st));
    check_launch("comm_emulation");
  }, "the collective stand-in kernel launched directly (tests)");
  m.def("amax", [](i64 x, i64 n, i64 out, int zero_first, i64 st) {
    pre_launch("amax");
    check(launch_amax(P(const float*, x), n, P(float*, out), zero_first, ST(st)), "amax");
  }, "|max| of n fp32 values (n % 4 == 0, 16-B aligned) atomically maxed into *out (cleared first if zero_first)");
  m.def("zero_segs", [](i64 base, i64 tab, int nblk, i64 st) {
    pre_launch("zero_segs");
    launch_zero_segs(P(float*, base), P(const int64_t*, tab), nblk, ST(st));
    check_launch("zero_segs");
  }, "zero the float4 ranges of a (lo, hi) block table from base (one launch)");
  m.def("amax_seg", [](i64 base, i64 tab, int nblk, i64 out, i64 st) {
    pre_launch("amax_seg");
    launch_amax_seg(P(const float*, base), P(const int64_t*, tab), nblk, P(float*, out), ST(st));
    check_launch("amax_seg");
  }, "per-segment |max| over a flat fp32 buffer: tab = [nblk][3] int64 (segment, first float4, end float4); out "
     "must be zeroed");

  m.def("set_attn_fp32_mode", &set_attn_fp32_mode, "fp32 attention products: 2 split-fp16 (h3), 0 exact-fp32 MFMA");
  m.def("attn_fp32_mode", &attn_fp32_mode);
  m.def("set_ln_bwd_lds", &set_ln_bwd_lds,
        "LN backward column partials: 1 = through a 3 KB LDS window (default), 0 = the [waves][H] LDS image");
  // amax: optional |max| slot of the output (ctx / dqkv); returns 1 when the kernel wrote it (h3 engine)
  m.def("attn_fwd", [](int dt, i64 qkv, i64 mask, i64 bqkv, i64 ctx, i64 lse, i64 dmask, int B, int S, int NH, int D,
                       float p, u64 seed, u64 off, i64 st, int bh0, i64 amax) {
    pre_launch("attn_fwd");
    int done = 0;
    check(launch_attn_fwd(dt, P(const void*, qkv), P(const int64_t*, mask), P(const float*, bqkv), P(void*, ctx),
                          P(float*, lse), P(uint32_t*, dmask), B, S, NH, D, p, seed, off, ST(st), bh0,
                          P(float*, amax), &done),
          "attn_fwd");
    return done;
  }, py::arg("dt"), py::arg("qkv"), py::arg("mask"), py::arg("bqkv"), py::arg("ctx"), py::arg("lse"), py::arg("dmask"),
     py::arg("B"), py::arg("S"), py::arg("NH"), py::arg("D"), py::arg("p"), py::arg("seed"), py::arg("off"),
     py::arg("st"), py::arg("bh0") = 0, py::arg("amax") = 0);
  m.def("attn_bwd", [](int dt, i64 qkv, i64 mask, i64 bqkv, i64 ctx, i64 dctx, i64 lse, i64 dbuf, i64 dqkv, i64 dmask,
                       int B, int S, int NH, int D, float p, i64 st, i64 amax) {
    pre_launch("attn_bwd");
    int done = 0;
    check(launch_attn_bwd(dt, P(const void*, qkv), P(const int64_t*, mask), P(const float*, bqkv),
                          P(const void*, ctx), P(const void*, dctx), P(const float*, lse), P(float*, dbuf),
                          P(void*, dqkv), P(const uint32_t*, dmask), B, S, NH, D, p, ST(st), P(float*, amax), &done),
          "attn_bwd");
    return done;
  }, py::arg("dt"), py::arg("qkv"), py::arg("mask"), py::arg("bqkv"), py::arg("ctx"), py::arg("dctx"), py::arg("lse"),
     py::arg("dbuf"), py::arg("dqkv"), py::arg("dmask"), py::arg("B"), py::arg("S"), py::arg("NH"), py::arg("D"),
     py::arg("p"), py::arg("st"), py::arg("amax") = 0);

  m.def("xent_fwd", [](int dt, i64 logits, i64 labels, int rows, int V, i64 ldv, int ignore, i64 row_loss, i64 lse,
                       i64 out, i64 st) {
    pre_launch("xent_fwd");
    launch_xent_fwd(dt, P(const void*, logits), P(const int64_t*, labels), rows, V, ldv, ignore, P(float*, row_loss),
                    P(float*, lse), P(float*, out), ST(st));
    check_launch("xent_fwd");
  });
  m.def("xent_bwd", [](int dt, i64 logits, i64 labels, i64 lse, int rows, int V, i64 ldv, int ignore, i64 dloss,
                       i64 stats, i64 st, i64 amax) {
    pre_launch("xent_bwd");
    launch_xent_bwd(dt, P(void*, logits), P(const int64_t*, labels), P(const float*, lse), rows, V, ldv, ignore,
                    P(const float*, dloss), P(const float*, stats), ST(st), P(float*, amax));
    check_launch("xent_bwd");
  }, pybind11::arg("dt"), pybind11::arg("logits"), pybind11::arg("labels"), pybind11::arg("lse"), pybind11::arg("rows"),
     pybind11::arg("V"), pybind11::arg("ldv"), pybind11::arg("ignore"), pybind11::arg("dloss"), pybind11::arg("stats"),
     pybind11::arg("st"), pybind11::arg("amax") = 0);

  // returns 0 when launched, -1 when the shape/epilogue is not served (caller falls back)
  m.def("set_skip_launches", [](int mask) { hs::g_hs_skip = mask; },
        "diagnostic ablation: 1 skip split-K finishing passes, 2 skip column-partial reductions (results invalid)");
  m.def("set_seed_ptr", [](i64 ptr) { hs::g_seed_dev = reinterpret_cast<const uint64_t*>(ptr); });
  m.def("stream_wait", [](i64 waiter, i64 signal) { stream_wait(ST(waiter), ST(signal)); });
  // After a failed (invalidated) capture: end the capture a stream may still be in -- a stream that
  // joined the capture through an event wait can be left capturing when the origin's capture fails --
  // and take the error it left pending.  Returns (1 if the stream was capturing, that error code).
  m.def("capture_status", [](i64 st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const hipError_t e = hipStreamIsCapturing(ST(st), &cs);
    return e == hipSuccess ? static_cast<int>(cs) : -static_cast<int>(e);
  }, "capture status of a stream: 0 none, 1 active, 2 invalidated (negative: the query's HIP error)");
  m.def("end_capture", [](i64 st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(ST(st), &cs) != hipSuccess) cs = hipStreamCaptureStatusNone;
    int was = cs != hipStreamCaptureStatusNone;
    if (was) {
      hipGraph_t g = nullptr;
      (void)hipStreamEndCapture(ST(st), &g);
      if (g) (void)hipGraphDestroy(g);
    }
    const int pending = static_cast<int>(hipGetLastError());
    return std::make_pair(was, pending);
  }, "end a (failed) capture the stream is still in; returns (was capturing, the pending error it took)");
  m.def("set_stream_wait_flags", [](int mode) {
    // 0: DisableTiming; 1: + DisableSystemFence; 2: + ReleaseToDevice; 3: + both
    g_wait_flags = hipEventDisableTiming | (mode & 1 ? hipEventDisableSystemFence : 0u) |
                   (mode & 2 ? hipEventReleaseToDevice : 0u);
  }, "event flags of stream_wait's ordering events (synchronises the device when they change)");
  // A non-blocking stream of the current device that lives for the whole process (runtime/streams.py
  // creates the engine's streams with it before RCCL and torch's stream pool create theirs, so each
  // role gets a hardware queue of its own; never destroyed).
  m.def("stream_create", [](int greatest_priority) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess)
      throw std::runtime_error("hipDeviceGetStreamPriorityRange failed");
    hipStream_t s = nullptr;
    if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest_priority ? greatest : least) != hipSuccess)
      throw std::runtime_error("hipStreamCreateWithPriority failed");
    return reinterpret_cast<i64>(s);
  });
  m.def("set_h3_occ3", &set_h3_occ3, "h3 GEMM engine, plain / bias epilogues at three blocks per CU (168 VGPRs): "
        "bit mask 1 forward, 2 data gradient, 4 weight gradient");
  m.def("gemm_last_ksplit", &gemm_last_ksplit,
        "K slices of the last split-bf16 GEMM launch (with C = 0 its partials stay in the slab)");
  m.def("gemm", [](int dt, int ta, int tb, int M, int N, int K, i64 A, i64 lda, i64 B, i64 ldb, i64 C, i64 ldc, i64 bias,
                   int epi, float beta, i64 aux, i64 ldaux, i64 part, i64 colsum, int colsum_acc, i64 st,
                   int tile, int ksplit, i64 slab, i64 slab_floats, int mv, int nv, int kv, i64 amax_a, int namax_a,
                   i64 amax_b, int namax_b, i64 amax_c) {
    pre_launch("gemm");
    const int rc = launch_gemm(dt, ta, tb, M, N, K, P(const void*, A), lda, P(const void*, B), ldb, P(void*, C), ldc,
                               P(const float*, bias), epi, beta, P(float*, aux), ldaux, P(float*, part),
                               P(float*, colsum), colsum_acc, tile, ST(st), ksplit, P(float*, slab), slab_floats, mv, nv,
                               kv, P(const float*, amax_a), namax_a, P(const float*, amax_b), namax_b,
                               P(float*, amax_c));
    if (rc == 0) check_launch("gemm");
    return rc;
  }, pybind11::arg("dt"), pybind11::arg("ta"), pybind11::arg("tb"), pybind11::arg("M"), pybind11::arg("N"),
     pybind11::arg("K"), pybind11::arg("A"), pybind11::arg("lda"), pybind11::arg("B"), pybind11::arg("ldb"),
     pybind11::arg("C"), pybind11::arg("ldc"), pybind11::arg("bias"), pybind11::arg("epi"), pybind11::arg("beta"),
     pybind11::arg("aux"), pybind11::arg("ldaux"), pybind11::arg("part"), pybind11::arg("colsum"),
     pybind11::arg("colsum_acc"), pybind11::arg("st"), pybind11::arg("tile") = -1, pybind11::arg("ksplit") = 0,
     pybind11::arg("slab") = 0, pybind11::arg("slab_floats") = 0, pybind11::arg("mv") = 0, pybind11::arg("nv") = 0,
     pybind11::arg("kv") = 0, pybind11::arg("amax_a") = 0, pybind11::arg("namax_a") = 0, pybind11::arg("amax_b") = 0,
     pybind11::arg("namax_b") = 0, pybind11::arg("amax_c") = 0);
  m.def("set_wcol_fold", &set_wcol_fold, "weight-gradient bias sums finished by the split-K pass (1) or reduce_rows (0)");
}
