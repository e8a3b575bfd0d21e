// Native launch path of the fused BERT encoder layer on the h3p engine (one host call per layer
// forward, one per layer backward).
//
// The Python layer (ops/bert_ops.py _layer_forward_h3p / _layer_backward_h3p) issues ~14 kernel
// launches per forward and ~16 per backward, each through a Python wrapper that allocates its
// outputs from the caching allocator, slices views and converts arguments: ~9 ms of host time per
// BERT-base step, within ~2 ms of the device time, and past it once data-parallel work is added.
// Here the launch sequence of a layer is resolved ONCE into a plan -- an int64 table (field names
// below) of every device address and size: the layer's weight planes, its persistent activation
// arena (ops/layer_prog.py allocates it per batch shape), the flat-store gradient views, the
// split-K slabs -- and each call only adds what changes per step: the layer input, the attention
// mask, the dropout seeds, the streams.
//
// Streams (runtime/streams.py): the forward's two half-batch chains run on `st0` (compute) and `st1`
// (the weight-gradient side stream, forked by the caller once per encoder forward); the backward's
// data-gradient chain runs on `st0` and its weight gradients / parameter-gradient finalisation on
// `st1`, forked at the same four points as the Python layer (one event each, shared by consecutive
// side-stream launches).
//
// Reference: one BertLayer forward / autograd backward (bert_modeling.py:361-441).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

int launch_gemm_h3p(int ta, int tb, int M, int N, int K, const void* A, int64_t lda, int64_t a_ps, const int8_t* ea,
                    int64_t lde_a, const void* B, int64_t ldb, int64_t b_ps, const int8_t* eb, int64_t lde_b, float* C,
                    int64_t ldc, const float* bias, int epi, float beta, float* aux, int64_t ldaux, float* part,
                    float* colsum, int colsum_acc, void* cp, int64_t ldcp, int64_t cp_ps, int8_t* ec, int64_t lde_c,
                    int ksplit, float* slab, int64_t slab_floats, int ablk, int bblk, hipStream_t st);
int launch_ln_fwd_h3p(const void*, const float*, const void*, const float*, const float*, void*, float*, float*, float*,
                      int, int, float, float, uint64_t, uint64_t, int, int, int64_t, int, float*, void*, int64_t, int8_t*,
                      uint32_t*, int, hipStream_t);
int launch_ln_bwd_h3p(const float*, const float*, const float*, const float*, const float*, float*, float*, float*,
                      float*, int, int, float, uint64_t, uint64_t, void*, int64_t, int8_t*, uint32_t*, hipStream_t);
int ln_bwd_h3p_part_rows(int coop);
int launch_attn_fwd_h3(const float*, const int64_t*, const float*, float*, float*, uint32_t*, int, int, int, int, float,
                       uint64_t, uint64_t, hipStream_t, int, float*, void*, int64_t, int8_t*);
int launch_attn_bwd_h3(const float*, const int64_t*, const float*, const float*, const float*, const float*, float*,
                       float*, const uint32_t*, int, int, int, int, float, hipStream_t, float*, void*, int64_t,
                       int8_t*, float*);
void launch_colpart_finalize(const float* const*, float* const*, int, int, int, int, hipStream_t);
int launch_h3p_colpart(const void*, int64_t, int64_t, const int8_t*, int64_t, int, int, float*, hipStream_t);
void hs_stream_wait(hipStream_t waiter, hipStream_t signal);
  // bindings.cpp (event ring)

// An h3p operand in the plan: planes address, leading dimension, plane stride, exponents address,
// exponent leading dimension, blocked layout (ops/h3p.py HP).
#define HPF(X, n) X(n##_p) X(n##_ld) X(n##_ps) X(n##_e) X(n##_lde) X(n##_blk)
#define LAYER_PLAN_FIELDS(X)                                                                                  \
  X(B) X(S) X(NH) X(H) X(F) X(rows) X(halves) X(ks_wo) X(ks_w2) X(ksg_qkv) X(ksg_wo) X(ksg_w1) X(ksg_w2)       \
  HPF(X, wqkv) HPF(X, wo) HPF(X, w1) HPF(X, w2)                                                               \
  X(bqkv) X(bo) X(g1) X(b1) X(bi) X(b2) X(g2) X(bb2)                                                          \
  X(qkv) X(ctx) X(lse) X(dmask) X(h1) X(z1) X(m1) X(r1) X(f1pre) X(h2) X(z2) X(m2) X(r2)                       \
  HPF(X, ctxp) HPF(X, h1p) HPF(X, f1p) HPF(X, h2p)                                                            \
  X(xp_ld) X(xp_ps) X(xp_lde) X(xp_blk)                                                                       \
  X(slab0) X(slab1) X(slab_floats)                                                                            \
  X(gwqkv) X(gbqkv) X(gwo) X(gbo) X(gg1) X(gb1) X(gw1) X(gbi) X(gw2) X(gb2) X(gg2) X(gbb2)                     \
  X(dz2) X(dz1) X(dctx) X(dbuf)                                                                              \
  HPF(X, da2p) HPF(X, df1p) HPF(X, da1p) HPF(X, dqkvp)                                                        \
  X(part2_g) X(part2_b) X(part2_bias) X(part1_g) X(part1_b) X(part1_bias) X(part_gelu) X(part_bq)            \
  X(psync_f) X(psync_b) X(dsbuf)

namespace {

enum Field : int {
#define X(n) f_##n,
  LAYER_PLAN_FIELDS(X)
#undef X
  kNumFields
};

const char* const kFieldNames[] = {
#define X(n) #n,
    LAYER_PLAN_FIELDS(X)
#undef X
};

struct HPv {
  int64_t p, ld, ps, e, lde, blk;
  HPv rows_from(int64_t r0) const {  // rows [r0, ...) of the operand (r0 a multiple of 32)
    return HPv{p + 2 * r0 * ld, ld, ps, e + (r0 / 32) * lde, lde, blk};
  }
};

template <class T>
T* ptr(int64_t v) {
  return reinterpret_cast<T*>(static_cast<uintptr_t>(v));
}

HPv hp_at(const int64_t* q, int f) { return HPv{q[f], q[f + 1], q[f + 2], q[f + 3], q[f + 4], q[f + 5]}; }

void req(int rc, const char* what) {
  if (rc != 0) throw std::invalid_argument(std::string("layer program: ") + what + " not served");
}

// h3p.gemm(a, b, ta, tb, ...) with the operand shapes resolved by the caller
void gemm(int ta, int tb, int M, int N, int K, const HPv& a, const HPv& b, float* C, int64_t ldc, const float* bias,
          int epi, float beta, float* aux, int64_t ldaux, float* part, float* colsum, int colsum_acc, const HPv* cp,
          int ksplit, float* slab, int64_t slab_floats, hipStream_t st, const char* what) {
  req(launch_gemm_h3p(ta, tb, M, N, K, ptr<const void>(a.p), a.ld, a.ps, ptr<const int8_t>(a.e), a.lde,
                      ptr<const void>(b.p), b.ld, b.ps, ptr<const int8_t>(b.e), b.lde, C, ldc, bias, epi, beta, aux,
                      ldaux, part, colsum, colsum_acc, cp ? ptr<void>(cp->p) : nullptr, cp ? cp->ld : 0,
                      cp ? cp->ps : 0, cp ? ptr<int8_t>(cp->e) : nullptr, cp ? cp->lde : 0, ksplit, slab, slab_floats,
                      (int)a.blk, (int)b.blk, st),
      what);
}

constexpr int kEpiGelu = 2, kEpiDgelu = 3;

// split-K product whose [ks, M, N] fp32 slices stay in the stream's slab for the LayerNorm that
// sums them (h3p.gemm slab_only)
float* gemm_slabs(int M, int N, int K, const HPv& a, const HPv& b, int ks, float* slab, int64_t slab_floats,
                  hipStream_t st, const char* what) {
  if ((int64_t)ks * M * N > slab_floats) throw std::invalid_argument("layer program: split-K slab too small");
  if (ks > 1)
    gemm(0, 1, M, N, K, a, b, nullptr, N, nullptr, 0, 0.f, nullptr, 0, nullptr, nullptr, 0, nullptr, ks, slab,
         slab_floats, st, what);
  else
    gemm(0, 1, M, N, K, a, b, slab, N, nullptr, 0, 0.f, nullptr, 0, nullptr, nullptr, 0, nullptr, 1, nullptr, 0, st,
         what);
  return slab;
}

}  // namespace

std::vector<std::string> layer_plan_fields() {
  return std::vector<std::string>(kFieldNames, kFieldNames + kNumFields);
}

// One layer forward.  x: the layer input [rows, H] fp32; xp / xe: its h3p planes / exponents (the
// plan holds their layout); mask [B, S] int64; seeds (a: attention, 1 / 2: the two LayerNorms);
// amax0 / amax1: |max| slots of each half's output (0: none).  stagger (the chains' first layer): the
// second chain waits for the first chain's QKV product (1), attention (2) or first LayerNorm (3), so
// the two chains run out of phase -- one chain's latency-bound attention / LayerNorm beside the other
// chain's GEMMs instead of both chains' attention at once.
void layer_fwd_h3p(int64_t plan, int64_t x, int64_t xp, int64_t xe, int64_t mask, uint64_t sa, uint64_t oa,
                   uint64_t s1, uint64_t o1, uint64_t s2, uint64_t o2, float eps, float p_h, float p_a, int64_t st0,
                   int64_t st1, int64_t amax0, int64_t amax1, int stagger) {
  const int64_t* q = ptr<const int64_t>(plan);
  const int B = (int)q[f_B], S = (int)q[f_S], NH = (int)q[f_NH], H = (int)q[f_H], F = (int)q[f_F];
  const int rows = (int)q[f_rows], nh = (int)q[f_halves];
  const int hr = rows / nh, hb = B / nh;
  const int64_t nl = (int64_t)hb * NH * S, nm = nl * (S / 32);
  const HPv Wqkv = hp_at(q, f_wqkv_p), Wo = hp_at(q, f_wo_p), W1 = hp_at(q, f_w1_p), W2 = hp_at(q, f_w2_p);
  const HPv X{xp, q[f_xp_ld], q[f_xp_ps], xe, q[f_xp_lde], q[f_xp_blk]};
  const HPv ctxp = hp_at(q, f_ctxp_p), h1p = hp_at(q, f_h1p_p), f1p = hp_at(q, f_f1p_p), h2p = hp_at(q, f_h2p_p);
  const int64_t slab_floats = q[f_slab_floats];
  for (int h = 0; h < nh; ++h) {
    hipStream_t st = ptr<ihipStream_t>(h == 0 ? st0 : st1);
    float* slab = ptr<float>(h == 0 ? q[f_slab0] : q[f_slab1]);
    const int64_t r0 = (int64_t)h * hr;
    float* qkv = ptr<float>(q[f_qkv]) + r0 * 3 * H;
    gemm(0, 1, hr, 3 * H, H, X.rows_from(r0), Wqkv, qkv, 3 * H, nullptr, 0, 0.f, nullptr, 0, nullptr, nullptr, 0,
         nullptr, 1, nullptr, 0, st, "qkv forward");
    const bool stag = h == 0 && nh > 1 && st1 != 0;
    if (stag && stagger == 1) hs_stream_wait(ptr<ihipStream_t>(st1), st);
    const HPv cp = ctxp.rows_from(r0);
    req(launch_attn_fwd_h3(qkv, ptr<const int64_t>(mask) + (int64_t)h * hb * S, ptr<const float>(q[f_bqkv]),
                           ptr<float>(q[f_ctx]) + r0 * H, ptr<float>(q[f_lse]) + h * nl,
                           q[f_dmask] ? ptr<uint32_t>(q[f_dmask]) + h * nm : nullptr, hb, S, NH, 64, p_a, sa, oa, st,
                           h * hb * NH, nullptr, ptr<void>(cp.p), cp.ps, ptr<int8_t>(cp.e)),
        "attention forward");
    if (stag && stagger == 2) hs_stream_wait(ptr<ihipStream_t>(st1), st);
    const int ks_wo = (int)q[f_ks_wo], ks_w2 = (int)q[f_ks_w2];
    gemm_slabs(hr, H, H, cp, Wo, ks_wo, slab, slab_floats, st, "attention-output forward");
    const HPv p1 = h1p.rows_from(r0);
    float* h1 = ptr<float>(q[f_h1]) + r0 * H;
    req(launch_ln_fwd_h3p(slab, ptr<const float>(q[f_bo]), ptr<const float>(x) + r0 * H, ptr<const float>(q[f_g1]),
                          ptr<const float>(q[f_b1]), h1, ptr<float>(q[f_z1]) + r0 * H, ptr<float>(q[f_m1]) + r0,
                          ptr<float>(q[f_r1]) + r0, hr, H, eps, p_h, s1, o1, 1, ks_wo, (int64_t)hr * H, (int)r0,
                          nullptr, ptr<void>(p1.p), p1.ps, ptr<int8_t>(p1.e), ptr<uint32_t>(q[f_psync_f]),
                          (int)(r0 / 32), st),
        "LayerNorm 1 forward");
    if (stag && stagger == 3) hs_stream_wait(ptr<ihipStream_t>(st1), st);
    const HPv pf = f1p.rows_from(r0);
    gemm(0, 1, hr, F, H, p1, W1, nullptr, F, ptr<const float>(q[f_bi]), kEpiGelu, 0.f,
         ptr<float>(q[f_f1pre]) + r0 * F, F, nullptr, nullptr, 0, &pf, 1, nullptr, 0, st, "FFN-in forward");
    gemm_slabs(hr, H, F, pf, W2, ks_w2, slab, slab_floats, st, "FFN-out forward");
    const HPv p2 = h2p.rows_from(r0);
    req(launch_ln_fwd_h3p(slab, ptr<const float>(q[f_b2]), h1, ptr<const float>(q[f_g2]), ptr<const float>(q[f_bb2]),
                          ptr<float>(q[f_h2]) + r0 * H, ptr<float>(q[f_z2]) + r0 * H, ptr<float>(q[f_m2]) + r0,
                          ptr<float>(q[f_r2]) + r0, hr, H, eps, p_h, s2, o2, 1, ks_w2, (int64_t)hr * H, (int)r0,
                          ptr<float>(h == 0 ? amax0 : amax1), ptr<void>(p2.p), p2.ps, ptr<int8_t>(p2.e),
                          ptr<uint32_t>(q[f_psync_f]), (int)(r0 / 32), st),
        "LayerNorm 2 forward");
  }
}

// One layer backward (flat-store gradients, side stream).  dh2: the output gradient [rows, H];
// xp / xe: the forward input's planes; wacc: the weight-gradient products accumulate (else store:
// the first backward after zero_grad).  The input gradient is left in the plan's dz1.
//
// events: 0, or the address of four hipEvent_t handles recorded on the side stream as each group of the
// layer's parameter gradients is complete -- FFN-out + LN2, FFN-in, attention output + LN1, QKV (the
// data-parallel engine reduces each group behind its event: parallel/ddp.py early buckets).
void layer_bwd_h3p(int64_t plan, int64_t dh2, int64_t xp, int64_t xe, int64_t mask, uint64_t s1, uint64_t o1,
                   uint64_t s2, uint64_t o2, float p_h, float p_a, int wacc, int64_t st0_, int64_t st1_,
                   int64_t events) {
  const int64_t* q = ptr<const int64_t>(plan);
  const int64_t* evs = ptr<const int64_t>(events);
  auto ready = [&](int g) {
    if (evs && hipEventRecord(ptr<ihipEvent_t>(evs[g]), ptr<ihipStream_t>(st1_)) != hipSuccess)
      throw std::runtime_error("layer program: hipEventRecord");
  };
  hipStream_t st0 = ptr<ihipStream_t>(st0_), st1 = ptr<ihipStream_t>(st1_);
  const int B = (int)q[f_B], S = (int)q[f_S], NH = (int)q[f_NH], H = (int)q[f_H], F = (int)q[f_F];
  const int rows = (int)q[f_rows], nb = rows / 32, npart = rows / ln_bwd_h3p_part_rows(q[f_psync_b] != 0);
  uint32_t* psb = ptr<uint32_t>(q[f_psync_b]);
  const HPv Wqkv = hp_at(q, f_wqkv_p), Wo = hp_at(q, f_wo_p), W1 = hp_at(q, f_w1_p), W2 = hp_at(q, f_w2_p);
  const HPv X{xp, q[f_xp_ld], q[f_xp_ps], xe, q[f_xp_lde], q[f_xp_blk]};
  const HPv ctxp = hp_at(q, f_ctxp_p), h1p = hp_at(q, f_h1p_p), f1p = hp_at(q, f_f1p_p);
  const HPv da2p = hp_at(q, f_da2p_p), df1p = hp_at(q, f_df1p_p), da1p = hp_at(q, f_da1p_p),
            dqkvp = hp_at(q, f_dqkvp_p);
  float* slab1 = ptr<float>(q[f_slab1]);
  const int64_t slab_floats = q[f_slab_floats];
  const float beta_w = wacc ? 1.f : 0.f;
  float* dz2 = ptr<float>(q[f_dz2]);
  float* dz1 = ptr<float>(q[f_dz1]);
  auto wgrad = [&](const HPv& dy, const HPv& xx, int M, int N, int64_t out, int ks, const char* what) {
    if ((int64_t)ks * M * N > slab_floats) throw std::invalid_argument("layer program: wgrad slab too small");
    gemm(1, 0, M, N, rows, dy, xx, ptr<float>(out), N, nullptr, 0, beta_w, nullptr, 0, nullptr, nullptr, 0, nullptr,
         ks, ks > 1 ? slab1 : nullptr, ks > 1 ? slab_floats : 0, st1, what);
  };
  auto finalize = [&](int64_t pg, int64_t pb, int64_t pbias, int64_t og, int64_t ob, int64_t obias) {
    const float* parts[3] = {ptr<const float>(pg), ptr<const float>(pb), ptr<const float>(pbias)};
    float* outs[3] = {ptr<float>(og), ptr<float>(ob), ptr<float>(obias)};
    launch_colpart_finalize(parts, outs, 3, npart, H, 1, st1);
  };
  // LN2 backward; its parameter gradients and the FFN-out weight gradient on the side stream
  req(launch_ln_bwd_h3p(ptr<const float>(dh2), ptr<const float>(q[f_z2]), ptr<const float>(q[f_m2]),
                        ptr<const float>(q[f_r2]), ptr<const float>(q[f_g2]), dz2, ptr<float>(q[f_part2_g]),
                        ptr<float>(q[f_part2_b]), ptr<float>(q[f_part2_bias]), rows, H, p_h, s2, o2,
                        ptr<void>(da2p.p), da2p.ps, ptr<int8_t>(da2p.e), psb, st0),
      "LayerNorm 2 backward");
  hs_stream_wait(st1, st0);
  finalize(q[f_part2_g], q[f_part2_b], q[f_part2_bias], q[f_gg2], q[f_gbb2], q[f_gb2]);
  wgrad(da2p, f1p, H, F, q[f_gw2], (int)q[f_ksg_w2], "FFN-out weight gradient");
  ready(0);
  // FFN-in data gradient through the GELU (planes only; the FFN-in bias gradient from the column
  // partials), its weight gradient beside it, then dh1 = dz2 + df1 @ W1
  gemm(0, 0, rows, F, H, da2p, W2, nullptr, F, ptr<const float>(q[f_bi]), kEpiDgelu, 0.f, ptr<float>(q[f_f1pre]), F,
       ptr<float>(q[f_part_gelu]), nullptr, 1, &df1p, 1, nullptr, 0, st0, "FFN-out data gradient");
  hs_stream_wait(st1, st0);
  {  // the FFN-in bias gradient from the dGELU epilogue's column partials, off the data-gradient chain
    const float* parts[1] = {ptr<const float>(q[f_part_gelu])};
    float* outs[1] = {ptr<float>(q[f_gbi])};
    launch_colpart_finalize(parts, outs, 1, rows / 128, F, 1, st1);
  }
  wgrad(df1p, h1p, F, H, q[f_gw1], (int)q[f_ksg_w1], "FFN-in weight gradient");
  ready(1);  // (the FFN-in bias gradient came from the compute stream before the fork)
  gemm(0, 0, rows, H, F, df1p, W1, dz2, H, nullptr, 0, 1.f, nullptr, 0, nullptr, nullptr, 0, nullptr, 1, nullptr, 0,
       st0, "FFN-in data gradient");
  // LN1 backward; its parameter gradients and the attention-output weight gradient on the side
  req(launch_ln_bwd_h3p(dz2, ptr<const float>(q[f_z1]), ptr<const float>(q[f_m1]), ptr<const float>(q[f_r1]),
                        ptr<const float>(q[f_g1]), dz1, ptr<float>(q[f_part1_g]), ptr<float>(q[f_part1_b]),
                        ptr<float>(q[f_part1_bias]), rows, H, p_h, s1, o1, ptr<void>(da1p.p), da1p.ps,
                        ptr<int8_t>(da1p.e), psb, st0),
      "LayerNorm 1 backward");
  hs_stream_wait(st1, st0);
  finalize(q[f_part1_g], q[f_part1_b], q[f_part1_bias], q[f_gg1], q[f_gb1], q[f_gbo]);
  wgrad(da1p, ctxp, H, H, q[f_gwo], (int)q[f_ksg_wo], "attention-output weight gradient");
  ready(2);
  float* dctx = ptr<float>(q[f_dctx]);
  gemm(0, 0, rows, H, H, da1p, Wo, dctx, H, nullptr, 0, 0.f, nullptr, 0, nullptr, nullptr, 0, nullptr, 1, nullptr, 0,
       st0, "attention-output data gradient");
  // dqkv only as planes (the QKV bias gradient from their column partials below)
  req(launch_attn_bwd_h3(ptr<const float>(q[f_qkv]), ptr<const int64_t>(mask), ptr<const float>(q[f_bqkv]),
                         ptr<const float>(q[f_ctx]), dctx, ptr<const float>(q[f_lse]), ptr<float>(q[f_dbuf]), nullptr,
                         q[f_dmask] ? ptr<const uint32_t>(q[f_dmask]) : nullptr, B, S, NH, 64, p_a, st0, nullptr,
                         ptr<void>(dqkvp.p), dqkvp.ps, ptr<int8_t>(dqkvp.e), ptr<float>(q[f_dsbuf])),
      "attention backward");
  // QKV weight and bias gradients on the side stream; dx = dz1 + dqkv @ Wqkv
  hs_stream_wait(st1, st0);
  wgrad(dqkvp, X, 3 * H, H, q[f_gwqkv], (int)q[f_ksg_qkv], "QKV weight gradient");
  {
    const float* parts[1] = {ptr<const float>(q[f_part_bq])};
    float* outs[1] = {ptr<float>(q[f_gbqkv])};
    req(launch_h3p_colpart(ptr<const void>(dqkvp.p), dqkvp.ld, dqkvp.ps, ptr<const int8_t>(dqkvp.e), dqkvp.lde, rows,
                           3 * H, ptr<float>(q[f_part_bq]), st1),
        "QKV bias-gradient partials");
    launch_colpart_finalize(parts, outs, 1, nb, 3 * H, 1, st1);
  }
  ready(3);
  gemm(0, 0, rows, H, 3 * H, dqkvp, Wqkv, dz1, H, nullptr, 0, 1.f, nullptr, 0, nullptr, nullptr, 0, nullptr, 1,
       nullptr, 0, st0, "QKV data gradient");
}
