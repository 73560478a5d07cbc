// pybind11 bindings for the tfk gfx950 kernel library. Every entry point validates device,
// dtype, alignment and the maximum element index each kernel will touch BEFORE launching, so a
// shape bug raises a Python exception instead of faulting the GPU. All launches go to the
// current HIP stream (graph-capturable: no allocation or synchronisation in here).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <vector>

#include "bind_util.h"
#include "../kernels/gemm_params.h"
#include "../kernels/bn_fin.h"

// common.h drop_thr8 (8-bit dropout threshold round(256 p)), host copy in the same float arithmetic
static inline int drop_thr8_host(float p) {
  const int t = (int)(p * 256.f + 0.5f);
  return t > 255 ? 255 : (t < 0 ? 0 : t);
}

extern "C" {
int tfk_gemm_launch(tfk::GemmParams p, int bm, int bn, int amode, int bmode, int epi, int batch, int splits, hipStream_t s);
int tfk_gemm_splits(int K, int splits);
void tfk_gemm_set_persist(int on);
void tfk_gemm_set_engine(int e);
void tfk_g4_set_shortk(int on);
extern "C" void tfk_fp8_set_engine(int e);
int tfk_mx_quant(const void*, void*, void*, long long, hipStream_t);
int tfk_mx_quant_t(const void*, void*, void*, int, int, hipStream_t);
int tfk_mx_quant_dual(const void*, void*, void*, void*, void*, int, int, hipStream_t);
int tfk_mx_quant_dual_group(const void*, int, int, hipStream_t);
int tfk_mx_probe(const int*, const int*, const int*, const int*, float*, hipStream_t);
int tfk_gemm_mxfp8(tfk::GemmParams p, int ext, int splits, hipStream_t s);
const unsigned long long* tfk_seed_key();
void tfk_set_seed_key(const unsigned long long* k);
int tfk_rng_advance(unsigned long long* st, unsigned long long stream, hipStream_t s);
void tfk_halo_set(int on);
void tfk_bn_fin_skip(int v);
void tfk_fp8_set_tile(int t);
void tfk_g8_set(int on);
void tfk_g5_set(int waves);
int tfk_bn_finalize(float*, int, int, float, const float*, const float*, float, float, float*, float*, float*, float*,
                    float*, float*, hipStream_t);
int tfk_bn_stats(const void*, long long, int, float*, int, hipStream_t);
int tfk_bn_apply(const void*, const float*, const float*, const void*, const float*, const float*, int, void*, long long,
                 int, uint8_t*, hipStream_t);
int tfk_bn_bwd_reduce(const void*, const void*, const void*, const float*, const float*, const void*, const float*,
                      const float*, long long, int, float*, int, const float*, const float*, const uint8_t*, hipStream_t);
int tfk_bn_bwd_finalize(float*, int, int, float, const float*, const float*, const float*, const float*, const float*,
                        const float*, float*, float*, float*, float*, float*, float*, hipStream_t);
int tfk_bn_bwd_apply(const void*, const void*, const void*, const float*, void*, const void*, const float*, void*, void*,
                     long long, int, const float*, const float*, const uint8_t*, hipStream_t);
int tfk_bn_fin_ok(int, int);
int tfk_bn_apply_fin(const void*, const tfk::BnFin*, const void*, const tfk::BnFin*, int, void*, long long, int, uint8_t*,
                     hipStream_t);
int tfk_bn_bwd_apply_fin(const void*, const void*, const float*, int, const tfk::BnBwdFin*, const void*,
                         const tfk::BnBwdFin*, void*, void*, void*, long long, int, const float*, const float*,
                         const uint8_t*, hipStream_t);
int tfk_bn_zero(float*, long long, hipStream_t);
int tfk_maxpool_fwd(const void*, void*, uint8_t*, int, int, int, int, int, int, int, int, int, int, int, int,
                    const float*, const float*, hipStream_t);
int tfk_maxpool_bwd(const void*, const uint8_t*, void*, int, int, int, int, int, int, int, int, int, int, int, int,
                    const void*, const float*, const float*, const float*, const float*, const uint8_t*, float*, int,
                    hipStream_t);
int tfk_avgpool_fwd(const void*, void*, int, int, int, hipStream_t);
int tfk_avgpool_bwd(const void*, void*, int, int, int, hipStream_t);
int tfk_softmax_xent(const void*, const int*, int, int, long long, float, int, float, float*, void*, float*, hipStream_t);
int tfk_xent_full_row(int, long long);
int tfk_sgd(float*, void*, const float*, float*, long long, float, float, float, int, float, const float*, const float*,
            hipStream_t);
int tfk_adamw(float*, void*, const float*, float*, float*, long long, float, float, float, float, float, float, float, float,
              const float*, const float*, hipStream_t);
int tfk_lamb(float*, void*, const float*, float*, float*, float*, const long long*, const int*, const int*, int, float*,
             float, float, float, float, float, float, float, float, const float*, const float*, hipStream_t);
int tfk_opt_hyper(int*, const float*, int, int, float, float, float*, hipStream_t);
int tfk_sumsq(const float*, long long, float*, hipStream_t);
int tfk_clip_coef(const float*, float, float*, float*, hipStream_t);
int tfk_splitk_reduce(const float*, int, long long, long long, float*, void*, int, float, hipStream_t);
void tfk_splitk_set_direct(int);
int tfk_hwgrad_slabs(int, int, int, int, int, int, int, int);
int tfk_stem_wgrad_slabs(int, int, int);
int tfk_stem_fwd_ok(int, int, int);
int tfk_stem_fwd_launch(const void*, const void*, void*, float*, int, int, int, int, hipStream_t);
int tfk_stem_wgrad_launch(const void*, const void*, float*, int, int, int, int, hipStream_t);
int tfk_hwgrad_launch(const void*, const void*, float*, int, int, int, int, int, int, int, int, int, hipStream_t);
int tfk_transpose_arb(const void*, void*, int, int, int, int, hipStream_t);
int tfk_transpose_f32(const float*, float*, int, int, hipStream_t);
int tfk_cast_f32_bf16(const float*, void*, long long, hipStream_t);
int tfk_cast_bf16_f32(const void*, float*, long long, hipStream_t);
int tfk_synth_uniform(void*, long long, int, int, float, float, unsigned long long, hipStream_t);
int tfk_synth_normal_f32(float*, long long, float, float, unsigned long long, hipStream_t);
int tfk_synth_labels(int*, long long, int, unsigned long long, hipStream_t);
int tfk_colsum(const void*, long long, int, long long, float*, hipStream_t);
int tfk_act_fwd(const void*, const float*, int, void*, long long, int, hipStream_t);
int tfk_act_bwd(const void*, const void*, void*, long long, int, hipStream_t);
int tfk_dropout(const void*, void*, long long, float, unsigned long long, hipStream_t);
int tfk_add(const void*, const void*, void*, long long, float, float, hipStream_t);
int tfk_gather_rows(const void*, const int*, int, int, int, long long, void*, hipStream_t);
int tfk_scatter_add_rows(void*, const void*, const int*, int, int, int, int, hipStream_t);
}

namespace {
enum { A_KIN = 0, A_KOUT = 1, A_CONV_FWD = 2, A_CONV_DGRAD = 3 };
enum { B_KIN = 0, B_KOUT = 1, B_CONV_WGRAD = 2 };

// conv = [Nimg, H, W, Cin, P, Q, Cout, R, S, sh, sw, ph, pw, dh, dw]
void gemm(torch::Tensor A, torch::Tensor B, torch::Tensor C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
          int amode, int bmode, int epi, int bm, int bn, double alpha, double beta, c10::optional<torch::Tensor> bias,
          c10::optional<torch::Tensor> resid, int act, c10::optional<torch::Tensor> stats, int shards, int splits,
          int batch, int64_t sA, int64_t sB, int64_t sC, int64_t split_stride, std::vector<int64_t> conv,
          std::vector<c10::optional<torch::Tensor>> bnr, int bn_relu, int bn_shards, c10::optional<torch::Tensor> aux,
          c10::optional<torch::Tensor> dact_src, int dact, double drop_p, int64_t drop_seed,
          std::vector<int64_t> rowmap, c10::optional<torch::Tensor> colsum) {
  need_bf16(A, "A");
  need_bf16(B, "B");
  TORCH_CHECK(epi == 0 || epi == 1, "epi");
  need(C, epi == 0 ? at::kBFloat16 : at::kFloat, "C");
  need_aligned(A, 16, "A");
  need_aligned(B, 16, "B");
  need_aligned(C, 16, "C");
  TORCH_CHECK(M > 0 && N > 0 && K > 0 && batch >= 1, "bad gemm dims M=", M, " N=", N, " K=", K);
  TORCH_CHECK(conv.size() == 15, "conv geometry must have 15 ints");
  tfk::GemmParams p{};
  p.A = A.data_ptr(); p.B = B.data_ptr(); p.C = C.data_ptr();
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.sA = sA; p.sB = sB; p.sC = sC;
  p.Nimg = conv[0]; p.H = conv[1]; p.W = conv[2]; p.Cin = conv[3]; p.P = conv[4]; p.Q = conv[5]; p.Cout = conv[6];
  p.R = conv[7]; p.S = conv[8]; p.sh = conv[9]; p.sw = conv[10]; p.ph = conv[11]; p.pw = conv[12]; p.dh = conv[13];
  p.dw = conv[14];
  p.alpha = (float)alpha; p.beta = (float)beta;
  p.act = act;
  p.stats_shards = shards;
  p.split_stride = split_stride;
  const long long bA = (long long)(batch - 1) * sA, bB = (long long)(batch - 1) * sB, bC = (long long)(batch - 1) * sC;
  // ---- operand A extents
  switch (amode) {
    case A_KIN:
      TORCH_CHECK(lda >= K, "A_KIN needs lda>=K");
      need_numel(A, bA + (long long)(M - 1) * lda + K, "A");
      break;
    case A_KOUT:
      TORCH_CHECK(lda >= M, "A_KOUT needs lda>=M");
      need_numel(A, bA + (long long)(K - 1) * lda + M, "A");
      break;
    case A_CONV_FWD:
      TORCH_CHECK(p.Cin % 8 == 0, "conv fwd needs Cin%8==0");
      TORCH_CHECK((long long)M == (long long)p.Nimg * p.P * p.Q && K == p.R * p.S * p.Cin, "conv fwd M/K mismatch");
      need_numel(A, (long long)p.Nimg * p.H * p.W * p.Cin, "X");
      break;
    case A_CONV_DGRAD:
      TORCH_CHECK(p.Cout % 8 == 0, "conv dgrad needs Cout%8==0");
      TORCH_CHECK((long long)M == (long long)p.Nimg * p.H * p.W && K == p.R * p.S * p.Cout, "conv dgrad M/K mismatch");
      need_numel(A, (long long)p.Nimg * p.P * p.Q * p.Cout, "dY");
      break;
    default: TORCH_CHECK(false, "bad amode");
  }
  switch (bmode) {
    case B_KIN:
      TORCH_CHECK(ldb >= K, "B_KIN needs ldb>=K");
      need_numel(B, bB + (long long)(N - 1) * ldb + K, "B");
      break;
    case B_KOUT:
      TORCH_CHECK(ldb >= N, "B_KOUT needs ldb>=N");
      need_numel(B, bB + (long long)(K - 1) * ldb + N, "B");
      break;
    case B_CONV_WGRAD:
      TORCH_CHECK(p.Cin % 8 == 0, "conv wgrad needs Cin%8==0");
      TORCH_CHECK(N == p.R * p.S * p.Cin && (long long)K == (long long)p.Nimg * p.P * p.Q, "conv wgrad N/K mismatch");
      need_numel(B, (long long)p.Nimg * p.H * p.W * p.Cin, "X");
      break;
    default: TORCH_CHECK(false, "bad bmode");
  }
  TORCH_CHECK(ldc >= N, "ldc < N");
  int ns = tfk_gemm_splits(K, splits);
  if (epi == 0) {
    TORCH_CHECK(ns == 1, "split-K requires the f32 epilogue");
    need_numel(C, bC + (long long)(M - 1) * ldc + N, "C");
  } else {
    TORCH_CHECK(ns == 1 || batch == 1, "split-K with batch>1 unsupported");
    // split_stride == -1: atomic split-K, every split accumulates into the one [M][ldc] C
    TORCH_CHECK(split_stride >= -1, "split_stride must be >= 0, or -1 for atomic split-K");
    TORCH_CHECK(split_stride >= 0 || (batch == 1 && beta == 0.0), "atomic split-K needs batch 1 and beta 0");
    need_numel(C, bC + (long long)(ns - 1) * std::max<int64_t>(split_stride, 0) + (long long)(M - 1) * ldc + N, "C");
  }
  if (bias.has_value() && bias->defined()) { need_f32(*bias, "bias"); need_numel(*bias, N, "bias"); }
  const bool resid_sub = rowmap.size() == 14 && rowmap[12] > 0;  // checked with the row maps below
  if (resid.has_value() && resid->defined()) {
    need_bf16(*resid, "resid");
    if (!resid_sub) need_numel(*resid, bC + (long long)(M - 1) * ldc + N, "resid");
  }
  if (stats.has_value() && stats->defined()) {
    need_f32(*stats, "stats");
    TORCH_CHECK(shards >= 1, "shards");
    need_numel(*stats, (long long)shards * 2 * N, "stats");
  }
  if (!bnr.empty()) {
    // [y, a, mean, invstd, scale, shift, y2, mean2, invstd2, sums]
    TORCH_CHECK(bnr.size() == 10, "bnr needs 10 entries");
    TORCH_CHECK(epi == 0 && N % 8 == 0 && ldc == N && batch == 1, "fused BN reduce needs bf16 out, N%8==0, ldc==N");
    for (int i : {0, 2, 3, 9}) TORCH_CHECK(bnr[i].has_value() && bnr[i]->defined(), "bnr missing required entry ", i);
    need_bf16(*bnr[0], "bn_y"); need_numel(*bnr[0], (long long)M * N, "bn_y");
    const void* bn_a = nullptr;
    p.bn_amask = relu_bitmask(bnr[1], (long long)M * N, &bn_a);
    TORCH_CHECK(!bn_a, "fused BN reduce: pass the activation's packed relu bitmask (uint8), not the bf16 tensor");
    if (bnr[6].has_value() && bnr[6]->defined()) { need_bf16(*bnr[6], "bn_y2"); need_numel(*bnr[6], (long long)M * N, "bn_y2"); }
    for (int i : {2, 3, 4, 5, 7, 8})
      if (bnr[i].has_value() && bnr[i]->defined()) { need_f32(*bnr[i], "bn vec"); need_numel(*bnr[i], N, "bn vec"); }
    need_f32(*bnr[9], "bn_sums");
    TORCH_CHECK(bn_shards >= 1, "bn_shards");
    need_numel(*bnr[9], (long long)bn_shards * 3 * N, "bn_sums");
    p.bn_y = bnr[0]->data_ptr();
    p.bn_mean = bnr[2]->data_ptr<float>();
    p.bn_invstd = bnr[3]->data_ptr<float>();
    p.bn_scale = opt_ptr<const float>(bnr[4]);
    p.bn_shift = opt_ptr<const float>(bnr[5]);
    p.bn_y2 = opt_ptr<const void>(bnr[6]);
    p.bn_mean2 = opt_ptr<const float>(bnr[7]);
    p.bn_invstd2 = opt_ptr<const float>(bnr[8]);
    p.bn_sums = bnr[9]->data_ptr<float>();
    p.bn_relu = bn_relu & 1;            // bit 0: relu mask from y*scale+shift
    p.bn_store_dz = (bn_relu >> 1) & 1;  // bit 1: store dz (masked dA) instead of dA
    p.bn_shards = bn_shards;
    TORCH_CHECK(!(p.bn_relu && !p.bn_amask && !(p.bn_scale && p.bn_shift)), "relu mask needs a or scale/shift");
  }
  p.bias = opt_ptr<const float>(bias);
  p.resid = opt_ptr<const void>(resid);
  p.stats = opt_ptr<float>(stats);
  for (auto* t : {&aux, &dact_src}) {
    if (t->has_value() && (*t)->defined()) {
      TORCH_CHECK(epi == 0, "aux/dact need the bf16 epilogue");
      if (relu_mask(**t, ldc, N, batch > 1 ? sC : 0, "aux/dact_src")) {
        need_numel(**t, (bC + (long long)(M - 1) * ldc + N + 7) / 8, "aux/dact_src relu mask");
      } else {
        need_bf16(**t, "aux/dact_src");
        need_numel(**t, bC + (long long)(M - 1) * ldc + N, "aux/dact_src");
      }
    }
  }
  p.aux = opt_ptr<void>(aux);
  p.dact_src = opt_ptr<const void>(dact_src);
  p.dact = dact;
  p.aux_bits = p.aux && aux->scalar_type() == at::kByte;
  p.dact_bits = p.dact_src && dact_src->scalar_type() == at::kByte;
  if (colsum.has_value() && colsum->defined()) {
    need_f32(*colsum, "colsum");
    need_numel(*colsum, N, "colsum");
    TORCH_CHECK(epi == 0 && batch == 1 && !(stats.has_value() && stats->defined()) && !p.resid &&
                    (p.dact_src || p.aux || drop_p > 0.0),
                "colsum: bf16 EXT epilogue (aux / dact / dropout), batch 1, no BN statistics, no residual");
  }
  p.colsum = opt_ptr<float>(colsum);
  TORCH_CHECK(!p.aux_bits || act == 1, "a relu-mask aux needs act relu");
  TORCH_CHECK(!p.dact_bits || dact == 1, "a relu-mask dact_src needs dact relu");
  TORCH_CHECK(!p.dact_src || (dact >= 1 && dact <= 3), "dact must be 1 (relu), 2 (gelu) or 3 (tanh) with dact_src");
  TORCH_CHECK(act >= 0 && act <= 3, "act");
  TORCH_CHECK(drop_p >= 0.0 && drop_p < 1.0, "drop_p");
  TORCH_CHECK(drop_p == 0.0 || (epi == 0 && ldc == N && batch == 1), "fused dropout needs bf16 out, ldc==N, batch 1");
  p.drop_p = (float)drop_p;
  p.drop_scale = drop_p > 0.0 ? 256.f / (float)(256 - drop_thr8_host((float)drop_p)) : 1.f;
  p.drop_seed = (unsigned long long)drop_seed;
  p.drop_seed_key = tfk_seed_key();
  const bool dense_a = amode == A_KIN || amode == A_KOUT;
  // the conv-fwd-gather / wgrad-gather 256x256 tiles and the 64x128 tile exist on the LDS-DMA engine
  // (gemm_g4.hip) only; the launcher falls back to 128x128 where that engine declines the shape
  TORCH_CHECK((bm == 128 && bn == 128) || (bm == 128 && bn == 64) || (bm == 64 && bn == 64) || (bm == 64 && bn == 128) ||
                  (bm == 256 && bn == 256 && (dense_a || amode == A_CONV_FWD) && (bmode == B_KIN || bmode == B_KOUT)) ||
                  (bm == 256 && bn == 256 && amode == A_KOUT && bmode == B_CONV_WGRAD) ||
                  (bm == 256 && bn == 64 && dense_a && !(amode == A_KOUT && bmode == B_KOUT && epi == 0)) ||
                  (bm == 256 && bn == 64 && amode == A_CONV_FWD && bmode == B_KIN) ||
                  (bm == 64 && bn == 256 && amode == A_KOUT && bmode == B_CONV_WGRAD && epi == 1) ||
                  (bm == 64 && bn == 256 && amode == A_KOUT && bmode == B_KOUT && epi == 1) ||
                  // 8-wave 3-stage g4 tiles (the launcher falls back to 128x128 where g4 declines)
                  ((bm == 256 && bn == 128) || (bm == 128 && bn == 256)),
              "unsupported tile ", bm, "x", bn, " for operand modes ", amode, "/", bmode);
  // row maps: [om_hp, om_wp, om_h, om_w, om_sh, om_sw, om_a, om_b, rs_h, rs_w, rs_p, rs_q, rs_sh, rs_sw]
  if (!rowmap.empty()) {
    TORCH_CHECK(rowmap.size() == 14, "rowmap needs 14 ints");
    TORCH_CHECK(!bnr.empty() && epi == 0 && batch == 1, "row maps need the fused BN-backward bf16 epilogue");
    const auto& r = rowmap;
    for (int i = 0; i < 14; ++i) TORCH_CHECK(r[i] >= 0, "rowmap entries must be >= 0");
    if (r[0] > 0) {
      TORCH_CHECK(r[4] >= 1 && r[5] >= 1 && r[6] < r[4] && r[7] < r[5], "out-map stride/phase");
      TORCH_CHECK(M % (r[0] * r[1]) == 0, "out-map: M must be images x om_hp x om_wp");
      TORCH_CHECK((r[0] - 1) * r[4] + r[6] < r[2] && (r[1] - 1) * r[5] + r[7] < r[3], "out-map exceeds the output grid");
      const long long rows = (long long)(M / (r[0] * r[1])) * r[2] * r[3];
      need_numel(C, (rows - 1) * ldc + N, "C (out-map)");
      for (int i : {0, 1, 6})
        if (bnr[i].has_value() && bnr[i]->defined())
          need_numel(*bnr[i], bnr[i]->scalar_type() == at::kByte ? rows * N / 8 : rows * N, "bn tensor (out-map)");
      if (resid.has_value() && resid->defined()) need_numel(*resid, (rows - 1) * ldc + N, "resid (out-map)");
    }
    if (r[12] > 0) {
      TORCH_CHECK(r[13] >= 1 && r[8] > 0 && r[9] > 0 && r[10] == (r[8] + r[12] - 1) / r[12] &&
                      r[11] == (r[9] + r[13] - 1) / r[13], "resid sub-sampling geometry");
      TORCH_CHECK(r[0] == 0, "resid sub-sampling and out-map are exclusive");
      TORCH_CHECK(M % (r[8] * r[9]) == 0, "resid sub-sampling: M must be images x rs_h x rs_w");
      TORCH_CHECK(resid.has_value() && resid->defined(), "resid sub-sampling needs resid");
      need_numel(*resid, (long long)(M / (r[8] * r[9])) * r[10] * r[11] * ldc, "resid (sub-sampled)");
    }
    p.om_hp = r[0]; p.om_wp = r[1]; p.om_h = r[2]; p.om_w = r[3]; p.om_sh = r[4]; p.om_sw = r[5]; p.om_a = r[6];
    p.om_b = r[7]; p.rs_h = r[8]; p.rs_w = r[9]; p.rs_p = r[10]; p.rs_q = r[11]; p.rs_sh = r[12]; p.rs_sw = r[13];
  }
  check_rc(tfk_gemm_launch(p, bm, bn, amode, bmode, epi, batch, splits, cur_stream()), "gemm");
}

int64_t gemm_splits(int K, int splits) { return tfk_gemm_splits(K, splits); }
// A/B switch for the persistent GEMM grid (tools/op_profile.py); default on.
void gemm_set_persist(int on) { tfk_gemm_set_persist(on); }
void gemm_set_engine(int e) { tfk_gemm_set_engine(e); }
void gemm_set_shortk(int on) { tfk_g4_set_shortk(on); }
void fp8_set_engine(int e) { tfk_fp8_set_engine(e); }

void mx_probe(torch::Tensor X, torch::Tensor Y, torch::Tensor sx, torch::Tensor sy, torch::Tensor D) {
  for (auto* t : {&X, &Y}) { need(*t, at::kInt, "probe operand"); need_numel(*t, 64 * 8, "probe operand"); }
  for (auto* t : {&sx, &sy}) { need(*t, at::kInt, "probe scale"); need_numel(*t, 64, "probe scale"); }
  need_f32(D, "D"); need_numel(D, 256, "D");
  check_rc(tfk_mx_probe(X.data_ptr<int>(), Y.data_ptr<int>(), sx.data_ptr<int>(), sy.data_ptr<int>(),
                        D.data_ptr<float>(), cur_stream()), "mx_probe");
}

// MX-fp8: x bf16 [rows][K] -> q uint8 (e4m3) [rows][K], s uint8 (e8m0) [rows][K/32]
void mx_quant(torch::Tensor x, torch::Tensor q, torch::Tensor s, int64_t rows, int64_t K) {
  need_bf16(x, "x"); need(q, at::kByte, "q"); need(s, at::kByte, "s");
  TORCH_CHECK(K % 32 == 0, "mx_quant needs K % 32 == 0");
  need_numel(x, rows * K, "x"); need_numel(q, rows * K, "q"); need_numel(s, rows * K / 32, "s");
  need_aligned(x, 16, "x"); need_aligned(q, 16, "q");
  check_rc(tfk_mx_quant(x.data_ptr(), q.data_ptr(), s.data_ptr(), rows * K / 32, cur_stream()), "mx_quant");
}

// MX-fp8 transposing quantizer: x bf16 [R][C] -> q uint8 [C][R], s uint8 [C][R/32]
void mx_quant_t(torch::Tensor x, torch::Tensor q, torch::Tensor s, int64_t R, int64_t C) {
  need_bf16(x, "x"); need(q, at::kByte, "q"); need(s, at::kByte, "s");
  TORCH_CHECK(R % 32 == 0 && R > 0 && C > 0, "mx_quant_t needs R % 32 == 0");
  need_numel(x, R * C, "x"); need_numel(q, R * C, "q"); need_numel(s, R * C / 32, "s");
  need_aligned(x, 16, "x"); need_aligned(q, 16, "q");
  check_rc(tfk_mx_quant_t(x.data_ptr(), q.data_ptr(), s.data_ptr(), (int)R, (int)C, cur_stream()), "mx_quant_t");
}

// Both MX quantizations in one read: x bf16 [R][C] -> row blocks (qr [R][C], sr [R][C/32]) and
// column blocks (qc [C][R], sc [C][R/32]); R % 32 == 0, C % 32 == 0
void mx_quant_dual(torch::Tensor x, torch::Tensor qr, torch::Tensor sr, torch::Tensor qc, torch::Tensor sc, int64_t R,
                   int64_t C) {
  need_bf16(x, "x");
  for (auto* t : {&qr, &sr, &qc, &sc}) need(*t, at::kByte, "mx dual out");
  TORCH_CHECK(R % 32 == 0 && C % 32 == 0 && R > 0 && C > 0, "mx_quant_dual needs R % 32 == 0 and C % 32 == 0");
  need_numel(x, R * C, "x"); need_numel(qr, R * C, "qr"); need_numel(qc, R * C, "qc");
  need_numel(sr, R * C / 32, "sr"); need_numel(sc, R * C / 32, "sc");
  for (auto* t : {&x, &qr, &qc}) need_aligned(*t, 16, "mx dual tensor");
  check_rc(tfk_mx_quant_dual(x.data_ptr(), qr.data_ptr(), sr.data_ptr(), qc.data_ptr(), sc.data_ptr(), (int)R, (int)C,
                             cur_stream()), "mx_quant_dual");
}

// Grouped dual quantization: table int64 [n][7] on the device, one QDesc per tensor (x, qr, sr, qc,
// sc, R | C << 32, t0 | tcols << 32), built and validated by ops/fp8.py GroupQuantizer.
void mx_quant_dual_group(torch::Tensor table, int64_t n, int64_t total) {
  need(table, at::kLong, "mx group table");
  TORCH_CHECK(table.is_cuda() && table.is_contiguous() && table.numel() == n * 7 && n > 0 && total > 0,
              "mx_quant_dual_group: table must be a contiguous device int64 [n][7]");
  check_rc(tfk_mx_quant_dual_group(table.data_ptr(), (int)n, (int)total, cur_stream()), "mx_quant_dual_group");
}

// C[M][N] = epilogue(Aq[M][K] . Bq[N][K]^T) with e8m0 block scales (one per 32 K-elements).
// C bf16: bias / act / resid / aux / dropout / activation backward (dact_src, dact);
// C f32: C = alpha * AB + beta * C (weight gradients).
void gemm_mxfp8(torch::Tensor A, torch::Tensor As, torch::Tensor B, torch::Tensor Bs, torch::Tensor C, int M, int N, int K,
                c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> resid, int act,
                c10::optional<torch::Tensor> aux, double drop_p, int64_t drop_seed,
                c10::optional<torch::Tensor> dact_src, int dact, double beta, int splits, int64_t split_stride,
                c10::optional<std::vector<torch::Tensor>> mx_out, bool mx_skip_c, c10::optional<torch::Tensor> colsum) {
  for (auto* t : {&A, &As, &B, &Bs}) need(*t, at::kByte, "mx operand");
  const bool f32 = C.scalar_type() == at::kFloat;
  if (!f32) need_bf16(C, "C");
  TORCH_CHECK(!f32 || (!bias.has_value() && !resid.has_value() && !aux.has_value() && !dact_src.has_value() &&
                       act == 0 && drop_p == 0.0), "gemm_mxfp8: f32 output takes no epilogue extras");
  TORCH_CHECK(M > 0 && N > 0 && K > 0 && K % 128 == 0, "gemm_mxfp8 needs K % 128 == 0, got ", K);
  need_numel(A, (long long)M * K, "A"); need_numel(B, (long long)N * K, "B");
  need_numel(As, (long long)M * K / 32, "As"); need_numel(Bs, (long long)N * K / 32, "Bs");
  TORCH_CHECK(splits >= 1 && (splits == 1 || (f32 && split_stride >= (long long)M * N)), "gemm_mxfp8: split-K needs f32 slabs");
  need_numel(C, splits > 1 ? (long long)(splits - 1) * split_stride + (long long)M * N : (long long)M * N, "C");
  for (auto* t : {&A, &B, &C}) need_aligned(*t, 16, "gemm_mxfp8 operand");
  for (auto* t : {&As, &Bs}) need_aligned(*t, 4, "gemm_mxfp8 scales");
  TORCH_CHECK(act >= 0 && act <= 3, "act");
  TORCH_CHECK(drop_p >= 0.0 && drop_p < 1.0, "drop_p");
  tfk::GemmParams p{};
  p.A = A.data_ptr(); p.B = B.data_ptr(); p.C = C.data_ptr();
  p.M = M; p.N = N; p.K = K; p.lda = K; p.ldb = K; p.ldc = N;
  p.alpha = 1.f; p.act = act;
  p.a_scale = As.data_ptr(); p.b_scale = Bs.data_ptr();
  if (bias.has_value() && bias->defined()) { need_f32(*bias, "bias"); need_numel(*bias, N, "bias"); }
  if (resid.has_value() && resid->defined()) { need_bf16(*resid, "resid"); need_numel(*resid, (long long)M * N, "resid"); }
  if (aux.has_value() && aux->defined()) {
    if (relu_mask(*aux, N, N, 0, "aux")) need_numel(*aux, (long long)M * N / 8, "aux relu mask");
    else { need_bf16(*aux, "aux"); need_numel(*aux, (long long)M * N, "aux"); }
  }
  p.bias = opt_ptr<const float>(bias);
  p.resid = opt_ptr<const void>(resid);
  p.aux = opt_ptr<void>(aux);
  p.aux_bits = p.aux && aux->scalar_type() == at::kByte;
  TORCH_CHECK(!p.aux_bits || act == 1, "a relu-mask aux needs act relu");
  p.drop_p = (float)drop_p;
  p.drop_scale = drop_p > 0.0 ? 256.f / (float)(256 - drop_thr8_host((float)drop_p)) : 1.f;
  p.drop_seed = (unsigned long long)drop_seed;
  p.drop_seed_key = tfk_seed_key();
  if (dact_src.has_value() && dact_src->defined()) {
    if (relu_mask(*dact_src, N, N, 0, "dact_src")) need_numel(*dact_src, (long long)M * N / 8, "dact_src relu mask");
    else { need_bf16(*dact_src, "dact_src"); need_numel(*dact_src, (long long)M * N, "dact_src"); }
    TORCH_CHECK(dact >= 1 && dact <= 3, "dact");
  }
  p.dact_src = opt_ptr<const void>(dact_src);
  p.dact = dact;
  p.dact_bits = p.dact_src && dact_src->scalar_type() == at::kByte;
  TORCH_CHECK(!p.dact_bits || dact == 1, "a relu-mask dact_src needs dact relu");
  p.beta = (float)beta;
  if (colsum.has_value() && colsum->defined()) {
    need_f32(*colsum, "colsum");
    need_numel(*colsum, N, "colsum");
    TORCH_CHECK(!f32 && !p.resid && (p.dact_src || p.aux || drop_p > 0.0),
                "colsum: bf16 EXT epilogue (aux / dact / dropout), no residual");
  }
  p.colsum = opt_ptr<float>(colsum);
  // an activated bf16 output takes the EXT epilogue (the plain bf16 one is activation-free)
  int ext = f32 ? 2 : ((p.aux || drop_p > 0.0 || p.dact_src || p.act) ? 1 : 0);
  if (mx_out.has_value()) {
    // MX-fp8 copies of C from the epilogue: [qr [M][N], sr [M][N/32], qc [N][M], sc [N][M/32]]
    const auto& o = *mx_out;
    TORCH_CHECK(!f32 && splits == 1 && o.size() == 4 && M % 32 == 0 && N % 32 == 0,
                "gemm_mxfp8 mx_out: bf16 output, no split, M, N % 32 == 0, 4 tensors");
    for (const auto& t : o) need(t, at::kByte, "mx_out");
    need_numel(o[0], (long long)M * N, "mx qr"); need_numel(o[1], (long long)M * N / 32, "mx sr");
    need_numel(o[2], (long long)M * N, "mx qc"); need_numel(o[3], (long long)M * N / 32, "mx sc");
    need_aligned(o[0], 16, "mx qr"); need_aligned(o[2], 16, "mx qc");
    p.mx_qr = o[0].data_ptr(); p.mx_sr = o[1].data_ptr(); p.mx_qc = o[2].data_ptr(); p.mx_sc = o[3].data_ptr();
    p.mx_skip_c = mx_skip_c ? 1 : 0;
    ext = 3;
  } else {
    TORCH_CHECK(!mx_skip_c, "gemm_mxfp8: mx_skip_c without mx_out");
  }
  // f32 split-K: split z writes its partial to the slab C + z * split_stride (ops.fp8 reduces them)
  p.split_stride = splits > 1 ? split_stride : 0;
  check_rc(tfk_gemm_mxfp8(p, ext, splits, cur_stream()), "gemm_mxfp8");
}

void bn_finalize(torch::Tensor stats, int shards, int C, double count, torch::Tensor gamma, torch::Tensor beta, double eps,
                 double momentum, c10::optional<torch::Tensor> run_mean, c10::optional<torch::Tensor> run_var,
                 torch::Tensor mean, torch::Tensor invstd, torch::Tensor scale, torch::Tensor shift) {
  need_f32(stats, "stats"); need_numel(stats, (long long)shards * 2 * C, "stats");
  for (auto* t : {&gamma, &beta, &mean, &invstd, &scale, &shift}) { need_f32(*t, "bn vec"); need_numel(*t, C, "bn vec"); }
  check_rc(tfk_bn_finalize(stats.data_ptr<float>(), shards, C, (float)count, gamma.data_ptr<float>(), beta.data_ptr<float>(),
                           (float)eps, (float)momentum, opt_ptr<float>(run_mean), opt_ptr<float>(run_var),
                           mean.data_ptr<float>(), invstd.data_ptr<float>(), scale.data_ptr<float>(),
                           shift.data_ptr<float>(), cur_stream()),
           "bn_finalize");
}

void bn_stats(torch::Tensor y, int64_t M, int C, torch::Tensor stats, int shards) {
  need_bf16(y, "y"); need_numel(y, M * C, "y"); TORCH_CHECK(C % 8 == 0, "C%8");
  need_f32(stats, "stats"); need_numel(stats, (long long)shards * 2 * C, "stats");
  check_rc(tfk_bn_stats(y.data_ptr(), M, C, stats.data_ptr<float>(), shards, cur_stream()), "bn_stats");
}

void bn_apply(torch::Tensor y, torch::Tensor scale, torch::Tensor shift, c10::optional<torch::Tensor> r,
              c10::optional<torch::Tensor> rscale, c10::optional<torch::Tensor> rshift, bool relu, torch::Tensor out,
              int64_t M, int C, c10::optional<torch::Tensor> mask) {
  need_bf16(y, "y"); need_bf16(out, "out"); need_numel(y, M * C, "y"); need_numel(out, M * C, "out");
  uint8_t* mk = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(relu && mask->scalar_type() == torch::kUInt8, "bn_apply: mask is the relu bitmask (uint8)");
    need_numel(*mask, M * C / 8, "mask");
    mk = mask->data_ptr<uint8_t>();
  }
  TORCH_CHECK(C % 8 == 0, "C%8");
  need_aligned(y, 16, "y"); need_aligned(out, 16, "out");
  need_f32(scale, "scale"); need_f32(shift, "shift"); need_numel(scale, C, "scale"); need_numel(shift, C, "shift");
  if (r.has_value() && r->defined()) { need_bf16(*r, "r"); need_numel(*r, M * C, "r"); }
  if (rscale.has_value() && rscale->defined()) { need_numel(*rscale, C, "rscale"); need_numel(*rshift, C, "rshift"); }
  check_rc(tfk_bn_apply(y.data_ptr(), scale.data_ptr<float>(), shift.data_ptr<float>(), opt_ptr<const void>(r),
                        opt_ptr<const float>(rscale), opt_ptr<const float>(rshift), relu ? 1 : 0, out.data_ptr(), M, C,
                        mk, cur_stream()),
           "bn_apply");
}

// Finalize-in-apply BN (bn.hip). f = [stats, gamma, beta, run_mean, run_var, mean, invstd, scale, shift]
// (stats undefined: apply with the given scale/shift, nothing finalized).
static tfk::BnFin bn_fin_of(const std::vector<c10::optional<torch::Tensor>>& f, double eps, double momentum, int shards,
                            int C) {
  TORCH_CHECK(f.size() == 9, "bn fin: [stats, gamma, beta, run_mean, run_var, mean, invstd, scale, shift]");
  tfk::BnFin b{};
  const bool fin = f[0].has_value() && f[0]->defined();
  if (fin) {
    need_f32(*f[0], "stats");
    need_numel(*f[0], (long long)shards * 2 * C, "stats");
    for (int i : {1, 2, 5, 6})
      TORCH_CHECK(f[i].has_value() && f[i]->defined(), "bn fin: gamma/beta/mean/invstd required");
  }
  for (int i = 1; i < 9; ++i)
    if (f[i].has_value() && f[i]->defined()) { need_f32(*f[i], "bn vec"); need_numel(*f[i], C, "bn vec"); }
  TORCH_CHECK(f[7].has_value() && f[7]->defined() && f[8].has_value() && f[8]->defined(), "bn fin: scale/shift required");
  b.stats = fin ? f[0]->data_ptr<float>() : nullptr;
  b.gamma = opt_ptr<const float>(f[1]);
  b.beta = opt_ptr<const float>(f[2]);
  b.run_mean = opt_ptr<float>(f[3]);
  b.run_var = opt_ptr<float>(f[4]);
  b.mean = opt_ptr<float>(f[5]);
  b.invstd = opt_ptr<float>(f[6]);
  b.scale = f[7]->data_ptr<float>();
  b.shift = f[8]->data_ptr<float>();
  b.eps = (float)eps;
  b.momentum = (float)momentum;
  b.shards = shards;
  return b;
}

bool bn_fin_ok(int C, int shards) { return tfk_bn_fin_ok(C, shards) != 0; }

void bn_apply_fin(torch::Tensor y, std::vector<c10::optional<torch::Tensor>> f, double eps, double momentum, int shards,
                  c10::optional<torch::Tensor> r, std::vector<c10::optional<torch::Tensor>> f2, double eps2,
                  double momentum2, int shards2, bool relu, torch::Tensor out, int64_t M, int C,
                  c10::optional<torch::Tensor> mask) {
  need_bf16(y, "y"); need_bf16(out, "out"); need_numel(y, M * C, "y"); need_numel(out, M * C, "out");
  need_aligned(y, 16, "y"); need_aligned(out, 16, "out");
  TORCH_CHECK(C % 64 == 0, "bn_apply_fin: C % 64");
  uint8_t* mk = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(relu && mask->scalar_type() == torch::kUInt8, "bn_apply_fin: mask is the relu bitmask (uint8)");
    need_numel(*mask, M * C / 8, "mask");
    mk = mask->data_ptr<uint8_t>();
  }
  const tfk::BnFin a = bn_fin_of(f, eps, momentum, shards, C);
  tfk::BnFin b{};
  const bool dual = !f2.empty();
  if (dual) b = bn_fin_of(f2, eps2, momentum2, shards2, C);
  if (r.has_value() && r->defined()) { need_bf16(*r, "r"); need_numel(*r, M * C, "r"); need_aligned(*r, 16, "r"); }
  TORCH_CHECK(!dual || (r.has_value() && r->defined()), "bn_apply_fin: a second BN needs r");
  check_rc(tfk_bn_apply_fin(y.data_ptr(), &a, opt_ptr<const void>(r), dual ? &b : nullptr, relu ? 1 : 0, out.data_ptr(),
                            M, C, mk, cur_stream()),
           "bn_apply_fin");
}

// g = [gamma, mean, invstd, dgamma, dbeta] per BN; g2 empty without a second BN.
static tfk::BnBwdFin bn_bwd_fin_of(const std::vector<torch::Tensor>& g, int C) {
  TORCH_CHECK(g.size() == 5, "bn bwd fin: [gamma, mean, invstd, dgamma, dbeta]");
  for (auto& t : g) { need_f32(t, "bn vec"); need_numel(t, C, "bn vec"); }
  return tfk::BnBwdFin{g[0].data_ptr<float>(), g[1].data_ptr<float>(), g[2].data_ptr<float>(), g[3].data_ptr<float>(),
                       g[4].data_ptr<float>()};
}

void bn_bwd_apply_fin(torch::Tensor da, c10::optional<torch::Tensor> amask_t, torch::Tensor y, torch::Tensor sums,
                      int shards, std::vector<torch::Tensor> g, c10::optional<torch::Tensor> y2,
                      std::vector<torch::Tensor> g2, torch::Tensor dy, c10::optional<torch::Tensor> dy2,
                      c10::optional<torch::Tensor> dres, int64_t M, int C, c10::optional<torch::Tensor> mscale,
                      c10::optional<torch::Tensor> mshift) {
  need_bf16(da, "da"); need_bf16(y, "y"); need_bf16(dy, "dy");
  for (auto* t : {&da, &y, &dy}) { need_numel(*t, M * C, "bn bwd tensor"); need_aligned(*t, 16, "bn bwd tensor"); }
  TORCH_CHECK(C % 64 == 0, "bn_bwd_apply_fin: C % 64");
  need_f32(sums, "sums"); need_numel(sums, (long long)shards * 3 * C, "sums");
  const uint8_t* amask = nullptr;
  if (amask_t.has_value() && amask_t->defined()) {
    TORCH_CHECK(amask_t->scalar_type() == torch::kUInt8, "bn_bwd_apply_fin: the relu mask is the packed bitmask");
    need_numel(*amask_t, M * C / 8, "mask");
    amask = amask_t->data_ptr<uint8_t>();
  }
  const tfk::BnBwdFin a = bn_bwd_fin_of(g, C);
  tfk::BnBwdFin b{};
  const bool two = y2.has_value() && y2->defined();
  if (two) {
    b = bn_bwd_fin_of(g2, C);
    TORCH_CHECK(dy2.has_value() && dy2->defined(), "bn_bwd_apply_fin: y2 needs dy2");
    need_numel(*y2, M * C, "y2"); need_numel(*dy2, M * C, "dy2");
  }
  if (dres.has_value() && dres->defined()) need_numel(*dres, M * C, "dres");
  if (mscale.has_value() && mscale->defined()) { need_numel(*mscale, C, "mscale"); need_numel(*mshift, C, "mshift"); }
  check_rc(tfk_bn_bwd_apply_fin(da.data_ptr(), y.data_ptr(), sums.data_ptr<float>(), shards, &a, opt_ptr<const void>(y2),
                                two ? &b : nullptr, dy.data_ptr(), opt_ptr<void>(dy2), opt_ptr<void>(dres), M, C,
                                opt_ptr<const float>(mscale), opt_ptr<const float>(mshift), amask, cur_stream()),
           "bn_bwd_apply_fin");
}

void bn_zero(torch::Tensor t) {
  need_f32(t, "bn accumulators");
  TORCH_CHECK(t.is_contiguous(), "bn_zero: contiguous");
  check_rc(tfk_bn_zero(t.data_ptr<float>(), t.numel(), cur_stream()), "bn_zero");
}

void bn_bwd_reduce(torch::Tensor da, c10::optional<torch::Tensor> a, torch::Tensor y, torch::Tensor mean,
                   torch::Tensor invstd, c10::optional<torch::Tensor> y2, c10::optional<torch::Tensor> mean2,
                   c10::optional<torch::Tensor> invstd2, int64_t M, int C, torch::Tensor sums, int shards,
                   c10::optional<torch::Tensor> mscale, c10::optional<torch::Tensor> mshift) {
  need_bf16(da, "da"); need_bf16(y, "y"); need_numel(da, M * C, "da"); need_numel(y, M * C, "y");
  TORCH_CHECK(C % 8 == 0, "C%8");
  const void* ap = nullptr;
  const uint8_t* amask = relu_bitmask(a, M * C, &ap);
  if (y2.has_value() && y2->defined()) need_numel(*y2, M * C, "y2");
  need_f32(sums, "sums"); need_numel(sums, (long long)shards * 3 * C, "sums");
  check_rc(tfk_bn_bwd_reduce(da.data_ptr(), ap, y.data_ptr(), mean.data_ptr<float>(),
                             invstd.data_ptr<float>(), opt_ptr<const void>(y2), opt_ptr<const float>(mean2),
                             opt_ptr<const float>(invstd2), M, C, sums.data_ptr<float>(), shards,
                             opt_ptr<const float>(mscale), opt_ptr<const float>(mshift), amask, cur_stream()),
           "bn_bwd_reduce");
}

void bn_bwd_finalize(torch::Tensor sums, int shards, int C, double count, torch::Tensor gamma, torch::Tensor mean,
                     torch::Tensor invstd, c10::optional<torch::Tensor> gamma2, c10::optional<torch::Tensor> mean2,
                     c10::optional<torch::Tensor> invstd2, torch::Tensor dgamma, torch::Tensor dbeta,
                     c10::optional<torch::Tensor> dgamma2, c10::optional<torch::Tensor> dbeta2, torch::Tensor coef,
                     c10::optional<torch::Tensor> coef2) {
  need_f32(sums, "sums"); need_numel(sums, (long long)shards * 3 * C, "sums");
  for (auto* t : {&gamma, &mean, &invstd, &dgamma, &dbeta}) { need_f32(*t, "bn vector"); need_numel(*t, C, "bn vector"); }
  need_numel(coef, 3 * C, "coef");
  if (coef2.has_value() && coef2->defined()) {
    need_numel(*coef2, 3 * C, "coef2");
    TORCH_CHECK(gamma2.has_value() && mean2.has_value() && invstd2.has_value() && dgamma2.has_value() &&
                    dbeta2.has_value(), "bn_bwd_finalize: second BN needs gamma2/mean2/invstd2/dgamma2/dbeta2");
  }
  check_rc(tfk_bn_bwd_finalize(sums.data_ptr<float>(), shards, C, (float)count, gamma.data_ptr<float>(),
                               mean.data_ptr<float>(), invstd.data_ptr<float>(), opt_ptr<const float>(gamma2),
                               opt_ptr<const float>(mean2), opt_ptr<const float>(invstd2), dgamma.data_ptr<float>(),
                               dbeta.data_ptr<float>(), opt_ptr<float>(dgamma2), opt_ptr<float>(dbeta2),
                               coef.data_ptr<float>(), opt_ptr<float>(coef2), cur_stream()),
           "bn_bwd_finalize");
}

void bn_bwd_apply(torch::Tensor da, c10::optional<torch::Tensor> a, torch::Tensor y, torch::Tensor coef, torch::Tensor dy,
                  c10::optional<torch::Tensor> y2, c10::optional<torch::Tensor> coef2, c10::optional<torch::Tensor> dy2,
                  c10::optional<torch::Tensor> dres, int64_t M, int C, c10::optional<torch::Tensor> mscale,
                  c10::optional<torch::Tensor> mshift) {
  need_bf16(da, "da"); need_bf16(y, "y"); need_bf16(dy, "dy");
  for (auto* t : {&da, &y, &dy}) need_numel(*t, M * C, "bn bwd tensor");
  need_f32(coef, "coef"); need_numel(coef, 3 * C, "coef");
  const void* ap = nullptr;
  const uint8_t* amask = relu_bitmask(a, M * C, &ap);
  if (y2.has_value() && y2->defined()) {
    TORCH_CHECK(coef2.has_value() && dy2.has_value(), "bn_bwd_apply: y2 needs coef2 and dy2");
    need_numel(*y2, M * C, "y2"); need_numel(*dy2, M * C, "dy2"); need_numel(*coef2, 3 * C, "coef2");
  }
  if (dres.has_value() && dres->defined()) need_numel(*dres, M * C, "dres");
  if (mscale.has_value() && mscale->defined()) { need_numel(*mscale, C, "mscale"); need_numel(*mshift, C, "mshift"); }
  TORCH_CHECK(C % 8 == 0, "C%8");
  check_rc(tfk_bn_bwd_apply(da.data_ptr(), ap, y.data_ptr(), coef.data_ptr<float>(), dy.data_ptr(),
                            opt_ptr<const void>(y2), opt_ptr<const float>(coef2), opt_ptr<void>(dy2),
                            opt_ptr<void>(dres), M, C, opt_ptr<const float>(mscale), opt_ptr<const float>(mshift),
                            amask, cur_stream()),
           "bn_bwd_apply");
}

// geom = [N, H, W, C, P, Q, KH, KW, sh, sw, ph, pw]
// bn (optional [scale, shift]): pool relu(x*scale + shift) -- the producer BN applied on the fly
void maxpool_fwd(torch::Tensor x, torch::Tensor y, torch::Tensor idx, std::vector<int64_t> g,
                 std::vector<torch::Tensor> bn) {
  TORCH_CHECK(g.size() == 12, "geom");
  TORCH_CHECK(bn.empty() || bn.size() == 2, "maxpool_fwd: bn = [scale, shift]");
  for (auto& t : bn) { need_f32(t, "bn vec"); need_numel(t, g[3], "bn vec"); }
  need_bf16(x, "x"); need_bf16(y, "y"); need(idx, at::kByte, "idx");
  TORCH_CHECK(g[3] % 8 == 0, "C%8");
  need_numel(x, g[0] * g[1] * g[2] * g[3], "x");
  need_numel(y, g[0] * g[4] * g[5] * g[3], "y");
  need_numel(idx, g[0] * g[4] * g[5] * g[3], "idx");
  TORCH_CHECK(g[6] * g[7] <= 255, "window too large");
  check_rc(tfk_maxpool_fwd(x.data_ptr(), y.data_ptr(), idx.data_ptr<uint8_t>(), g[0], g[1], g[2], g[3], g[4], g[5], g[6],
                           g[7], g[8], g[9], g[10], g[11], bn.empty() ? nullptr : bn[0].data_ptr<float>(),
                           bn.empty() ? nullptr : bn[1].data_ptr<float>(), cur_stream()),
           "maxpool_fwd");
}
// bnr (optional, the gemm's 10-entry BN-reduce spec without y2): also accumulate the BN-backward
// channel sums of the layer that produced the pooled input from the final dx
void maxpool_bwd(torch::Tensor dy, torch::Tensor idx, torch::Tensor dx, std::vector<int64_t> g,
                 std::vector<c10::optional<torch::Tensor>> bnr, int bn_shards) {
  TORCH_CHECK(g.size() == 12, "geom");
  need_bf16(dy, "dy"); need_bf16(dx, "dx"); need(idx, at::kByte, "idx");
  const long long nx = g[0] * g[1] * g[2] * g[3];
  need_numel(dx, nx, "dx");
  need_numel(dy, g[0] * g[4] * g[5] * g[3], "dy");
  need_numel(idx, g[0] * g[4] * g[5] * g[3], "idx");
  const void* y = nullptr;
  const float *mean = nullptr, *invstd = nullptr, *msc = nullptr, *msh = nullptr;
  const uint8_t* amask = nullptr;
  float* sums = nullptr;
  if (!bnr.empty()) {
    TORCH_CHECK(bnr.size() == 10, "bnr needs 10 entries");
    for (int i : {0, 2, 3, 9}) TORCH_CHECK(bnr[i].has_value() && bnr[i]->defined(), "bnr missing required entry ", i);
    TORCH_CHECK(!(bnr[6].has_value() && bnr[6]->defined()), "maxpool_bwd BN reduce: no second BN");
    TORCH_CHECK(g[3] % 8 == 0 && g[3] >= 8 && 256 % (g[3] / 8) == 0, "maxpool_bwd BN reduce needs C % 8 == 0 and (C/8) | 256");
    need_bf16(*bnr[0], "bn_y"); need_numel(*bnr[0], nx, "bn_y");
    const void* bn_a = nullptr;
    amask = relu_bitmask(bnr[1], nx, &bn_a);
    TORCH_CHECK(!bn_a, "maxpool_bwd BN reduce: pass the packed relu bitmask");
    for (int i : {2, 3, 4, 5})
      if (bnr[i].has_value() && bnr[i]->defined()) { need_f32(*bnr[i], "bn vec"); need_numel(*bnr[i], g[3], "bn vec"); }
    need_f32(*bnr[9], "bn_sums");
    TORCH_CHECK(bn_shards >= 1, "bn_shards");
    need_numel(*bnr[9], (long long)bn_shards * 3 * g[3], "bn_sums");
    y = bnr[0]->data_ptr();
    mean = bnr[2]->data_ptr<float>();
    invstd = bnr[3]->data_ptr<float>();
    msc = opt_ptr<const float>(bnr[4]);
    msh = opt_ptr<const float>(bnr[5]);
    TORCH_CHECK((msc == nullptr) == (msh == nullptr), "scale and shift go together");
    sums = bnr[9]->data_ptr<float>();
  }
  check_rc(tfk_maxpool_bwd(dy.data_ptr(), idx.data_ptr<uint8_t>(), dx.data_ptr(), g[0], g[1], g[2], g[3], g[4], g[5], g[6],
                           g[7], g[8], g[9], g[10], g[11], y, mean, invstd, msc, msh, amask, sums, bn_shards,
                           cur_stream()),
           "maxpool_bwd");
}
void avgpool_fwd(torch::Tensor x, torch::Tensor y, int N, int HW, int C) {
  need_bf16(x, "x"); need_bf16(y, "y"); TORCH_CHECK(C % 8 == 0, "C%8");
  need_numel(x, (long long)N * HW * C, "x"); need_numel(y, (long long)N * C, "y");
  check_rc(tfk_avgpool_fwd(x.data_ptr(), y.data_ptr(), N, HW, C, cur_stream()), "avgpool_fwd");
}
void avgpool_bwd(torch::Tensor dy, torch::Tensor dx, int N, int HW, int C) {
  need_bf16(dy, "dy"); need_bf16(dx, "dx"); TORCH_CHECK(C % 8 == 0, "C%8");
  need_numel(dx, (long long)N * HW * C, "dx"); need_numel(dy, (long long)N * C, "dy");
  check_rc(tfk_avgpool_bwd(dy.data_ptr(), dx.data_ptr(), N, HW, C, cur_stream()), "avgpool_bwd");
}

void softmax_xent(torch::Tensor logits, torch::Tensor labels, int B, int V, int64_t ld, double smoothing, int ignore_index,
                  double scale, torch::Tensor loss, c10::optional<torch::Tensor> dlogits,
                  c10::optional<torch::Tensor> correct) {
  need_bf16(logits, "logits"); need(labels, at::kInt, "labels"); need_f32(loss, "loss");
  need_numel(logits, (long long)(B - 1) * ld + V, "logits"); need_numel(labels, B, "labels"); need_numel(loss, B, "loss");
  if (dlogits.has_value() && dlogits->defined()) { need_bf16(*dlogits, "dlogits"); need_numel(*dlogits, (long long)(B - 1) * ld + V, "dlogits"); }
  if (correct.has_value() && correct->defined()) need_numel(*correct, B, "correct");
  check_rc(tfk_softmax_xent(logits.data_ptr(), labels.data_ptr<int>(), B, V, ld, (float)smoothing, ignore_index,
                            (float)scale, loss.data_ptr<float>(), opt_ptr<void>(dlogits), opt_ptr<float>(correct),
                            cur_stream()),
           "softmax_xent");
}

// hp (optional): device f32[3] {lr, bc1, bc2} from opt_hyper -- overrides the host lr / bias corrections
static const float* hp_ptr(const c10::optional<torch::Tensor>& hp) {
  if (!hp.has_value() || !hp->defined()) return nullptr;
  need_f32(*hp, "hp");
  need_numel(*hp, 3, "hp");
  return hp->data_ptr<float>();
}
void sgd(torch::Tensor w, c10::optional<torch::Tensor> wb, torch::Tensor g, torch::Tensor m, double lr, double mu,
         double wd, bool nesterov, double gs, c10::optional<torch::Tensor> gs_dev, c10::optional<torch::Tensor> hp) {
  need_f32(w, "w"); need_f32(g, "g"); need_f32(m, "m");
  long long n = w.numel();
  need_numel(g, n, "g"); need_numel(m, n, "m");
  need_aligned(w, 16, "w"); need_aligned(g, 16, "g"); need_aligned(m, 16, "m");
  if (wb.has_value() && wb->defined()) { need_bf16(*wb, "wb"); need_numel(*wb, n, "wb"); need_aligned(*wb, 8, "wb"); }
  check_rc(tfk_sgd(w.data_ptr<float>(), opt_ptr<void>(wb), g.data_ptr<float>(), m.data_ptr<float>(), n, (float)lr,
                   (float)mu, (float)wd, nesterov ? 1 : 0, (float)gs, opt_ptr<const float>(gs_dev), hp_ptr(hp),
                   cur_stream()),
           "sgd");
}
void adamw(torch::Tensor w, c10::optional<torch::Tensor> wb, torch::Tensor g, torch::Tensor m, torch::Tensor v, double lr,
           double b1, double b2, double eps, double wd, double bc1, double bc2, double gs,
           c10::optional<torch::Tensor> gs_dev, c10::optional<torch::Tensor> hp) {
  need_f32(w, "w"); need_f32(g, "g"); need_f32(m, "m"); need_f32(v, "v");
  long long n = w.numel();
  need_numel(g, n, "g"); need_numel(m, n, "m"); need_numel(v, n, "v");
  if (wb.has_value() && wb->defined()) { need_bf16(*wb, "wb"); need_numel(*wb, n, "wb"); }
  check_rc(tfk_adamw(w.data_ptr<float>(), opt_ptr<void>(wb), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                     n, (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (float)bc1, (float)bc2, (float)gs,
                     opt_ptr<const float>(gs_dev), hp_ptr(hp), cur_stream()),
           "adamw");
}
void lamb(torch::Tensor w, c10::optional<torch::Tensor> wb, torch::Tensor g, torch::Tensor m, torch::Tensor v,
          torch::Tensor u, torch::Tensor cstart, torch::Tensor clen, torch::Tensor cseg, torch::Tensor seg_norms, double lr,
          double b1, double b2, double eps, double wd, double bc1, double bc2, double gs,
          c10::optional<torch::Tensor> gs_dev, c10::optional<torch::Tensor> hp) {
  need_f32(w, "w"); need_f32(g, "g"); need_f32(m, "m"); need_f32(v, "v"); need_f32(u, "u");
  need(cstart, at::kLong, "cstart"); need(clen, at::kInt, "clen"); need(cseg, at::kInt, "cseg");
  need_f32(seg_norms, "seg_norms");
  long long n = w.numel();
  for (auto* t : {&g, &m, &v, &u}) need_numel(*t, n, "lamb buf");
  int nch = (int)cstart.numel();
  TORCH_CHECK(clen.numel() == nch && cseg.numel() == nch, "chunk table");
  check_rc(tfk_lamb(w.data_ptr<float>(), opt_ptr<void>(wb), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                    u.data_ptr<float>(), cstart.data_ptr<int64_t>() ? (const long long*)cstart.data_ptr<int64_t>() : nullptr,
                    clen.data_ptr<int>(), cseg.data_ptr<int>(), nch, seg_norms.data_ptr<float>(), (float)lr, (float)b1,
                    (float)b2, (float)eps, (float)wd, (float)bc1, (float)bc2, (float)gs, opt_ptr<const float>(gs_dev),
                    hp_ptr(hp), cur_stream()),
           "lamb");
}
// Advance the device optimizer step and write hp = {lr_table[step-1+off], 1-b1^step, 1-b2^step}.
void opt_hyper(torch::Tensor step, torch::Tensor lr_table, int64_t lr_offset, double b1, double b2, torch::Tensor hp) {
  need(step, at::kInt, "step"); need_numel(step, 1, "step");
  need_f32(lr_table, "lr_table"); TORCH_CHECK(lr_table.numel() >= 1, "lr_table");
  need_f32(hp, "hp"); need_numel(hp, 3, "hp");
  check_rc(tfk_opt_hyper(step.data_ptr<int>(), lr_table.data_ptr<float>(), (int)lr_table.numel(), (int)lr_offset,
                         (float)b1, (float)b2, hp.data_ptr<float>(), cur_stream()),
           "opt_hyper");
}
void sumsq(torch::Tensor x, torch::Tensor out) {
  need_f32(x, "x"); need_f32(out, "out");
  check_rc(tfk_sumsq(x.data_ptr<float>(), x.numel(), out.data_ptr<float>(), cur_stream()), "sumsq");
}
void clip_coef(torch::Tensor ss, double max_norm, torch::Tensor coef, c10::optional<torch::Tensor> norm) {
  need_f32(ss, "ss"); need_f32(coef, "coef");
  check_rc(tfk_clip_coef(ss.data_ptr<float>(), (float)max_norm, coef.data_ptr<float>(), opt_ptr<float>(norm), cur_stream()),
           "clip_coef");
}

void splitk_reduce(torch::Tensor slabs, int S, int64_t stride, int64_t n, c10::optional<torch::Tensor> out,
                   c10::optional<torch::Tensor> outb, bool accumulate, double alpha) {
  need_f32(slabs, "slabs");
  need_numel(slabs, (long long)(S - 1) * stride + n, "slabs");
  TORCH_CHECK(stride % 4 == 0, "stride%4");
  need_aligned(slabs, 16, "slabs");
  if (out.has_value() && out->defined()) { need_f32(*out, "out"); need_numel(*out, n, "out"); need_aligned(*out, 16, "out"); }
  else { TORCH_CHECK(outb.has_value() && outb->defined(), "need out"); need_bf16(*outb, "outb"); need_numel(*outb, n, "outb"); need_aligned(*outb, 8, "outb"); }
  check_rc(tfk_splitk_reduce(slabs.data_ptr<float>(), S, stride, n, opt_ptr<float>(out), opt_ptr<void>(outb),
                             accumulate ? 1 : 0, (float)alpha, cur_stream()),
           "splitk_reduce");
}
// Halo-tile 3x3 weight gradient (conv_hwgrad.hip): per-block f32 slabs of dW [K][3][3][C] into ws
int64_t hwgrad_slabs(int N, int H, int W, int P, int Q, int C, int K, int st) {
  return tfk_hwgrad_slabs(H, W, P, Q, C, K, st, N);
}
void hwgrad(torch::Tensor x, torch::Tensor dy, torch::Tensor ws, int N, int H, int W, int P, int Q, int C, int K, int st,
            int slabs) {
  need_bf16(x, "x"); need_bf16(dy, "dy"); need_f32(ws, "ws");
  TORCH_CHECK(x.dim() == 4 && x.size(0) == N && x.size(1) == H && x.size(2) == W && x.size(3) == C, "hwgrad: x shape");
  TORCH_CHECK(dy.dim() == 4 && dy.size(0) == N && dy.size(1) == P && dy.size(2) == Q && dy.size(3) == K, "hwgrad: dy shape");
  need_aligned(x, 16, "x"); need_aligned(dy, 16, "dy"); need_aligned(ws, 16, "ws");
  TORCH_CHECK(slabs > 0 && slabs == tfk_hwgrad_slabs(H, W, P, Q, C, K, st, N), "hwgrad: shape not served / slab count");
  need_numel(ws, (long long)slabs * K * 9 * C, "ws");
  check_rc(tfk_hwgrad_launch(x.data_ptr(), dy.data_ptr(), ws.data_ptr<float>(), N, H, W, P, Q, C, K, st, slabs,
                             cur_stream()), "hwgrad");
}
// Stem 7x7/s2/p3 weight gradient (conv_hwgrad.hip): x [N][H][W][8] (channels >= 4 zero), dy [N][H/2][W/2][64]
int64_t stem_wgrad_slabs(int N, int H, int W) { return tfk_stem_wgrad_slabs(N, H, W); }
void stem_wgrad(torch::Tensor x, torch::Tensor dy, torch::Tensor ws, int N, int H, int W, int slabs) {
  need_bf16(x, "x"); need_bf16(dy, "dy"); need_f32(ws, "ws");
  TORCH_CHECK(x.dim() == 4 && x.size(0) == N && x.size(1) == H && x.size(2) == W && x.size(3) == 8, "stem_wgrad: x shape");
  TORCH_CHECK(dy.dim() == 4 && dy.size(0) == N && dy.size(1) == H / 2 && dy.size(2) == W / 2 && dy.size(3) == 64,
              "stem_wgrad: dy shape");
  need_aligned(x, 16, "x"); need_aligned(dy, 16, "dy"); need_aligned(ws, 16, "ws");
  TORCH_CHECK(slabs > 0 && slabs == tfk_stem_wgrad_slabs(N, H, W), "stem_wgrad: shape not served / slab count");
  need_numel(ws, (long long)slabs * 64 * 49 * 8, "ws");
  check_rc(tfk_stem_wgrad_launch(x.data_ptr(), dy.data_ptr(), ws.data_ptr<float>(), N, H, W, slabs, cur_stream()),
           "stem_wgrad");
}
// Stem 7x7/s2/p3 forward + BN statistics (conv_stem.hip): x [N][H][W][8] (channels >= 4 zero),
// w [64][7][7][8], y [N][H/2][W/2][64], stats [shards][2][64] (accumulated)
bool stem_fwd_ok(int N, int H, int W) { return tfk_stem_fwd_ok(N, H, W) != 0; }
void stem_fwd(torch::Tensor x, torch::Tensor w, torch::Tensor y, c10::optional<torch::Tensor> stats, int shards) {
  need_bf16(x, "x"); need_bf16(w, "w"); need_bf16(y, "y");
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 8, "stem_fwd: x must be [N][H][W][8]");
  const int N = x.size(0), H = x.size(1), W = x.size(2);
  TORCH_CHECK(tfk_stem_fwd_ok(N, H, W), "stem_fwd: shape not served");
  TORCH_CHECK(w.numel() == 64 * 49 * 8, "stem_fwd: w must be [64][7][7][8]");
  TORCH_CHECK(y.dim() == 4 && y.size(0) == N && y.size(1) == H / 2 && y.size(2) == W / 2 && y.size(3) == 64,
              "stem_fwd: y shape");
  need_aligned(x, 16, "x"); need_aligned(w, 16, "w"); need_aligned(y, 16, "y");
  float* st = nullptr;
  if (stats.has_value() && stats->defined()) {
    need_f32(*stats, "stats");
    need_numel(*stats, (long long)(shards < 1 ? 1 : shards) * 2 * 64, "stats");
    st = stats->data_ptr<float>();
  }
  check_rc(tfk_stem_fwd_launch(x.data_ptr(), w.data_ptr(), y.data_ptr(), st, shards, N, H, W, cur_stream()), "stem_fwd");
}
void transpose_arb(torch::Tensor in, torch::Tensor out, int A, int R, int B, int flip) {
  need_bf16(in, "in"); need_bf16(out, "out");
  need_numel(in, (long long)A * R * B, "in"); need_numel(out, (long long)A * R * B, "out");
  check_rc(tfk_transpose_arb(in.data_ptr(), out.data_ptr(), A, R, B, flip, cur_stream()), "transpose_arb");
}
void transpose_f32(torch::Tensor in, torch::Tensor out, int rows, int cols) {
  need_f32(in, "in"); need_f32(out, "out");
  need_numel(in, (long long)rows * cols, "in"); need_numel(out, (long long)rows * cols, "out");
  check_rc(tfk_transpose_f32(in.data_ptr<float>(), out.data_ptr<float>(), rows, cols, cur_stream()), "transpose_f32");
}
void cast_f32_bf16(torch::Tensor x, torch::Tensor y) {
  need_f32(x, "x"); need_bf16(y, "y"); need_numel(y, x.numel(), "y");
  check_rc(tfk_cast_f32_bf16(x.data_ptr<float>(), y.data_ptr(), x.numel(), cur_stream()), "cast_f32_bf16");
}
void cast_bf16_f32(torch::Tensor x, torch::Tensor y) {
  need_bf16(x, "x"); need_f32(y, "y"); need_numel(y, x.numel(), "y");
  check_rc(tfk_cast_bf16_f32(x.data_ptr(), y.data_ptr<float>(), x.numel(), cur_stream()), "cast_bf16_f32");
}
void synth_uniform(torch::Tensor y, int64_t rows, int Creal, int Cpad, double lo, double hi, int64_t seed) {
  need_bf16(y, "y"); need_numel(y, rows * Cpad, "y");
  check_rc(tfk_synth_uniform(y.data_ptr(), rows, Creal, Cpad, (float)lo, (float)hi, (unsigned long long)seed, cur_stream()),
           "synth_uniform");
}
void synth_normal_f32(torch::Tensor y, double mean, double std, int64_t seed) {
  need_f32(y, "y");
  check_rc(tfk_synth_normal_f32(y.data_ptr<float>(), y.numel(), (float)mean, (float)std, (unsigned long long)seed,
                                cur_stream()),
           "synth_normal");
}
void synth_labels(torch::Tensor y, int classes, int64_t seed) {
  need(y, at::kInt, "labels");
  check_rc(tfk_synth_labels(y.data_ptr<int>(), y.numel(), classes, (unsigned long long)seed, cur_stream()), "synth_labels");
}
void colsum(torch::Tensor x, int64_t M, int N, int64_t ld, torch::Tensor out) {
  need_bf16(x, "x"); need_f32(out, "out");
  need_numel(x, (M - 1) * ld + N, "x"); need_numel(out, N, "out");
  check_rc(tfk_colsum(x.data_ptr(), M, N, ld, out.data_ptr<float>(), cur_stream()), "colsum");
}
void act_fwd(torch::Tensor x, c10::optional<torch::Tensor> bias, int N, torch::Tensor y, int act) {
  need_bf16(x, "x"); need_bf16(y, "y"); need_numel(y, x.numel(), "y");
  if (bias.has_value() && bias->defined()) { need_f32(*bias, "bias"); need_numel(*bias, N, "bias"); TORCH_CHECK(x.numel() % N == 0, "bias N"); }
  check_rc(tfk_act_fwd(x.data_ptr(), opt_ptr<const float>(bias), N, y.data_ptr(), x.numel(), act, cur_stream()), "act_fwd");
}
void act_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor dx, int act) {
  need_bf16(dy, "dy"); need_bf16(x, "x"); need_bf16(dx, "dx");
  need_numel(x, dy.numel(), "x"); need_numel(dx, dy.numel(), "dx");
  check_rc(tfk_act_bwd(dy.data_ptr(), x.data_ptr(), dx.data_ptr(), dy.numel(), act, cur_stream()), "act_bwd");
}
// rng state of a model: int64 [counter, key]. set_rng_key registers &state[1] as the per-step key
// every dropout-capable launch adds to its salt (None: unregister); rng_advance steps it on device.
void set_rng_key(c10::optional<torch::Tensor> st) {
  if (!st.has_value() || !st->defined()) {
    tfk_set_seed_key(nullptr);
    return;
  }
  need(*st, at::kLong, "rng state");
  need_numel(*st, 2, "rng state");
  tfk_set_seed_key(reinterpret_cast<const unsigned long long*>(st->data_ptr<int64_t>()) + 1);
}
void rng_advance(torch::Tensor st, int64_t stream) {
  need(st, at::kLong, "rng state");
  need_numel(st, 2, "rng state");
  check_rc(tfk_rng_advance(reinterpret_cast<unsigned long long*>(st.data_ptr<int64_t>()), (unsigned long long)stream,
                           cur_stream()),
           "rng_advance");
}

void dropout(torch::Tensor x, torch::Tensor y, double p, int64_t seed) {
  need_bf16(x, "x"); need_bf16(y, "y"); need_numel(y, x.numel(), "y");
  check_rc(tfk_dropout(x.data_ptr(), y.data_ptr(), x.numel(), (float)p, (unsigned long long)seed, cur_stream()), "dropout");
}
// Head rows of a [B*S][W] activation: row r -> (r / P) * S + pos[r] (pos int32 [B*P]) or the
// first row of each sequence (pos = None, P = 1).
void gather_rows(torch::Tensor src, c10::optional<torch::Tensor> pos, int64_t P, int64_t S, torch::Tensor dst) {
  need_bf16(src, "src"); need_bf16(dst, "dst");
  TORCH_CHECK(src.dim() == 2 && dst.dim() == 2 && src.size(1) == dst.size(1), "gather_rows: [rows][W] operands");
  const long long n = dst.size(0);
  TORCH_CHECK(n % P == 0 && (n / P) * S <= src.size(0), "gather_rows: ", n, " rows of ", P, " per sequence exceed src");
  const int* pp = nullptr;
  if (pos.has_value() && pos->defined()) { need(*pos, at::kInt, "pos"); need_numel(*pos, n, "pos"); pp = pos->data_ptr<int>(); }
  else TORCH_CHECK(P == 1, "gather_rows: without pos, one row (the first) per sequence");
  check_rc(tfk_gather_rows(src.data_ptr(), pp, (int)P, (int)S, (int)src.size(1), n, dst.data_ptr(), cur_stream()), "gather_rows");
}
void scatter_add_rows(torch::Tensor dst, torch::Tensor src, c10::optional<torch::Tensor> pos, int64_t P, int64_t S) {
  need_bf16(src, "src"); need_bf16(dst, "dst");
  TORCH_CHECK(src.dim() == 2 && dst.dim() == 2 && src.size(1) == dst.size(1), "scatter_add_rows: [rows][W] operands");
  const long long n = src.size(0);
  TORCH_CHECK(n % P == 0 && (n / P) * S <= dst.size(0), "scatter_add_rows: rows exceed dst");
  const int* pp = nullptr;
  if (pos.has_value() && pos->defined()) { need(*pos, at::kInt, "pos"); need_numel(*pos, n, "pos"); pp = pos->data_ptr<int>(); }
  else TORCH_CHECK(P == 1, "scatter_add_rows: without pos, one row (the first) per sequence");
  check_rc(tfk_scatter_add_rows(dst.data_ptr(), src.data_ptr(), pp, (int)P, (int)S, (int)src.size(1), (int)(n / P),
                                cur_stream()), "scatter_add_rows");
}

void add(torch::Tensor a, torch::Tensor b, torch::Tensor y, double alpha, double beta) {
  need_bf16(a, "a"); need_bf16(b, "b"); need_bf16(y, "y");
  need_numel(b, a.numel(), "b"); need_numel(y, a.numel(), "y");
  check_rc(tfk_add(a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), (float)alpha, (float)beta, cur_stream()), "add");
}
}  // namespace

void register_transformer_ops(pybind11::module& m);
void register_ckpt_ops(pybind11::module& m);
void register_comm_ops(pybind11::module& m);

PYBIND11_MODULE(_C, m) {
  m.doc() = "tfk gfx950 HIP kernel library";
  m.def("gemm", &gemm);
  m.def("gemm_splits", &gemm_splits);
  m.def("gemm_set_persist", &gemm_set_persist);
  m.def("gemm_set_engine", &gemm_set_engine);
  m.def("gemm_set_shortk", &gemm_set_shortk);
  m.def("fp8_set_engine", &fp8_set_engine);
  m.def("mx_quant", &mx_quant);
  m.def("mx_quant_t", &mx_quant_t);
  m.def("mx_quant_dual", &mx_quant_dual);
  m.def("mx_quant_dual_group", &mx_quant_dual_group);
  m.def("mx_probe", &mx_probe);
  m.def("gemm_mxfp8", &gemm_mxfp8, py::arg("A"), py::arg("As"), py::arg("B"), py::arg("Bs"), py::arg("C"), py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("bias"), py::arg("resid"), py::arg("act"), py::arg("aux"), py::arg("drop_p"),
        py::arg("drop_seed"), py::arg("dact_src") = py::none(), py::arg("dact") = 0, py::arg("beta") = 0.0,
        py::arg("splits") = 1, py::arg("split_stride") = 0, py::arg("mx_out") = py::none(), py::arg("mx_skip_c") = false,
        py::arg("colsum") = py::none());
  m.def("bn_finalize", &bn_finalize);
  m.def("bn_stats", &bn_stats);
  m.def("bn_apply", &bn_apply);
  m.def("bn_bwd_reduce", &bn_bwd_reduce);
  m.def("bn_bwd_finalize", &bn_bwd_finalize);
  m.def("bn_bwd_apply", &bn_bwd_apply);
  m.def("bn_fin_ok", &bn_fin_ok);
  m.def("bn_apply_fin", &bn_apply_fin);
  m.def("bn_bwd_apply_fin", &bn_bwd_apply_fin);
  m.def("bn_zero", &bn_zero);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("softmax_xent", &softmax_xent);
  m.def("xent_full_row", [](int V, int64_t ld) { return tfk_xent_full_row(V, ld) != 0; });
  m.def("sgd", &sgd);
  m.def("adamw", &adamw);
  m.def("lamb", &lamb);
  m.def("opt_hyper", &opt_hyper);
  m.def("sumsq", &sumsq);
  m.def("clip_coef", &clip_coef);
  m.def("splitk_reduce", &splitk_reduce);
  m.def("splitk_set_direct", &tfk_splitk_set_direct);  // A/B: 0 two-pass only, 1/2 direct for S <= 8
  m.def("hwgrad_slabs", &hwgrad_slabs);
  m.def("hwgrad", &hwgrad);
  m.def("stem_wgrad_slabs", &stem_wgrad_slabs);
  m.def("stem_wgrad", &stem_wgrad);
  m.def("stem_fwd_ok", &stem_fwd_ok);
  m.def("stem_fwd", &stem_fwd);
  m.def("transpose_arb", &transpose_arb, py::arg("in"), py::arg("out"), py::arg("A"), py::arg("R"), py::arg("B"),
        py::arg("flip") = 0);
  m.def("transpose_f32", &transpose_f32);
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("cast_bf16_f32", &cast_bf16_f32);
  m.def("synth_uniform", &synth_uniform);
  m.def("synth_normal_f32", &synth_normal_f32);
  m.def("synth_labels", &synth_labels);
  m.def("colsum", &colsum);
  m.def("act_fwd", &act_fwd);
  m.def("act_bwd", &act_bwd);
  m.def("dropout", &dropout);
  m.def("set_rng_key", &set_rng_key);
  m.def("halo_set", &tfk_halo_set);
  m.def("bn_fin_skip", &tfk_bn_fin_skip);
  m.def("g5_set", &tfk_g5_set);  // 256x256 GEMMs on the mid-tile-barrier engine: 4 / 8 waves, 0 off
  m.def("g8_set", &tfk_g8_set);  // 256x256 dense GEMMs on the 8-phase engine: 1 on, 0 off
  m.def("fp8_set_tile", &tfk_fp8_set_tile);  // fp8 g4 tile: 0 by shape, 128 / 256 forced, -1 -> TFK_FP8_TILE
  m.def("rng_advance", &rng_advance);
  m.def("add", &add);
  m.def("gather_rows", &gather_rows);
  m.def("scatter_add_rows", &scatter_add_rows);
  register_transformer_ops(m);
  register_ckpt_ops(m);
  register_comm_ops(m);
}
