// Bindings for the transformer kernel family: LayerNorm, embedding, fused attention
// (csrc/kernels/transformer.hip, attention.hip). Same contract as ops.cpp: validate device,
// dtype, layout and every extent a kernel will touch before launching on the current stream.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <vector>

#include "bind_util.h"

extern "C" {
void tfk_attn_set_waves(int w);
int tfk_layernorm_fwd(const void*, const float*, const float*, void*, float*, float*, int, int, float, hipStream_t);
int tfk_layernorm_fwd_mx(const void*, const float*, const float*, void*, float*, float*, int, int, float, void*, void*, void*,
                         void*, hipStream_t);
int tfk_layernorm_bwd(const void*, const void*, const float*, const float*, const float*, const void*, void*, float*,
                      float*, int, int, void*, float, unsigned long long, float*, void*, void*, void*, void*, float*,
                      hipStream_t);
int tfk_ln_bwd_blocks(int M, int mxo);
void tfk_ln_bwd_set_rows(int r);
void tfk_ln_bwd_set_fast(int on);
void tfk_ln_fwd_set_fast(int on);
int tfk_embedding_fwd(const int*, const void*, int, const void*, int, const int*, const void*, int, void*, long long, int,
                      float, hipStream_t);
int tfk_embedding_bwd(const int*, const void*, int, float*, float*, int, const int*, float*, int, long long, int, float,
                      int*, hipStream_t);
int tfk_emb_guard_count();
int tfk_attn_fwd(const void*, const void*, const void*, void*, float*, const long long*, const long long*, const int*,
                 float, int, float, unsigned long long, hipStream_t);
int tfk_attn_bwd(const void*, const void*, const void*, const void*, const void*, const float*, float*, void*, void*,
                 void*, const long long*, const long long*, const long long*, const int*, float, int, float,
                 unsigned long long, hipStream_t);
}

namespace {
void layernorm_fwd(torch::Tensor x, torch::Tensor gamma, torch::Tensor beta, torch::Tensor y, torch::Tensor mean,
                   torch::Tensor rstd, int64_t M, int W, double eps) {
  need_bf16(x, "x"); need_bf16(y, "y"); need_f32(gamma, "gamma"); need_f32(beta, "beta");
  need_f32(mean, "mean"); need_f32(rstd, "rstd");
  TORCH_CHECK(W % 8 == 0 && W <= 2048, "layernorm needs W%8==0 and W<=2048, got ", W);
  need_numel(x, M * W, "x"); need_numel(y, M * W, "y"); need_numel(gamma, W, "gamma"); need_numel(beta, W, "beta");
  need_numel(mean, M, "mean"); need_numel(rstd, M, "rstd");
  check_rc(tfk_layernorm_fwd(x.data_ptr(), gamma.data_ptr<float>(), beta.data_ptr<float>(), y.data_ptr(),
                             mean.data_ptr<float>(), rstd.data_ptr<float>(), (int)M, W, (float)eps, cur_stream()),
           "layernorm_fwd");
}

// LayerNorm forward + both MX-fp8 quantizations of y (qr [M][W], sr [M][W/32], qc [W][M], sc [W][M/32]);
// y optional (no bf16 store). M % 32 == 0, W % 32 == 0, W <= 1024.
void layernorm_fwd_mx(torch::Tensor x, torch::Tensor gamma, torch::Tensor beta, c10::optional<torch::Tensor> y,
                      torch::Tensor mean, torch::Tensor rstd, int64_t M, int W, double eps, torch::Tensor qr,
                      torch::Tensor sr, torch::Tensor qc, torch::Tensor sc) {
  need_bf16(x, "x"); need_f32(gamma, "gamma"); need_f32(beta, "beta"); need_f32(mean, "mean"); need_f32(rstd, "rstd");
  TORCH_CHECK(M % 32 == 0 && W % 32 == 0 && W <= 1024, "layernorm_fwd_mx needs M, W % 32 == 0 and W <= 1024");
  need_numel(x, M * W, "x"); need_numel(gamma, W, "gamma"); need_numel(beta, W, "beta");
  need_numel(mean, M, "mean"); need_numel(rstd, M, "rstd");
  if (y.has_value() && y->defined()) { need_bf16(*y, "y"); need_numel(*y, M * W, "y"); }
  for (auto* t : {&qr, &sr, &qc, &sc}) need(*t, at::kByte, "mx out");
  need_numel(qr, M * W, "qr"); need_numel(qc, M * W, "qc"); need_numel(sr, M * W / 32, "sr"); need_numel(sc, M * W / 32, "sc");
  need_aligned(qr, 16, "qr"); need_aligned(qc, 16, "qc");
  check_rc(tfk_layernorm_fwd_mx(x.data_ptr(), gamma.data_ptr<float>(), beta.data_ptr<float>(),
                                (y.has_value() && y->defined()) ? y->data_ptr() : nullptr, mean.data_ptr<float>(),
                                rstd.data_ptr<float>(), (int)M, W, (float)eps, qr.data_ptr(), sr.data_ptr(), qc.data_ptr(),
                                sc.data_ptr(), cur_stream()),
           "layernorm_fwd_mx");
}

void layernorm_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor gamma, torch::Tensor mean, torch::Tensor rstd,
                   c10::optional<torch::Tensor> dres, torch::Tensor dx, torch::Tensor dgamma, torch::Tensor dbeta,
                   int64_t M, int W, c10::optional<torch::Tensor> dxd, double drop_p, int64_t drop_seed,
                   c10::optional<torch::Tensor> dbias, c10::optional<std::vector<torch::Tensor>> mx_out) {
  if (dbias.has_value() && dbias->defined()) { need_f32(*dbias, "dbias"); need_numel(*dbias, W, "dbias"); }
  void* mxp[4] = {nullptr, nullptr, nullptr, nullptr};
  if (mx_out.has_value()) {
    const auto& o = *mx_out;
    TORCH_CHECK(o.size() == 4 && M % 32 == 0 && W % 32 == 0 && W <= 1024, "layernorm_bwd mx_out: 4 tensors, M, W % 32 == 0, W <= 1024");
    for (const auto& t : o) need(t, at::kByte, "mx_out");
    need_numel(o[0], M * W, "mx qr"); need_numel(o[1], M * W / 32, "mx sr");
    need_numel(o[2], M * W, "mx qc"); need_numel(o[3], M * W / 32, "mx sc");
    need_aligned(o[0], 16, "mx qr"); need_aligned(o[2], 16, "mx qc");
    for (int i = 0; i < 4; ++i) mxp[i] = o[i].data_ptr();
  }
  need_bf16(dy, "dy"); need_bf16(x, "x"); need_bf16(dx, "dx");
  for (auto* t : {&gamma, &mean, &rstd, &dgamma, &dbeta}) need_f32(*t, "ln vector");
  TORCH_CHECK(W % 8 == 0 && W <= 2048, "layernorm needs W%8==0 and W<=2048");
  for (auto* t : {&dy, &x, &dx}) need_numel(*t, M * W, "ln tensor");
  need_numel(gamma, W, "gamma"); need_numel(dgamma, W, "dgamma"); need_numel(dbeta, W, "dbeta");
  need_numel(mean, M, "mean"); need_numel(rstd, M, "rstd");
  if (dres.has_value() && dres->defined()) { need_bf16(*dres, "dres"); need_numel(*dres, M * W, "dres"); }
  if (dxd.has_value() && dxd->defined()) {
    need_bf16(*dxd, "dxd"); need_numel(*dxd, M * W, "dxd");
    TORCH_CHECK(drop_p > 0.0 && drop_p < 1.0, "dxd needs 0 < drop_p < 1");
  }
  // per-block column partials (caching allocator: graph-capture safe), reduced by a second launch
  const int NS = (dbias.has_value() && dbias->defined()) ? 3 : 2;
  torch::Tensor part = torch::empty({(long long)tfk_ln_bwd_blocks((int)M, mxp[0] != nullptr) * NS * W},
                                    dgamma.options());
  check_rc(tfk_layernorm_bwd(dy.data_ptr(), x.data_ptr(), gamma.data_ptr<float>(), mean.data_ptr<float>(),
                             rstd.data_ptr<float>(), opt_ptr<const void>(dres), dx.data_ptr(), dgamma.data_ptr<float>(),
                             dbeta.data_ptr<float>(), (int)M, W, opt_ptr<void>(dxd), (float)drop_p,
                             (unsigned long long)drop_seed, opt_ptr<float>(dbias), mxp[0], mxp[1], mxp[2], mxp[3],
                             part.data_ptr<float>(), cur_stream()),
           "layernorm_bwd");
}

void embedding_fwd(torch::Tensor ids, torch::Tensor word, c10::optional<torch::Tensor> pos, int64_t S,
                   c10::optional<torch::Tensor> tt, c10::optional<torch::Tensor> type, torch::Tensor out, double scale) {
  need(ids, at::kInt, "ids"); need_bf16(word, "word"); need_bf16(out, "out");
  TORCH_CHECK(word.dim() == 2, "word table must be [V, W]");
  const int V = (int)word.size(0), W = (int)word.size(1);
  TORCH_CHECK(W % 8 == 0, "embedding width %8");
  const long long ntok = ids.numel();
  need_numel(out, ntok * W, "out");
  if (pos.has_value() && pos->defined()) {
    need_bf16(*pos, "pos"); TORCH_CHECK(S >= 1, "S"); need_numel(*pos, S * W, "pos");
    TORCH_CHECK(ntok % S == 0, "tokens must be a multiple of S");
  }
  int T = 0;
  if (type.has_value() && type->defined()) {
    need_bf16(*type, "type"); TORCH_CHECK(tt.has_value() && tt->defined(), "type table needs type ids");
    need(*tt, at::kInt, "type ids"); need_numel(*tt, ntok, "type ids");
    T = (int)type->size(0); need_numel(*type, (long long)T * W, "type");
  }
  check_rc(tfk_embedding_fwd(ids.data_ptr<int>(), word.data_ptr(), V, opt_ptr<const void>(pos), (int)S,
                             opt_ptr<const int>(tt), opt_ptr<const void>(type), T, out.data_ptr(), ntok, W,
                             (float)scale, cur_stream()),
           "embedding_fwd");
}

void embedding_bwd(torch::Tensor ids, torch::Tensor dy, torch::Tensor dword, c10::optional<torch::Tensor> dpos,
                   int64_t S, c10::optional<torch::Tensor> tt, c10::optional<torch::Tensor> dtype, int64_t W,
                   double scale) {
  need(ids, at::kInt, "ids"); need_bf16(dy, "dy"); need_f32(dword, "dword");
  TORCH_CHECK(W % 8 == 0, "embedding width %8");
  const long long ntok = ids.numel();
  need_numel(dy, ntok * W, "dy");
  const int V = (int)(dword.numel() / W);
  TORCH_CHECK(V >= 1, "dword");
  if (dpos.has_value() && dpos->defined()) {
    need_f32(*dpos, "dpos"); need_numel(*dpos, S * W, "dpos");
    TORCH_CHECK(S >= 1 && ntok % S == 0, "tokens must be a multiple of S");
  }
  int T = 0;
  if (dtype.has_value() && dtype->defined()) {
    need_f32(*dtype, "dtype"); TORCH_CHECK(tt.has_value() && tt->defined(), "type grads need type ids");
    need(*tt, at::kInt, "type ids"); need_numel(*tt, ntok, "type ids");
    T = (int)(dtype->numel() / W);
    TORCH_CHECK(T >= 1 && T <= 4, "at most 4 token types");
  }
  // row-bucketed word gradient (no f32 atomics): int32 scratch [3 V + ntok] from the caching allocator
  // (graph-capture safe); rows that are not 16-B aligned fall back to the scattered-atomic kernel
  torch::Tensor scratch = torch::empty({3 * (long long)V + ntok}, ids.options());
  check_rc(tfk_embedding_bwd(ids.data_ptr<int>(), dy.data_ptr(), V, dword.data_ptr<float>(), opt_ptr<float>(dpos),
                             (int)S, opt_ptr<const int>(tt), opt_ptr<float>(dtype), T, ntok, (int)W, (float)scale,
                             scratch.data_ptr<int>(), cur_stream()),
           "embedding_bwd");
}

// Attention views: each of q/k/v/o is a bf16 buffer holding [B, S, H, 64] at element offset 0 of
// `t` with token stride rs and batch stride bs (e.g. q/k/v are column slices of a fused QKV
// projection). `off` = element offset of the view inside the buffer.
void check_view(const torch::Tensor& t, long long off, long long bs, long long rs, long long B, long long S, int H,
                const char* n) {
  need_bf16(t, n);
  TORCH_CHECK(rs % 8 == 0 && bs % 8 == 0 && off % 8 == 0, n, ": strides/offset must be multiples of 8 elements");
  TORCH_CHECK(rs >= (long long)H * 64, n, ": token stride < H*64");
  need_numel(t, off + (B - 1) * bs + (S - 1) * rs + (long long)H * 64, n);
}

void attn_fwd(torch::Tensor q, int64_t qo, torch::Tensor k, int64_t ko, torch::Tensor v, int64_t vo, torch::Tensor out,
              torch::Tensor lse, std::vector<int64_t> shape, std::vector<int64_t> strides,
              c10::optional<torch::Tensor> kv_len, double scale, bool causal, double p_drop, int64_t seed) {
  TORCH_CHECK(shape.size() == 4 && strides.size() == 8, "attn shape [B,H,Sq,Sk], strides [q_bs,q_rs,k_bs,k_rs,v_bs,v_rs,o_bs,o_rs]");
  const long long B = shape[0], H = shape[1], Sq = shape[2], Sk = shape[3];
  TORCH_CHECK(B >= 1 && H >= 1 && Sq >= 1 && Sk >= 1 && H <= 65535 && B <= 65535, "bad attention shape");
  check_view(q, qo, strides[0], strides[1], B, Sq, (int)H, "q");
  check_view(k, ko, strides[2], strides[3], B, Sk, (int)H, "k");
  check_view(v, vo, strides[4], strides[5], B, Sk, (int)H, "v");
  check_view(out, 0, strides[6], strides[7], B, Sq, (int)H, "out");
  need_f32(lse, "lse"); need_numel(lse, B * H * Sq, "lse");
  if (kv_len.has_value() && kv_len->defined()) { need(*kv_len, at::kInt, "kv_len"); need_numel(*kv_len, B, "kv_len"); }
  TORCH_CHECK(p_drop >= 0.0 && p_drop < 1.0, "p_drop");
  std::vector<long long> sh(shape.begin(), shape.end()), st(strides.begin(), strides.end());
  const auto* qp = (const at::BFloat16*)q.data_ptr() + qo;
  const auto* kp = (const at::BFloat16*)k.data_ptr() + ko;
  const auto* vp = (const at::BFloat16*)v.data_ptr() + vo;
  check_rc(tfk_attn_fwd(qp, kp, vp, out.data_ptr(), lse.data_ptr<float>(), sh.data(), st.data(),
                        opt_ptr<const int>(kv_len), (float)scale, causal ? 1 : 0, (float)p_drop,
                        (unsigned long long)seed, cur_stream()),
           "attn_fwd");
}

void attn_bwd(torch::Tensor q, int64_t qo, torch::Tensor k, int64_t ko, torch::Tensor v, int64_t vo, torch::Tensor out,
              torch::Tensor dout, torch::Tensor lse, torch::Tensor delta, torch::Tensor dq, int64_t dqo, torch::Tensor dk,
              int64_t dko, torch::Tensor dv, int64_t dvo, std::vector<int64_t> shape, std::vector<int64_t> strides,
              std::vector<int64_t> gstrides, c10::optional<torch::Tensor> kv_len, double scale, bool causal,
              double p_drop, int64_t seed) {
  TORCH_CHECK(shape.size() == 4 && strides.size() == 8 && gstrides.size() == 6, "attn_bwd shape/strides");
  const long long B = shape[0], H = shape[1], Sq = shape[2], Sk = shape[3];
  TORCH_CHECK(B >= 1 && H >= 1 && Sq >= 1 && Sk >= 1, "bad attention shape");
  check_view(q, qo, strides[0], strides[1], B, Sq, (int)H, "q");
  check_view(k, ko, strides[2], strides[3], B, Sk, (int)H, "k");
  check_view(v, vo, strides[4], strides[5], B, Sk, (int)H, "v");
  check_view(out, 0, strides[6], strides[7], B, Sq, (int)H, "out");
  check_view(dout, 0, strides[6], strides[7], B, Sq, (int)H, "dout");
  check_view(dq, dqo, gstrides[0], gstrides[1], B, Sq, (int)H, "dq");
  check_view(dk, dko, gstrides[2], gstrides[3], B, Sk, (int)H, "dk");
  check_view(dv, dvo, gstrides[4], gstrides[5], B, Sk, (int)H, "dv");
  need_f32(lse, "lse"); need_numel(lse, B * H * Sq, "lse");
  need_f32(delta, "delta"); need_numel(delta, B * H * Sq, "delta");
  if (kv_len.has_value() && kv_len->defined()) { need(*kv_len, at::kInt, "kv_len"); need_numel(*kv_len, B, "kv_len"); }
  std::vector<long long> sh(shape.begin(), shape.end()), st(strides.begin(), strides.end()),
      gs(gstrides.begin(), gstrides.end());
  auto base = [](torch::Tensor& t, int64_t o) { return (void*)((at::BFloat16*)t.data_ptr() + o); };
  check_rc(tfk_attn_bwd(base(q, qo), base(k, ko), base(v, vo), out.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(),
                        delta.data_ptr<float>(), base(dq, dqo), base(dk, dko), base(dv, dvo), sh.data(), st.data(),
                        gs.data(), opt_ptr<const int>(kv_len), (float)scale, causal ? 1 : 0, (float)p_drop,
                        (unsigned long long)seed, cur_stream()),
           "attn_bwd");
}
}  // namespace

void register_transformer_ops(pybind11::module& m) {
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("ln_bwd_set_rows", &tfk_ln_bwd_set_rows);
  m.def("ln_bwd_set_fast", &tfk_ln_bwd_set_fast);
  m.def("ln_fwd_set_fast", &tfk_ln_fwd_set_fast);
  m.def("layernorm_fwd_mx", &layernorm_fwd_mx);
  m.def("layernorm_bwd", &layernorm_bwd, py::arg("dy"), py::arg("x"), py::arg("gamma"), py::arg("mean"),
        py::arg("rstd"), py::arg("dres"), py::arg("dx"), py::arg("dgamma"), py::arg("dbeta"), py::arg("M"), py::arg("W"),
        py::arg("dxd"), py::arg("drop_p"), py::arg("drop_seed"), py::arg("dbias") = py::none(),
        py::arg("mx_out") = py::none());
  m.def("embedding_fwd", &embedding_fwd);
  m.def("embedding_bwd", &embedding_bwd);
  // out-of-range events the bucketed embedding backward skipped since the last call (0 when healthy)
  m.def("emb_guard_count", [] { return tfk_emb_guard_count(); });
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd);
  m.def("attn_set_waves", [](int w) { tfk_attn_set_waves(w); });
}
