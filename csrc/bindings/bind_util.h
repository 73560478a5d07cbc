// Shared host-side validation helpers of the _C bindings: every op checks device, dtype,
// contiguity, alignment and extents before a kernel launch, so a bad call fails loudly in Python
// instead of faulting the GPU.
#pragma once
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace {
inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

inline void check_rc(int rc, const char* what) { TORCH_CHECK(rc == 0, "tfk kernel launch failed: ", what, " rc=", rc); }

inline void need(const torch::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
inline void need_bf16(const torch::Tensor& t, const char* n) { need(t, at::kBFloat16, n); }
inline void need_f32(const torch::Tensor& t, const char* n) { need(t, at::kFloat, n); }
inline void need_aligned(const torch::Tensor& t, int bytes, const char* n) {
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % bytes == 0, n, " must be ", bytes, "-byte aligned");
}
inline void need_numel(const torch::Tensor& t, long long n, const char* name) {
  TORCH_CHECK(t.numel() >= n, name, " too small: numel=", t.numel(), " < required ", n);
}
// uint8 aux / dact_src of a GEMM epilogue = relu bitmask [rows][ld/8] (gemm_params.h aux_bits,
// the same bit layout as relu_bitmask below): contiguous, every 8-column chunk starting on a byte
inline bool relu_mask(const torch::Tensor& t, long long ld, long long N, long long off, const char* what) {
  if (t.scalar_type() != at::kByte) return false;
  TORCH_CHECK(t.is_contiguous(), what, ": relu mask must be contiguous");
  TORCH_CHECK(ld % 8 == 0 && N % 8 == 0 && off % 8 == 0, what, ": relu mask needs 8-column aligned rows");
  return true;
}
template <typename T>
T* opt_ptr(const c10::optional<torch::Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

// A relu-mask operand of the BN-backward ops: either the post-activation bf16 tensor a (mask a > 0,
// *bf16_out = a) or its packed bitmask (uint8, bit e of byte i/8 = a[i+e] > 0; returned).
inline const uint8_t* relu_bitmask(const c10::optional<torch::Tensor>& a, long long n, const void** bf16_out) {
  *bf16_out = nullptr;
  if (!a.has_value() || !a->defined()) return nullptr;
  if (a->scalar_type() == at::kByte) {
    need(*a, at::kByte, "relu bitmask");
    TORCH_CHECK(n % 8 == 0, "relu bitmask needs a multiple of 8 elements");
    need_numel(*a, n / 8, "relu bitmask");
    return a->data_ptr<uint8_t>();
  }
  need_bf16(*a, "a");
  need_numel(*a, n, "a");
  *bf16_out = a->data_ptr();
  return nullptr;
}

}  // namespace
