// Python bindings for the C++ TF V2 checkpoint bundle (cpp/runtime/tfbundle.cc): zero-copy writes
// from CPU torch tensors, crc-verified reads into fresh CPU tensors, and the `checkpoint` state file.
#include <torch/extension.h>

#include "../../cpp/runtime/tfbundle.h"

namespace {
using namespace tfk::ckpt;

int dtype_of(const torch::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return DT_FLOAT;
    case at::kDouble: return DT_DOUBLE;
    case at::kInt: return DT_INT32;
    case at::kLong: return DT_INT64;
    case at::kByte: return DT_UINT8;
    case at::kChar: return DT_INT8;
    case at::kShort: return DT_INT16;
    case at::kBool: return DT_BOOL;
    case at::kBFloat16: return DT_BFLOAT16;
    case at::kHalf: return DT_HALF;
    default: TORCH_CHECK(false, "unsupported checkpoint dtype ", t.scalar_type());
  }
}
at::ScalarType scalar_of(int dt) {
  switch (dt) {
    case DT_FLOAT: return at::kFloat;
    case DT_DOUBLE: return at::kDouble;
    case DT_INT32: return at::kInt;
    case DT_INT64: return at::kLong;
    case DT_UINT8: return at::kByte;
    case DT_INT8: return at::kChar;
    case DT_INT16: return at::kShort;
    case DT_BOOL: return at::kBool;
    case DT_BFLOAT16: return at::kBFloat16;
    case DT_HALF: return at::kHalf;
    default: TORCH_CHECK(false, "unsupported TF dtype ", dt);
  }
}

void bundle_write(const std::string& prefix, const std::vector<std::string>& names, const std::vector<torch::Tensor>& ts) {
  TORCH_CHECK(names.size() == ts.size(), "names/tensors length mismatch");
  std::vector<torch::Tensor> keep;
  std::vector<TensorRef> refs;
  for (size_t i = 0; i < ts.size(); ++i) {
    auto t = ts[i].contiguous();
    TORCH_CHECK(!t.is_cuda(), "checkpoint tensors must be on the CPU (D2H first)");
    keep.push_back(t);
    TensorRef r;
    r.name = names[i];
    r.dtype = dtype_of(t);
    for (auto d : t.sizes()) r.shape.push_back(d);
    r.data = t.data_ptr();
    r.nbytes = t.numel() * t.element_size();
    refs.push_back(r);
  }
  std::string err;
  bool ok;
  {
    pybind11::gil_scoped_release nogil;
    ok = write_bundle(prefix, refs, &err);
  }
  TORCH_CHECK(ok, "checkpoint write failed: ", err);
}

std::vector<std::tuple<std::string, std::string, std::vector<int64_t>>> list(const std::string& prefix) {
  BundleReader r;
  std::string err;
  TORCH_CHECK(r.open(prefix, &err), err);
  std::vector<std::tuple<std::string, std::string, std::vector<int64_t>>> out;
  for (auto& kv : r.entries()) out.emplace_back(kv.first, dtype_name(kv.second.dtype), kv.second.shape);
  return out;
}

std::map<std::string, torch::Tensor> bundle_read(const std::string& prefix, const std::vector<std::string>& only) {
  BundleReader r;
  std::string err;
  TORCH_CHECK(r.open(prefix, &err), err);
  std::map<std::string, torch::Tensor> out;
  for (auto& kv : r.entries()) {
    if (!only.empty() && std::find(only.begin(), only.end(), kv.first) == only.end()) continue;
    std::string data;
    TORCH_CHECK(r.read(kv.first, &data, &err), err);
    auto t = torch::empty(kv.second.shape, torch::TensorOptions().dtype(scalar_of(kv.second.dtype)));
    TORCH_CHECK((size_t)(t.numel() * t.element_size()) == data.size(), "size mismatch for ", kv.first);
    memcpy(t.data_ptr(), data.data(), data.size());
    out[kv.first] = t;
  }
  return out;
}

void state_write(const std::string& dir, const std::string& latest, const std::vector<std::string>& all) {
  std::string err;
  TORCH_CHECK(write_checkpoint_state(dir, latest, all, &err), err);
}
std::pair<std::string, std::vector<std::string>> state_read(const std::string& dir) {
  std::string latest;
  std::vector<std::string> all;
  read_checkpoint_state(dir, &latest, &all);
  return {latest, all};
}
}  // namespace

void register_ckpt_ops(pybind11::module& m) {
  m.def("ckpt_write", &bundle_write);
  m.def("ckpt_list", &list);
  m.def("ckpt_read", &bundle_read, pybind11::arg("prefix"), pybind11::arg("only") = std::vector<std::string>{});
  m.def("ckpt_state_write", &state_write);
  m.def("ckpt_state_read", &state_read);
}
