// Bindings for the transformer kernel family (LayerNorm, embedding, flash attention).
#include <torch/extension.h>
void register_transformer_ops(pybind11::module& m) {}
