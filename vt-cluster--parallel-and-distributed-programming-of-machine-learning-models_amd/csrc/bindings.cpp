// Python bindings for the mift gfx950 extension (`mift._C`).
// Every function takes/returns at::Tensor and launches on torch's current
// HIP stream, so the ops compose with torch streams/events and are
// capturable into hipGraphs (torch.cuda.graph).
#include <torch/extension.h>
#include "ops.h"
#include "common.h"

void mift_bind_runtime(pybind11::module& m);  // runtime/loader.cpp

// Device micro-step counter for graph-replayed dropout seeds (common.h mift_seed).
static at::Tensor g_seed_step;
const int64_t* mift_seed_step() { return g_seed_step.defined() ? g_seed_step.data_ptr<int64_t>() : nullptr; }
static void mift_set_seed_step(const c10::optional<at::Tensor>& t) {
  if (!t || !t->defined()) {
    g_seed_step = at::Tensor();
    return;
  }
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong && t->numel() >= 1, "set_seed_step: int64 GPU tensor");
  g_seed_step = *t;
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "mift: MI355X (gfx950) HIP kernels + native runtime";
  // K4 LayerNorm
  m.def("layer_norm_fwd", &mift_layer_norm_fwd, "LayerNorm forward -> (y, mean, rstd)");
  m.def("layer_norm_bwd", &mift_layer_norm_bwd,
        "LayerNorm backward (+residual add, +dropout-masked branch copy, +optional dgamma/dbeta)");
  m.def("set_seed_step", &mift_set_seed_step,
        "bind (tensor) / unbind (None) the device micro-step counter mixed into every dropout seed");
  MIFT_BIND_MORE(m);
  mift_bind_runtime(m);
}
