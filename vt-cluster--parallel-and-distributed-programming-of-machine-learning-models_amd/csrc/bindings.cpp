// Python bindings for the mift gfx950 extension (`mift._C`).
// Every function takes/returns at::Tensor and launches on torch's current
// HIP stream, so the ops compose with torch streams/events and are
// capturable into hipGraphs (torch.cuda.graph).
#include <torch/extension.h>
#include "ops.h"

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "mift: MI355X (gfx950) HIP kernels + native runtime";
  // K4 LayerNorm
  m.def("layer_norm_fwd", &mift_layer_norm_fwd, "LayerNorm forward -> (y, mean, rstd)");
  m.def("layer_norm_bwd", &mift_layer_norm_bwd,
        "LayerNorm backward (+residual add, +dropout-masked branch copy, +optional dgamma/dbeta)");
  MIFT_BIND_MORE(m);
}
