// Host-side declarations of every op exported by mift._C.
#pragma once
#include <torch/extension.h>
#include <vector>

// ---- K4 LayerNorm (kernels/layernorm.hip)
std::vector<at::Tensor> mift_layer_norm_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b,
                                            double eps);
std::vector<at::Tensor> mift_layer_norm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                            const at::Tensor& mean, const at::Tensor& rstd,
                                            const c10::optional<at::Tensor>& dres, bool want_branch, double p,
                                            int64_t seed, bool want_wgrad);

// ---- K1/K2 MFMA GEMM NT with fused epilogue (kernels/gemm.hip)
std::vector<at::Tensor> mift_gemm_nt(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& bias,
                                     const c10::optional<at::Tensor>& a2, const c10::optional<at::Tensor>& b2,
                                     int64_t act, const c10::optional<at::Tensor>& aux,
                                     const c10::optional<at::Tensor>& residual, double dropout_p, int64_t seed,
                                     bool want_preact, double alpha, const c10::optional<at::Tensor>& out,
                                     int64_t tile);

#define MIFT_BIND_MORE(m) \
  m.def("gemm_nt", &mift_gemm_nt, "C = epi(A @ B^T [+ A2 @ B2^T]) MFMA bf16/fp16");
