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
// lora_proj on the rowproj.hip MFMA form when the shape fits (called by mift_lora_proj)
bool mift_rowproj_lora_proj(const at::Tensor& x, const at::Tensor& w, at::Tensor& out, double alpha, double p,
                            int64_t seed, int64_t rows);

std::vector<at::Tensor> mift_gemm_nt(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& bias,
                                     const c10::optional<at::Tensor>& a2, const c10::optional<at::Tensor>& b2,
                                     int64_t act, const c10::optional<at::Tensor>& aux,
                                     const c10::optional<at::Tensor>& residual, double dropout_p, int64_t seed,
                                     bool want_preact, double alpha, const c10::optional<at::Tensor>& out,
                                     int64_t tile, const c10::optional<at::Tensor>& alpha_t,
                                     const c10::optional<at::Tensor>& pre_add, double ext_p, int64_t ext_seed,
                                     const c10::optional<at::Tensor>& proj_w, int64_t proj_rows, double proj_p,
                                     int64_t proj_seed, double proj_alpha, const c10::optional<at::Tensor>& sbits);

// ---- K2/K7 fused LM head + cross-entropy (kernels/gemm.hip, EPI 1/2)
std::vector<at::Tensor> mift_lmhead_fwd(const at::Tensor& a, const at::Tensor& w, const at::Tensor& labels, int64_t V,
                                        int64_t shift, int64_t ignore, const c10::optional<at::Tensor>& ws);
at::Tensor mift_lmhead_dgrad(const at::Tensor& E, const at::Tensor& wt, const at::Tensor& w, const at::Tensor& labels,
                             int64_t V, const at::Tensor& stats, const at::Tensor& lse, const at::Tensor& gscale,
                             int64_t shift, int64_t ignore, const c10::optional<at::Tensor>& gmul);

// ---- LoRA side path (kernels/lora.hip)
at::Tensor mift_lora_proj(const at::Tensor& x, const at::Tensor& w, double alpha, double p, int64_t seed,
                          int64_t rows);
void mift_lora_wgrad(const at::Tensor& x, const at::Tensor& y, at::Tensor& out, double p, int64_t seed, int64_t mode,
                     int64_t rank, int64_t offset, int64_t qoff);
void mift_lora_wgrad_group(at::Tensor& out, const std::vector<at::Tensor>& xs, const std::vector<at::Tensor>& ys,
                           const std::vector<int64_t>& meta, const std::vector<double>& ps);
void mift_pack_lora_all(const at::Tensor& arena, const at::Tensor& table, const at::Tensor& scales, at::Tensor& out,
                        int64_t max_elems);
void mift_pack_lora_multi(const at::Tensor& arena, const at::Tensor& table, const at::Tensor& scales,
                          int64_t max_elems, bool bf16_out);

// ---- row producers fused with the LoRA projection (kernels/rowproj.hip)
std::vector<at::Tensor> mift_layer_norm_fwd_proj(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b,
                                                 double eps, const at::Tensor& pw, int64_t rank, double alpha,
                                                 double p, int64_t seed);
bool mift_ln_bwd_mask_proj_ok(int64_t D);
std::vector<at::Tensor> mift_ln_bwd_mask_proj(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                              const at::Tensor& mean, const at::Tensor& rstd,
                                              const c10::optional<at::Tensor>& dres, double p, int64_t seed,
                                              const at::Tensor& pw, int64_t rank, double alpha);
std::vector<at::Tensor> mift_mask_proj(const at::Tensor& x, double p, int64_t seed, const at::Tensor& pw,
                                       int64_t rank, double alpha);

// ---- elementwise / embedding / LoRA pack (kernels/elementwise.hip)
at::Tensor mift_mask_scale(const at::Tensor& x, double p, int64_t seed, const c10::optional<at::Tensor>& out,
                           bool accumulate);
at::Tensor mift_act_bwd(const at::Tensor& g, const at::Tensor& z, int64_t act, double p, int64_t seed);
std::vector<at::Tensor> mift_mask_positions(const at::Tensor& mask);
at::Tensor mift_embed_fwd(const at::Tensor& ids, const c10::optional<at::Tensor>& pos, const at::Tensor& wte,
                          const c10::optional<at::Tensor>& wpe, int64_t pos_offset, double p, int64_t seed,
                          at::ScalarType out_dtype);
std::vector<at::Tensor> mift_pack_lora(const at::Tensor& A, const at::Tensor& B, double a_scale, at::ScalarType dt);

// ---- K7 cross-entropy (kernels/xent.hip)
std::vector<at::Tensor> mift_xent_fwd_bwd(at::Tensor& logits, const at::Tensor& labels, int64_t V,
                                          int64_t ignore_index, bool write_grad);

// ---- K9 fused optimizer (kernels/adamw.hip)
void mift_grad_stats(const at::Tensor& g, at::Tensor& stats);
void mift_opt_finalize(const at::Tensor& stats, at::Tensor& state, double max_norm, bool dynamic_scale,
                       double growth_factor, double backoff_factor, int64_t growth_interval);
void mift_opt_stats(const at::Tensor& g, at::Tensor& stats, at::Tensor& ws, at::Tensor& state, bool finalize,
                    double max_norm, bool dynamic_scale, double growth_factor, double backoff_factor,
                    int64_t growth_interval);
void mift_opt_apply(at::Tensor& p, at::Tensor& g, at::Tensor& m, at::Tensor& v, double lr, at::Tensor& state,
                    const at::Tensor& stats, at::Tensor& ws, bool finalize, double max_norm, bool dynamic_scale,
                    double growth_factor, double backoff_factor, int64_t growth_interval, double beta1, double beta2,
                    double eps, double wd);
void mift_adamw(at::Tensor& p, at::Tensor& g, at::Tensor& m, at::Tensor& v, const at::Tensor& lr_t,
                const at::Tensor& state, double beta1, double beta2, double eps, double wd);

// ---- K3 flash attention (kernels/attention.hip)
std::vector<at::Tensor> mift_attn_fwd(const at::Tensor& qkv, int64_t B, int64_t S, int64_t H, int64_t HD, double scale,
                                      double p, int64_t seed, const c10::optional<at::Tensor>& kv_len);
at::Tensor mift_attn_bwd(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& o, const at::Tensor& lse,
                         int64_t B, int64_t S, int64_t H, int64_t HD, double scale, double p, int64_t seed,
                         const c10::optional<at::Tensor>& kv_len);
std::vector<at::Tensor> mift_attn_fwd_bits(const at::Tensor& qkv, int64_t B, int64_t S, int64_t H, int64_t HD,
                                           double scale, double p, int64_t seed,
                                           const c10::optional<at::Tensor>& kv_len);
at::Tensor mift_attn_bwd_bits(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& o, const at::Tensor& lse,
                              int64_t B, int64_t S, int64_t H, int64_t HD, double scale, double p, int64_t seed,
                              const c10::optional<at::Tensor>& kv_len, const c10::optional<at::Tensor>& bits);

// ---- K12 decode attention over a KV cache (kernels/decode.hip)
void mift_gemm_set_stamps(const c10::optional<at::Tensor>& buf);
bool mift_gemm_ln_ok(int64_t M, int64_t N, int64_t K);
std::vector<at::Tensor> mift_gemm_ln(const at::Tensor& x, const at::Tensor& ln_w, const at::Tensor& ln_b, double eps,
                                     const at::Tensor& w, const c10::optional<at::Tensor>& bias, int64_t act,
                                     bool want_preact);
at::Tensor mift_gemm_ln_fold(const at::Tensor& x, const at::Tensor& wf, const at::Tensor& c1, const at::Tensor& c2,
                             double eps, int64_t act);
void mift_decode_tail(const at::Tensor& logits, int64_t V, at::Tensor& done, at::Tensor& ids, at::Tensor& out,
                      at::Tensor& col, at::Tensor& pos, at::Tensor& t, int64_t fill, int64_t pad, int64_t eos);
void mift_kv_store(const at::Tensor& qkv, at::Tensor& kc, at::Tensor& vc, int64_t S);
at::Tensor mift_decode_attn(const at::Tensor& qkv, at::Tensor& kc, at::Tensor& vc, int64_t t, double scale,
                            const c10::optional<at::Tensor>& start, const c10::optional<at::Tensor>& plen,
                            int64_t gend, const c10::optional<at::Tensor>& t_dev);

#define MIFT_BIND_MORE(m) \
  m.def("gemm_set_stamps", &mift_gemm_set_stamps, "diagnostics: per-block cycle stamps of later gemm_nt launches"); \
  m.def("gemm_ln_ok", &mift_gemm_ln_ok, "shapes the LN-prologue skinny GEMM takes"); \
  m.def("gemm_ln", &mift_gemm_ln, "act(LN(x) w^T + bias) for M <= 64 rows (decode), LN applied in the GEMM"); \
  m.def("gemm_ln_fold", &mift_gemm_ln_fold, "act(rstd (x wf^T - mean c1) + c2): LN folded into the weights (decode)"); \
  m.def("decode_tail", &mift_decode_tail, "greedy decode step tail: argmax, pad/eos, next ids, out/col/pos/t advance"); \
  m.def("kv_store", &mift_kv_store, "prefill: K / V rows [0, S) of qkv into the caches, one launch"); \
  m.def("decode_attn", &mift_decode_attn, "single-token attention over a KV cache; appends k/v at t (left padding: start; prompt gap: plen, gend)"); \
  m.def("lora_proj", &mift_lora_proj, "out[M,32] = alpha*drop(x)@w^T (tall-skinny MFMA)"); \
  m.def("layer_norm_fwd_proj", &mift_layer_norm_fwd_proj, "LN fwd + alpha*drop(y)@pw^T -> (y, mean, rstd, proj)"); \
  m.def("mask_proj", &mift_mask_proj, "y = dropout(x) (p>0), proj = alpha*y@pw^T -> (y, proj)"); \
  m.def("ln_bwd_mask_proj_ok", &mift_ln_bwd_mask_proj_ok, "ln_bwd_mask_proj applies at this width");            \
  m.def("ln_bwd_mask_proj", &mift_ln_bwd_mask_proj, "dh = LN-bwd + dres, y = dropout-bwd(dh), proj = alpha*y@pw^T"); \
  m.def("lora_wgrad", &mift_lora_wgrad, "out[P,32] += drop(x)^T @ y (tr_b16 split-M MFMA); arena modes"); \
  m.def("lora_wgrad_group", &mift_lora_wgrad_group, "grouped LoRA weight grads (<= 16 problems, one launch)"); \
  m.def("pack_lora_multi", &mift_pack_lora_multi, "one-launch pack of every shared-input adapter group (q/k/v)"); \
  m.def("pack_lora_all", &mift_pack_lora_all, "pack every adapter's 16-bit operands from the fp32 arena"); \
  m.def("attn_fwd", &mift_attn_fwd, "causal flash attention fwd on fused qkv -> (o, lse)"); \
  m.def("attn_bwd", &mift_attn_bwd, "causal flash attention bwd -> dqkv"); \
  m.def("attn_fwd_bits", &mift_attn_fwd_bits, "attn fwd that also records its dropout keep bits -> (o, lse, bits)"); \
  m.def("attn_bwd_bits", &mift_attn_bwd_bits, "attn bwd reading the forward's keep bits -> dqkv"); \
  m.def("gemm_nt", &mift_gemm_nt, "C = epi(A @ B^T [+ A2 @ B2^T]) MFMA bf16/fp16 -> (C, preact, proj)", \
        pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("bias"), pybind11::arg("a2"), pybind11::arg("b2"), \
        pybind11::arg("act"), pybind11::arg("aux"), pybind11::arg("residual"), pybind11::arg("dropout_p"), \
        pybind11::arg("seed"), pybind11::arg("want_preact"), pybind11::arg("alpha"), pybind11::arg("out"), \
        pybind11::arg("tile"), pybind11::arg("alpha_t"), pybind11::arg("pre_add"), pybind11::arg("ext_p"), \
        pybind11::arg("ext_seed"), pybind11::arg("proj_w") = pybind11::none(), pybind11::arg("proj_rows") = 32, \
        pybind11::arg("proj_p") = 0.0, pybind11::arg("proj_seed") = 0, pybind11::arg("proj_alpha") = 1.0, \
        pybind11::arg("sbits") = pybind11::none()); \
  m.def("lmhead_fwd", &mift_lmhead_fwd, "fused LM head + CE fwd -> (E, stats, lse, loss, zlab[, total])"); \
  m.def("lmhead_dgrad", &mift_lmhead_dgrad, "fused LM head + CE dgrad -> dX (no dlogits)"); \
  m.def("grad_stats", &mift_grad_stats, "sum(g^2), nonfinite count -> stats[2]"); \
  m.def("opt_finalize", &mift_opt_finalize, "clip coef / found_inf / step / loss-scale update"); \
  m.def("adamw", &mift_adamw, "fused AdamW over a flat fp32 arena (zeroes grads)"); \
  m.def("opt_stats", &mift_opt_stats, "grad stats + in-launch fixed-order reduce [+ finalize]"); \
  m.def("arrive_ints", []() { return (int64_t)MIFT_ARRIVE_INTS; }, "int32 words of an in-launch arrival-counter set"); \
  m.def("opt_apply", &mift_opt_apply, "AdamW [+ finalize from all-reduced stats] (zeroes grads)"); \
  m.def("mask_scale", &mift_mask_scale, "counter-hash dropout (fwd == bwd), optional accumulate"); \
  m.def("act_bwd", &mift_act_bwd, "dz = dropmask(g) * act'(z)"); \
  m.def("mask_positions", &mift_mask_positions, "OPT positions cumsum(mask)*mask-1 and key lengths, one launch"); \
  m.def("embed_fwd", &mift_embed_fwd, "token + position gather (+dropout)"); \
  m.def("pack_lora", &mift_pack_lora, "fp32 LoRA A,B -> padded 16-bit A32[32,K], B32[N,32]"); \
  m.def("xent_fwd_bwd", &mift_xent_fwd_bwd, "row cross-entropy; dlogits written in place");
