// K9: fused optimizer step over the flat LoRA arena (mift.lora.LoraArena).
//
// Launches, everything stays on the device (no host sync, capturable into a hipGraph):
//   1. grad_stats:  per-block partial sum(g^2) and non-finite counts of the arena, then ONE block
//                   sums the partials in a fixed order into stats[0..1] (fp32).  No float atomics:
//                   the result is bit-identical run to run, so DDP replicas that hold identical
//                   all-reduced grads derive identical clip coefficients (SURVEY §5.2 deterministic
//                   mode).  For PP / ZeRO-1 the caller all-reduces `stats` over
//                   the model-parallel group between 1 and 2.
//   2. opt_finalize (1 thread): unscale (fp16 loss scaling), global-norm clip
//                   coefficient (max_norm, reference clip 1.0), found_inf,
//                   step += !found_inf, dynamic loss-scale update.
//   3. adamw_apply: decoupled weight decay AdamW (torch/HF semantics,
//                   betas (0.9,0.999), eps 1e-8) on every element; skipped
//                   entirely when found_inf; grads zeroed in the same pass.
// Reference semantics: HF Trainer defaults and DeepSpeed
// `gradient_clipping: 1.0` (P2 deepspeed_pp_zero1_cpu_activ.json).
#include "common.h"
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

namespace {

// Pass 1: block b writes (sum g^2, non-finite count) of its grid-strided elements to part[b].
// The element -> thread assignment and the block reduction tree are fixed, so each partial is too.
__global__ __launch_bounds__(256) void grad_stats_kernel(const float* __restrict__ g, int64_t n,
                                                         float2* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  float bad = 0.f;
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 3 < n) {
      float4 v = *reinterpret_cast<const float4*>(g + i);
      s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      if (!isfinite(v.x) || !isfinite(v.y) || !isfinite(v.z) || !isfinite(v.w)) bad += 1.f;
    } else {
      for (int64_t j = i; j < n; ++j) {
        s += g[j] * g[j];
        if (!isfinite(g[j])) bad += 1.f;
      }
    }
  }
  s = block_sum<4>(s, red);
  __syncthreads();
  bad = block_sum<4>(bad, red);
  if (threadIdx.x == 0) part[blockIdx.x] = make_float2(s, bad);
}

// Pass 2 (one block): thread t sums partials t, t + 256, ... in index order, then the fixed block
// tree — the same bits for the same gradients on every run and every replica.
__global__ __launch_bounds__(256) void grad_stats_reduce_kernel(const float2* __restrict__ part, int np,
                                                                float* __restrict__ stats) {
  __shared__ float red[4];
  float s = 0.f, bad = 0.f;
  for (int i = threadIdx.x; i < np; i += 256) {
    const float2 v = part[i];
    s += v.x;
    bad += v.y;
  }
  s = block_sum<4>(s, red);
  __syncthreads();
  bad = block_sum<4>(bad, red);
  if (threadIdx.x == 0) {
    stats[0] = s;
    stats[1] = bad;
  }
}

// state: [0]=step, [1]=loss_scale, [2]=good_steps, [3]=clip_coef (out),
//        [4]=found_inf (out), [5]=grad_norm (out, unscaled)
__global__ void opt_finalize_kernel(const float* __restrict__ stats, float* __restrict__ state, float max_norm,
                                    int dynamic_scale, float growth_factor, float backoff_factor,
                                    int growth_interval) {
  const float scale = state[1];
  const float inv_scale = 1.f / scale;
  const bool inf = !(stats[1] == 0.f) || !isfinite(stats[0]);
  const float norm = sqrtf(fmaxf(stats[0], 0.f)) * inv_scale;
  float coef = inv_scale;
  if (max_norm > 0.f && norm > max_norm) coef = inv_scale * (max_norm / (norm + 1e-6f));
  state[3] = coef;
  state[4] = inf ? 1.f : 0.f;
  state[5] = norm;
  if (!inf) state[0] += 1.f;
  if (dynamic_scale) {
    if (inf) {
      state[1] = fmaxf(scale * backoff_factor, 1.f);
      state[2] = 0.f;
    } else {
      state[2] += 1.f;
      if (state[2] >= (float)growth_interval) {
        state[1] = scale * growth_factor;
        state[2] = 0.f;
      }
    }
  }
}

__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                    const float* __restrict__ lr_t, const float* __restrict__ state,
                                                    float beta1, float beta2, float eps, float wd) {
  const bool inf = state[4] != 0.f;
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  if (inf) {  // skip the update, only clear grads
    for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride)
      for (int64_t j = i; j < min(i + 4, n); ++j) g[j] = 0.f;
    return;
  }
  const float step = state[0];
  const float coef = state[3];
  const float lr = lr_t[0];
  const float bc1 = 1.f - powf(beta1, step);
  const float bc2 = 1.f - powf(beta2, step);
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = rsqrtf(bc2);
  const float decay = 1.f - lr * wd;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 3 < n) {
      float4 pp = *reinterpret_cast<float4*>(p + i);
      float4 gg = *reinterpret_cast<float4*>(g + i);
      float4 mm = *reinterpret_cast<float4*>(m + i);
      float4 vv = *reinterpret_cast<float4*>(v + i);
      float* P = &pp.x; float* G = &gg.x; float* Mv = &mm.x; float* V = &vv.x;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float gk = G[k] * coef;
        Mv[k] = beta1 * Mv[k] + (1.f - beta1) * gk;
        V[k] = beta2 * V[k] + (1.f - beta2) * gk * gk;
        float denom = sqrtf(V[k]) * inv_sqrt_bc2 + eps;
        P[k] = P[k] * decay - step_size * Mv[k] / denom;
      }
      *reinterpret_cast<float4*>(p + i) = pp;
      *reinterpret_cast<float4*>(m + i) = mm;
      *reinterpret_cast<float4*>(v + i) = vv;
      *reinterpret_cast<float4*>(g + i) = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      for (int64_t j = i; j < n; ++j) {
        float gk = g[j] * coef;
        m[j] = beta1 * m[j] + (1.f - beta1) * gk;
        v[j] = beta2 * v[j] + (1.f - beta2) * gk * gk;
        float denom = sqrtf(v[j]) * inv_sqrt_bc2 + eps;
        p[j] = p[j] * decay - step_size * m[j] / denom;
        g[j] = 0.f;
      }
    }
  }
}

int grid_for(int64_t n) {
  int64_t b = (n / 4 + 255) / 256;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, 2048));
}

}  // namespace

void mift_grad_stats(const at::Tensor& g, at::Tensor& stats) {
  TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kFloat && g.is_contiguous(), "grad_stats: fp32 contiguous");
  TORCH_CHECK(stats.is_cuda() && stats.scalar_type() == at::kFloat && stats.numel() >= 2, "grad_stats: stats[2]");
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const int nb = grid_for(g.numel());
  auto part = at::empty({2 * (int64_t)nb}, g.options());
  grad_stats_kernel<<<nb, 256, 0, st>>>(g.data_ptr<float>(), g.numel(), reinterpret_cast<float2*>(part.data_ptr<float>()));
  grad_stats_reduce_kernel<<<1, 256, 0, st>>>(reinterpret_cast<const float2*>(part.data_ptr<float>()), nb,
                                              stats.data_ptr<float>());
}

void mift_opt_finalize(const at::Tensor& stats, at::Tensor& state, double max_norm, bool dynamic_scale,
                       double growth_factor, double backoff_factor, int64_t growth_interval) {
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  opt_finalize_kernel<<<1, 1, 0, st>>>(stats.data_ptr<float>(), state.data_ptr<float>(), (float)max_norm,
                                       dynamic_scale ? 1 : 0, (float)growth_factor, (float)backoff_factor,
                                       (int)growth_interval);
}

void mift_adamw(at::Tensor& p, at::Tensor& g, at::Tensor& m, at::Tensor& v, const at::Tensor& lr_t,
                const at::Tensor& state, double beta1, double beta2, double eps, double wd) {
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "adamw: sizes");
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  adamw_kernel<<<grid_for(p.numel()), 256, 0, st>>>(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(),
                                                    v.data_ptr<float>(), p.numel(), lr_t.data_ptr<float>(),
                                                    state.data_ptr<float>(), (float)beta1, (float)beta2, (float)eps,
                                                    (float)wd);
}
