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
//
// The training step uses the TWO-launch form (opt_stats + opt_apply, VERDICT r3 hygiene):
//   opt_stats:  pass 1 above, and the LAST block to finish (a self-resetting arrival counter in
//               the optimizer's workspace) sums the partials in the same fixed order and — when no
//               model-parallel all-reduce follows — runs the finalize of 2 in the same launch;
//   opt_apply:  pass 3; when the stats were all-reduced after opt_stats, every block derives the
//               finalize values itself from (stats, state) — identical inputs, identical bits — and
//               the last block to arrive commits the new state (no fence: no block reads another's
//               writes, see the kernel).  The learning rate is a launch
//               argument (no per-step device fill).
// Cross-block visibility: partials are stored write-through (sc1) before the arrival atomic, the last
// block takes an agent-scope acquire before reading them (common.h mift_last_block_arrival).
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
struct FinArgs {
  float max_norm, growth_factor, backoff_factor;
  int dynamic_scale, growth_interval;
};

// new state from (stats, old state) — pure, so every block of opt_apply derives the same values
__device__ inline void finalize_state(const float* __restrict__ stats, const float* __restrict__ old, FinArgs f,
                                      float* __restrict__ ns) {
  const float scale = old[1];
  const float inv_scale = 1.f / scale;
  const bool inf = !(stats[1] == 0.f) || !isfinite(stats[0]);
  const float norm = sqrtf(fmaxf(stats[0], 0.f)) * inv_scale;
  float coef = inv_scale;
  if (f.max_norm > 0.f && norm > f.max_norm) coef = inv_scale * (f.max_norm / (norm + 1e-6f));
  ns[0] = inf ? old[0] : old[0] + 1.f;
  ns[1] = scale;
  ns[2] = old[2];
  ns[3] = coef;
  ns[4] = inf ? 1.f : 0.f;
  ns[5] = norm;
  if (f.dynamic_scale) {
    if (inf) {
      ns[1] = fmaxf(scale * f.backoff_factor, 1.f);
      ns[2] = 0.f;
    } else {
      ns[2] = old[2] + 1.f;
      if (ns[2] >= (float)f.growth_interval) {
        ns[1] = scale * f.growth_factor;
        ns[2] = 0.f;
      }
    }
  }
}

__global__ void opt_finalize_kernel(const float* __restrict__ stats, float* __restrict__ state, FinArgs f) {
  float ns[6];
  finalize_state(stats, state, f, ns);
#pragma unroll
  for (int k = 0; k < 6; ++k) state[k] = ns[k];
}

// opt_stats: partial (sum g^2, non-finite) per block; the last block reduces them in index order
// (the grad_stats_reduce_kernel order) and optionally finalizes the state.
__global__ __launch_bounds__(256) void opt_stats_kernel(const float* __restrict__ g, int64_t n,
                                                        float2* __restrict__ part, float* __restrict__ stats,
                                                        unsigned* __restrict__ counter, float* __restrict__ state,
                                                        int finalize, FinArgs f) {
  __shared__ float red[4];
  __shared__ int flag;
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
  if (threadIdx.x == 0) mift_st_sc1(&part[blockIdx.x], make_float2(s, bad));
  if (!mift_last_block_arrival(counter, &flag)) return;
  const int np = gridDim.x;
  float t = 0.f, tb = 0.f;
  for (int i = threadIdx.x; i < np; i += 256) {
    const float2 v = part[i];
    t += v.x;
    tb += v.y;
  }
  __syncthreads();
  t = block_sum<4>(t, red);
  __syncthreads();
  tb = block_sum<4>(tb, red);
  if (threadIdx.x == 0) {
    stats[0] = t;
    stats[1] = tb;
    if (finalize) {
      float ns[6];
      finalize_state(stats, state, f, ns);
#pragma unroll
      for (int k = 0; k < 6; ++k) state[k] = ns[k];
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

// opt_apply: AdamW over the arena.  finalize = 1: the state is still the previous step's — every
// block derives the new values from (stats, state) and the last block to finish writes them.
__global__ __launch_bounds__(256) void opt_apply_kernel(float* __restrict__ p, float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                        float lr, float* __restrict__ state,
                                                        const float* __restrict__ stats,
                                                        unsigned* __restrict__ counter, int finalize, FinArgs f,
                                                        float beta1, float beta2, float eps, float wd) {
  float ns[6];
  if (finalize) {
    finalize_state(stats, state, f, ns);
  } else {
#pragma unroll
    for (int k = 0; k < 6; ++k) ns[k] = state[k];
  }
  const bool inf = ns[4] != 0.f;
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  if (inf) {  // skip the update, only clear grads
    for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride)
      for (int64_t j = i; j < min(i + 4, n); ++j) g[j] = 0.f;
  } else {
    const float step = ns[0];
    const float coef = ns[3];
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
  if (!finalize) return;
  // Arrival WITHOUT a release fence: nothing this block wrote is read by another block, only its
  // (completed — the values were consumed above) reads of `state` must precede the last block's
  // write.  A release here would write back the XCD's L2 (dirty p/m/v/g lines) from every block —
  // the cost that sank the in-kernel LoRA wgrad finisher in round 3.
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(counter, 1u) == gridDim.x - 1) {
    counter[0] = 0u;
#pragma unroll
    for (int k = 0; k < 6; ++k) state[k] = ns[k];
  }
}

FinArgs fin_args(double max_norm, bool dynamic_scale, double growth_factor, double backoff_factor,
                 int64_t growth_interval) {
  FinArgs f;
  f.max_norm = (float)max_norm;
  f.growth_factor = (float)growth_factor;
  f.backoff_factor = (float)backoff_factor;
  f.dynamic_scale = dynamic_scale ? 1 : 0;
  f.growth_interval = (int)growth_interval;
  return f;
}

void check_ws(const at::Tensor& ws, const at::Tensor& state) {
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == at::kInt && ws.numel() >= MIFT_ARRIVE_INTS + 1 &&
                  ws.is_contiguous(),
              "optimizer workspace: int32[MIFT_ARRIVE_INTS + 1] (zero-initialised, self-resetting arrival counters)");
  TORCH_CHECK(state.is_cuda() && state.scalar_type() == at::kFloat && state.numel() >= 6, "optimizer state: fp32[6]");
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
  opt_finalize_kernel<<<1, 1, 0, st>>>(stats.data_ptr<float>(), state.data_ptr<float>(),
                                       fin_args(max_norm, dynamic_scale, growth_factor, backoff_factor,
                                                growth_interval));
}

void mift_opt_stats(const at::Tensor& g, at::Tensor& stats, at::Tensor& ws, at::Tensor& state, bool finalize,
                    double max_norm, bool dynamic_scale, double growth_factor, double backoff_factor,
                    int64_t growth_interval) {
  TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kFloat && g.is_contiguous(), "opt_stats: fp32 contiguous");
  TORCH_CHECK(stats.is_cuda() && stats.scalar_type() == at::kFloat && stats.numel() >= 2, "opt_stats: stats[2]");
  check_ws(ws, state);
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const int nb = grid_for(g.numel());
  auto part = at::empty({2 * (int64_t)nb}, g.options());
  opt_stats_kernel<<<nb, 256, 0, st>>>(g.data_ptr<float>(), g.numel(), reinterpret_cast<float2*>(part.data_ptr<float>()),
                                       stats.data_ptr<float>(), reinterpret_cast<unsigned*>(ws.data_ptr<int>()),
                                       state.data_ptr<float>(), finalize ? 1 : 0,
                                       fin_args(max_norm, dynamic_scale, growth_factor, backoff_factor, growth_interval));
}

void mift_opt_apply(at::Tensor& p, at::Tensor& g, at::Tensor& m, at::Tensor& v, double lr, at::Tensor& state,
                    const at::Tensor& stats, at::Tensor& ws, bool finalize, double max_norm, bool dynamic_scale,
                    double growth_factor, double backoff_factor, int64_t growth_interval, double beta1, double beta2,
                    double eps, double wd) {
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "opt_apply: sizes");
  TORCH_CHECK(stats.is_cuda() && stats.scalar_type() == at::kFloat && stats.numel() >= 2, "opt_apply: stats[2]");
  check_ws(ws, state);
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  opt_apply_kernel<<<grid_for(p.numel()), 256, 0, st>>>(
      p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), p.numel(), (float)lr,
      state.data_ptr<float>(), stats.data_ptr<float>(), reinterpret_cast<unsigned*>(ws.data_ptr<int>()) + MIFT_ARRIVE_INTS,
      finalize ? 1 : 0, fin_args(max_norm, dynamic_scale, growth_factor, backoff_factor, growth_interval),
      (float)beta1, (float)beta2, (float)eps, (float)wd);
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
