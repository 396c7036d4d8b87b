// Elementwise / small fused ops (memory-bound, 16-B vector I/O, Guideline 13).
//
//   mask_scale(x, p, seed[, out, accumulate]):  y = keep(seed, i) ? x/(1-p) : 0
//       — dropout forward AND its backward (same seed => same mask); with
//         `accumulate` it adds into `out` (LoRA input-dropout backward).
//   act_bwd(g, z, act, p, seed): dz = dropmask(g) * act'(z)
//   embed_fwd(ids, wte, wpe, pos_offset, p, seed): h = wte[ids] + wpe[pos] (+dropout)
//       K8: token + learned-position gather; OPT passes explicit positions
//       (cumsum(mask)*mask - 1 + 2).
//   pack_lora(A[r,K] f32, B[N,r] f32) -> A32[32,K], B32[N,32] (T, zero padded)
#include "common.h"
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

namespace {

template <typename T>
__global__ __launch_bounds__(256) void mask_scale_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                         uint64_t seed, const int64_t* __restrict__ sstep, uint32_t thr, float inv_keep,
                                                         int accumulate) {
  seed = mift_seed(seed, sstep);
  const int64_t stride = (int64_t)gridDim.x * 256 * 8;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8; i < n; i += stride) {
    if (i + 8 <= n) {
      float v[8], o[8];
      load8<T>(x + i, v);
      if (accumulate) load8<T>(y + i, o);
      bool kp[8];
      mift_keep8(seed, (uint64_t)i, thr, kp);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float r = kp[e] ? v[e] * inv_keep : 0.f;
        o[e] = accumulate ? o[e] + r : r;
      }
      store8<T>(y + i, o);
    } else {
      for (int64_t j = i; j < n; ++j) {
        float r = mift_keep(seed, (uint64_t)j, thr) ? (float)x[j] * inv_keep : 0.f;
        y[j] = (T)(accumulate ? (float)y[j] + r : r);
      }
    }
  }
}

MIFT_HD float act_grad(int act, float z) {
  switch (act) {
    case 1: return gelu_tanh_grad(z);
    case 2: return z > 0.f ? 1.f : 0.f;
    case 3: return gelu_erf_grad(z);
    default: return 1.f;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void act_bwd_kernel(const T* __restrict__ g, const T* __restrict__ z,
                                                      T* __restrict__ out, int64_t n, int act, uint64_t seed,
                                                      const int64_t* __restrict__ sstep, uint32_t thr, float inv_keep) {
  seed = mift_seed(seed, sstep);
  const int64_t stride = (int64_t)gridDim.x * 256 * 8;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8; i < n; i += stride) {
    if (i + 8 <= n) {
      float gv[8], zv[8];
      load8<T>(g + i, gv);
      load8<T>(z + i, zv);
      bool kp[8] = {true, true, true, true, true, true, true, true};
      if (thr != 0) mift_keep8(seed, (uint64_t)i, thr, kp);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float m = kp[e] ? inv_keep : 0.f;
        gv[e] = gv[e] * m * act_grad(act, zv[e]);
      }
      store8<T>(out + i, gv);
    } else {
      for (int64_t j = i; j < n; ++j) {
        float m = (thr == 0 || mift_keep(seed, (uint64_t)j, thr)) ? inv_keep : 0.f;
        out[j] = (T)((float)g[j] * m * act_grad(act, (float)z[j]));
      }
    }
  }
}

template <typename T, typename W>
__global__ __launch_bounds__(256) void embed_kernel(const int64_t* __restrict__ ids, const int64_t* __restrict__ pos,
                                                    const W* __restrict__ wte, const W* __restrict__ wpe,
                                                    T* __restrict__ h, int S, int D, int pos_offset,
                                                    uint64_t seed, const int64_t* __restrict__ sstep, uint32_t thr, float inv_keep,
                                                    int64_t vocab, int64_t npos) {
  seed = mift_seed(seed, sstep);
  const int row = blockIdx.x;
  const int64_t tok = ids[row];
  const int64_t p = (pos != nullptr ? pos[row] : (int64_t)(row % S)) + pos_offset;
  MIFT_ASSERT(tok >= 0 && tok < vocab);
  MIFT_ASSERT(wpe == nullptr || (p >= 0 && p < npos));
  for (int c = threadIdx.x * 8; c < D; c += 256 * 8) {
    float a[8], b[8];
    load8<W>(wte + tok * D + c, a);
    if (wpe != nullptr) load8<W>(wpe + p * D + c, b);
    else for (int e = 0; e < 8; ++e) b[e] = 0.f;
    bool kp[8] = {true, true, true, true, true, true, true, true};
    if (thr != 0) mift_keep8(seed, (uint64_t)row * D + c, thr, kp);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = a[e] + b[e];
      if (thr != 0) v = kp[e] ? v * inv_keep : 0.f;
      a[e] = v;
    }
    store8<T>(h + (int64_t)row * D + c, a);
  }
}

// OPT's learned positions and key lengths from the attention mask, one block per row:
// pos[b, t] = cumsum(mask[b])[t]·mask[b, t] - 1 (HF OPTLearnedPositionalEmbedding; pad -> -1) and
// kv_len[b] = Σ_t mask[b, t] — one launch in place of the six torch kernels (cumsum, mul, sub, cast,
// sum) the replayed OPT step ran per micro-batch.  Chunks of 256 tokens, block-wide inclusive scan
// (wave shuffles + one LDS word per wave), running carry.
__global__ __launch_bounds__(256) void mask_positions_kernel(const int64_t* __restrict__ mask, int S,
                                                             int64_t* __restrict__ pos, int* __restrict__ kv_len) {
  __shared__ int wsum[4];
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t* m = mask + (int64_t)b * S;
  int carry = 0;
  for (int t0 = 0; t0 < S; t0 += 256) {
    const int t = t0 + threadIdx.x;
    const int v = t < S ? (int)m[t] : 0;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int before = carry;
    for (int k = 0; k < w; ++k) before += wsum[k];
    const int total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (t < S) pos[(int64_t)b * S + t] = (int64_t)(before + x) * v - 1;
    carry += total;
    __syncthreads();
  }
  if (threadIdx.x == 0) kv_len[b] = carry;
}

template <typename T>
__global__ void pack_lora_kernel(const float* __restrict__ A, const float* __restrict__ B, T* __restrict__ A32,
                                 T* __restrict__ B32, int r, int K, int N, float a_scale) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t na = 32LL * K, nb = (int64_t)N * 32;
  if (i < na) {
    int row = i / K, col = i % K;
    A32[i] = (T)(row < r ? A[(int64_t)row * K + col] * a_scale : 0.f);
  } else if (i < na + nb) {
    int64_t j = i - na;
    int row = j / 32, col = j % 32;
    B32[j] = (T)(col < r ? B[(int64_t)row * r + col] : 0.f);
  }
}

int ew_grid(int64_t n) {
  int64_t b = (n / 8 + 255) / 256;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, 4096));
}

uint32_t thr_of(double p) { return mift_thr16(p); }

}  // namespace

#define DISPATCH_16(dt, ...)                                           \
  do {                                                                 \
    if (dt == at::kBFloat16) { using T = bf16; __VA_ARGS__; }          \
    else if (dt == at::kHalf) { using T = fp16; __VA_ARGS__; }         \
    else if (dt == at::kFloat) { using T = float; __VA_ARGS__; }       \
    else TORCH_CHECK(false, "unsupported dtype ", dt);                 \
  } while (0)

at::Tensor mift_mask_scale(const at::Tensor& x, double p, int64_t seed, const c10::optional<at::Tensor>& out,
                           bool accumulate) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "mask_scale: contiguous GPU tensor");
  at::Tensor y = out ? *out : at::empty_like(x);
  TORCH_CHECK(y.is_contiguous() && y.numel() == x.numel() && y.scalar_type() == x.scalar_type(), "mask_scale: out");
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const int64_t n = x.numel();
  float inv = p > 0 ? mift_inv_keep(p) : 1.f;
  DISPATCH_16(x.scalar_type(), mask_scale_kernel<T><<<ew_grid(n), 256, 0, st>>>((const T*)x.data_ptr(), (T*)y.data_ptr(), n,
                                                                                 (uint64_t)seed, mift_seed_step(), thr_of(p), inv,
                                                                                 accumulate ? 1 : 0));
  return y;
}

at::Tensor mift_act_bwd(const at::Tensor& g, const at::Tensor& z, int64_t act, double p, int64_t seed) {
  TORCH_CHECK(g.is_contiguous() && z.is_contiguous() && g.numel() == z.numel(), "act_bwd: shapes");
  auto out = at::empty_like(g);
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const int64_t n = g.numel();
  float inv = p > 0 ? mift_inv_keep(p) : 1.f;
  DISPATCH_16(g.scalar_type(), act_bwd_kernel<T><<<ew_grid(n), 256, 0, st>>>((const T*)g.data_ptr(), (const T*)z.data_ptr(),
                                                                              (T*)out.data_ptr(), n, (int)act,
                                                                              (uint64_t)seed, mift_seed_step(), thr_of(p), inv));
  return out;
}

at::Tensor mift_embed_fwd(const at::Tensor& ids, const c10::optional<at::Tensor>& pos, const at::Tensor& wte,
                          const c10::optional<at::Tensor>& wpe, int64_t pos_offset, double p, int64_t seed,
                          at::ScalarType out_dtype) {
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous(), "embed: int64 ids");
  const int D = wte.size(1);
  TORCH_CHECK(D % 8 == 0, "embed: D % 8");
  const int S = ids.size(-1);
  const int64_t rows = ids.numel();
  auto h = at::empty({rows, D}, wte.options().dtype(out_dtype));
  if (rows == 0) return h;
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  float inv = p > 0 ? mift_inv_keep(p) : 1.f;
  TORCH_CHECK(wte.scalar_type() == out_dtype, "embed: table dtype must equal out dtype");
  DISPATCH_16(out_dtype, embed_kernel<T, T><<<rows, 256, 0, st>>>(
                             ids.data_ptr<int64_t>(), pos ? pos->data_ptr<int64_t>() : nullptr, (const T*)wte.data_ptr(),
                             wpe ? (const T*)wpe->data_ptr() : nullptr, (T*)h.data_ptr(), S, D, (int)pos_offset,
                             (uint64_t)seed, mift_seed_step(), thr_of(p), inv, (int64_t)wte.size(0),
                             wpe ? (int64_t)wpe->size(0) : (int64_t)0));
  return h;
}

std::vector<at::Tensor> mift_mask_positions(const at::Tensor& mask) {
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == at::kLong && mask.dim() == 2 && mask.is_contiguous(),
              "mask_positions: int64 [B, S] contiguous mask");
  const int B = mask.size(0), S = mask.size(1);
  auto pos = at::empty({B, S}, mask.options());
  auto kv = at::empty({B}, mask.options().dtype(at::kInt));
  if (B == 0 || S == 0) return {pos, kv};
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  mask_positions_kernel<<<B, 256, 0, st>>>(mask.data_ptr<int64_t>(), S, pos.data_ptr<int64_t>(), kv.data_ptr<int>());
  return {pos, kv};
}

std::vector<at::Tensor> mift_pack_lora(const at::Tensor& A, const at::Tensor& B, double a_scale,
                                       at::ScalarType dt) {
  TORCH_CHECK(A.scalar_type() == at::kFloat && B.scalar_type() == at::kFloat, "pack_lora: fp32 masters");
  const int r = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == r && r <= 32, "pack_lora: rank <= 32");
  auto A32 = at::empty({32, K}, A.options().dtype(dt));
  auto B32 = at::empty({N, 32}, A.options().dtype(dt));
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const int64_t tot = 32LL * K + (int64_t)N * 32;
  const int grid = (tot + 255) / 256;
  if (dt == at::kBFloat16)
    pack_lora_kernel<bf16><<<grid, 256, 0, st>>>(A.data_ptr<float>(), B.data_ptr<float>(), (bf16*)A32.data_ptr(),
                                                 (bf16*)B32.data_ptr(), r, K, N, (float)a_scale);
  else
    pack_lora_kernel<fp16><<<grid, 256, 0, st>>>(A.data_ptr<float>(), B.data_ptr<float>(), (fp16*)A32.data_ptr(),
                                                 (fp16*)B32.data_ptr(), r, K, N, (float)a_scale);
  return {A32, B32};
}
