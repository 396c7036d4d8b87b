// Row-wise producers fused with the rank-r LoRA projection.
//
// A LoRA linear needs the tall-skinny product P = alpha · f(x) · W^T
// ([M,32], W = [32,D], only the first r <= 32 rows non-zero) next to its base
// GEMM: T = s·drop(x)·A^T in the forward and dT = s·gz·B in the backward
// (mift.ops.fused.AdapterOps).  When x is produced by a one-wave-per-row
// kernel the row is already in registers, so the product costs a few FMAs
// per element plus one cross-lane reduction instead of a separate launch
// that re-reads x (the stand-alone lora_proj kernel, csrc/kernels/lora.hip):
//
//   ln_fwd_proj    y = LN(x); T = alpha·drop(y)·W^T        (GPT-2 ln_1 -> c_attn)
//   mask_proj      y = keep⊙x/(1-p) (residual-dropout bwd); P = alpha·y·W^T
//                  (grad of attn.c_proj / mlp.c_proj outputs -> dT)
//
// Numerics match lora_proj: the projection consumes the 16-bit value the
// consumer GEMM sees (y rounded to T); dropped elements are zeroed and the
// 1/(1-p) scale is applied once to the fp32 sums (folded into alpha by the
// host), accumulation is fp32, the output rounded once.
//
// Cross-lane reduction of the LR per-lane partial sums: a reduce-scatter
// butterfly (each xor step sends the half of the partials the lane does not
// keep: LR/2 + LR/4 + ... shuffles) followed by a plain butterfly over the
// remaining lane bits — 10 shuffles for LR = 8 instead of 8 × 6.
#include "common.h"
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

namespace {

constexpr int VEC = 4;

template <typename T>
MIFT_HD void ld4(const T* p, float* o) {
  short4_ v = *reinterpret_cast<const short4_*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) { short s = v[i]; T t; __builtin_memcpy(&t, &s, 2); o[i] = (float)t; }
}
template <typename W>
MIFT_HD void ldw4(const W* p, float* o) {
  if constexpr (sizeof(W) == 4) {
    float4 v = *reinterpret_cast<const float4*>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else {
    ld4<W>(p, o);
  }
}
template <typename T>
MIFT_HD void st4(T* p, const float* o) {
  short4_ v;
#pragma unroll
  for (int i = 0; i < 4; ++i) { T t = (T)o[i]; short s; __builtin_memcpy(&s, &t, 2); v[i] = s; }
  *reinterpret_cast<short4_*>(p) = v;
}
template <typename T>
MIFT_HD float rnd(float v) { return (float)(T)v; }

// acc + x·w over 4 packed 16-bit values with two v_dot2_f32_{bf16,f16} (no unpacking to fp32: the
// per-element converts of the weight rows were most of these kernels' vector instructions)
typedef __bf16 bf16x2_ __attribute__((ext_vector_type(2)));
typedef _Float16 fp16x2_ __attribute__((ext_vector_type(2)));
template <typename T>
MIFT_HD float dot4(short4_ x, short4_ w, float acc) {
  if constexpr (std::is_same<T, bf16>::value) {
    bf16x2_ x0, x1, w0, w1;
    __builtin_memcpy(&x0, &x, 4);
    __builtin_memcpy(&x1, reinterpret_cast<const char*>(&x) + 4, 4);
    __builtin_memcpy(&w0, &w, 4);
    __builtin_memcpy(&w1, reinterpret_cast<const char*>(&w) + 4, 4);
    acc = __builtin_amdgcn_fdot2_f32_bf16(x0, w0, acc, false);
    return __builtin_amdgcn_fdot2_f32_bf16(x1, w1, acc, false);
  } else {
    fp16x2_ x0, x1, w0, w1;
    __builtin_memcpy(&x0, &x, 4);
    __builtin_memcpy(&x1, reinterpret_cast<const char*>(&x) + 4, 4);
    __builtin_memcpy(&w0, &w, 4);
    __builtin_memcpy(&w1, reinterpret_cast<const char*>(&w) + 4, 4);
    acc = __builtin_amdgcn_fdot2(x0, w0, acc, false);
    return __builtin_amdgcn_fdot2(x1, w1, acc, false);
  }
}
template <typename T>
MIFT_HD short4_ pack4(const float* o) {
  short4_ v;
#pragma unroll
  for (int i = 0; i < 4; ++i) { T t = (T)o[i]; short s; __builtin_memcpy(&s, &t, 2); v[i] = s; }
  return v;
}

// acc[0..LR) partial sums per lane -> out[row, 0..32) (cols >= LR zero), times alpha
template <typename T, int LR>
MIFT_HD void reduce_store(float (&acc)[LR], T* out_row, int lane, float alpha) {
  int n = LR;
  int off = 32;
#pragma unroll
  for (int step = 0; step < 5; ++step) {
    if (n > 1) {
      const bool upper = (lane & off) != 0;
      n >>= 1;
#pragma unroll
      for (int j = 0; j < LR / 2; ++j) {
        if (j < n) {
          const float send = upper ? acc[j] : acc[j + n];
          const float keep = upper ? acc[j + n] : acc[j];
          acc[j] = keep + __shfl_xor(send, off, 64);
        }
      }
      off >>= 1;
    }
  }
  // n == 1: acc[0] holds index lane / (64 / LR) partially summed over the remaining lane bits
#pragma unroll
  for (int o = 32 / LR; o > 0; o >>= 1) acc[0] += __shfl_xor(acc[0], o, 64);
  const float v = __shfl(acc[0], (lane % LR) * (64 / LR), 64);
  if (lane < 32) out_row[lane] = (T)(lane < LR ? v * alpha : 0.f);
}

template <typename T, typename W, int NIT, int LR>
__global__ __launch_bounds__(256) void ln_fwd_proj_kernel(const T* __restrict__ x, const W* __restrict__ w,
                                                          const W* __restrict__ b, T* __restrict__ y,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                          const T* __restrict__ pw, T* __restrict__ pout, int M, int D,
                                                          float eps, float alpha, uint64_t seed, const int64_t* __restrict__ sstep, uint32_t thr,
                                                          float inv_keep) {
  seed = mift_seed(seed, sstep);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* xr = x + (size_t)row * D;
  float v[NIT][VEC];
  float s = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = (it * 64 + lane) * VEC;
    if (c < D) {
      ld4<T>(xr + c, v[it]);
#pragma unroll
      for (int i = 0; i < VEC; ++i) s += v[it][i];
    } else {
#pragma unroll
      for (int i = 0; i < VEC; ++i) v[it][i] = 0.f;
    }
  }
  const float mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = (it * 64 + lane) * VEC;
    if (c < D) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) { const float d = v[it][i] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / D + eps);
  T* yr = y + (size_t)row * D;
  float acc[LR];
#pragma unroll
  for (int j = 0; j < LR; ++j) acc[j] = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = (it * 64 + lane) * VEC;
    if (c < D) {
      float wv[VEC], bv[VEC], o[VEC];
      ldw4<W>(w + c, wv);
      ldw4<W>(b + c, bv);
#pragma unroll
      for (int i = 0; i < VEC; ++i) o[i] = (v[it][i] - mean) * rstd * wv[i] + bv[i];
      short4_ yb = pack4<T>(o);  // the 16-bit y the consumer GEMM sees
      *reinterpret_cast<short4_*>(yr + c) = yb;
      if (thr != 0) {  // dropped elements zeroed; 1/(1-p) folded into alpha by the host
        bool kp[VEC];
        mift_keep4(seed, (uint64_t)row * D + c, thr, kp);
#pragma unroll
        for (int i = 0; i < VEC; ++i) yb[i] = kp[i] ? yb[i] : (short)0;
      }
#pragma unroll
      for (int j = 0; j < LR; ++j)
        acc[j] = dot4<T>(yb, *reinterpret_cast<const short4_*>(pw + (size_t)j * D + c), acc[j]);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
  reduce_store<T, LR>(acc, pout + (size_t)row * 32, lane, alpha);
}

template <typename T, int NIT, int LR>
__global__ __launch_bounds__(256) void mask_proj_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                        const T* __restrict__ pw, T* __restrict__ pout, int M, int D,
                                                        float alpha, uint64_t seed, const int64_t* __restrict__ sstep, uint32_t thr, float inv_keep) {
  seed = mift_seed(seed, sstep);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* xr = x + (size_t)row * D;
  T* yr = y + (size_t)row * D;
  float acc[LR];
#pragma unroll
  for (int j = 0; j < LR; ++j) acc[j] = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = (it * 64 + lane) * VEC;
    if (c < D) {
      short4_ yb = *reinterpret_cast<const short4_*>(xr + c);
      if (thr != 0) {
        float v[VEC];
        ld4<T>(xr + c, v);
        bool kp[VEC];
        mift_keep4(seed, (uint64_t)row * D + c, thr, kp);
#pragma unroll
        for (int i = 0; i < VEC; ++i) v[i] = kp[i] ? v[i] * inv_keep : 0.f;
        yb = pack4<T>(v);  // the 16-bit y written out is the one projected
        *reinterpret_cast<short4_*>(yr + c) = yb;
      }
#pragma unroll
      for (int j = 0; j < LR; ++j)
        acc[j] = dot4<T>(yb, *reinterpret_cast<const short4_*>(pw + (size_t)j * D + c), acc[j]);
    }
  }
  reduce_store<T, LR>(acc, pout + (size_t)row * 32, lane, alpha);
}

template <int LR, typename F>
void by_nit(int D, F&& f) {
  const int nit = (D + 255) / 256;
  if (nit <= 1) f(std::integral_constant<int, 1>{});
  else if (nit <= 2) f(std::integral_constant<int, 2>{});
  else if (nit <= 3) f(std::integral_constant<int, 3>{});
  else if (nit <= 4) f(std::integral_constant<int, 4>{});
  else if (nit <= 8) f(std::integral_constant<int, 8>{});
  else if (nit <= 10) f(std::integral_constant<int, 10>{});
  else if (nit <= 16) f(std::integral_constant<int, 16>{});
  else TORCH_CHECK(false, "rowproj: hidden size too large: ", D);
}

template <typename F>
void by_rank(int r, F&& f) {
  if (r <= 8) f(std::integral_constant<int, 8>{});
  else if (r <= 16) f(std::integral_constant<int, 16>{});
  else f(std::integral_constant<int, 32>{});
}

void check_pw(const at::Tensor& x, const at::Tensor& pw, int D, int64_t rank) {
  TORCH_CHECK(pw.is_contiguous() && pw.dim() == 2 && pw.size(0) == 32 && pw.size(1) == D,
              "rowproj: projection weight must be [32, D] contiguous");
  TORCH_CHECK(pw.scalar_type() == x.scalar_type(), "rowproj: projection dtype");
  TORCH_CHECK(rank >= 1 && rank <= 32, "rowproj: rank in [1, 32]");
}

}  // namespace

// (y, mean, rstd, proj[M,32]) = LN(x), alpha·drop(y)·pw^T (only rows < rank of pw may be non-zero)
std::vector<at::Tensor> mift_layer_norm_fwd_proj(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b,
                                                 double eps, const at::Tensor& pw, int64_t rank, double alpha,
                                                 double p, int64_t seed) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "layer_norm_fwd_proj: x must be contiguous GPU");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "layer_norm_fwd_proj: bf16/fp16");
  const int D = x.size(-1);
  const int M = x.numel() / D;
  TORCH_CHECK(D % 4 == 0, "layer_norm_fwd_proj: D must be a multiple of 4");
  TORCH_CHECK(w.numel() == D && b.numel() == D && w.scalar_type() == b.scalar_type(), "layer_norm_fwd_proj: w/b");
  check_pw(x, pw, D, rank);
  auto y = at::empty_like(x);
  auto mean = at::empty({M}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({M}, x.options().dtype(at::kFloat));
  auto pout = at::empty({M, 32}, x.options());
  if (M == 0) return {y, mean, rstd, pout};
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const uint32_t thr = mift_thr16(p);
  const float inv = p > 0 ? mift_inv_keep(p) : 1.f;
  const bool wf32 = w.scalar_type() == at::kFloat;
  TORCH_CHECK(wf32 || w.scalar_type() == x.scalar_type(), "layer_norm_fwd_proj: LN weight dtype");
  auto go = [&](auto tt) {
    using T = decltype(tt);
    by_rank(rank, [&](auto lr) {
      constexpr int LR = decltype(lr)::value;
      by_nit<LR>(D, [&](auto nit) {
        constexpr int NIT = decltype(nit)::value;
        if (wf32)
          ln_fwd_proj_kernel<T, float, NIT, LR><<<(M + 3) / 4, 256, 0, st>>>(
              (const T*)x.data_ptr(), w.data_ptr<float>(), b.data_ptr<float>(), (T*)y.data_ptr(),
              mean.data_ptr<float>(), rstd.data_ptr<float>(), (const T*)pw.data_ptr(), (T*)pout.data_ptr(), M, D,
              (float)eps, (float)alpha * inv, (uint64_t)seed, mift_seed_step(), thr, inv);
        else
          ln_fwd_proj_kernel<T, T, NIT, LR><<<(M + 3) / 4, 256, 0, st>>>(
              (const T*)x.data_ptr(), (const T*)w.data_ptr(), (const T*)b.data_ptr(), (T*)y.data_ptr(),
              mean.data_ptr<float>(), rstd.data_ptr<float>(), (const T*)pw.data_ptr(), (T*)pout.data_ptr(), M, D,
              (float)eps, (float)alpha * inv, (uint64_t)seed, mift_seed_step(), thr, inv);
      });
    });
  };
  if (x.scalar_type() == at::kBFloat16) go(bf16{});
  else go(fp16{});
  return {y, mean, rstd, pout};
}

// (y, proj[M,32]) = keep⊙x/(1-p) (x itself when p == 0: y aliases x), alpha·y·pw^T
std::vector<at::Tensor> mift_mask_proj(const at::Tensor& x, double p, int64_t seed, const at::Tensor& pw,
                                       int64_t rank, double alpha) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 2, "mask_proj: contiguous 2-D GPU x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "mask_proj: bf16/fp16");
  const int D = x.size(1);
  const int M = x.size(0);
  TORCH_CHECK(D % 4 == 0, "mask_proj: D must be a multiple of 4");
  check_pw(x, pw, D, rank);
  const uint32_t thr = mift_thr16(p);
  at::Tensor y = thr != 0 ? at::empty_like(x) : x;
  auto pout = at::empty({M, 32}, x.options());
  if (M == 0) return {y, pout};
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const float inv = p > 0 ? mift_inv_keep(p) : 1.f;
  auto go = [&](auto tt) {
    using T = decltype(tt);
    by_rank(rank, [&](auto lr) {
      constexpr int LR = decltype(lr)::value;
      by_nit<LR>(D, [&](auto nit) {
        constexpr int NIT = decltype(nit)::value;
        mask_proj_kernel<T, NIT, LR><<<(M + 3) / 4, 256, 0, st>>>((const T*)x.data_ptr(), (T*)y.data_ptr(),
                                                                  (const T*)pw.data_ptr(), (T*)pout.data_ptr(), M, D,
                                                                  (float)alpha, (uint64_t)seed, mift_seed_step(), thr, inv);
      });
    });
  };
  if (x.scalar_type() == at::kBFloat16) go(bf16{});
  else go(fp16{});
  return {y, pout};
}
