// K4: LayerNorm forward / backward (GPT-2 ln_1/ln_2/ln_f, OPT pre-LN,
// BERT post-LN).  Reference op: HF nn.LayerNorm (eps 1e-5 GPT-2/OPT,
// 1e-12 BERT) — see SURVEY §2.4 K4.
//
// Mapping: one wave per row, 4 rows per 256-thread block, the row held in
// registers (VEC=4 elements per lane per pass, NIT passes), so x is read
// exactly once from HBM.  Statistics in fp32 (two-pass mean/var on the
// register copy: no E[x^2]-E[x]^2 cancellation).
//
// Backward fuses (a) the residual-stream gradient add (dx += dres) and
// (b) the dropout-masked copy for the parallel branch of a pre-LN block
// (dbranch = keep(seed, idx) * dx / (1-p)), so the block backward reads the
// residual gradient once instead of three times.
#include "common.h"
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

namespace {

constexpr int VEC = 4;

template <typename T>
MIFT_HD void ld4(const T* p, float* o) {
  if constexpr (sizeof(T) == 4) {
    float4 v = *reinterpret_cast<const float4*>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else {
    short4_ v = *reinterpret_cast<const short4_*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) { short s = v[i]; T t; __builtin_memcpy(&t, &s, 2); o[i] = (float)t; }
  }
}
template <typename T>
MIFT_HD void st4(T* p, const float* o) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  } else {
    short4_ v;
#pragma unroll
    for (int i = 0; i < 4; ++i) { T t = (T)o[i]; short s; __builtin_memcpy(&s, &t, 2); v[i] = s; }
    *reinterpret_cast<short4_*>(p) = v;
  }
}

template <typename T, typename W, int NIT>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const W* __restrict__ w,
                                                     const W* __restrict__ b, T* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* xr = x + (size_t)row * D;
  float v[NIT][VEC];
  float s = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    int c = (it * 64 + lane) * VEC;
    if (c < D) {
      ld4(xr + c, v[it]);
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
    int c = (it * 64 + lane) * VEC;
    if (c < D) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) { float d = v[it][i] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / D + eps);
  T* yr = y + (size_t)row * D;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    int c = (it * 64 + lane) * VEC;
    if (c < D) {
      float wv[VEC], bv[VEC], o[VEC];
      ld4(w + c, wv);
      ld4(b + c, bv);
#pragma unroll
      for (int i = 0; i < VEC; ++i) o[i] = (v[it][i] - mean) * rstd * wv[i] + bv[i];
      st4(yr + c, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * w
template <typename T, typename W, int NIT>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const W* __restrict__ w, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, const T* __restrict__ dres,
                                                     T* __restrict__ dx, T* __restrict__ dbranch,
                                                     float* __restrict__ dw, float* __restrict__ db, int M, int D,
                                                     uint64_t seed, const int64_t* __restrict__ sstep, uint32_t thr, float inv_keep) {
  seed = mift_seed(seed, sstep);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float mean = mean_in[row], rstd = rstd_in[row];
  const T* xr = x + (size_t)row * D;
  const T* dyr = dy + (size_t)row * D;
  float xh[NIT][VEC], g[NIT][VEC];
  float sg = 0.f, sgx = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    int c = (it * 64 + lane) * VEC;
    if (c < D) {
      float xv[VEC], dv[VEC], wv[VEC];
      ld4(xr + c, xv);
      ld4(dyr + c, dv);
      ld4(w + c, wv);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        xh[it][i] = (xv[i] - mean) * rstd;
        g[it][i] = dv[i] * wv[i];
        sg += g[it][i];
        sgx += g[it][i] * xh[it][i];
      }
    }
  }
  sg = wave_sum(sg) / D;
  sgx = wave_sum(sgx) / D;
  T* dxr = dx + (size_t)row * D;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    int c = (it * 64 + lane) * VEC;
    if (c < D) {
      float o[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i) o[i] = rstd * (g[it][i] - sg - xh[it][i] * sgx);
      if (dres != nullptr) {
        float r[VEC];
        ld4(dres + (size_t)row * D + c, r);
#pragma unroll
        for (int i = 0; i < VEC; ++i) o[i] += r[i];
      }
      st4(dxr + c, o);
      if (dbranch != nullptr) {
        float m[VEC];
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          uint64_t idx = (uint64_t)row * D + c + i;
          m[i] = mift_keep(seed, idx, thr) ? o[i] * inv_keep : 0.f;
        }
        st4(dbranch + (size_t)row * D + c, m);
      }
    }
  }
}

// dgamma / dbeta (trainable LayerNorm, e.g. full fine-tuning), deterministic: pass 1 sums a chunk
// of LN_WG_ROWS rows per (column, chunk) in row order, pass 2 sums the chunks in order — no
// float atomics.
constexpr int LN_WG_ROWS = 128;
template <typename T>
__global__ __launch_bounds__(256) void ln_wgrad_partial_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ rstd, float* __restrict__ pw,
                                                               float* __restrict__ pb, int M, int D) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= D) return;
  const int r0 = blockIdx.y * LN_WG_ROWS, r1 = min(M, r0 + LN_WG_ROWS);
  float sw = 0.f, sb = 0.f;
  for (int r = r0; r < r1; ++r) {
    const float g = (float)dy[(size_t)r * D + c];
    sw += g * ((float)x[(size_t)r * D + c] - mean[r]) * rstd[r];
    sb += g;
  }
  pw[(size_t)blockIdx.y * D + c] = sw;
  pb[(size_t)blockIdx.y * D + c] = sb;
}

__global__ __launch_bounds__(256) void ln_wgrad_reduce_kernel(const float* __restrict__ pw, const float* __restrict__ pb,
                                                              float* __restrict__ dw, float* __restrict__ db, int nch,
                                                              int D) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= D) return;
  float sw = 0.f, sb = 0.f;
  for (int k = 0; k < nch; ++k) {
    sw += pw[(size_t)k * D + c];
    sb += pb[(size_t)k * D + c];
  }
  dw[c] = sw;
  db[c] = sb;
}

// ---- 16-B vector form (16-bit T, D % (8·LPR) == 0): RPW rows per wave, LPR = 64/RPW lanes per row,
// 8 elements per lane per pass.  The 4-element form above issues 8-B loads and, at distilgpt2's
// D = 768, three passes of one row per wave; ln_bwd read x, dy, w and dres that way at ~4.4 TB/s
// (11.5-14.5 us per call at M = 8192).  Two rows per wave at D <= 1024 keep every lane busy with
// whole 16-B pieces (D = 768: 32 lanes x 3 passes).  Same two-pass fp32 statistics.
template <int LPR>
MIFT_HD float lpr_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T, typename W, int RPW, int NIT>
__global__ __launch_bounds__(256) void ln_fwd8_kernel(const T* __restrict__ x, const W* __restrict__ w,
                                                      const W* __restrict__ b, T* __restrict__ y,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                      int M, int D, float eps) {
  constexpr int LPR = 64 / RPW;
  const int lane = threadIdx.x & 63, l = lane % LPR;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= M) return;  // wave-uniform
  const int row = min(row0 + lane / LPR, M - 1);
  const bool live = row0 + lane / LPR < M;
  const T* xr = x + (size_t)row * D + l * 8;
  short8 xv[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) xv[it] = *reinterpret_cast<const short8*>(xr + it * LPR * 8);
  float s = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    float v[8];
    unpack8<T>(xv[it], v);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[e];
  }
  const float mean = lpr_sum<LPR>(s) / D;
  float q = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    float v[8];
    unpack8<T>(xv[it], v);
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float d = v[e] - mean; q += d * d; }
  }
  const float rstd = rsqrtf(lpr_sum<LPR>(q) / D + eps);
  T* yr = y + (size_t)row * D + l * 8;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = (it * LPR + l) * 8;
    float v[8], wv[8], bv[8];
    unpack8<T>(xv[it], v);
    load8<W>(w + c, wv);
    load8<W>(b + c, bv);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (v[e] - mean) * rstd * wv[e] + bv[e];
    if (live) store8<T>(yr + it * LPR * 8, v);
  }
  if (live && l == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) (+ dres),  g = dy * w
template <typename T, typename W, int RPW, int NIT>
__global__ __launch_bounds__(256) void ln_bwd8_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                      const W* __restrict__ w, const float* __restrict__ mean_in,
                                                      const float* __restrict__ rstd_in, const T* __restrict__ dres,
                                                      T* __restrict__ dx, int M, int D) {
  constexpr int LPR = 64 / RPW;
  const int lane = threadIdx.x & 63, l = lane % LPR;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= M) return;  // wave-uniform
  const int row = min(row0 + lane / LPR, M - 1);
  const bool live = row0 + lane / LPR < M;
  const size_t base = (size_t)row * D + l * 8;
  short8 xv[NIT], gv[NIT], rv[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    xv[it] = *reinterpret_cast<const short8*>(x + base + it * LPR * 8);
    gv[it] = *reinterpret_cast<const short8*>(dy + base + it * LPR * 8);
    if (dres != nullptr) rv[it] = *reinterpret_cast<const short8*>(dres + base + it * LPR * 8);
  }
  const float mean = mean_in[row], rstd = rstd_in[row];
  float sg = 0.f, sgx = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = (it * LPR + l) * 8;
    float xf[8], df[8], wv[8];
    unpack8<T>(xv[it], xf);
    unpack8<T>(gv[it], df);
    load8<W>(w + c, wv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float g = df[e] * wv[e];
      sg += g;
      sgx += g * ((xf[e] - mean) * rstd);
    }
  }
  sg = lpr_sum<LPR>(sg) / D;
  sgx = lpr_sum<LPR>(sgx) / D;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = (it * LPR + l) * 8;
    float xf[8], df[8], wv[8], o[8];
    unpack8<T>(xv[it], xf);
    unpack8<T>(gv[it], df);
    load8<W>(w + c, wv);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = rstd * (df[e] * wv[e] - sg - (xf[e] - mean) * rstd * sgx);
    if (dres != nullptr) {
      float r[8];
      unpack8<T>(rv[it], r);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += r[e];
    }
    if (live) store8<T>(dx + base + it * LPR * 8, o);
  }
}

// (RPW, NIT) of the 16-B form for this D, or false (4-element form)
inline bool ln8_shape(int D, int& rpw, int& nit) {
  const char* e = getenv("MIFT_LN_V");  // 1 = the 4-element kernels (A/B knob, read per call)
  if (e && atoi(e) == 1) return false;
  rpw = D <= 1024 ? 2 : 1;
  const int per = 8 * (64 / rpw);
  if (D % per != 0) return false;
  nit = D / per;
  return nit == 1 || nit == 2 || nit == 3 || nit == 4 || nit == 5 || nit == 6 || nit == 8 || nit == 10;
}

inline bool a16(const at::Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; }

template <int RPW, typename F>
void ln8_nit(int nit, F&& f) {
  switch (nit) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 3: f(std::integral_constant<int, 3>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 5: f(std::integral_constant<int, 5>{}); break;
    case 6: f(std::integral_constant<int, 6>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    default: f(std::integral_constant<int, 10>{}); break;  // ln8_shape admits no other value
  }
}

template <typename T, typename W, int N>
void ln_fwd_launch(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b, at::Tensor& y, at::Tensor& mean,
                   at::Tensor& rstd, int M, int D, float eps, hipStream_t st) {
  dim3 grid((M + 3) / 4), block(256);
  ln_fwd_kernel<T, W, N><<<grid, block, 0, st>>>((const T*)x.data_ptr(), (const W*)w.data_ptr(),
                                                 (const W*)b.data_ptr(), (T*)y.data_ptr(), mean.data_ptr<float>(),
                                                 rstd.data_ptr<float>(), M, D, eps);
}

template <typename T, typename W>
void launch_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b, at::Tensor& y, at::Tensor& mean,
                at::Tensor& rstd, int M, int D, float eps, hipStream_t st) {
  if (M == 0) return;
  int rpw8 = 0, nit8 = 0;
  if constexpr (sizeof(T) == 2) {
    if (ln8_shape(D, rpw8, nit8) && a16(x) && a16(w) && a16(b) && a16(y)) {
      auto go = [&](auto rpwc) {
        constexpr int RPW = decltype(rpwc)::value;
        ln8_nit<RPW>(nit8, [&](auto nc) {
          constexpr int NIT = decltype(nc)::value;
          const int waves = (M + RPW - 1) / RPW;
          ln_fwd8_kernel<T, W, RPW, NIT><<<(waves + 3) / 4, 256, 0, st>>>(
              (const T*)x.data_ptr(), (const W*)w.data_ptr(), (const W*)b.data_ptr(), (T*)y.data_ptr(),
              mean.data_ptr<float>(), rstd.data_ptr<float>(), M, D, eps);
        });
      };
      if (rpw8 == 2) go(std::integral_constant<int, 2>{});
      else go(std::integral_constant<int, 1>{});
      return;
    }
  }
  int nit = (D + 255) / 256;
  if (nit <= 1) ln_fwd_launch<T, W, 1>(x, w, b, y, mean, rstd, M, D, eps, st);
  else if (nit <= 2) ln_fwd_launch<T, W, 2>(x, w, b, y, mean, rstd, M, D, eps, st);
  else if (nit <= 3) ln_fwd_launch<T, W, 3>(x, w, b, y, mean, rstd, M, D, eps, st);
  else if (nit <= 4) ln_fwd_launch<T, W, 4>(x, w, b, y, mean, rstd, M, D, eps, st);
  else if (nit <= 6) ln_fwd_launch<T, W, 6>(x, w, b, y, mean, rstd, M, D, eps, st);
  else if (nit <= 8) ln_fwd_launch<T, W, 8>(x, w, b, y, mean, rstd, M, D, eps, st);
  else if (nit <= 10) ln_fwd_launch<T, W, 10>(x, w, b, y, mean, rstd, M, D, eps, st);
  else if (nit <= 12) ln_fwd_launch<T, W, 12>(x, w, b, y, mean, rstd, M, D, eps, st);
  else if (nit <= 16) ln_fwd_launch<T, W, 16>(x, w, b, y, mean, rstd, M, D, eps, st);
  else if (nit <= 32) ln_fwd_launch<T, W, 32>(x, w, b, y, mean, rstd, M, D, eps, st);
  else TORCH_CHECK(false, "layer_norm: hidden size too large: ", D);
}

template <typename T, typename W, int N>
void ln_bwd_launch(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w, const at::Tensor& mean,
                   const at::Tensor& rstd, const c10::optional<at::Tensor>& dres, at::Tensor& dx,
                   const c10::optional<at::Tensor>& dbranch, const c10::optional<at::Tensor>& dw,
                   const c10::optional<at::Tensor>& db, int M, int D, uint64_t seed, uint32_t thr, float inv_keep,
                   hipStream_t st) {
  dim3 grid((M + 3) / 4), block(256);
  ln_bwd_kernel<T, W, N><<<grid, block, 0, st>>>(
      (const T*)dy.data_ptr(), (const T*)x.data_ptr(), (const W*)w.data_ptr(), mean.data_ptr<float>(),
      rstd.data_ptr<float>(), dres ? (const T*)dres->data_ptr() : nullptr, (T*)dx.data_ptr(),
      dbranch ? (T*)dbranch->data_ptr() : nullptr, dw ? dw->data_ptr<float>() : nullptr,
      db ? db->data_ptr<float>() : nullptr, M, D, seed, mift_seed_step(), thr, inv_keep);
}

template <typename T, typename W>
void launch_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w, const at::Tensor& mean,
                const at::Tensor& rstd, const c10::optional<at::Tensor>& dres, at::Tensor& dx,
                const c10::optional<at::Tensor>& dbranch, const c10::optional<at::Tensor>& dw,
                const c10::optional<at::Tensor>& db, int M, int D, uint64_t seed, uint32_t thr, float inv_keep,
                hipStream_t st) {
  if (M == 0) return;
  int rpw8 = 0, nit8 = 0;
  if constexpr (sizeof(T) == 2) {
    if (!dbranch && ln8_shape(D, rpw8, nit8) && a16(dy) && a16(x) && a16(w) && a16(dx) && (!dres || a16(*dres))) {
      auto go = [&](auto rpwc) {
        constexpr int RPW = decltype(rpwc)::value;
        ln8_nit<RPW>(nit8, [&](auto nc) {
          constexpr int NIT = decltype(nc)::value;
          const int waves = (M + RPW - 1) / RPW;
          ln_bwd8_kernel<T, W, RPW, NIT><<<(waves + 3) / 4, 256, 0, st>>>(
              (const T*)dy.data_ptr(), (const T*)x.data_ptr(), (const W*)w.data_ptr(), mean.data_ptr<float>(),
              rstd.data_ptr<float>(), dres ? (const T*)dres->data_ptr() : nullptr, (T*)dx.data_ptr(), M, D);
        });
      };
      if (rpw8 == 2) go(std::integral_constant<int, 2>{});
      else go(std::integral_constant<int, 1>{});
      return;
    }
  }
  int nit = (D + 255) / 256;
  if (nit <= 1) ln_bwd_launch<T, W, 1>(dy, x, w, mean, rstd, dres, dx, dbranch, dw, db, M, D, seed, thr, inv_keep, st);
  else if (nit <= 2) ln_bwd_launch<T, W, 2>(dy, x, w, mean, rstd, dres, dx, dbranch, dw, db, M, D, seed, thr, inv_keep, st);
  else if (nit <= 3) ln_bwd_launch<T, W, 3>(dy, x, w, mean, rstd, dres, dx, dbranch, dw, db, M, D, seed, thr, inv_keep, st);
  else if (nit <= 4) ln_bwd_launch<T, W, 4>(dy, x, w, mean, rstd, dres, dx, dbranch, dw, db, M, D, seed, thr, inv_keep, st);
  else if (nit <= 6) ln_bwd_launch<T, W, 6>(dy, x, w, mean, rstd, dres, dx, dbranch, dw, db, M, D, seed, thr, inv_keep, st);
  else if (nit <= 8) ln_bwd_launch<T, W, 8>(dy, x, w, mean, rstd, dres, dx, dbranch, dw, db, M, D, seed, thr, inv_keep, st);
  else if (nit <= 10) ln_bwd_launch<T, W, 10>(dy, x, w, mean, rstd, dres, dx, dbranch, dw, db, M, D, seed, thr, inv_keep, st);
  else if (nit <= 12) ln_bwd_launch<T, W, 12>(dy, x, w, mean, rstd, dres, dx, dbranch, dw, db, M, D, seed, thr, inv_keep, st);
  else if (nit <= 16) ln_bwd_launch<T, W, 16>(dy, x, w, mean, rstd, dres, dx, dbranch, dw, db, M, D, seed, thr, inv_keep, st);
  else if (nit <= 32) ln_bwd_launch<T, W, 32>(dy, x, w, mean, rstd, dres, dx, dbranch, dw, db, M, D, seed, thr, inv_keep, st);
  else TORCH_CHECK(false, "layer_norm_bwd: hidden size too large: ", D);
}

}  // namespace

#define DISPATCH_TW(xdt, wdt, ...)                                                                   \
  do {                                                                                               \
    if (xdt == at::kBFloat16 && wdt == at::kBFloat16) { using T = bf16; using W = bf16; __VA_ARGS__; } \
    else if (xdt == at::kBFloat16 && wdt == at::kFloat) { using T = bf16; using W = float; __VA_ARGS__; } \
    else if (xdt == at::kHalf && wdt == at::kHalf) { using T = fp16; using W = fp16; __VA_ARGS__; }   \
    else if (xdt == at::kHalf && wdt == at::kFloat) { using T = fp16; using W = float; __VA_ARGS__; }  \
    else if (xdt == at::kFloat && wdt == at::kFloat) { using T = float; using W = float; __VA_ARGS__; } \
    else TORCH_CHECK(false, "layer_norm: unsupported dtypes ", xdt, " / ", wdt);                  \
  } while (0)

std::vector<at::Tensor> mift_layer_norm_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b,
                                            double eps) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "layer_norm: x must be contiguous GPU");
  const int D = x.size(-1);
  const int M = x.numel() / D;
  TORCH_CHECK(D % 4 == 0, "layer_norm: D must be a multiple of 4");
  TORCH_CHECK(w.numel() == D && b.numel() == D, "layer_norm: weight/bias size");
  auto y = at::empty_like(x);
  auto mean = at::empty({M}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({M}, x.options().dtype(at::kFloat));
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  DISPATCH_TW(x.scalar_type(), w.scalar_type(), launch_fwd<T, W>(x, w, b, y, mean, rstd, M, D, (float)eps, st));
  return {y, mean, rstd};
}

std::vector<at::Tensor> mift_layer_norm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                            const at::Tensor& mean, const at::Tensor& rstd,
                                            const c10::optional<at::Tensor>& dres, bool want_branch, double p,
                                            int64_t seed, bool want_wgrad) {
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous(), "layer_norm_bwd: contiguous inputs");
  const int D = x.size(-1);
  const int M = x.numel() / D;
  auto dx = at::empty_like(x);
  c10::optional<at::Tensor> dbranch, dw, db;
  if (want_branch) dbranch = at::empty_like(x);
  uint32_t thr = mift_thr16(p);
  float inv_keep = p > 0 ? mift_inv_keep(p) : 1.f;
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const c10::optional<at::Tensor> none;
  DISPATCH_TW(x.scalar_type(), w.scalar_type(),
              launch_bwd<T, W>(dy, x, w, mean, rstd, dres, dx, dbranch, none, none, M, D, (uint64_t)seed, thr,
                               inv_keep, st));
  if (want_wgrad) {
    dw = at::empty({D}, x.options().dtype(at::kFloat));
    db = at::empty({D}, x.options().dtype(at::kFloat));
    const int nch = std::max(1, (M + LN_WG_ROWS - 1) / LN_WG_ROWS);
    auto part = at::empty({2, (int64_t)nch, D}, x.options().dtype(at::kFloat));
    float* pw = part.data_ptr<float>();
    float* pb = pw + (size_t)nch * D;
    const dim3 g1((D + 255) / 256, nch);
    if (M > 0) {
      if (x.scalar_type() == at::kBFloat16)
        ln_wgrad_partial_kernel<bf16><<<g1, 256, 0, st>>>((const bf16*)dy.data_ptr(), (const bf16*)x.data_ptr(),
                                                          mean.data_ptr<float>(), rstd.data_ptr<float>(), pw, pb, M, D);
      else if (x.scalar_type() == at::kHalf)
        ln_wgrad_partial_kernel<fp16><<<g1, 256, 0, st>>>((const fp16*)dy.data_ptr(), (const fp16*)x.data_ptr(),
                                                          mean.data_ptr<float>(), rstd.data_ptr<float>(), pw, pb, M, D);
      else
        ln_wgrad_partial_kernel<float><<<g1, 256, 0, st>>>(dy.data_ptr<float>(), x.data_ptr<float>(),
                                                           mean.data_ptr<float>(), rstd.data_ptr<float>(), pw, pb, M, D);
      ln_wgrad_reduce_kernel<<<(D + 255) / 256, 256, 0, st>>>(pw, pb, dw->data_ptr<float>(), db->data_ptr<float>(), nch, D);
    } else {
      dw->zero_();
      db->zero_();
    }
  }
  std::vector<at::Tensor> out{dx};
  out.push_back(want_branch ? *dbranch : at::Tensor());
  out.push_back(want_wgrad ? *dw : at::Tensor());
  out.push_back(want_wgrad ? *db : at::Tensor());
  return out;
}
