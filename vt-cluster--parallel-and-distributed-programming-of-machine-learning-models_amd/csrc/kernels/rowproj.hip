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

// ---- MFMA form (D = 32·NK): one NW-wave block per 16 rows (NW = 4 / 8 / 16 by width, by_nk) ----
// The one-wave-per-row kernels above re-read the [LR, D] projection operand from cache for every
// row and do LR dot2 per element pair on the VALU: at LR = 32 (OPT's three q/k/v adapters) they
// ran 136 us at M = 16384, D = 768, 10x the LN alone.  Here a block owns a 16-row MFMA A-tile and
// its 4 waves split the k-steps (NK/4 each, 32 columns per k-step): lane (fr = lane & 15,
// g = lane >> 4) of wave w holds row fr's columns 32·s + 8·g .. +7 of the wave's k-steps s, so
//   * row statistics = per-lane partials + 2 cross-lane steps (xor 16, 32) + one LDS exchange of
//     the 4 waves' [16] partials (two for LN: mean, then the centred sum of squares);
//   * the row is normalised / masked in registers and stored as 16-B pieces;
//   * the projection is NK/4 (rank <= 16) or 2·NK/4 MFMA 16x16x32 per wave on weight fragments
//     read straight from global (L2 hits), reduced over the waves through LDS.
// A first version with one wave per 16 rows (whole row per wave) had 2 waves per CU at
// M = 8192 and ran 18.5 us against 7.1 us for the plain LN (latency-bound: one long chain per
// wave).  Same numerics as the row kernels: y rounded to T before it is projected, dropped
// elements zeroed (1/(1-p) folded into alpha by the host for LN), fp32 accumulation.
// MODE: 0 = residual-dropout backward (y = keep·x/(1-p) stored and projected), 1 = LN (y = LN(x)
// stored, LoRA-input dropout on the projection), 2 = plain LoRA projection (lora_proj semantics:
// T = alpha·drop(x)·Wᵀ, nothing stored; replaces lora_proj's 16-row blocks at these widths),
// 3 = LN backward feeding a residual-dropout backward: x = dY of the LN, xin = its input, lw its
// weight, mean_out / rstd_out its saved statistics (read); dh = LN-bwd(dY) + dres is stored (the
// residual-stream gradient), then MODE 0 on the rounded dh (the upstream LoRA linear's dropout and
// dT = s·y·Bᵀ) — the separate MODE 0 pass re-read dh (one launch and 12.6 MB per site at distilgpt2).
template <typename T, typename W, int NK, int NTI, int MODE, int NW>
__global__ __launch_bounds__(NW * 64) void rowproj_mfma_kernel(const T* __restrict__ x, const W* __restrict__ lw,
                                                           const W* __restrict__ lb, T* __restrict__ y,
                                                           float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                           const T* __restrict__ pw, T* __restrict__ pout, int M,
                                                           float eps, float alpha, uint64_t seed,
                                                           const int64_t* __restrict__ sstep, uint32_t thr,
                                                           float inv_keep, int wrows, int write_y,
                                                           const T* __restrict__ xin, const T* __restrict__ dres,
                                                           T* __restrict__ dh) {
  using frag = typename std::conditional<std::is_same<T, bf16>::value, bf16x8, fp16x8>::type;
  constexpr int D = NK * 32;
  constexpr int NKW = NK / NW;  // k-steps per wave
  static_assert(NK % NW == 0, "k-steps split evenly over the waves");
  __shared__ float red[NW][16];
  __shared__ float pred[NW][16][33];
  seed = mift_seed(seed, sstep);
  const int tid = threadIdx.x, lane = tid & 63, fr = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = blockIdx.x * 16;
  const int row = min(m0 + fr, M - 1);
  const bool live = m0 + fr < M;
  const int c00 = wave * NKW * 32 + g * 8;  // this lane's first column
  const T* xr = x + (size_t)row * D + c00;
  short8 xv[NKW];
#pragma unroll
  for (int s = 0; s < NKW; ++s) xv[s] = *reinterpret_cast<const short8*>(xr + s * 32);
  T* yr = y + (size_t)row * D + c00;
  // sum over the block's NW waves (in wave order) of a per-row value held by lanes g = 0..3 of every wave
  auto row_sum = [&](float v) {
    v = xor16_add(v);
    v = xor32_add(v);
    if (g == 0) red[wave][fr] = v;
    __syncthreads();
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) r += red[q][fr];
    __syncthreads();  // red is reused by the next call
    return r;
  };
  constexpr bool LN = MODE == 1;
  if constexpr (LN) {
    float sum = 0.f;
#pragma unroll
    for (int s = 0; s < NKW; ++s) {
      float v[8];
      unpack8<T>(xv[s], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) sum += v[e];
    }
    const float mean = row_sum(sum) * (1.f / D);
    float q = 0.f;
#pragma unroll
    for (int s = 0; s < NKW; ++s) {
      float v[8];
      unpack8<T>(xv[s], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[e] - mean; q += d * d; }
    }
    const float rstd = rsqrtf(row_sum(q) * (1.f / D) + eps);
#pragma unroll
    for (int s = 0; s < NKW; ++s) {
      const int c = c00 + s * 32;
      float v[8], wv[8], bv[8];
      unpack8<T>(xv[s], v);
      load8<W>(lw + c, wv);
      load8<W>(lb + c, bv);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (v[e] - mean) * rstd * wv[e] + bv[e];
      short8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) { T t = (T)v[e]; short h; __builtin_memcpy(&h, &t, 2); o[e] = h; }
      xv[s] = o;  // the 16-bit y the consumer GEMM sees
      if (live) *reinterpret_cast<short8*>(yr + s * 32) = o;
    }
    if (live && wave == 0 && g == 0) {
      mean_out[m0 + fr] = mean;
      rstd_out[m0 + fr] = rstd;
    }
  } else if constexpr (MODE == 3) {
    const float mean = mean_out[row], rstd = rstd_out[row];
    // the 4-wave widths (768 / 1024) request dres with the other row operands; the wide forms (8 / 16
    // waves, up to 10 pieces per operand) load it in the output loop: all three operands live across
    // the statistics barrier spilled 114-253 VGPRs there
    constexpr bool RV_EARLY = NW == 4;
    short8 hv[NKW], rv[RV_EARLY ? NKW : 1];
    const T* hr = xin + (size_t)row * D + c00;
#pragma unroll
    for (int s = 0; s < NKW; ++s) {
      hv[s] = *reinterpret_cast<const short8*>(hr + s * 32);
      if constexpr (RV_EARLY)
        rv[s] = dres != nullptr ? *reinterpret_cast<const short8*>(dres + (size_t)row * D + c00 + s * 32)
                                : short8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    float sg = 0.f, sgx = 0.f;
    // wide forms: the per-step LN weight / dres loads go one step ahead of their use, and a scheduling
    // barrier per step keeps hipcc from hoisting every step's loads to the top of the unrolled loop
    // (what made the register footprint)
    float wn[8];
    short8 rn = short8{0, 0, 0, 0, 0, 0, 0, 0};
    if constexpr (!RV_EARLY) load8<W>(lw + c00, wn);
#pragma unroll
    for (int s = 0; s < NKW; ++s) {
      float dv[8], xf[8], wv[8];
      unpack8<T>(xv[s], dv);
      unpack8<T>(hv[s], xf);
      if constexpr (RV_EARLY) {
        load8<W>(lw + c00 + s * 32, wv);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) wv[e] = wn[e];
        load8<W>(lw + c00 + min(s + 1, NKW - 1) * 32, wn);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float gg = dv[e] * wv[e];
        sg += gg;
        sgx += gg * ((xf[e] - mean) * rstd);
      }
      if constexpr (!RV_EARLY) __builtin_amdgcn_sched_barrier(0);
    }
    {  // both row sums in one LDS exchange (one barrier pair instead of two)
      __shared__ float red2[NW][16][2];
      sg = xor16_add(sg);
      sg = xor32_add(sg);
      sgx = xor16_add(sgx);
      sgx = xor32_add(sgx);
      if (g == 0) {
        red2[wave][fr][0] = sg;
        red2[wave][fr][1] = sgx;
      }
      if constexpr (!RV_EARLY) {  // step 0's operands requested before the barrier
        load8<W>(lw + c00, wn);
        if (dres != nullptr) rn = *reinterpret_cast<const short8*>(dres + (size_t)row * D + c00);
      }
      __syncthreads();
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        s0 += red2[q][fr][0];
        s1 += red2[q][fr][1];
      }
      sg = s0 * (1.f / D);
      sgx = s1 * (1.f / D);
    }
    T* dhr = dh + (size_t)row * D + c00;
#pragma unroll
    for (int s = 0; s < NKW; ++s) {
      float dv[8], xf[8], wv[8], r[8], o[8];
      unpack8<T>(xv[s], dv);
      unpack8<T>(hv[s], xf);
      if constexpr (RV_EARLY) {
        unpack8<T>(rv[s], r);
        load8<W>(lw + c00 + s * 32, wv);
      } else {
        unpack8<T>(rn, r);
#pragma unroll
        for (int e = 0; e < 8; ++e) wv[e] = wn[e];
        const int sn = min(s + 1, NKW - 1);
        load8<W>(lw + c00 + sn * 32, wn);
        if (dres != nullptr) rn = *reinterpret_cast<const short8*>(dres + (size_t)row * D + c00 + sn * 32);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = rstd * (dv[e] * wv[e] - sg - (xf[e] - mean) * rstd * sgx) + r[e];
      short8 hq;
#pragma unroll
      for (int e = 0; e < 8; ++e) { T t = (T)o[e]; short h; __builtin_memcpy(&h, &t, 2); hq[e] = h; }
      if (live) *reinterpret_cast<short8*>(dhr + s * 32) = hq;
      if (thr != 0) {
        bool kp[8];
        mift_keep8(seed, (uint64_t)row * D + c00 + s * 32, thr, kp);
        float v[8];
        unpack8<T>(hq, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          T t = (T)(kp[e] ? v[e] * inv_keep : 0.f);
          short h;
          __builtin_memcpy(&h, &t, 2);
          hq[e] = h;
        }
        if (live) *reinterpret_cast<short8*>(yr + s * 32) = hq;
      }
      xv[s] = hq;
      if constexpr (!RV_EARLY) __builtin_amdgcn_sched_barrier(0);
    }
  } else if (MODE == 0 && thr != 0) {  // residual-dropout backward: y = keep ? x/(1-p) : 0, stored and projected
#pragma unroll
    for (int s = 0; s < NKW; ++s) {
      float v[8];
      bool kp[8];
      unpack8<T>(xv[s], v);
      mift_keep8(seed, (uint64_t)row * D + c00 + s * 32, thr, kp);
      short8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        T t = (T)(kp[e] ? v[e] * inv_keep : 0.f);
        short h;
        __builtin_memcpy(&h, &t, 2);
        o[e] = h;
      }
      xv[s] = o;
      if (live && write_y) *reinterpret_cast<short8*>(yr + s * 32) = o;
    }
  }
  // projection partial over this wave's k-steps: acc[j] = y[16 rows] · pw[16j .. 16j+15]^T (rows
  // >= wrows of pw are zero: not read)
  const bool mask_in = (MODE == 1 || MODE == 2) && thr != 0;  // LoRA-input dropout (1/(1-p) folded into alpha)
  const uint32_t hm0 = mift_hmix(seed, 0);
  const bool hz = (uint64_t)M * D < (1ull << 33);
  float4_ acc[NTI];
#pragma unroll
  for (int j = 0; j < NTI; ++j) acc[j] = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NKW; ++s) {
    const int c = c00 + s * 32;
    short8 a = xv[s];
    if (mask_in) {
      uint32_t w[4], km[4];
      __builtin_memcpy(w, &a, 16);
      mift_andmask8(seed, hm0, hz, (uint64_t)row * D + c, thr, km);
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] &= km[e];
      __builtin_memcpy(&a, w, 16);
    }
    frag af;
    __builtin_memcpy(&af, &a, 16);
#pragma unroll
    for (int j = 0; j < NTI; ++j) {
      const int wr = j * 16 + fr;
      const short8 b = wr < wrows ? *reinterpret_cast<const short8*>(pw + (size_t)wr * D + c)
                                  : short8{0, 0, 0, 0, 0, 0, 0, 0};
      frag bfv;
      __builtin_memcpy(&bfv, &b, 16);
      if constexpr (std::is_same<T, bf16>::value)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfv, acc[j], 0, 0, 0);
      else
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bfv, acc[j], 0, 0, 0);
    }
  }
  // lane (fr, g) holds the partial out[4g + r][16j + fr]; sum the NW waves' partials in LDS (wave order)
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int j = 0; j < 2; ++j) pred[wave][4 * g + r][j * 16 + fr] = j < NTI ? acc[j < NTI ? j : 0][r] : 0.f;
  __syncthreads();
  for (int e = tid; e < 16 * 32; e += NW * 64) {
    const int r = e >> 5, c = e & 31;
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) v += pred[q][r][c];
    if (m0 + r < M) pout[(size_t)(m0 + r) * 32 + c] = (T)(v * alpha);
  }
}

// MFMA-form widths: D = 32·NK, split over NW waves (NK / NW k-steps of 32 columns per wave, so a wave
// holds <= 10 16-B pieces of each row operand): 768 / 1024 on 4 waves (distilgpt2, OPT-125m / 350m),
// 2048 / 2560 on 8 (OPT-1.3b / 2.7b), 4096 on 16 (OPT-6.7b).  MIFT_ROWPROJ_V=1 (A/B knob, read per
// call): the row kernels.  Other widths take the row kernels (the LN / mask producers) or lora_proj.
inline bool rowproj_width(int D) { return D == 768 || D == 1024 || D == 2048 || D == 2560 || D == 4096; }
inline bool rowproj_mfma_ok(int D) {
  const char* e = getenv("MIFT_ROWPROJ_V");
  return !(e && atoi(e) == 1) && rowproj_width(D);
}

// waves per block at the distilgpt2 / OPT-125m widths: 12 (16 at 1024; 2 k-steps per wave).  More waves
// per row block shorten each wave's load chain and register footprint (the LN-backward pass: ~100 VGPRs
// on 8 waves against 174 on 4) so more waves per SIMD hide the row loads — distilgpt2 step 4.727 ->
// 4.664 ms on 8 waves (LN-bwd + dropout-bwd + dT 17.5 -> 15 us, LN + T 11.1 -> 9.5, c_attn dT 14.3 ->
// 10.7), 4.659 on 12 (profiles/r5/step_ab_rowproj_nw*.json).  MIFT_ROWPROJ_NW = 4 / 8 / 12 (read per
// call): A/B.
inline int rowproj_nw() {
  const char* e = getenv("MIFT_ROWPROJ_NW");
  const int v = e ? atoi(e) : 12;
  return v == 4 || v == 8 ? v : 12;
}

// f(integral_constant NK, integral_constant NW) for a rowproj_width D
template <typename F>
void by_nk(int D, F&& f) {
  using std::integral_constant;
  const int nw = rowproj_nw();
  switch (D) {
    case 768:
      if (nw == 4) f(integral_constant<int, 24>{}, integral_constant<int, 4>{});
      else if (nw == 12) f(integral_constant<int, 24>{}, integral_constant<int, 12>{});
      else f(integral_constant<int, 24>{}, integral_constant<int, 8>{});
      break;
    case 1024:
      if (nw == 4) f(integral_constant<int, 32>{}, integral_constant<int, 4>{});
      else if (nw == 12) f(integral_constant<int, 32>{}, integral_constant<int, 16>{});
      else f(integral_constant<int, 32>{}, integral_constant<int, 8>{});
      break;
    case 2048: f(integral_constant<int, 64>{}, integral_constant<int, 8>{}); break;
    case 2560: f(integral_constant<int, 80>{}, integral_constant<int, 8>{}); break;
    default: f(integral_constant<int, 128>{}, integral_constant<int, 16>{}); break;  // 4096
  }
}

// the plain projection (MODE 2): the rowproj widths plus K = 2304 (distilgpt2's c_attn dT)
// (K = 7680, OPT-2.7B's fused q/k/v dT, on 16 waves x 15 k-steps measured 40.7 / 131 us against
// lora_proj's own kernel's 39.6 / 106 us at 6144 / 24576 rows: profiles/r5/bench_rowproj_opt_k7680.json)
inline bool rowproj_proj_width(int K) { return rowproj_width(K) || K == 2304; }
template <typename F>
void by_nk_proj(int K, F&& f) {
  if (K == 2304) {
    const int nw = rowproj_nw();
    if (nw == 4) f(std::integral_constant<int, 72>{}, std::integral_constant<int, 4>{});
    else if (nw == 12) f(std::integral_constant<int, 72>{}, std::integral_constant<int, 12>{});
    else f(std::integral_constant<int, 72>{}, std::integral_constant<int, 8>{});
  } else {
    by_nk(K, f);
  }
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
  if (rowproj_mfma_ok(D)) {
    auto go2 = [&](auto tt, auto wt) {
      using T = decltype(tt);
      using Wt = decltype(wt);
      by_nk(D, [&](auto nk, auto nw) {
        constexpr int NK = decltype(nk)::value, NW = decltype(nw)::value;
        auto kern = rank <= 16 ? rowproj_mfma_kernel<T, Wt, NK, 1, 1, NW> : rowproj_mfma_kernel<T, Wt, NK, 2, 1, NW>;
        hipLaunchKernelGGL(kern, dim3((M + 15) / 16), dim3(NW * 64), 0, st, (const T*)x.data_ptr(),
                           (const Wt*)w.data_ptr(), (const Wt*)b.data_ptr(), (T*)y.data_ptr(), mean.data_ptr<float>(),
                           rstd.data_ptr<float>(), (const T*)pw.data_ptr(), (T*)pout.data_ptr(), M, (float)eps,
                           (float)alpha * inv, (uint64_t)seed, mift_seed_step(), thr, inv, (int)rank, 1,
                           (const T*)nullptr, (const T*)nullptr, (T*)nullptr);
      });
    };
    if (x.scalar_type() == at::kBFloat16) {
      if (wf32) go2(bf16{}, 0.f); else go2(bf16{}, bf16{});
    } else {
      if (wf32) go2(fp16{}, 0.f); else go2(fp16{}, fp16{});
    }
    return {y, mean, rstd, pout};
  }
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
  if (rowproj_mfma_ok(D)) {
    auto go2 = [&](auto tt) {
      using T = decltype(tt);
      by_nk(D, [&](auto nk, auto nw) {
        constexpr int NK = decltype(nk)::value, NW = decltype(nw)::value;
        auto kern = rank <= 16 ? rowproj_mfma_kernel<T, T, NK, 1, 0, NW> : rowproj_mfma_kernel<T, T, NK, 2, 0, NW>;
        hipLaunchKernelGGL(kern, dim3((M + 15) / 16), dim3(NW * 64), 0, st, (const T*)x.data_ptr(), (const T*)nullptr,
                           (const T*)nullptr, (T*)y.data_ptr(), (float*)nullptr, (float*)nullptr,
                           (const T*)pw.data_ptr(), (T*)pout.data_ptr(), M, 0.f, (float)alpha, (uint64_t)seed,
                           mift_seed_step(), thr, inv, (int)rank, thr != 0 ? 1 : 0, (const T*)nullptr,
                           (const T*)nullptr, (T*)nullptr);
      });
    };
    if (x.scalar_type() == at::kBFloat16) go2(bf16{});
    else go2(fp16{});
    return {y, pout};
  }
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

// (dh, y, proj[M,32]): dh = LN-bwd(dy; x, w, mean, rstd) + dres, y = keep⊙dh/(1-p) (dh itself when
// p == 0), proj = alpha·y·pw^T — layer_norm_bwd followed by mask_proj in one pass (MFMA form only:
// the rowproj widths; the caller checks mift_ln_bwd_mask_proj_ok)
// (not at 4096: the 16-wave MODE 3 form spills ~110 VGPRs at its 128-register budget and ran 155 us
// against 81 for layer_norm_bwd + mask_scale + lora_proj at M = 6144, tools/bench_rowproj_opt.py)
bool mift_ln_bwd_mask_proj_ok(int64_t D) { return rowproj_mfma_ok((int)D) && D != 4096; }

std::vector<at::Tensor> mift_ln_bwd_mask_proj(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                              const at::Tensor& mean, const at::Tensor& rstd,
                                              const c10::optional<at::Tensor>& dres, double p, int64_t seed,
                                              const at::Tensor& pw, int64_t rank, double alpha) {
  TORCH_CHECK(dy.is_cuda() && dy.is_contiguous() && dy.dim() == 2, "ln_bwd_mask_proj: contiguous 2-D GPU dy");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 || dy.scalar_type() == at::kHalf, "ln_bwd_mask_proj: bf16/fp16");
  const int D = dy.size(1);
  const int M = dy.size(0);
  TORCH_CHECK(mift_ln_bwd_mask_proj_ok(D), "ln_bwd_mask_proj: D in {768, 1024, 2048, 2560}");
  TORCH_CHECK(x.is_contiguous() && x.sizes() == dy.sizes() && x.scalar_type() == dy.scalar_type(), "ln_bwd_mask_proj: x");
  TORCH_CHECK(!dres || (dres->is_contiguous() && dres->sizes() == dy.sizes() && dres->scalar_type() == dy.scalar_type()),
              "ln_bwd_mask_proj: dres");
  TORCH_CHECK(w.numel() == D && (w.scalar_type() == dy.scalar_type() || w.scalar_type() == at::kFloat), "ln_bwd_mask_proj: w");
  TORCH_CHECK(mean.scalar_type() == at::kFloat && rstd.scalar_type() == at::kFloat && mean.numel() == M &&
              rstd.numel() == M, "ln_bwd_mask_proj: mean / rstd");
  check_pw(dy, pw, D, rank);
  const uint32_t thr = mift_thr16(p);
  auto dh = at::empty_like(dy);
  at::Tensor y = thr != 0 ? at::empty_like(dy) : dh;
  auto pout = at::empty({M, 32}, dy.options());
  if (M == 0) return {dh, y, pout};
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const float inv = p > 0 ? mift_inv_keep(p) : 1.f;
  const bool wf32 = w.scalar_type() == at::kFloat;
  auto go = [&](auto tt, auto wt) {
    using T = decltype(tt);
    using Wt = decltype(wt);
    by_nk(D, [&](auto nk, auto nw) {
      constexpr int NK = decltype(nk)::value, NW = decltype(nw)::value;
      auto kern = rank <= 16 ? rowproj_mfma_kernel<T, Wt, NK, 1, 3, NW> : rowproj_mfma_kernel<T, Wt, NK, 2, 3, NW>;
      hipLaunchKernelGGL(kern, dim3((M + 15) / 16), dim3(NW * 64), 0, st, (const T*)dy.data_ptr(), (const Wt*)w.data_ptr(),
                         (const Wt*)nullptr, (T*)y.data_ptr(), const_cast<float*>(mean.data_ptr<float>()),
                         const_cast<float*>(rstd.data_ptr<float>()), (const T*)pw.data_ptr(), (T*)pout.data_ptr(), M,
                         0.f, (float)alpha, (uint64_t)seed, mift_seed_step(), thr, inv, (int)rank, thr != 0 ? 1 : 0,
                         (const T*)x.data_ptr(), dres ? (const T*)dres->data_ptr() : (const T*)nullptr,
                         (T*)dh.data_ptr());
    });
  };
  if (dy.scalar_type() == at::kBFloat16) {
    if (wf32) go(bf16{}, 0.f); else go(bf16{}, bf16{});
  } else {
    if (wf32) go(fp16{}, 0.f); else go(fp16{}, fp16{});
  }
  return {dh, y, pout};
}

// lora_proj on the 16-row MFMA form (MODE 2) for contiguous x at the rowproj widths and K = 2304:
// out = alpha·(1/(1-p))·drop(x)·wᵀ.  Returns false (caller runs lora_proj's own kernel) otherwise.
// lora_proj's own kernel (16-row blocks, K split over the waves, 8 k-steps of loads in flight) ran
// 8.5 / 20.2 us at M = 8192, K = 768 / 2304 against 6.4 / 18.2 here (profiles/r3/bench_rowproj_r3k.jsonl).
bool mift_rowproj_lora_proj(const at::Tensor& x, const at::Tensor& w, at::Tensor& out, double alpha, double p,
                            int64_t seed, int64_t rows) {
  const int M = x.size(0), K = x.size(1);
  const char* e = getenv("MIFT_ROWPROJ_V");  // 1 = off (A/B knob, read per call)
  // (K = 3072 measured slower here than lora_proj's kernel: 24.2 vs 21.9 us at M = 8192)
  if ((e && atoi(e) == 1) || !rowproj_proj_width(K) || x.stride(0) != K ||
      reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 != 0)
    return false;
  if (M == 0) return true;
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const uint32_t thr = mift_thr16(p);
  const float ik = p > 0 ? mift_inv_keep(p) : 1.f;
  auto go = [&](auto tt) {
    using T = decltype(tt);
    by_nk_proj(K, [&](auto nk, auto nw) {
      constexpr int NK = decltype(nk)::value, NW = decltype(nw)::value;
      auto kern = rows <= 16 ? rowproj_mfma_kernel<T, T, NK, 1, 2, NW> : rowproj_mfma_kernel<T, T, NK, 2, 2, NW>;
      hipLaunchKernelGGL(kern, dim3((M + 15) / 16), dim3(NW * 64), 0, st, (const T*)x.data_ptr(), (const T*)nullptr,
                         (const T*)nullptr, (T*)nullptr, (float*)nullptr, (float*)nullptr, (const T*)w.data_ptr(),
                         (T*)out.data_ptr(), M, 0.f, (float)alpha * ik, (uint64_t)seed, mift_seed_step(), thr, ik,
                         (int)rows, 0, (const T*)nullptr, (const T*)nullptr, (T*)nullptr);
    });
  };
  if (x.scalar_type() == at::kBFloat16) go(bf16{});
  else go(fp16{});
  return true;
}
