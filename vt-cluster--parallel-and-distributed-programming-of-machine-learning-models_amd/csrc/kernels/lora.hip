// LoRA side-path kernels (rank r <= 32, padded to 32).
//
//   lora_proj  out[M,32] = alpha · drop(X)[M,K] · W[32,K]^T
//       forward  T  = s·drop(x)·A^T   (W = A pre-scaled by s, padded rows 0)
//       backward dT = s·gz·B          (W = B^T padded, no mask)
//     Tall-skinny MFMA product: one 256-thread block per 32 rows, the four
//     waves split K and reduce through LDS; operands go straight from global
//     to registers (no reuse to stage); the dropout mask of X is applied to the
//     A fragments in registers (counter hash, no mask tensor, no x_drop copy).
//
//   lora_wgrad out[P,32] += Σ_m drop(X)[m,p] · Y[m,q]
//       dB   = gz^T · T         (X = gz [M,N], Y = T)
//       dA^T = drop(x)^T · dT   (X = x  [M,K], Y = s·dT, mask regenerated)
//     Reduction over the token dimension: both MFMA operands are columns of
//     row-major tiles, read with the gfx950 hardware transpose
//     ds_read_b64_tr_b16 (guide T10).  Rows are consumed in a permuted order
//     (group g takes rows 4g..4g+3 and 16+4g..16+4g+3 of each 32-row step) so a
//     half-wave's 8 rows sit at an odd multiple of 32 B apart -> conflict-free.
//     Split over M across blocks, fp32 atomics into the small [P,32] output.
#include "common.h"
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

namespace {

typedef short v4s __attribute__((ext_vector_type(4)));

template <typename T>
using frag_t = typename std::conditional<std::is_same<T, bf16>::value, bf16x8, fp16x8>::type;

template <typename T>
MIFT_HD float4_ mfma16(frag_t<T> a, frag_t<T> b, float4_ c) {
  if constexpr (std::is_same<T, bf16>::value)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

template <typename T>
MIFT_HD frag_t<T> masked_frag(const T* p, uint64_t seed, uint64_t idx0, uint32_t thr, float inv_keep) {
  short8 v = *reinterpret_cast<const short8*>(p);
  if (thr != 0) {
    bool kp[8];
    mift_keep8(seed, idx0, thr, kp);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      short s = v[e];
      T t;
      __builtin_memcpy(&t, &s, 2);
      t = kp[e] ? (T)((float)t * inv_keep) : (T)0.f;
      __builtin_memcpy(&s, &t, 2);
      v[e] = s;
    }
  }
  frag_t<T> f;
  __builtin_memcpy(&f, &v, 16);
  return f;
}

// ------------------------------------------------------------------ lora_proj
// Grid = (M/32 row blocks) x KS K-splits: with only M/32 row blocks (128 for
// M = 4096) the kernel filled half of the 256 CUs and ran latency-bound; the
// K-splits give ~1024 blocks.  KS > 1: every block stores its [32,32] fp32
// partial to ws[kss] with plain stores and lora_proj_reduce sums the KS
// partials into the 16-bit output (an in-kernel last-block reduction needs a
// device-scope fence per block, ~3.5 us on gfx950 — slower than a launch).
template <typename T, int NW>
__global__ __launch_bounds__(NW * 64) void lora_proj_kernel(const T* __restrict__ X, const T* __restrict__ W,
                                                        T* __restrict__ out, int M, int K, int ldx, float alpha,
                                                        uint64_t seed, const int64_t* __restrict__ sstep, uint32_t thr, float inv_keep, int KS,
                                                        float* __restrict__ ws) {
  seed = mift_seed(seed, sstep);
  __shared__ float red[NW][32][33];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on it
  const int g = lane >> 4, fr = lane & 15;
  const int mb = blockIdx.x / KS, kss = blockIdx.x % KS;
  const int m0 = mb * 32;
  float4_ acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = float4_{0.f, 0.f, 0.f, 0.f};
  const int rows[2] = {min(m0 + fr, M - 1), min(m0 + 16 + fr, M - 1)};
  const int nks_all = K / 32;
  const int per_blk = (nks_all + KS - 1) / KS;
  const int kb0 = kss * per_blk, nks = min(nks_all, kb0 + per_blk);
  // each wave owns a contiguous K range of the block's split; UNR k-steps of
  // loads are issued back to back before their MFMAs (memory-level
  // parallelism: one 16-B load per lane per operand per k-step).  NW = 8 for
  // long K halves every wave's chain of dependent load rounds.
  constexpr int UNR = 4;
  const int per = (nks - kb0 + NW - 1) / NW;
  const int kbeg = kb0 + wave * per, kend = min(nks, kbeg + per);
  for (int ks0 = kbeg; ks0 < kend; ks0 += UNR) {
    short8 ra[UNR][2], rb[UNR][2];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int col = min(ks0 + u, nks - 1) * 32 + g * 8;
#pragma unroll
      for (int i = 0; i < 2; ++i) ra[u][i] = *reinterpret_cast<const short8*>(X + (int64_t)rows[i] * ldx + col);
#pragma unroll
      for (int j = 0; j < 2; ++j) rb[u][j] = *reinterpret_cast<const short8*>(W + (int64_t)(j * 16 + fr) * K + col);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (ks0 + u >= kend) break;
      const int col = (ks0 + u) * 32 + g * 8;
      frag_t<T> a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        short8 v = ra[u][i];
        if (thr != 0) {
          bool kp[8];
          mift_keep8(seed, (uint64_t)rows[i] * K + col, thr, kp);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            short s = v[e];
            T t;
            __builtin_memcpy(&t, &s, 2);
            t = kp[e] ? (T)((float)t * inv_keep) : (T)0.f;
            __builtin_memcpy(&s, &t, 2);
            v[e] = s;
          }
        }
        __builtin_memcpy(&a[i], &v, 16);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) __builtin_memcpy(&b[j], &rb[u][j], 16);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16<T>(a[i], b[j], acc[i][j]);
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][i * 16 + g * 4 + r][j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  auto rsum = [&](int r, int c) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][r][c];
    return v;
  };
  if (KS == 1) {
    for (int e = tid; e < 32 * 32; e += NW * 64) {
      const int r = e >> 5, c = e & 31;
      if (m0 + r < M) out[(int64_t)(m0 + r) * 32 + c] = (T)(rsum(r, c) * alpha);
    }
    return;
  }
  float* wp = ws + (int64_t)kss * M * 32;
  for (int e = tid; e < 32 * 32; e += NW * 64) {
    const int r = e >> 5, c = e & 31;
    if (m0 + r < M) wp[(int64_t)(m0 + r) * 32 + c] = rsum(r, c);
  }
}

// out[m, c] = alpha * sum_s ws[s, m, c]  (8 outputs per thread, 16-B stores)
template <typename T>
__global__ __launch_bounds__(256) void lora_proj_reduce(const float* __restrict__ ws, T* __restrict__ out, int M,
                                                         int KS, float alpha) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  const int64_t n = (int64_t)M * 32;
  if (i >= n) return;
  float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int s = 0; s < KS; ++s) {
    const float4 a = *reinterpret_cast<const float4*>(ws + s * n + i);
    const float4 b = *reinterpret_cast<const float4*>(ws + s * n + i + 4);
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
    v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] *= alpha;
  store8<T>(out + i, v);
}

// ----------------------------------------------------------------- lora_wgrad
constexpr int XS = 160;  // X tile row stride (bytes): 64 cols (128 B) padded to an odd multiple of 32 B
constexpr int YS = 96;   // Y tile row stride: 32 cols (64 B) -> 96 B

template <typename T>
MIFT_HD v4s tr_read(const char* lds_base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(lds_base + off));
}

template <typename T>
__global__ __launch_bounds__(256) void lora_wgrad_kernel(const T* __restrict__ X, const T* __restrict__ Y,
                                                         float* __restrict__ out, int M, int P, int ldx,
                                                         int rows_per_block, uint64_t seed, const int64_t* __restrict__ sstep, uint32_t thr,
                                                         float inv_keep, int mode, int rank, int qoff) {
  seed = mift_seed(seed, sstep);
  // NB 32-row steps per group: the whole group's global loads are in flight
  // together (one 16-B X load + half a Y load per thread per step), staged
  // into NB LDS buffers, then consumed; the next group's loads are issued
  // before this group's transpose reads + MFMAs.
  constexpr int NB = 4;
  __shared__ __attribute__((aligned(16))) char Xs[NB][32 * XS];
  __shared__ __attribute__((aligned(16))) char Ys[NB][32 * YS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on it
  const int g = lane >> 4, li = lane & 15;
  const int ntp = P / 64;
  const int pt = blockIdx.x % ntp, ms = blockIdx.x / ntp;
  const int p0 = pt * 64;
  const int mbeg = ms * rows_per_block;
  const int mend = min(mbeg + rows_per_block, M);
  float4_ acc[2] = {float4_{0.f, 0.f, 0.f, 0.f}, float4_{0.f, 0.f, 0.f, 0.f}};

  const int xr = tid >> 3, xc = tid & 7;
  const int yr = (tid & 127) >> 2, yc = tid & 3;
  short8 xv[NB], yv[NB];
  auto gload = [&](int m0g) {
#pragma unroll
    for (int s = 0; s < NB; ++s) {
      const int m = m0g + 32 * s;
      const int gm = min(m + xr, M - 1);
      xv[s] = *reinterpret_cast<const short8*>(X + (int64_t)gm * ldx + p0 + xc * 8);
      if (tid < 128) {
        const int gy = min(m + yr, M - 1);
        yv[s] = *reinterpret_cast<const short8*>(Y + (int64_t)gy * 32 + yc * 8);
      }
    }
  };
  auto lstore = [&](int m0g) {
#pragma unroll
    for (int s = 0; s < NB; ++s) {
      const int m = m0g + 32 * s;
      const bool valid = (m + xr) < mend;
      short8 v = xv[s];
      if (thr != 0 || !valid) {
        bool kp[8];
        if (thr != 0) mift_keep8(seed, (uint64_t)min(m + xr, M - 1) * P + p0 + xc * 8, thr, kp);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          short sh = v[e];
          T t;
          __builtin_memcpy(&t, &sh, 2);
          float f = (float)t;
          f = !valid ? 0.f : (thr != 0 ? (kp[e] ? f * inv_keep : 0.f) : f);
          t = (T)f;
          __builtin_memcpy(&sh, &t, 2);
          v[e] = sh;
        }
      }
      *reinterpret_cast<short8*>(Xs[s] + xr * XS + xc * 16) = v;
      if (tid < 128) {
        short8 w = yv[s];
        if ((m + yr) >= mend) w = short8{0, 0, 0, 0, 0, 0, 0, 0};
        *reinterpret_cast<short8*>(Ys[s] + yr * YS + yc * 16) = w;
      }
    }
  };

  // transpose-read addresses (permuted rows: first read rows 4g+q', second 16+4g+q')
  const int q4 = li >> 2, p4 = li & 3;
  const int rowA = 4 * g + q4;
  const int xoff = rowA * XS + (wave * 16 + p4 * 4) * 2;
  const int yoff0 = rowA * YS + (0 * 16 + p4 * 4) * 2;
  const int yoff1 = rowA * YS + (1 * 16 + p4 * 4) * 2;

  if (mbeg < mend) gload(mbeg);
  for (int mg = mbeg; mg < mend; mg += 32 * NB) {
    __syncthreads();
    lstore(mg);
    __syncthreads();
    if (mg + 32 * NB < mend) gload(mg + 32 * NB);
#pragma unroll
    for (int s = 0; s < NB; ++s) {
      if (mg + 32 * s >= mend) break;
      const char* xb = Xs[s];
      const char* yb = Ys[s];
      v4s a0 = tr_read<T>(xb, xoff), a1 = tr_read<T>(xb, xoff + 16 * XS);
      v4s b00 = tr_read<T>(yb, yoff0), b01 = tr_read<T>(yb, yoff0 + 16 * YS);
      v4s b10 = tr_read<T>(yb, yoff1), b11 = tr_read<T>(yb, yoff1 + 16 * YS);
      frag_t<T> af, bf0, bf1;
      {
        short8 t = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        __builtin_memcpy(&af, &t, 16);
        short8 u = {b00[0], b00[1], b00[2], b00[3], b01[0], b01[1], b01[2], b01[3]};
        __builtin_memcpy(&bf0, &u, 16);
        short8 w = {b10[0], b10[1], b10[2], b10[3], b11[0], b11[1], b11[2], b11[3]};
        __builtin_memcpy(&bf1, &w, 16);
      }
      acc[0] = mfma16<T>(af, bf0, acc[0]);
      acc[1] = mfma16<T>(af, bf1, acc[1]);
    }
  }
  // acc[c][r] = out[p = p0 + wave*16 + g*4 + r][q = c*16 + li]
  // mode 0: dense [P,32]; mode 1: dB layout [P, rank]; mode 2: dA layout [rank, P]
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t pp = p0 + wave * 16 + g * 4 + r;
      const int q = c * 16 + li;
      if (mode == 0) atomicAdd(out + pp * 32 + q, acc[c][r]);
      else if (q >= qoff && q < qoff + rank) atomicAdd(out + (mode == 1 ? pp * rank + (q - qoff) : (int64_t)(q - qoff) * P + pp), acc[c][r]);
    }
}

}  // namespace

at::Tensor mift_lora_proj(const at::Tensor& x, const at::Tensor& w, double alpha, double p, int64_t seed) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "lora_proj: x [M,K] row-major");
  TORCH_CHECK(w.is_contiguous() && w.size(0) == 32 && w.size(1) == x.size(1), "lora_proj: w [32,K]");
  TORCH_CHECK(x.scalar_type() == w.scalar_type(), "lora_proj: dtype");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(K % 32 == 0 && x.stride(0) % 8 == 0, "lora_proj: K % 32, aligned rows");
  auto out = at::empty({M, 32}, x.options());
  if (M == 0) return out;
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const uint32_t thr = mift_thr16(p);
  const float ik = p > 0 ? mift_inv_keep(p) : 1.f;
  const int mblocks = (M + 31) / 32, nks = K / 32;
  // K-splits so the launch covers the chip (>= ~1024 blocks), >= 4 k-steps (one per wave) each
  static const int ks_env = [] { const char* e = getenv("MIFT_LORA_KS"); return e ? atoi(e) : 0; }();
  // split K only when the row blocks alone leave CUs idle (measured: distilgpt2, M = 8192 ->
  // 256 row blocks, is 3 % faster unsplit; OPT micro-batches of M = 4096 gain 2 % from KS = 8)
  int KS = mblocks >= 192 ? 1 : std::max(1, std::min(std::max(1, nks / 4), (1024 + mblocks - 1) / mblocks));
  if (ks_env > 0) KS = std::max(1, std::min(ks_env, std::max(1, nks / 4)));  // A/B override
  float* ws = nullptr;
  at::Tensor wsb;
  if (KS > 1) {
    wsb = at::empty({(int64_t)KS * M * 32}, x.options().dtype(at::kFloat));
    ws = wsb.data_ptr<float>();
  }
  const int grid = mblocks * KS;
  // 4 waves per row block (MIFT_LORA_NW=8 for 8): the 8-wave variant for long K measured slower
  // at OPT-2.7B shapes (M = 24576: K = 2560 35.6 vs 30.3 us, K = 7680 118 vs 105, K = 10240 155 vs
  // 140; tools/bench_rowproj.py) and even at distilgpt2's
  static const int nw_env = [] { const char* e = getenv("MIFT_LORA_NW"); return e ? atoi(e) : 4; }();
  const bool wide = nw_env == 8;
  auto go = [&](auto tt) {
    using T = decltype(tt);
    if (wide)
      lora_proj_kernel<T, 8><<<grid, 512, 0, st>>>((const T*)x.data_ptr(), (const T*)w.data_ptr(),
                                                   (T*)out.data_ptr(), M, K, (int)x.stride(0), (float)alpha,
                                                   (uint64_t)seed, mift_seed_step(), thr, ik, KS, ws);
    else
      lora_proj_kernel<T, 4><<<grid, 256, 0, st>>>((const T*)x.data_ptr(), (const T*)w.data_ptr(),
                                                   (T*)out.data_ptr(), M, K, (int)x.stride(0), (float)alpha,
                                                   (uint64_t)seed, mift_seed_step(), thr, ik, KS, ws);
  };
  if (x.scalar_type() == at::kBFloat16) go(bf16{});
  else go(fp16{});
  if (KS > 1) {
    const int rg = (int)(((int64_t)M * 32 / 8 + 255) / 256);
    if (x.scalar_type() == at::kBFloat16)
      lora_proj_reduce<bf16><<<rg, 256, 0, st>>>(ws, (bf16*)out.data_ptr(), M, KS, (float)alpha);
    else
      lora_proj_reduce<fp16><<<rg, 256, 0, st>>>(ws, (fp16*)out.data_ptr(), M, KS, (float)alpha);
  }
  return out;
}

// out fp32, accumulated: mode 0 -> out[P,32]; mode 1/2 -> out is a flat arena
// and the result lands at out[offset:] in dB [P,r] / dA [r,P] layout.
void mift_lora_wgrad(const at::Tensor& x, const at::Tensor& y, at::Tensor& out, double p, int64_t seed, int64_t mode,
                     int64_t rank, int64_t offset, int64_t qoff) {
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && y.is_contiguous() && y.size(1) == 32, "lora_wgrad: shapes");
  const int M = x.size(0), P = x.size(1);
  TORCH_CHECK(y.size(0) == M && P % 64 == 0, "lora_wgrad: P % 64 == 0");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous(), "lora_wgrad: out fp32 contiguous");
  if (mode == 0) {
    TORCH_CHECK(out.numel() == (int64_t)P * 32, "lora_wgrad: out [P,32]");
  } else {
    TORCH_CHECK(offset + (int64_t)P * rank <= out.numel() && rank <= 32, "lora_wgrad: arena range");
  }
  if (M == 0) return;
  const int ntp = P / 64;
  int splits = std::max(1, std::min((512 + ntp - 1) / ntp, (M + 127) / 128));
  int rows = ((M + splits - 1) / splits + 127) / 128 * 128;
  splits = (M + rows - 1) / rows;
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const uint32_t thr = mift_thr16(p);
  const float ik = p > 0 ? mift_inv_keep(p) : 1.f;
  if (x.scalar_type() == at::kBFloat16)
    lora_wgrad_kernel<bf16><<<ntp * splits, 256, 0, st>>>((const bf16*)x.data_ptr(), (const bf16*)y.data_ptr(),
                                                          out.data_ptr<float>() + offset, M, P, (int)x.stride(0), rows,
                                                          (uint64_t)seed, mift_seed_step(), thr, ik, (int)mode, (int)rank, (int)qoff);
  else
    lora_wgrad_kernel<fp16><<<ntp * splits, 256, 0, st>>>((const fp16*)x.data_ptr(), (const fp16*)y.data_ptr(),
                                                          out.data_ptr<float>() + offset, M, P, (int)x.stride(0), rows,
                                                          (uint64_t)seed, mift_seed_step(), thr, ik, (int)mode, (int)rank, (int)qoff);
}

// ------------------------------------------------------------ pack_lora_all
// One launch packs the 16-bit operands of EVERY adapted Linear from the flat
// fp32 arena (done once per optimizer step, not per micro-batch):
//   table[i] = {r, K, N, offA, offB, offOut}; out + offOut holds, in order,
//   A32s [32,K] = s·A | B32 [N,32] | B32t [32,N] | At32 [K,32]   (zero padded)
namespace {
template <typename T>
__global__ __launch_bounds__(256) void pack_lora_all_kernel(const float* __restrict__ arena,
                                                            const int64_t* __restrict__ table,
                                                            const float* __restrict__ scales, T* __restrict__ out) {
  const int mi = blockIdx.y;
  const int64_t* t = table + mi * 6;
  const int r = (int)t[0], K = (int)t[1], N = (int)t[2];
  const float* A = arena + t[3];
  const float* B = arena + t[4];
  T* o = out + t[5];
  const float s = scales[mi];
  const int64_t nA = 32LL * K, nB = 32LL * N;
  const int64_t total = 2 * nA + 2 * nB;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    float v;
    if (i < nA) {  // A32s [32,K]
      const int row = i / K, col = i % K;
      v = row < r ? A[(int64_t)row * K + col] * s : 0.f;
    } else if (i < nA + nB) {  // B32 [N,32]
      const int64_t j = i - nA;
      const int row = j / 32, col = j % 32;
      v = col < r ? B[(int64_t)row * r + col] : 0.f;
    } else if (i < nA + 2 * nB) {  // B32t [32,N]
      const int64_t j = i - nA - nB;
      const int row = j / N, col = j % N;
      v = row < r ? B[(int64_t)col * r + row] : 0.f;
    } else {  // At32 [K,32]
      const int64_t j = i - nA - 2 * nB;
      const int row = j / 32, col = j % 32;
      v = col < r ? A[(int64_t)col * K + row] : 0.f;
    }
    o[i] = (T)v;
  }
}
}  // namespace

void mift_pack_lora_all(const at::Tensor& arena, const at::Tensor& table, const at::Tensor& scales, at::Tensor& out,
                        int64_t max_elems) {
  TORCH_CHECK(arena.scalar_type() == at::kFloat && table.scalar_type() == at::kLong && table.size(1) == 6,
              "pack_lora_all: arena fp32, table int64 [n,6]");
  const int n = table.size(0);
  if (n == 0) return;
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const int gx = (int)std::min<int64_t>(256, (max_elems + 255) / 256);
  dim3 grid(gx, n);
  if (out.scalar_type() == at::kBFloat16)
    pack_lora_all_kernel<bf16><<<grid, 256, 0, st>>>(arena.data_ptr<float>(), table.data_ptr<int64_t>(),
                                                     scales.data_ptr<float>(), (bf16*)out.data_ptr());
  else
    pack_lora_all_kernel<fp16><<<grid, 256, 0, st>>>(arena.data_ptr<float>(), table.data_ptr<int64_t>(),
                                                     scales.data_ptr<float>(), (fp16*)out.data_ptr());
}
