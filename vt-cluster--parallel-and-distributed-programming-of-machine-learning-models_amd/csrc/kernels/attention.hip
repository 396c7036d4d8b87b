// K3: causal flash attention (forward + backward) for gfx950.
//
// Layout: the fused projection output qkv [B*S, 3*H*HD] (token-major, as the
// qkv GEMM writes it) is read in place — no head split / transpose kernels.
// Output o [B*S, H*HD]; lse [B, H, S] fp32 (natural log of the softmax
// denominator of scale*QK^T) for the backward.  Head dims 64 (GPT-2),
// 80 (OPT-2.7B; QK^T K-steps zero-padded to 96) and 128 (OPT-6.7B).
//
// MFMA mapping (16x16x32 bf16, "swapped" products, guide §3):
//   forward  S^T[key, q] = K · Q^T   A = K rows (LDS), B = Q rows (registers)
//            -> each lane owns ONE query (lane & 15) and 4 keys per 16-key
//               sub-tile, so the P tile is already the A operand of P·V up to
//               a k-permutation; V is staged transposed + key-permuted in LDS
//               so the matching B fragment is one 16-B ds_read (no P round
//               trip through LDS, no cross-lane shuffles for P).
//   Online softmax in exp2 with per-query running max/sum; O rescale factors
//   are moved to the accumulator layout with 4 shuffles per KV tile.
// Backward (FA2 split, no atomics): attn_bwd_dq (mirror of the forward: Q,
// dO in registers, loop over key tiles, dQ += dS·K) and attn_bwd_dkdv (one
// key tile per block, loop over query tiles, S = Q·K^T in the lane-per-key
// layout, dV += P^T dO and dK += dS^T Q with transposed/permuted dO^T, Q^T
// images in LDS).  D = rowsum(dO ∘ O) comes from attn_bwd_pre.
// Dropout (GPT-2 attn_pdrop 0.1): counter hash of idx = ((b*H+h)*S+q)*S+k,
// identical in all kernels (see common.h).
#include "common.h"
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

namespace {

constexpr int BQ = 64, BKV = 64;
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

MIFT_HD float4_ mfma_bf16(bf16x8 a, bf16x8 b, float4_ c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// key position inside a 64-key "permuted" row so that the 8 keys a lane group
// g contributes to K-step s2 of the P·V product are contiguous:
//   key = 32*s2 + 16*t + 4*g + r  ->  pos = 32*s2 + 8*g + 4*t + r
MIFT_HD int perm_pos(int key) {
  const int s2 = key >> 5, t = (key >> 4) & 1, g = (key >> 2) & 3, r = key & 3;
  return (s2 << 5) | (g << 3) | (t << 2) | r;
}

template <int HD>
struct Geo {
  static constexpr int HDP = (HD + 31) / 32 * 32;  // padded for 32-deep K steps
  static constexpr int NKS = HDP / 32;             // K-steps over head dim
  static constexpr int NOT = HD / 16;              // 16-wide output tiles
  static constexpr int RS = HDP * 2 + 16;          // row-tile stride (bytes)
  static constexpr int CS = BKV * 2 + 16;          // col-tile stride (bytes)
  static constexpr int ROW_BYTES = 64 * RS;
  static constexpr int COL_BYTES = HD * CS;
  static constexpr int CH = HD / 8;                // 16-B chunks per row
};

MIFT_HD bf16x8 ld_frag(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

MIFT_HD bf16x8 zero_frag() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.f;
  return z;
}

// Load a 64-row x HD tile (rows row0.., clamped to [0,nrows)) from a strided
// bf16 matrix into a row tile (stride RS, padded columns zeroed once by caller).
template <int HD>
MIFT_HD void load_row_tile(char* dst, const bf16* src, int64_t ld, int row0, int nrows, int tid) {
  using G = Geo<HD>;
  for (int i = tid; i < 64 * G::CH; i += 256) {
    const int r = i / G::CH, c = i % G::CH;
    const int gr = min(row0 + r, nrows - 1);
    short8 v = *reinterpret_cast<const short8*>(src + (int64_t)gr * ld + c * 8);
    *reinterpret_cast<short8*>(dst + r * G::RS + c * 16) = v;
  }
}

// Same source, written transposed + key-permuted: dst[hd][perm_pos(row)].
template <int HD>
MIFT_HD void load_col_tile(char* dst, const bf16* src, int64_t ld, int row0, int nrows, int tid) {
  using G = Geo<HD>;
  for (int i = tid; i < 64 * G::CH; i += 256) {
    const int r = i % 64, c = i / 64;
    const int gr = min(row0 + r, nrows - 1);
    short8 v = *reinterpret_cast<const short8*>(src + (int64_t)gr * ld + c * 8);
    const int pos = perm_pos(r);
#pragma unroll
    for (int e = 0; e < 8; ++e) *reinterpret_cast<short*>(dst + (c * 8 + e) * G::CS + pos * 2) = v[e];
  }
}

template <int HD>
MIFT_HD void zero_row_pad(char* dst, int tid) {
  using G = Geo<HD>;
  if (G::HDP == HD) return;
  constexpr int PADC = (G::HDP - HD) / 8;
  for (int i = tid; i < 64 * PADC; i += 256) {
    const int r = i / PADC, c = HD / 8 + i % PADC;
    *reinterpret_cast<short8*>(dst + r * G::RS + c * 16) = short8{0, 0, 0, 0, 0, 0, 0, 0};
  }
}

// Q-style fragments for 16 rows straight from global: frag[s] = X[row0 + (lane&15)][32s + 8(lane>>4) ..]
template <int HD>
MIFT_HD void load_reg_frags(bf16x8* f, const bf16* src, int64_t ld, int row, int nrows, int lane) {
  using G = Geo<HD>;
  const int gr = min(row, nrows - 1);
#pragma unroll
  for (int s = 0; s < G::NKS; ++s) {
    const int col = 32 * s + 8 * (lane >> 4);
    f[s] = col < HD ? *reinterpret_cast<const bf16x8*>(src + (int64_t)gr * ld + col) : zero_frag();
  }
}

MIFT_HD bool drop_keep(uint64_t seed, uint32_t thr, int64_t bh, int S, int q, int k) {
  return mift_keep(seed, ((uint64_t)bh * S + q) * S + k, thr);
}

// ============================== forward ====================================
template <int HD>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                       float* __restrict__ lse, const int* __restrict__ kv_len,
                                                       int B, int S, int H, float scale, uint64_t seed,
                                                       uint32_t thr, float inv_keep) {
  using G = Geo<HD>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ks = smem;
  char* Vt = smem + G::ROW_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, qc = lane & 15;
  const int nqt = (S + BQ - 1) / BQ;
  const int qt = nqt - 1 - (blockIdx.x % nqt);  // heavy (late) query tiles first
  const int bh = blockIdx.x / nqt;
  const int b = bh / H, h = bh % H;
  const int D = H * HD;
  const int64_t ld = 3LL * D;
  const bf16* Qg = qkv + (int64_t)b * S * ld + h * HD;
  const bf16* Kg = Qg + D;
  const bf16* Vg = Qg + 2 * D;
  const int klen = kv_len ? kv_len[b] : S;
  const int q0 = qt * BQ + wave * 16;
  const int myq = q0 + qc;
  const float c2 = scale * LOG2E;

  bf16x8 qf[G::NKS];
  load_reg_frags<HD>(qf, Qg, ld, myq, S, lane);
  zero_row_pad<HD>(Ks, tid);

  float m = -INFINITY, l = 0.f;
  float4_ o[G::NOT];
#pragma unroll
  for (int i = 0; i < G::NOT; ++i) o[i] = float4_{0.f, 0.f, 0.f, 0.f};

  const int kend = min((qt + 1) * BQ, klen);
  const int nkt = (kend + BKV - 1) / BKV;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * BKV;
    __syncthreads();
    load_row_tile<HD>(Ks, Kg, ld, k0, S, tid);
    load_col_tile<HD>(Vt, Vg, ld, k0, S, tid);
    __syncthreads();
    // S^T tile: 4 sub-tiles of 16 keys
    float4_ st[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st[t] = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < G::NKS; ++s) {
        bf16x8 kf = ld_frag(Ks + (t * 16 + qc) * G::RS + (4 * s + g) * 16);
        st[t] = mfma_bf16(kf, qf[s], st[t]);
      }
    }
    // mask + tile max (per query: lane-local 16 values, then across the 4 groups)
    float tmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + t * 16 + g * 4 + r;
        float v = st[t][r] * c2;
        if (key > myq || key >= klen) v = -INFINITY;
        st[t][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(m, tmax);
    const float alpha = (m == -INFINITY) ? 0.f : exp2f(m - mnew);
    m = mnew;
    float psum = 0.f;
    bf16x8 pf[2];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float p = (mnew == -INFINITY) ? 0.f : exp2f(st[t][r] - mnew);
        psum += p;
        if (thr != 0) {
          const int key = k0 + t * 16 + g * 4 + r;
          p = drop_keep(seed, thr, bh, S, myq, key) ? p * inv_keep : 0.f;
        }
        pf[t >> 1][(t & 1) * 4 + r] = (bf16)p;
      }
    l = l * alpha + psum;
    // rescale O (acc layout: row = g*4 + r -> query q0 + g*4 + r lives in lane g*4+r)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float ar = __shfl(alpha, g * 4 + r, 64);
#pragma unroll
      for (int i = 0; i < G::NOT; ++i) o[i][r] *= ar;
    }
    // O += P · V
#pragma unroll
    for (int i = 0; i < G::NOT; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 vf = ld_frag(Vt + (i * 16 + qc) * G::CS + (32 * s2 + 8 * g) * 2);
        o[i] = mfma_bf16(pf[s2], vf, o[i]);
      }
  }
  // finalize
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float inv_l = l > 0.f ? 1.f / l : 0.f;
  if (g == 0 && myq < S) lse[(int64_t)bh * S + myq] = (l > 0.f) ? (m + log2f(l)) * LN2 : -INFINITY;
  bf16* Og = out + (int64_t)b * S * D + h * HD;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float il = __shfl(inv_l, g * 4 + r, 64);
    const int q = q0 + g * 4 + r;
    if (q < S) {
#pragma unroll
      for (int i = 0; i < G::NOT; ++i) Og[(int64_t)q * D + i * 16 + qc] = (bf16)(o[i][r] * il);
    }
  }
}

// ======================== backward: D = rowsum(dO∘O) ========================
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(const bf16* __restrict__ o, const bf16* __restrict__ dout,
                                                           float* __restrict__ Dv, int BS, int H, int S) {
  // one wave per (token, head)
  const int lane = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= (int64_t)BS * H) return;
  const int64_t tok = item / H;
  const int h = item % H;
  const int D = H * HD;
  float s = 0.f;
  for (int c = lane; c < HD; c += 64) s += (float)o[tok * D + h * HD + c] * (float)dout[tok * D + h * HD + c];
  s = wave_sum(s);
  if (lane == 0) {
    const int b = tok / S, q = tok % S;
    Dv[((int64_t)b * H + h) * S + q] = s;
  }
}

// ============================ backward: dQ =================================
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                                          const float* __restrict__ lse, const float* __restrict__ Dv,
                                                          bf16* __restrict__ dqkv, const int* __restrict__ kv_len,
                                                          int B, int S, int H, float scale, uint64_t seed,
                                                          uint32_t thr, float inv_keep) {
  using G = Geo<HD>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ks = smem;                       // K rows (A of S^T)
  char* Vs = smem + G::ROW_BYTES;        // V rows (A of dP^T)
  char* Kt = smem + 2 * G::ROW_BYTES;    // K^T permuted (B of dQ)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, qc = lane & 15;
  const int nqt = (S + BQ - 1) / BQ;
  const int qt = nqt - 1 - (blockIdx.x % nqt);
  const int bh = blockIdx.x / nqt;
  const int b = bh / H, h = bh % H;
  const int D = H * HD;
  const int64_t ld = 3LL * D;
  const bf16* Qg = qkv + (int64_t)b * S * ld + h * HD;
  const bf16* Kg = Qg + D;
  const bf16* Vg = Qg + 2 * D;
  const bf16* dOg = dout + (int64_t)b * S * D + h * HD;
  const int klen = kv_len ? kv_len[b] : S;
  const int q0 = qt * BQ + wave * 16;
  const int myq = q0 + qc;
  const float c2 = scale * LOG2E;

  bf16x8 qf[G::NKS], df[G::NKS];
  load_reg_frags<HD>(qf, Qg, ld, myq, S, lane);
  load_reg_frags<HD>(df, dOg, D, myq, S, lane);
  const float lse2 = myq < S ? lse[(int64_t)bh * S + myq] * LOG2E : 0.f;
  const float Dq = myq < S ? Dv[(int64_t)bh * S + myq] : 0.f;
  zero_row_pad<HD>(Ks, tid);
  zero_row_pad<HD>(Vs, tid);

  float4_ dq[G::NOT];
#pragma unroll
  for (int i = 0; i < G::NOT; ++i) dq[i] = float4_{0.f, 0.f, 0.f, 0.f};

  const int kend = min((qt + 1) * BQ, klen);
  const int nkt = (kend + BKV - 1) / BKV;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * BKV;
    __syncthreads();
    load_row_tile<HD>(Ks, Kg, ld, k0, S, tid);
    load_row_tile<HD>(Vs, Vg, ld, k0, S, tid);
    load_col_tile<HD>(Kt, Kg, ld, k0, S, tid);
    __syncthreads();
    bf16x8 dsf[2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float4_ sa = float4_{0.f, 0.f, 0.f, 0.f}, pa = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < G::NKS; ++s) {
        sa = mfma_bf16(ld_frag(Ks + (t * 16 + qc) * G::RS + (4 * s + g) * 16), qf[s], sa);
        pa = mfma_bf16(ld_frag(Vs + (t * 16 + qc) * G::RS + (4 * s + g) * 16), df[s], pa);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + t * 16 + g * 4 + r;
        float p = (key > myq || key >= klen) ? 0.f : exp2f(sa[r] * c2 - lse2);
        float dp = pa[r];
        if (thr != 0) dp = drop_keep(seed, thr, bh, S, myq, key) ? dp * inv_keep : 0.f;
        const float ds = p * (dp - Dq);
        dsf[t >> 1][(t & 1) * 4 + r] = (bf16)ds;
      }
    }
#pragma unroll
    for (int i = 0; i < G::NOT; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        dq[i] = mfma_bf16(dsf[s2], ld_frag(Kt + (i * 16 + qc) * G::CS + (32 * s2 + 8 * g) * 2), dq[i]);
  }
  bf16* dQg = dqkv + (int64_t)b * S * ld + h * HD;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = q0 + g * 4 + r;
    if (q < S) {
#pragma unroll
      for (int i = 0; i < G::NOT; ++i) dQg[(int64_t)q * ld + i * 16 + qc] = (bf16)(dq[i][r] * scale);
    }
  }
}

// ========================== backward: dK, dV ===============================
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                                            const float* __restrict__ lse, const float* __restrict__ Dv,
                                                            bf16* __restrict__ dqkv, const int* __restrict__ kv_len,
                                                            int B, int S, int H, float scale, uint64_t seed,
                                                            uint32_t thr, float inv_keep) {
  using G = Geo<HD>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Qs = smem;                                   // Q rows (A of S)
  char* dOs = smem + G::ROW_BYTES;                   // dO rows (A of dP)
  char* Qt = smem + 2 * G::ROW_BYTES;                // Q^T permuted (B of dK)
  char* dOt = Qt + G::COL_BYTES;                     // dO^T permuted (B of dV)
  float* lse_s = reinterpret_cast<float*>(dOt + G::COL_BYTES);
  float* D_s = lse_s + 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, kc = lane & 15;
  const int nkt = (S + BKV - 1) / BKV;
  const int kt = blockIdx.x % nkt;
  const int bh = blockIdx.x / nkt;
  const int b = bh / H, h = bh % H;
  const int D = H * HD;
  const int64_t ld = 3LL * D;
  const bf16* Qg = qkv + (int64_t)b * S * ld + h * HD;
  const bf16* Kg = Qg + D;
  const bf16* Vg = Qg + 2 * D;
  const bf16* dOg = dout + (int64_t)b * S * D + h * HD;
  const int klen = kv_len ? kv_len[b] : S;
  const int k0 = kt * BKV + wave * 16;
  const int mykey = k0 + kc;
  const float c2 = scale * LOG2E;

  // K, V fragments of this wave's 16 keys as B operands: B[k=hd][n=key] = X[key][hd]
  bf16x8 kf[G::NKS], vf[G::NKS];
  load_reg_frags<HD>(kf, Kg, ld, mykey, S, lane);
  load_reg_frags<HD>(vf, Vg, ld, mykey, S, lane);
  zero_row_pad<HD>(Qs, tid);
  zero_row_pad<HD>(dOs, tid);

  float4_ dk[G::NOT], dv[G::NOT];
#pragma unroll
  for (int i = 0; i < G::NOT; ++i) {
    dk[i] = float4_{0.f, 0.f, 0.f, 0.f};
    dv[i] = float4_{0.f, 0.f, 0.f, 0.f};
  }
  const int nqt = (S + BQ - 1) / BQ;
  const bool active = kt * BKV < klen;
  for (int qt = active ? kt : nqt; qt < nqt; ++qt) {
    const int qb = qt * BQ;
    __syncthreads();
    load_row_tile<HD>(Qs, Qg, ld, qb, S, tid);
    load_row_tile<HD>(dOs, dOg, D, qb, S, tid);
    load_col_tile<HD>(Qt, Qg, ld, qb, S, tid);
    load_col_tile<HD>(dOt, dOg, D, qb, S, tid);
    if (tid < 64) {
      const int q = min(qb + tid, S - 1);
      lse_s[tid] = lse[(int64_t)bh * S + q] * LOG2E;
      D_s[tid] = Dv[(int64_t)bh * S + q];
    }
    __syncthreads();
    bf16x8 pf[2], dsf[2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float4_ sa = float4_{0.f, 0.f, 0.f, 0.f}, pa = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < G::NKS; ++s) {
        sa = mfma_bf16(ld_frag(Qs + (t * 16 + kc) * G::RS + (4 * s + g) * 16), kf[s], sa);
        pa = mfma_bf16(ld_frag(dOs + (t * 16 + kc) * G::RS + (4 * s + g) * 16), vf[s], pa);
      }
      // acc layout: row = query t*16 + g*4 + r, col = key kc
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = t * 16 + g * 4 + r;
        const int q = qb + ql;
        const bool valid = q < S && mykey <= q && mykey < klen;
        const float p = valid ? exp2f(sa[r] * c2 - lse_s[ql]) : 0.f;
        float pd = p, dp = pa[r];
        if (thr != 0) {
          const bool kp = valid && drop_keep(seed, thr, bh, S, q, mykey);
          pd = kp ? p * inv_keep : 0.f;
          dp = kp ? dp * inv_keep : 0.f;
        }
        const float ds = p * (dp - D_s[ql]);
        pf[t >> 1][(t & 1) * 4 + r] = (bf16)pd;
        dsf[t >> 1][(t & 1) * 4 + r] = (bf16)ds;
      }
    }
#pragma unroll
    for (int i = 0; i < G::NOT; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        dv[i] = mfma_bf16(pf[s2], ld_frag(dOt + (i * 16 + kc) * G::CS + (32 * s2 + 8 * g) * 2), dv[i]);
        dk[i] = mfma_bf16(dsf[s2], ld_frag(Qt + (i * 16 + kc) * G::CS + (32 * s2 + 8 * g) * 2), dk[i]);
      }
  }
  bf16* dKg = dqkv + (int64_t)b * S * ld + D + h * HD;
  bf16* dVg = dKg + D;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int key = k0 + g * 4 + r;
    if (key < S) {
#pragma unroll
      for (int i = 0; i < G::NOT; ++i) {
        dKg[(int64_t)key * ld + i * 16 + kc] = (bf16)(dk[i][r] * scale);
        dVg[(int64_t)key * ld + i * 16 + kc] = (bf16)dv[i][r];
      }
    }
  }
}

uint32_t thr_of(double p) { return mift_thr16(p); }

template <int HD>
void fwd_launch(const at::Tensor& qkv, at::Tensor& o, at::Tensor& lse, const int* kvl, int B, int S, int H, float scale,
                uint64_t seed, uint32_t thr, float inv_keep, hipStream_t st) {
  using G = Geo<HD>;
  const int nqt = (S + BQ - 1) / BQ;
  const int smem = G::ROW_BYTES + G::COL_BYTES;
  hipLaunchKernelGGL((attn_fwd_kernel<HD>), dim3(B * H * nqt), dim3(256), smem, st, (const bf16*)qkv.data_ptr(),
                     (bf16*)o.data_ptr(), lse.data_ptr<float>(), kvl, B, S, H, scale, seed, thr, inv_keep);
}

template <int HD>
void bwd_launch(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& o, const at::Tensor& lse,
                at::Tensor& Dv, at::Tensor& dqkv, const int* kvl, int B, int S, int H, float scale, uint64_t seed,
                uint32_t thr, float inv_keep, hipStream_t st) {
  using G = Geo<HD>;
  const int BS = B * S;
  hipLaunchKernelGGL((attn_bwd_pre_kernel<HD>), dim3(((int64_t)BS * H + 3) / 4), dim3(256), 0, st,
                     (const bf16*)o.data_ptr(), (const bf16*)dout.data_ptr(), Dv.data_ptr<float>(), BS, H, S);
  const int nqt = (S + BQ - 1) / BQ, nkt = (S + BKV - 1) / BKV;
  const int smem_dq = 2 * G::ROW_BYTES + G::COL_BYTES;
  hipLaunchKernelGGL((attn_bwd_dq_kernel<HD>), dim3(B * H * nqt), dim3(256), smem_dq, st, (const bf16*)qkv.data_ptr(),
                     (const bf16*)dout.data_ptr(), lse.data_ptr<float>(), Dv.data_ptr<float>(),
                     (bf16*)dqkv.data_ptr(), kvl, B, S, H, scale, seed, thr, inv_keep);
  const int smem_kv = 2 * G::ROW_BYTES + 2 * G::COL_BYTES + 2 * 64 * 4;
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HD>), dim3(B * H * nkt), dim3(256), smem_kv, st,
                     (const bf16*)qkv.data_ptr(), (const bf16*)dout.data_ptr(), lse.data_ptr<float>(),
                     Dv.data_ptr<float>(), (bf16*)dqkv.data_ptr(), kvl, B, S, H, scale, seed, thr, inv_keep);
}

}  // namespace

std::vector<at::Tensor> mift_attn_fwd(const at::Tensor& qkv, int64_t B, int64_t S, int64_t H, int64_t HD, double scale,
                                      double p, int64_t seed, const c10::optional<at::Tensor>& kv_len) {
  TORCH_CHECK(qkv.is_cuda() && qkv.is_contiguous() && qkv.scalar_type() == at::kBFloat16, "attn: bf16 contiguous qkv");
  TORCH_CHECK(qkv.numel() == B * S * 3 * H * HD, "attn: qkv shape");
  auto o = at::empty({B * S, H * HD}, qkv.options());
  auto lse = at::empty({B, H, S}, qkv.options().dtype(at::kFloat));
  const int* kvl = nullptr;
  if (kv_len) {
    TORCH_CHECK(kv_len->scalar_type() == at::kInt && kv_len->numel() == B, "attn: kv_len int32 [B]");
    kvl = kv_len->data_ptr<int>();
  }
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const float inv_keep = p > 0 ? mift_inv_keep(p) : 1.f;
  switch (HD) {
    case 64: fwd_launch<64>(qkv, o, lse, kvl, B, S, H, (float)scale, (uint64_t)seed, thr_of(p), inv_keep, st); break;
    case 80: fwd_launch<80>(qkv, o, lse, kvl, B, S, H, (float)scale, (uint64_t)seed, thr_of(p), inv_keep, st); break;
    case 128: fwd_launch<128>(qkv, o, lse, kvl, B, S, H, (float)scale, (uint64_t)seed, thr_of(p), inv_keep, st); break;
    case 32: fwd_launch<32>(qkv, o, lse, kvl, B, S, H, (float)scale, (uint64_t)seed, thr_of(p), inv_keep, st); break;
    default: TORCH_CHECK(false, "attn: unsupported head dim ", HD);
  }
  return {o, lse};
}

at::Tensor mift_attn_bwd(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& o, const at::Tensor& lse,
                         int64_t B, int64_t S, int64_t H, int64_t HD, double scale, double p, int64_t seed,
                         const c10::optional<at::Tensor>& kv_len) {
  TORCH_CHECK(dout.is_contiguous() && o.is_contiguous(), "attn_bwd: contiguous");
  auto dqkv = at::empty_like(qkv);
  auto Dv = at::empty({B, H, S}, qkv.options().dtype(at::kFloat));
  const int* kvl = kv_len ? kv_len->data_ptr<int>() : nullptr;
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const float inv_keep = p > 0 ? mift_inv_keep(p) : 1.f;
  switch (HD) {
    case 64: bwd_launch<64>(dout, qkv, o, lse, Dv, dqkv, kvl, B, S, H, (float)scale, (uint64_t)seed, thr_of(p), inv_keep, st); break;
    case 80: bwd_launch<80>(dout, qkv, o, lse, Dv, dqkv, kvl, B, S, H, (float)scale, (uint64_t)seed, thr_of(p), inv_keep, st); break;
    case 128: bwd_launch<128>(dout, qkv, o, lse, Dv, dqkv, kvl, B, S, H, (float)scale, (uint64_t)seed, thr_of(p), inv_keep, st); break;
    case 32: bwd_launch<32>(dout, qkv, o, lse, Dv, dqkv, kvl, B, S, H, (float)scale, (uint64_t)seed, thr_of(p), inv_keep, st); break;
    default: TORCH_CHECK(false, "attn_bwd: unsupported head dim ", HD);
  }
  return dqkv;
}
