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
//     Split over M across blocks.  Deterministic (default, MIFT_DETERMINISTIC != 0): every block
//     stores its fp32 partial tile to a slab and lora_wgrad_reduce adds the row-chunk partials of a
//     column tile in chunk order into the output (bit-identical run to run); with
//     MIFT_DETERMINISTIC=0 the blocks add into the output with fp32 atomics instead.
#include "common.h"
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <algorithm>
#include <tuple>
#include <vector>

// rowproj.hip: the 4-wave 16-row MFMA projection, used for contiguous x at K in {768, 1024, 2304}
bool mift_rowproj_lora_proj(const at::Tensor& x, const at::Tensor& w, at::Tensor& out, double alpha, double p,
                            int64_t seed, int64_t rows);

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
// Grid = (M/(16·MT) row blocks) x KS K-splits.  MT = 1 (16 rows per block) doubles the blocks of a
// distilgpt2-size M (8192 rows -> 512 blocks, two per CU) so more X bytes are in flight per CU;
// NTI = 1 when only the first 16 rows of W are non-zero (one adapter, r <= 16): half the MFMAs
// and W loads of the 32-column product.  KS > 1: every block stores its fp32 partial to ws[kss]
// write-through (sc1) and the LAST of a row block's KS blocks to arrive (counter per row block,
// common.h mift_group_arrival: no release fence) sums the KS partials in split order into the
// 16-bit output — no lora_proj_reduce launch (OPT micro-batches ran 7 per layer, 4.7 us each).
// The round-2 form fenced every block (~3.5 us each) and kept the separate reduction.
template <typename T, int NW, int MT, int NTI>
__global__ __launch_bounds__(NW * 64) void lora_proj_kernel(const T* __restrict__ X, const T* __restrict__ W,
                                                        T* __restrict__ out, int M, int K, int ldx, float alpha,
                                                        uint64_t seed, const int64_t* __restrict__ sstep, uint32_t thr, float inv_keep, int KS,
                                                        float* __restrict__ ws, int wrows, unsigned* __restrict__ flags) {
  seed = mift_seed(seed, sstep);
  constexpr int RB = 16 * MT;  // rows per block
  __shared__ float red[NW][RB][33];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on it
  const int g = lane >> 4, fr = lane & 15;
  const int mb = blockIdx.x / KS, kss = blockIdx.x % KS;
  const int m0 = mb * RB;
  float4_ acc[MT][NTI];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTI; ++j) acc[i][j] = float4_{0.f, 0.f, 0.f, 0.f};
  int rows[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) rows[i] = min(m0 + 16 * i + fr, M - 1);
  const int nks_all = K / 32;
  const int per_blk = (nks_all + KS - 1) / KS;
  const int kb0 = kss * per_blk, nks = min(nks_all, kb0 + per_blk);
  // each wave owns a contiguous K range of the block's split; UNR k-steps of loads are issued
  // back to back before their MFMAs (memory-level parallelism: one 16-B X load per lane per
  // M-tile per k-step)
  constexpr int UNR = MT == 1 ? 8 : 4;
  const int per = (nks - kb0 + NW - 1) / NW;
  const int kbeg = kb0 + wave * per, kend = min(nks, kbeg + per);
  // LoRA-input dropout: kept elements enter the MFMA unscaled (AND on packed pairs); the host folds
  // 1/(1-p) into alpha, applied once to the fp32 sums
  const bool hz = (uint64_t)M * K < (1ull << 33);
  const uint32_t hm0 = mift_hmix(seed, 0);
  for (int ks0 = kbeg; ks0 < kend; ks0 += UNR) {
    short8 ra[UNR][MT], rb[UNR][NTI];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int col = min(ks0 + u, nks - 1) * 32 + g * 8;
#pragma unroll
      for (int i = 0; i < MT; ++i) ra[u][i] = *reinterpret_cast<const short8*>(X + (int64_t)rows[i] * ldx + col);
      // rows >= wrows of W are zero padding: not fetched (the rank-8 adapters' 16-row tile is half
      // padding, and every block re-reads W from L2)
#pragma unroll
      for (int j = 0; j < NTI; ++j)
        rb[u][j] = j * 16 + fr < wrows ? *reinterpret_cast<const short8*>(W + (int64_t)(j * 16 + fr) * K + col)
                                       : short8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (ks0 + u >= kend) break;
      const int col = (ks0 + u) * 32 + g * 8;
      frag_t<T> a[MT], b[NTI];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        short8 v = ra[u][i];
        if (thr != 0) {
          uint32_t w[4], km[4];
          __builtin_memcpy(w, &v, 16);
          mift_andmask8(seed, hm0, hz, (uint64_t)rows[i] * K + col, thr, km);
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] &= km[e];
          __builtin_memcpy(&v, w, 16);
        }
        __builtin_memcpy(&a[i], &v, 16);
      }
#pragma unroll
      for (int j = 0; j < NTI; ++j) __builtin_memcpy(&b[j], &rb[u][j], 16);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTI; ++j) acc[i][j] = mfma16<T>(a[i], b[j], acc[i][j]);
    }
  }
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][i * 16 + g * 4 + r][j * 16 + fr] = j < NTI ? acc[i][j < NTI ? j : 0][r] : 0.f;
  __syncthreads();
  auto rsum = [&](int r, int c) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][r][c];
    return v;
  };
  if (KS == 1) {
    for (int e = tid; e < RB * 32; e += NW * 64) {
      const int r = e >> 5, c = e & 31;
      if (m0 + r < M) out[(int64_t)(m0 + r) * 32 + c] = (T)(rsum(r, c) * alpha);
    }
    return;
  }
  float* wp = ws + (int64_t)kss * M * 32;
  for (int e = tid; e < RB * 32; e += NW * 64) {
    const int r = e >> 5, c = e & 31;
    if (m0 + r < M) mift_st_sc1(wp + (int64_t)(m0 + r) * 32 + c, rsum(r, c));
  }
  __shared__ int last;
  if (!mift_group_arrival(flags + mb, (unsigned)KS, &last)) return;
  for (int e = tid; e < RB * 32; e += NW * 64) {
    const int r = e >> 5, c = e & 31;
    if (m0 + r >= M) continue;
    float v = 0.f;
    for (int s = 0; s < KS; ++s) v += ws[((int64_t)s * M + m0 + r) * 32 + c];
    out[(int64_t)(m0 + r) * 32 + c] = (T)(v * alpha);
  }
}

// ----------------------------------------------------------------- lora_wgrad
constexpr int XS = 160;  // X tile row stride (bytes): 64 cols (128 B) padded to an odd multiple of 32 B
constexpr int YS = 96;   // Y tile row stride: 32 cols (64 B) -> 96 B

template <typename T>
MIFT_HD v4s tr_read(const char* lds_base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(lds_base + off));
}

// Grouped: ONE launch reduces every weight-gradient problem of a layer's backward (dB and dA of
// each adapter, up to WG_MAXP).  Block b belongs to the problem whose [blk0, next blk0) holds it;
// a problem is split into P/64 column tiles x ceil(M / rows) row chunks.  One launch per layer
// instead of two per adapter: the per-adapter launches were ~10 us each for 12-50 MB of reads
// (ramp + tail dominate), 0.43 ms of the 5.8 ms distilgpt2 step on the critical path even on the
// side stream (tools/step_ab.py, MIFT_DIAG_SKIP=wgrad).
constexpr int WG_MAXP = 16, WG_MAXS = 4;
struct WgSlot {
  int qoff, rank;   // columns [qoff, qoff + rank) of the 32-wide product ...
  int64_t offset;   // ... land at out + offset in dB [P, rank] (mode 1) / dA [rank, P] (mode 2) layout
};
struct WgProb {
  const void* X;    // [M, P] rows of stride ldx (a column slice of a wider tensor is fine)
  const void* Y;    // [M, 32] contiguous
  int ldx, P, M, rows, blk0, mode, nslot;
  int tile0;        // first column tile of this problem in the reduction launch (deterministic mode)
  uint32_t thr;     // LoRA-input dropout on X (dA): keep iff hash >= thr, index = row * P + col
  float inv_keep;
  uint64_t seed;
  WgSlot slot[WG_MAXS];
};
struct WgArgs {
  float* out;
  float* ws;        // deterministic mode: [blocks][NQT*16][64] fp32 partial slabs (nullptr: atomics)
  int* flags;       // (unused: the slabs are always reduced by lora_wgrad_reduce_kernel)
  const int64_t* sstep;
  int np;
  WgProb p[WG_MAXP];
};

// Output index of element (pp, q) of problem pr's [P, 32] product (-1: column q feeds no slot).
// mode 0: dense [P,32] at slot 0; mode 1: dB [P, rank]; mode 2: dA [rank, P] per slot.
MIFT_HD int64_t wg_out_index(const WgProb& pr, int64_t pp, int q, int si) {
  if (pr.mode == 0) return si == 0 ? pr.slot[0].offset + pp * 32 + q : -1;
  const WgSlot& sl = pr.slot[si];
  if (q < sl.qoff || q >= sl.qoff + sl.rank) return -1;
  return sl.offset + (pr.mode == 1 ? pp * sl.rank + (q - sl.qoff) : (int64_t)(q - sl.qoff) * pr.P + pp);
}

// Block epilogue of both wgrad kernels: acc[c][r] = product[p0 + wave*16 + g*4 + r][c*16 + li].
template <int NQT>
MIFT_HD void wg_store(const WgArgs& args, const WgProb& pr, const float4_ (&acc)[NQT], int p0, int wave, int g, int li) {
  if (args.ws != nullptr) {  // deterministic: slab [c][li][64 rows of p], one 16-B store per (c)
    float* slab = args.ws + (size_t)blockIdx.x * (NQT * 16 * 64);
#pragma unroll
    for (int c = 0; c < NQT; ++c)
      *reinterpret_cast<float4_*>(slab + (c * 16 + li) * 64 + wave * 16 + g * 4) = acc[c];
    return;
  }
#pragma unroll
  for (int c = 0; c < NQT; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t pp = p0 + wave * 16 + g * 4 + r;
      const int q = c * 16 + li;
#pragma unroll 1
      for (int si = 0; si < (pr.mode == 0 ? 1 : pr.nslot); ++si) {
        const int64_t o = wg_out_index(pr, pp, q, si);
        if (o >= 0) atomicAdd(args.out + o, acc[c][r]);
      }
    }
}

template <int NQT>
MIFT_HD void wg_reduce_tile(const WgArgs& args, const WgProb& pr, int pt);

// Split-M weight gradients: each block reduces a row chunk of one 64-column tile of one problem
// (X^T·Y over its rows) with MFMA from LDS images of the X and Y row groups.  Two register sets of
// NB-step load groups alternate, so group g+2's global loads are issued as soon as group g has been
// written to LDS and group g+1's have had a whole iteration to land (round 2's one-group loop paid the
// full load latency per group; removed in round 6).  NQT = 1 when every
// slot of the launch lives in columns [0, 16) (rank <= 16, one adapter per input): one MFMA per
// 32-row step instead of two and half the Y bytes.
template <typename T, int NQT>
__global__ __launch_bounds__(256) void lora_wgrad2_kernel(const WgArgs args) {
  int pi = 0;
#pragma unroll 1
  while (pi + 1 < args.np && (int)blockIdx.x >= args.p[pi + 1].blk0) ++pi;
  const WgProb& pr = args.p[pi];
  const T* __restrict__ X = reinterpret_cast<const T*>(pr.X);
  const T* __restrict__ Y = reinterpret_cast<const T*>(pr.Y);
  const int M = pr.M, P = pr.P, ldx = pr.ldx, rows_per_block = pr.rows;
  const uint32_t thr = pr.thr;
  const float inv_keep = pr.inv_keep;
  const uint64_t seed = mift_seed(pr.seed, args.sstep);
  const int lb = blockIdx.x - pr.blk0;
  constexpr int NB = 4;
  constexpr int YT = NQT == 2 ? 128 : 64;  // threads loading Y (16 B each: 4 or 2 chunks per 32-col row)
  __shared__ __attribute__((aligned(16))) char Xs[NB][32 * XS];
  __shared__ __attribute__((aligned(16))) char Ys[NB][32 * YS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int ntp = P / 64;
  const int pt = lb % ntp, ms = lb / ntp;
  const int p0 = pt * 64;
  const int mbeg = ms * rows_per_block;
  const int mend = min(mbeg + rows_per_block, M);
  MIFT_ASSERT(P % 64 == 0 && mbeg < M);
  float4_ acc[NQT];
#pragma unroll
  for (int c = 0; c < NQT; ++c) acc[c] = float4_{0.f, 0.f, 0.f, 0.f};

  const int xr = tid >> 3, xc = tid & 7;
  const int yr = NQT == 2 ? (tid & 127) >> 2 : (tid & 63) >> 1, yc = NQT == 2 ? tid & 3 : tid & 1;
  short8 xa[NB], ya[NB], xb[NB], yb[NB];
  auto gload = [&](short8 (&xv)[NB], short8 (&yv)[NB], int m0g) {
#pragma unroll
    for (int s = 0; s < NB; ++s) {
      const int m = m0g + 32 * s;
      const int gm = min(m + xr, M - 1);
      xv[s] = *reinterpret_cast<const short8*>(X + (int64_t)gm * ldx + p0 + xc * 8);
      if (tid < YT) {
        const int gy = min(m + yr, M - 1);
        yv[s] = *reinterpret_cast<const short8*>(Y + (int64_t)gy * 32 + yc * 8);
      }
    }
  };
  // LoRA-input dropout on X: the kept elements enter the MFMA unscaled (a bitwise AND on the packed
  // 16-bit pairs) and the 1/(1-p) factor is applied to the fp32 accumulators once at the end —
  // the per-element unpack/scale/round/repack cost as much VALU as the hash itself (the masked dA
  // problems were VALU-issue bound: +28 % over unmasked ones).  The pair hashes share one hoisted
  // high-word mix (element indices < 2^33).
  const bool hz = (uint64_t)M * P < (1ull << 33);
  const uint32_t hm0 = mift_hmix(seed, 0);
  auto lstore = [&](short8 (&xv)[NB], short8 (&yv)[NB], int m0g) {
#pragma unroll
    for (int s = 0; s < NB; ++s) {
      const int m = m0g + 32 * s;
      const bool valid = (m + xr) < mend;
      short8 v = xv[s];
      if (!valid) {
        v = short8{0, 0, 0, 0, 0, 0, 0, 0};
      } else if (thr != 0) {
        uint32_t w[4], km[4];
        __builtin_memcpy(w, &v, 16);
        mift_andmask8(seed, hm0, hz, (uint64_t)(m + xr) * P + p0 + xc * 8, thr, km);  // 8-aligned columns
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] &= km[e];
        __builtin_memcpy(&v, w, 16);
      }
      *reinterpret_cast<short8*>(Xs[s] + xr * XS + xc * 16) = v;
      if (tid < YT) {
        short8 w = yv[s];
        if ((m + yr) >= mend) w = short8{0, 0, 0, 0, 0, 0, 0, 0};
        *reinterpret_cast<short8*>(Ys[s] + yr * YS + yc * 16) = w;
      }
    }
  };
  const int q4 = li >> 2, p4 = li & 3;
  const int rowA = 4 * g + q4;
  const int xoff = rowA * XS + (wave * 16 + p4 * 4) * 2;
  const int yoff0 = rowA * YS + (0 * 16 + p4 * 4) * 2;
  const int yoff1 = rowA * YS + (1 * 16 + p4 * 4) * 2;
  auto compute = [&](int mg) {
#pragma unroll
    for (int s = 0; s < NB; ++s) {
      if (mg + 32 * s >= mend) break;
      const char* xbp = Xs[s];
      const char* ybp = Ys[s];
      v4s a0 = tr_read<T>(xbp, xoff), a1 = tr_read<T>(xbp, xoff + 16 * XS);
      v4s b00 = tr_read<T>(ybp, yoff0), b01 = tr_read<T>(ybp, yoff0 + 16 * YS);
      frag_t<T> af, bf0;
      short8 t = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      __builtin_memcpy(&af, &t, 16);
      short8 u = {b00[0], b00[1], b00[2], b00[3], b01[0], b01[1], b01[2], b01[3]};
      __builtin_memcpy(&bf0, &u, 16);
      acc[0] = mfma16<T>(af, bf0, acc[0]);
      if constexpr (NQT == 2) {
        v4s b10 = tr_read<T>(ybp, yoff1), b11 = tr_read<T>(ybp, yoff1 + 16 * YS);
        frag_t<T> bf1;
        short8 w = {b10[0], b10[1], b10[2], b10[3], b11[0], b11[1], b11[2], b11[3]};
        __builtin_memcpy(&bf1, &w, 16);
        acc[1] = mfma16<T>(af, bf1, acc[1]);
      }
    }
  };
  constexpr int GR = 32 * NB;  // rows per load group
  if (mbeg < mend) gload(xa, ya, mbeg);
  if (mbeg + GR < mend) gload(xb, yb, mbeg + GR);
  for (int mg = mbeg; mg < mend; mg += 2 * GR) {
    __syncthreads();
    lstore(xa, ya, mg);
    __syncthreads();
    if (mg + 2 * GR < mend) gload(xa, ya, mg + 2 * GR);
    compute(mg);
    if (mg + GR >= mend) break;
    __syncthreads();
    lstore(xb, yb, mg + GR);
    __syncthreads();
    if (mg + 3 * GR < mend) gload(xb, yb, mg + 3 * GR);
    compute(mg + GR);
  }
  if (thr != 0) {
#pragma unroll
    for (int c = 0; c < NQT; ++c) acc[c] *= inv_keep;
  }
  wg_store<NQT>(args, pr, acc, p0, wave, g, li);
}

// Deterministic reduction: block t = column tile t of the launch (problem pi, tile pt) sums the
// row-chunk slabs of that tile in chunk order and adds the result to the output — each output
// element is owned by exactly one thread (the host checks that the problems' slots are disjoint).
// Sum the chunk slabs of column tile pt of problem pr in chunk order and add the result into the
// output (one thread per 4 slab elements of each 16-column group).
template <int NQT>
MIFT_HD void wg_reduce_tile(const WgArgs& args, const WgProb& pr, int pt) {
  const int ntp = pr.P / 64;
  const int nch = (pr.M + pr.rows - 1) / pr.rows;
  constexpr int SL = NQT * 16 * 64;
  const size_t cstep = (size_t)ntp * SL;
  const float* base = args.ws + (size_t)(pr.blk0 + pt) * SL;
  // chunk slabs added strictly in chunk order (the deterministic result); the loads of all NQT
  // column groups and CB chunks are issued together (the serial dependent-load chain was
  // latency-bound, ~10 us per distilgpt2 layer; 8 chunks of one group at a time paid more trips)
  constexpr int CB = 16 / NQT;  // chunk slabs per batch: 16 float4 loads in flight per thread
  float4_ sum[NQT];
#pragma unroll
  for (int k = 0; k < NQT; ++k) sum[k] = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int ch0 = 0; ch0 < nch; ch0 += CB) {
    float4_ v[NQT][CB];
#pragma unroll
    for (int k = 0; k < NQT; ++k)
#pragma unroll
      for (int u = 0; u < CB; ++u)
        v[k][u] = *reinterpret_cast<const float4_*>(base + (threadIdx.x + 256 * k) * 4 +
                                                     (size_t)min(ch0 + u, nch - 1) * cstep);
#pragma unroll
    for (int k = 0; k < NQT; ++k)
#pragma unroll
      for (int u = 0; u < CB; ++u)
        if (ch0 + u < nch) sum[k] += v[k][u];
  }
#pragma unroll
  for (int k = 0; k < NQT; ++k) {
    const int e = (threadIdx.x + 256 * k) * 4;  // slab element: [c][li][p]
    const int c = e / 1024, li = (e / 64) % 16, pl = e % 64;
    const int q = c * 16 + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t pp = (int64_t)pt * 64 + pl + r;
#pragma unroll 1
      for (int si = 0; si < (pr.mode == 0 ? 1 : pr.nslot); ++si) {
        const int64_t o = wg_out_index(pr, pp, q, si);
        if (o >= 0) args.out[o] += sum[k][r];
      }
    }
  }
}

template <int NQT>
__global__ __launch_bounds__(256) void lora_wgrad_reduce_kernel(const WgArgs args) {
  int pi = 0;
#pragma unroll 1
  while (pi + 1 < args.np && (int)blockIdx.x >= args.p[pi + 1].tile0) ++pi;
  wg_reduce_tile<NQT>(args, args.p[pi], blockIdx.x - args.p[pi].tile0);
}

}  // namespace

namespace {
// persistent per-row-block arrival counters of lora_proj's K-split reduction (zeroed once, re-armed by
// each row block's last arriver; stream-ordered users; first allocated by an eager call)
unsigned* lp_flags(int n) {
  static at::Tensor flags;
  if (!flags.defined() || flags.numel() < n)
    flags = at::zeros({std::max<int64_t>(n, 1 << 14)}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA));
  return reinterpret_cast<unsigned*>(flags.data_ptr<int>());
}
}  // namespace

at::Tensor mift_lora_proj(const at::Tensor& x, const at::Tensor& w, double alpha, double p, int64_t seed,
                          int64_t rows) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "lora_proj: x [M,K] row-major");
  TORCH_CHECK(w.is_contiguous() && w.size(0) == 32 && w.size(1) == x.size(1), "lora_proj: w [32,K]");
  TORCH_CHECK(x.scalar_type() == w.scalar_type(), "lora_proj: dtype");
  TORCH_CHECK(rows >= 1 && rows <= 32, "lora_proj: non-zero rows of w in [1, 32]");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(K % 32 == 0 && x.stride(0) % 8 == 0, "lora_proj: K % 32, aligned rows");
  auto out = at::empty({M, 32}, x.options());
  if (M == 0) return out;
  if (mift_rowproj_lora_proj(x, w, out, alpha, p, seed, rows)) return out;  // rowproj.hip, MODE 2
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const uint32_t thr = mift_thr16(p);
  const float ik = p > 0 ? mift_inv_keep(p) : 1.f;
  const int cus = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
  }();
  // 16-row blocks while 32-row blocks would leave fewer than two per CU (MIFT_LORA_MT=1|2 forces)
  const char* mte = getenv("MIFT_LORA_MT");
  const int MT = mte ? (atoi(mte) == 1 ? 1 : 2) : ((M + 31) / 32 >= 2 * cus ? 2 : 1);
  const int mblocks = (M + 16 * MT - 1) / (16 * MT), nks = K / 32;
  static const int ks_env = [] { const char* e = getenv("MIFT_LORA_KS"); return e ? atoi(e) : 0; }();
  // K-splits only when the row blocks alone leave CUs idle (>= ~1024 blocks, >= 4 k-steps each).  With
  // at least one row block per CU the split's hand-off costs more than the extra blocks give: OPT-2.7B
  // at micro-batch 12 (M = 6144, 384 row blocks, K = 2560) ran its projections at 22.3 / 39.1 us with
  // KS = 3 and 19.4 / 35.2 us unsplit, step 675 -> 669 ms (profiles/r4/lora_proj_ks_opt27b_mb12.txt)
  int KS = mblocks >= cus ? 1 : std::max(1, std::min(std::max(1, nks / 4), (1024 + mblocks - 1) / mblocks));
  if (ks_env > 0) KS = std::max(1, std::min(ks_env, std::max(1, nks / 4)));  // A/B override
  float* ws = nullptr;
  unsigned* flags = nullptr;
  at::Tensor wsb;
  if (KS > 1) {
    wsb = at::empty({(int64_t)KS * M * 32}, x.options().dtype(at::kFloat));
    ws = wsb.data_ptr<float>();
    flags = lp_flags(mblocks);
  }
  const int grid = mblocks * KS;
  const bool one_tile = rows <= 16;
  auto go = [&](auto tt) {
    using T = decltype(tt);
    auto args = std::make_tuple((const T*)x.data_ptr(), (const T*)w.data_ptr(), (T*)out.data_ptr(), M, K,
                                (int)x.stride(0), (float)alpha * ik, (uint64_t)seed, mift_seed_step(), thr, ik, KS, ws,
                                (int)rows, flags);
    auto launch = [&](auto kern, int threads) {
      std::apply([&](auto... a) { hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, st, a...); }, args);
    };
    // MIFT_LORA_NW=8 (A/B only): 8-wave blocks, each wave half the k-steps — measured slower at OPT-2.7B
    // mb 12 (20.7 / 37.8 vs 19.4 / 35.2 us, step 647 vs 644 ms: profiles/r4/lora_proj_nw8_rejected.txt)
    static const int nw_env = [] { const char* e = getenv("MIFT_LORA_NW"); return e ? atoi(e) : 0; }();
    const bool nw8 = nw_env == 8;
    if (nw8) {
      if (MT == 1 && one_tile) launch(lora_proj_kernel<T, 8, 1, 1>, 512);
      else if (MT == 1) launch(lora_proj_kernel<T, 8, 1, 2>, 512);
      else if (one_tile) launch(lora_proj_kernel<T, 8, 2, 1>, 512);
      else launch(lora_proj_kernel<T, 8, 2, 2>, 512);
    } else if (MT == 1 && one_tile) launch(lora_proj_kernel<T, 4, 1, 1>, 256);
    else if (MT == 1) launch(lora_proj_kernel<T, 4, 1, 2>, 256);
    else if (one_tile) launch(lora_proj_kernel<T, 4, 2, 1>, 256);
    else launch(lora_proj_kernel<T, 4, 2, 2>, 256);
  };
  if (x.scalar_type() == at::kBFloat16) go(bf16{});
  else go(fp16{});
  return out;
}

namespace {
// persistent per-column-tile arrival counters of the in-kernel slab reduction (zeroed once; every
// finisher re-arms its own; first allocated by an eager call, outside any hipGraph capture)

template <typename T>
void launch_wgrad(WgArgs& args, hipStream_t st) {
  // rows per block: ~2048 blocks over the group (eight per CU: loads of several blocks in flight
  // per CU), a multiple of the 128-row load group, >= 128 (MIFT_WGRAD_BLOCKS: A/B knob)
  const char* te = getenv("MIFT_WGRAD_BLOCKS");
  const int64_t target = te ? std::max(1, atoi(te)) : 2048;
  int64_t work = 0;
  for (int i = 0; i < args.np; ++i) work += (int64_t)(args.p[i].P / 64) * args.p[i].M;
  const int64_t rows = std::max<int64_t>(128, (work / target + 127) / 128 * 128);
  int blk = 0;
  for (int i = 0; i < args.np; ++i) {
    WgProb& p = args.p[i];
    p.rows = (int)std::min<int64_t>(rows, (p.M + 127) / 128 * 128);
    p.blk0 = blk;
    blk += (p.P / 64) * ((p.M + p.rows - 1) / p.rows);
  }
  if (blk == 0) return;
  bool narrow = true;  // every slot within columns [0, 16)
  for (int i = 0; i < args.np; ++i) {
    if (args.p[i].mode == 0) narrow = false;
    for (int si = 0; si < args.p[i].nslot; ++si)
      if (args.p[i].slot[si].qoff + args.p[i].slot[si].rank > 16) narrow = false;
  }
  const int nqt = narrow ? 1 : 2;
  at::Tensor ws;
  args.flags = nullptr;
  if (mift_deterministic()) {
    ws = at::empty({(int64_t)blk * nqt * 16 * 64}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA));
    args.ws = ws.data_ptr<float>();
    int tiles = 0;
    for (int i = 0; i < args.np; ++i) {
      args.p[i].tile0 = tiles;
      tiles += args.p[i].P / 64;
    }
    if (narrow) lora_wgrad2_kernel<T, 1><<<blk, 256, 0, st>>>(args);
    else lora_wgrad2_kernel<T, 2><<<blk, 256, 0, st>>>(args);
    // (an in-launch slab reduction by each column tile's last chunk block was measured cost-neutral at
    // best, round 4, profiles/r4/step_ab_wgrad_fin_write_through.jsonl, and removed in round 6)
    if (nqt == 1) lora_wgrad_reduce_kernel<1><<<tiles, 256, 0, st>>>(args);
    else lora_wgrad_reduce_kernel<2><<<tiles, 256, 0, st>>>(args);
    return;
  }
  args.ws = nullptr;
  if (narrow) lora_wgrad2_kernel<T, 1><<<blk, 256, 0, st>>>(args);
  else lora_wgrad2_kernel<T, 2><<<blk, 256, 0, st>>>(args);
}
}  // namespace

// Grouped LoRA weight gradients into a flat fp32 tensor `out` (the grad arena, or a dense [P,32]):
//   xs[i] [M_i, P_i] (row stride free, unit column stride), ys[i] [M_i, 32];
//   meta[i] = {mode, nslot, (qoff, rank, offset) x WG_MAXS, seed};  ps[i] = LoRA-input dropout p on xs[i].
void mift_lora_wgrad_group(at::Tensor& out, const std::vector<at::Tensor>& xs, const std::vector<at::Tensor>& ys,
                           const std::vector<int64_t>& meta, const std::vector<double>& ps) {
  const int np = (int)xs.size();
  constexpr int MW = 3 + 3 * WG_MAXS;
  TORCH_CHECK(np >= 1 && np <= WG_MAXP && (int)ys.size() == np && (int)ps.size() == np &&
                  (int)meta.size() == np * MW, "lora_wgrad_group: 1..16 problems, meta/ps sizes");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.is_cuda(), "lora_wgrad_group: out fp32");
  const auto dt = xs[0].scalar_type();
  TORCH_CHECK(dt == at::kBFloat16 || dt == at::kHalf, "lora_wgrad_group: bf16/fp16");
  WgArgs args{};
  args.out = out.data_ptr<float>();
  args.sstep = mift_seed_step();
  int n = 0;
  for (int i = 0; i < np; ++i) {
    const at::Tensor& x = xs[i];
    const at::Tensor& y = ys[i];
    const int64_t* m = meta.data() + i * MW;
    TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 && x.scalar_type() == dt,
                "lora_wgrad_group: x [M,P] with 16-B aligned rows");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "lora_wgrad_group: x 16-B aligned");
    TORCH_CHECK(y.dim() == 2 && y.is_contiguous() && y.size(1) == 32 && y.size(0) == x.size(0) && y.scalar_type() == dt,
                "lora_wgrad_group: y [M,32]");
    const int P = x.size(1), M = x.size(0);
    TORCH_CHECK(P % 64 == 0, "lora_wgrad_group: P % 64 == 0");
    const int mode = (int)m[0], nslot = (int)m[1];
    TORCH_CHECK(mode >= 0 && mode <= 2 && nslot >= 1 && nslot <= WG_MAXS, "lora_wgrad_group: mode / slots");
    if (M == 0) continue;
    WgProb& p = args.p[n++];
    p.X = x.data_ptr();
    p.Y = y.data_ptr();
    p.ldx = (int)x.stride(0);
    p.P = P;
    p.M = M;
    p.mode = mode;
    p.nslot = nslot;
    p.thr = mift_thr16(ps[i]);
    p.inv_keep = ps[i] > 0 ? mift_inv_keep(ps[i]) : 1.f;
    p.seed = (uint64_t)m[2 + 3 * WG_MAXS];
    for (int si = 0; si < nslot; ++si) {
      const int qoff = (int)m[2 + 3 * si], rank = (int)m[3 + 3 * si];
      const int64_t off = m[4 + 3 * si];
      TORCH_CHECK(qoff >= 0 && rank >= 1 && qoff + rank <= 32, "lora_wgrad_group: slot columns");
      const int64_t need = mode == 0 ? (int64_t)P * 32 : (int64_t)P * rank;
      TORCH_CHECK(off >= 0 && off + need <= out.numel(), "lora_wgrad_group: slot range outside out");
      p.slot[si] = WgSlot{qoff, rank, off};
    }
  }
  args.np = n;
  if (n == 0) return;
  if (mift_deterministic()) {  // the reduction kernel writes each output element from ONE thread
    std::vector<std::pair<int64_t, int64_t>> iv;
    for (int i = 0; i < n; ++i)
      for (int si = 0; si < (args.p[i].mode == 0 ? 1 : args.p[i].nslot); ++si) {
        const WgSlot& sl = args.p[i].slot[si];
        iv.emplace_back(sl.offset, sl.offset + (int64_t)args.p[i].P * (args.p[i].mode == 0 ? 32 : sl.rank));
      }
    std::sort(iv.begin(), iv.end());
    for (size_t k = 1; k < iv.size(); ++k)
      TORCH_CHECK(iv[k].first >= iv[k - 1].second, "lora_wgrad_group: overlapping output slots in one launch");
  }
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  if (dt == at::kBFloat16) launch_wgrad<bf16>(args, st);
  else launch_wgrad<fp16>(args, st);
}

// one problem (tests, non-arena paths): out fp32, accumulated; mode 0 -> out[P,32];
// mode 1/2 -> out is a flat arena and the result lands at out[offset:] in dB [P,r] / dA [r,P] layout
void mift_lora_wgrad(const at::Tensor& x, const at::Tensor& y, at::Tensor& out, double p, int64_t seed, int64_t mode,
                     int64_t rank, int64_t offset, int64_t qoff) {
  TORCH_CHECK(y.is_contiguous() && y.size(1) == 32, "lora_wgrad: shapes");
  if (mode == 0) TORCH_CHECK(out.numel() == x.size(1) * 32, "lora_wgrad: out [P,32]");
  std::vector<int64_t> meta(3 + 3 * WG_MAXS, 0);
  meta[0] = mode;
  meta[1] = 1;
  meta[2] = mode == 0 ? 0 : qoff;
  meta[3] = mode == 0 ? 32 : rank;
  meta[4] = offset;
  meta[2 + 3 * WG_MAXS] = seed;
  mift_lora_wgrad_group(out, {x}, {y}, meta, {p});
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

// ------------------------------------------------------------ pack_lora_multi
// The shared-input adapter groups (OPT's q/k/v as one [3d, d] GEMM, ops/fused.py MultiAdapterOps):
// adapter j of a group owns rank columns [q_j, q_j + r_j) of the 32 and output rows [n0_j, n1_j).
// Group g's operands (one buffer, address in its table row): A32s [32,K] (s_j·A_j in rows q_j..),
// B32 [N,32] (B_j in its row span / rank columns), B32t [32,N] (s_j·B_jᵀ), At32 [K,32] (A_jᵀ); zeros
// elsewhere.  One launch per optimizer step for every group (the torch-op form ran ~22 kernels per
// layer inside the replayed OPT step: zero fills, scaled slice copies, casts).
//   table[g] = {K, N, nslots, out_ptr, then per slot j < 4: r, q, n0, n1, offA, offB};  scales[g][j]
constexpr int MULTI_COLS = 4 + 4 * 6;
namespace {
template <typename T>
__global__ __launch_bounds__(256) void pack_lora_multi_kernel(const float* __restrict__ arena,
                                                              const int64_t* __restrict__ table,
                                                              const float* __restrict__ scales) {
  const int64_t* t = table + (int64_t)blockIdx.y * MULTI_COLS;
  const int K = (int)t[0], N = (int)t[1], ns = (int)t[2];
  T* o = reinterpret_cast<T*>(t[3]);
  const float* sc = scales + blockIdx.y * 4;
  const int64_t nA = 32LL * K, nB = 32LL * N;
  const int64_t total = 2 * nA + 2 * nB;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    int rk, other;  // rank column (0..31), and the row index along K or N
    int part;       // 0 A32s, 1 B32, 2 B32t, 3 At32
    if (i < nA) { part = 0; rk = (int)(i / K); other = (int)(i % K); }
    else if (i < nA + nB) { const int64_t j = i - nA; part = 1; other = (int)(j / 32); rk = (int)(j % 32); }
    else if (i < nA + 2 * nB) { const int64_t j = i - nA - nB; part = 2; rk = (int)(j / N); other = (int)(j % N); }
    else { const int64_t j = i - nA - 2 * nB; part = 3; other = (int)(j / 32); rk = (int)(j % 32); }
    float v = 0.f;
    for (int s = 0; s < ns; ++s) {
      const int64_t* u = t + 4 + 6 * s;
      const int r = (int)u[0], q = (int)u[1], n0 = (int)u[2], n1 = (int)u[3];
      if (rk < q || rk >= q + r) continue;
      const float* A = arena + u[4];
      const float* B = arena + u[5];
      if (part == 0) v = A[(int64_t)(rk - q) * K + other] * sc[s];
      else if (part == 3) v = A[(int64_t)(rk - q) * K + other];
      else if (other >= n0 && other < n1) {
        const float b = B[(int64_t)(other - n0) * r + (rk - q)];
        v = part == 1 ? b : b * sc[s];
      }
      break;
    }
    o[i] = (T)v;
  }
}
}  // namespace

void mift_pack_lora_multi(const at::Tensor& arena, const at::Tensor& table, const at::Tensor& scales,
                          int64_t max_elems, bool bf16_out) {
  TORCH_CHECK(arena.scalar_type() == at::kFloat && table.scalar_type() == at::kLong &&
                  table.size(1) == MULTI_COLS && scales.scalar_type() == at::kFloat && scales.numel() == table.size(0) * 4,
              "pack_lora_multi: arena fp32, table int64 [g, 28], scales fp32 [g, 4]");
  const int n = table.size(0);
  if (n == 0) return;
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const int gx = (int)std::min<int64_t>(512, (max_elems + 255) / 256);
  dim3 grid(gx, n);
  if (bf16_out)
    pack_lora_multi_kernel<bf16><<<grid, 256, 0, st>>>(arena.data_ptr<float>(), table.data_ptr<int64_t>(),
                                                       scales.data_ptr<float>());
  else
    pack_lora_multi_kernel<fp16><<<grid, 256, 0, st>>>(arena.data_ptr<float>(), table.data_ptr<int64_t>(),
                                                       scales.data_ptr<float>());
}

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
