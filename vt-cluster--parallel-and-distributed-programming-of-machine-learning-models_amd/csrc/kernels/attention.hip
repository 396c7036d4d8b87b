// K3: causal flash attention (forward + backward) for gfx950.
//
// Layout: the fused projection output qkv [B*S, 3*H*HD] (token-major, as the
// qkv GEMM writes it) is read in place — no head split / transpose kernels.
// Output o [B*S, H*HD]; lse [B, H, S] fp32 (natural log of the softmax
// denominator of scale*QK^T) for the backward.  Head dims 32, 64 (GPT-2),
// 80 (OPT-2.7B; QK^T K-steps zero-padded to 96) and 128 (OPT-6.7B).
//
// MFMA mapping (16x16x32 bf16/f16, "swapped" products, guide §3):
//   forward  S^T[key, q] = K · Q^T   A = K rows (LDS, ds_read_b128),
//            B = Q rows (registers) -> each lane owns ONE query (lane & 15)
//            and 4 keys per 16-key sub-tile, so the P tile already is the A
//            operand of P·V up to a k-permutation (keys 4g..4g+3 and
//            16+4g..16+4g+3 of each 32-key step).  The matching V^T fragment
//            is two gfx950 hardware-transpose reads (ds_read_b64_tr_b16,
//            guide T10) of the row-major V tile: no transposed LDS writes, no
//            P round trip, no cross-lane shuffles for P.
//   Tiles stream through registers: tile t+1's K/V global loads are issued
//   before tile t's MFMAs (T14 issue-early / write-late).
//   LDS row strides: every image row is an odd multiple of 32 B, so b128 reads and
//   transpose reads are bank-conflict free on the same image; the 16-B staging writes are made
//   conflict-free by the chunk order of tile_chunk (hd 80's 10-chunk rows would otherwise put a
//   ds_write_b128 8-lane group across two rows: 2-way, 0.9-1.8 M conflict cycles per dispatch in
//   round 3's PMC).
// Backward (FA2 split, no atomics): attn_bwd_dq (mirror of the forward, also
// computes D = rowsum(dO∘O) for its queries) then attn_bwd_dkdv (one key tile
// per block, loop over query tiles; S = Q·K^T in the lane-per-key layout,
// dV += P^T dO and dK += dS^T Q with tr-read B operands).
// Dropout (GPT-2 attn_pdrop 0.1): counter hash of idx = ((b*H+h)*S+q)*S+k,
// identical in all kernels (see common.h).
#include "common.h"
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

namespace {

constexpr int BQ = 64, BKV = 64;
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

typedef short v4s __attribute__((ext_vector_type(4)));

MIFT_HD float4_ mfma16(bf16x8 a, bf16x8 b, float4_ c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
MIFT_HD float4_ mfma16(fp16x8 a, fp16x8 b, float4_ c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// 8 x 16-bit MFMA operand vector of element type T (bf16 or fp16)
template <typename T> struct V8;
template <> struct V8<bf16> { using type = bf16x8; };
template <> struct V8<fp16> { using type = fp16x8; };
template <typename T> using vec8 = typename V8<T>::type;

template <int HD>
struct Geo {
  static constexpr int HDP = (HD + 31) / 32 * 32;  // padded for 32-deep K steps
  static constexpr int NKS = HDP / 32;             // K-steps over head dim
  static constexpr int NOT = HD / 16;              // 16-wide output tiles
  // b128-read image stride: an odd multiple of 32 B >= HDP*2, so the 8 rows a ds_read_b128 lane group
  // (and a ds_read_b64_tr_b16 group) touches land on 8 distinct 32-B bank slots — conflict-free for
  // BOTH access kinds (the old HDP*2+16 stride was 2-way on b128 groups and on transpose reads of
  // the same image: 1-4 M conflicts per dispatch, profiles/r2/pmc_attention_seq.txt).  Leaves >= 32 B
  // of padding per row (the dkdv seq kernel keeps a query's lse / D there).
  static constexpr int RS = (((HDP * 2 + 31) / 32) | 1) * 32;
  static constexpr int TS = ((HD * 2 + 31) / 32) | 1;  // tr-read image stride / 32 (odd)
  static constexpr int TRS = TS * 32;
  static constexpr int ROW_BYTES = 64 * RS;
  static constexpr int TR_BYTES = 64 * TRS;
  static constexpr int CH = HD / 8;                // 16-B chunks per row
  static constexpr int NCH = (64 * CH + 255) / 256;  // chunks per thread per 64-row tile
};

template <typename T>
MIFT_HD vec8<T> ld_frag(const char* p) { return *reinterpret_cast<const vec8<T>*>(p); }

template <typename T>
MIFT_HD vec8<T> zero_frag() {
  vec8<T> z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (T)0.f;
  return z;
}

// B fragment from a row-major [key][hd] image by two transpose reads:
// lane (li, g) gets X[kbase + 4g + 0..3][col0 + li] and X[kbase + 16 + 4g + 0..3][col0 + li]
template <typename T>
MIFT_HD vec8<T> tr_frag(const char* img, int stride, int kbase, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15;
  const int off = (kbase + 4 * g + (li >> 2)) * stride + (col0 + (li & 3) * 4) * 2;
  v4s a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(img + off));
  v4s b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(img + off + 16 * stride));
  short8 t = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  vec8<T> f;
  __builtin_memcpy(&f, &t, 16);
  return f;
}

// Chunk i of a 64-row tile -> (row r, 16-B chunk c) for the staging copies.  A ds_write_b128
// serves 8 consecutive lanes per LDS cycle, conflict-free when their 16-B slots (r·stride/16 + c) mod 8
// are distinct.  Rows of CH % 8 == 0 chunks give every 8-lane group one row.  Head dim 80 (CH = 10)
// would straddle rows at the b128 image stride 224 B (2-way); there the first 8 chunks of each row go
// first and chunks 8, 9 of four consecutive rows form the remaining groups — slots (6r + c) mod 8 and
// (2r + c) mod 8 (b128 / transpose image strides) are then distinct (bank model: 128 -> 0 extra
// cycles per tile store).  Global loads stay 128-B row segments per 8 lanes.
template <int HD>
MIFT_HD void tile_chunk(int i, int& r, int& c) {
  constexpr int CH = Geo<HD>::CH;
  if constexpr (CH == 10) {
    if (i < 64 * 8) {
      r = i >> 3;
      c = i & 7;
    } else {
      const int j = i - 64 * 8;
      r = j >> 1;
      c = 8 + (j & 1);
    }
  } else {
    r = i / CH;
    c = i % CH;
  }
}

// register-staged 64-row tile: global -> regs (issue early) -> LDS image(s) (write late)
template <int HD>
struct TileRegs {
  short8 v[Geo<HD>::NCH];
  template <typename T>
  MIFT_HD void load(const T* src, int64_t ld, int row0, int nrows, int tid) {
    using G = Geo<HD>;
    // 64·CH is a multiple of 64 for every head dim, so the chunk guard is wave-uniform:
    // test it on the scalar wave index (no per-lane exec-mask branches)
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
#pragma unroll
    for (int k = 0; k < G::NCH; ++k) {
      const int i = tid + k * 256;
      if ((64 * G::CH) % 256 == 0 || k + 1 < G::NCH || wv * 64 + k * 256 < 64 * G::CH) {
        int r, c;
        tile_chunk<HD>(i, r, c);
        const int gr = min(row0 + r, nrows - 1);
        v[k] = *reinterpret_cast<const short8*>(src + (int64_t)gr * ld + c * 8);
      }
    }
  }
  MIFT_HD void store(char* img, int stride, int tid) const {
    using G = Geo<HD>;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
#pragma unroll
    for (int k = 0; k < G::NCH; ++k) {
      const int i = tid + k * 256;
      if ((64 * G::CH) % 256 == 0 || k + 1 < G::NCH || wv * 64 + k * 256 < 64 * G::CH) {
        int r, c;
        tile_chunk<HD>(i, r, c);
        *reinterpret_cast<short8*>(img + r * stride + c * 16) = v[k];
      }
    }
  }
};

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

// fragments for 16 rows straight from global: frag[s] = X[row][32s + 8(lane>>4) ..]
template <typename T, int HD>
MIFT_HD void load_reg_frags(vec8<T>* f, const T* src, int64_t ld, int row, int nrows, int lane) {
  using G = Geo<HD>;
  const int gr = min(row, nrows - 1);
#pragma unroll
  for (int s = 0; s < G::NKS; ++s) {
    const int col = 32 * s + 8 * (lane >> 4);
    f[s] = col < HD ? *reinterpret_cast<const vec8<T>*>(src + (int64_t)gr * ld + col) : zero_frag<T>();
  }
}

// Block -> (head, tile) for the tiled kernels: the tiles of one head share K/V (forward, dQ) or Q/dO
// (dK/dV), re-read once per tile.  Blocks are dealt round-robin over the 8 XCDs (b and b + 8 share
// one), so consecutive block ids — one head's tiles — sat on 8 different L2s and every re-read went to
// the Infinity Cache.  The bijective remap (gemm.hip, guide T1) gives each XCD a contiguous run of
// block ids: a head's tiles run on one XCD and re-read its L2.  MIFT_ATTN_XCD=0: off (A/B).
MIFT_HD int attn_block_id(int xcd_remap) {
  const int b = blockIdx.x;
  if (!xcd_remap) return b;
  const int n = gridDim.x, q = n / 8, r = n % 8, xcd = b % 8, loc = b / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}
inline int attn_xcd_env() {
  const char* e = getenv("MIFT_ATTN_XCD");
  return e ? atoi(e) : 1;
}

MIFT_HD bool drop_keep(uint64_t seed, uint32_t thr, int64_t bh, int S, int q, int k) {
  return mift_keep(seed, ((uint64_t)bh * S + q) * S + k, thr);
}

// ============================== forward ====================================
// QG query groups of 16 per wave (block = 64·QG queries): every K fragment
// (ds_read_b128) and V^T fragment (two ds_read_b64_tr_b16) read from LDS feeds
// QG MFMAs instead of one.  With QG = 1 a 16x16x32 MFMA (8 cycles on its
// SIMD) needs 1 KiB of LDS reads (8 cycles of the CU's shared 128 B/clk LDS
// port), so four waves are LDS-bound 4:1; QG = 2 halves the LDS bytes per
// MFMA and the K/V global->LDS traffic per query.  Groups whose 16 queries all
// precede a key tile skip it (wave-uniform branch; same result as a fully
// masked tile).
// OT (output transposed, default): P·V is issued with the operands swapped, mfma(Vᵀ frag, P frag),
// which computes Oᵀ: lane (g, qc) then holds hd columns 16i + 4g .. +3 of ITS OWN query qc instead of
// one column of queries 4g .. 4g+3.  The softmax state (m, l, alpha) is per query = per lane already,
// so the rescale and the final 1/l need no cross-lane shuffles, and the output leaves as one 8-B store
// per 16 columns (NOT per lane) instead of 4·NOT 2-B stores — the attention store tail is issue-bound
// (MI355X_MICROARCH.md constants: 16 dwordx2 per lane ≈ 9.3k cycles for the last-finishing half).
template <typename T, int HD, int QG, bool OT = true>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const T* __restrict__ qkv, T* __restrict__ out,
                                                       float* __restrict__ lse, const int* __restrict__ kv_len,
                                                       int B, int S, int H, float scale, uint64_t seed,
                                                       const int64_t* __restrict__ sstep, uint32_t thr, float inv_keep,
                                                       int xcd) {
  seed = mift_seed(seed, sstep);
  using G = Geo<HD>;
  constexpr int BQB = BQ * QG;  // queries per block
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ks = smem;                    // [64][HDP] b128 image
  char* Vs = smem + G::ROW_BYTES;     // [64][HD] tr image
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on it
  const int g = lane >> 4, qc = lane & 15;
  const int nqt = (S + BQB - 1) / BQB;
  const int bid = attn_block_id(xcd);
  const int qt = nqt - 1 - (bid % nqt);  // heavy (late) query tiles first
  const int bh = bid / nqt;
  const int b = bh / H, h = bh % H;
  const int D = H * HD;
  const int64_t ld = 3LL * D;
  const T* Qg = qkv + (int64_t)b * S * ld + h * HD;
  const T* Kg = Qg + D;
  const T* Vg = Qg + 2 * D;
  const int klen = kv_len ? kv_len[b] : S;
  MIFT_ASSERT(klen >= 0 && klen <= S);
  const int q0 = qt * BQB + wave * 16 * QG;  // first query of this wave; group j: q0 + 16 j
  const float c2 = scale * LOG2E;
  const bool hz = (uint64_t)B * H * S * S < (1ull << 33);  // dropout pairs' high word is 0: hoisted hash
  const uint32_t hm0 = mift_hmix(seed, 0);

  vec8<T> qf[QG][G::NKS];
#pragma unroll
  for (int j = 0; j < QG; ++j) load_reg_frags<T, HD>(qf[j], Qg, ld, q0 + 16 * j + qc, S, lane);
  zero_row_pad<HD>(Ks, tid);

  float m[QG], l[QG];
  float4_ o[QG][G::NOT];
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    m[j] = -INFINITY;
    l[j] = 0.f;
#pragma unroll
    for (int i = 0; i < G::NOT; ++i) o[j][i] = float4_{0.f, 0.f, 0.f, 0.f};
  }

  const int kend = min((qt + 1) * BQB, klen);
  const int nkt = (kend + BKV - 1) / BKV;
  TileRegs<HD> kr, vr;
  if (nkt > 0) {
    kr.load(Kg, ld, 0, S, tid);
    vr.load(Vg, ld, 0, S, tid);
  }
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * BKV;
    __syncthreads();
    kr.store(Ks, G::RS, tid);
    vr.store(Vs, G::TRS, tid);
    __syncthreads();
    if (kt + 1 < nkt) {  // next tile in flight during this tile's math
      kr.load(Kg, ld, k0 + BKV, S, tid);
      vr.load(Vg, ld, k0 + BKV, S, tid);
    }
    bool act[QG];
#pragma unroll
    for (int j = 0; j < QG; ++j) act[j] = k0 <= q0 + 16 * j + 15;
    if (!act[0]) continue;  // groups are in query order: none of this wave's queries sees the tile
    float4_ st[QG][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int j = 0; j < QG; ++j) st[j][t] = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < G::NKS; ++s) {
        const vec8<T> kf = ld_frag<T>(Ks + (t * 16 + qc) * G::RS + (4 * s + g) * 16);
#pragma unroll
        for (int j = 0; j < QG; ++j)
          if (act[j]) st[j][t] = mfma16(kf, qf[j][s], st[j][t]);
      }
    }
    vec8<T> pf[QG][2];
#pragma unroll
    for (int j = 0; j < QG; ++j) {
      if (!act[j]) continue;
      const int q0j = q0 + 16 * j, myq = q0j + qc;
      const bool diag = (k0 + BKV > q0j) || (k0 + BKV > klen);
      float tmax = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = st[j][t][r] * c2;
          if (diag) {
            const int key = k0 + t * 16 + g * 4 + r;
            if (key > myq || key >= klen) v = -INFINITY;
          }
          st[j][t][r] = v;
          tmax = fmaxf(tmax, v);
        }
      tmax = xor16_max(tmax);
      tmax = xor32_max(tmax);
      // lazy rescale: the running max only moves when some row's tile max exceeds it by
      // > 2^8 (p <= 256 stays exact in fp32 and representable in bf16/fp16), so most tiles
      // skip the O rescale and its accumulator round trips (wave-uniform branch)
      const bool resc = __any(tmax > m[j] + 8.f);
      float alpha = 1.f;
      if (resc) {
        const float mnew = fmaxf(m[j], tmax);
        alpha = (m[j] == -INFINITY) ? 0.f : fast_exp2(m[j] - mnew);
        m[j] = mnew;
      }
      float psum = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        bool kp[4] = {true, true, true, true};
        if (thr != 0) {
          const uint64_t i0 = ((uint64_t)bh * S + myq) * S + k0 + t * 16 + g * 4;
          if (hz && !(i0 & 1)) mift_keep4_hm(seed, hm0, i0, thr, kp);
          else mift_keep4(seed, i0, thr, kp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = (m[j] == -INFINITY) ? 0.f : fast_exp2(st[j][t][r] - m[j]);
          psum += p;
          if (thr != 0) p = kp[r] ? p * inv_keep : 0.f;
          pf[j][t >> 1][(t & 1) * 4 + r] = (T)p;
        }
      }
      l[j] = l[j] * alpha + psum;
      if (resc) {
        if constexpr (OT) {
#pragma unroll
          for (int i = 0; i < G::NOT; ++i) o[j][i] *= alpha;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float ar = __shfl(alpha, g * 4 + r, 64);
#pragma unroll
            for (int i = 0; i < G::NOT; ++i) o[j][i][r] *= ar;
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < G::NOT; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const vec8<T> vf = tr_frag<T>(Vs, G::TRS, 32 * s2, i * 16, lane);
#pragma unroll
        for (int j = 0; j < QG; ++j)
          if (act[j]) o[j][i] = OT ? mfma16(vf, pf[j][s2], o[j][i]) : mfma16(pf[j][s2], vf, o[j][i]);
      }
  }
  T* Og = out + (int64_t)b * S * D + h * HD;
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    float lj = l[j];
    lj = xor16_add(lj);
    lj = xor32_add(lj);
    const float inv_l = lj > 0.f ? 1.f / lj : 0.f;
    const int q0j = q0 + 16 * j, myq = q0j + qc;
    if (g == 0 && myq < S) lse[(int64_t)bh * S + myq] = (lj > 0.f) ? (m[j] + log2f(lj)) * LN2 : -INFINITY;
    if constexpr (OT) {
      if (myq < S) {
#pragma unroll
        for (int i = 0; i < G::NOT; ++i) {
          float v4[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v4[r] = o[j][i][r] * inv_l;
          store4<T>(Og + (int64_t)myq * D + i * 16 + g * 4, v4);
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float il = __shfl(inv_l, g * 4 + r, 64);
        const int q = q0j + g * 4 + r;
        if (q < S) {
#pragma unroll
          for (int i = 0; i < G::NOT; ++i) Og[(int64_t)q * D + i * 16 + qc] = (T)(o[j][i][r] * il);
        }
      }
    }
  }
}

// ===================== forward, whole sequence in LDS ======================
// Short sequences (distilgpt2 S = 256): one block of NW waves per (batch, head) stages ALL of K
// (b128 image) and V (transpose-read image) in LDS once — one barrier per block instead of two
// per 64-key tile, and K/V read from HBM once per head instead of once per query tile.  Each
// wave takes 16-query groups in snake order (w, 2NW-1-w, 2NW+w, ...) so the causal work is
// balanced across waves; the per-group math is the tiled kernel's, tile by tile from LDS.
template <int HD>
constexpr int seq_row_bytes() { return Geo<HD>::RS + Geo<HD>::TRS; }

// Head split of the whole-sequence kernels (forward, dq).  Two blocks fit per CU (LDS), so with
// C < B·H < 2C heads (distilgpt2: 384 over 256 CUs) half the CUs ran two heads and half one, and the
// kernel took as long as a two-head CU.  The first nfull blocks take whole heads; each of the
// remaining 2C - B·H heads is split into two blocks by causal work (query groups [0, gs) and
// [gs, ng), gs balancing the 64-key tiles visited), so every CU gets one head and one half head
// (blocks dispatch in index order: full heads fill the first slot of every CU, halves the second).
// MIFT_ATTN_SPLIT=0 turns it off (A/B).
int num_cus_attn() {
  static int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
  }();
  return n;
}

struct SeqSplit {
  int nfull, gs;
};
MIFT_HD void seq_block(const SeqSplit& sp, int ng, int& bh, int& g0, int& g1) {
  const int b = blockIdx.x;
  if (b < sp.nfull) {
    bh = b; g0 = 0; g1 = ng;
  } else {
    const int t = b - sp.nfull;
    bh = sp.nfull + (t >> 1);
    g0 = (t & 1) ? sp.gs : 0;
    g1 = (t & 1) ? ng : sp.gs;
  }
}
inline SeqSplit seq_split_plan(int BH, int S, int cus, int& blocks) {
  SeqSplit sp{BH, 0};
  blocks = BH;
  const char* e = getenv("MIFT_ATTN_SPLIT");
  const int ng = (S + 15) / 16;
  if ((e && atoi(e) == 0) || BH <= cus || BH >= 2 * cus || ng < 4) return sp;
  const int k = 2 * cus - BH;  // heads split in two
  sp.nfull = BH - k;
  long tot = 0;
  for (int g = 0; g < ng; ++g) tot += (16 * g + 16 + BKV - 1) / BKV;
  long acc = 0;
  int gs = 1;
  for (; gs < ng; ++gs) {
    acc += (16 * (gs - 1) + 16 + BKV - 1) / BKV;
    if (2 * acc >= tot) break;
  }
  sp.gs = gs;
  blocks = BH + k;
  return sp;
}
// dK/dV: key groups [0, gs) and [gs, ng); a key group visits the 64-query tiles from its own to
// the last, so the weights run the other way
inline SeqSplit seq_split_plan_kv(int BH, int S, int cus, int& blocks) {
  SeqSplit sp = seq_split_plan(BH, S, cus, blocks);
  if (sp.nfull == BH) return sp;
  const int ng = (S + 15) / 16, nqt = (S + BQ - 1) / BQ;
  long tot = 0;
  for (int g = 0; g < ng; ++g) tot += nqt - (16 * g) / BQ;
  long acc = 0;
  int gs = 1;
  for (; gs < ng; ++gs) {
    acc += nqt - (16 * (gs - 1)) / BQ;
    if (2 * acc >= tot) break;
  }
  sp.gs = gs;
  return sp;
}

// MIFT_ATTN_SEQ: 0 = tiled kernels only, 1 = whole-sequence kernels when they fit and there are
// >= 256 heads to fill the chip (default), 2 = whenever they fit (tests, A/B); read per call
int attn_seq_mode() {
  const char* e = getenv("MIFT_ATTN_SEQ");
  return e ? atoi(e) : 1;
}

template <typename T, int HD, int NW, bool OT = true>  // OT: see attn_fwd_kernel
__global__ __launch_bounds__(NW * 64, HD <= 80 ? 4 : 2) void attn_fwd_seq_kernel(const T* __restrict__ qkv, T* __restrict__ out,
                                                              float* __restrict__ lse, const int* __restrict__ kv_len,
                                                              int B, int S, int H, float scale, uint64_t seed,
                                                              const int64_t* __restrict__ sstep, uint32_t thr,
                                                              float inv_keep, uint16_t* __restrict__ dmask,
                                                              SeqSplit split) {
  seed = mift_seed(seed, sstep);
  using G = Geo<HD>;
  constexpr int NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int SP = (S + BKV - 1) / BKV * BKV;  // image rows (zero padded to whole key tiles)
  const int NR = SP / 16;                    // keep-bit record: uint16 elements per query (see KEEP BITS)
  char* Ks = smem;                           // [SP][RS] b128 image
  char* Vs = smem + (size_t)SP * G::RS;      // [SP][TRS] tr image
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, qc = lane & 15;
  int bh, g0, g1;
  seq_block(split, (S + 15) / 16, bh, g0, g1);
  const int SPB = min(SP, (16 * g1 + BKV - 1) / BKV * BKV);  // keys this block's queries can see
  const int b = bh / H, h = bh % H;
  const int D = H * HD;
  const int64_t ld = 3LL * D;
  const T* Qg = qkv + (int64_t)b * S * ld + h * HD;
  const T* Kg = Qg + D;
  const T* Vg = Qg + 2 * D;
  const int klen = kv_len ? kv_len[b] : S;
  MIFT_ASSERT(klen >= 0 && klen <= S);
  const float c2 = scale * LOG2E;
  // hoisted-hash path: pair indices < 2^32 and (S even) every lane's element index i0 is even
  const bool hze = (uint64_t)B * H * S * S < (1ull << 33) && S % 2 == 0;
  const uint32_t hm0 = mift_hmix(seed, 0);

  const int ng = g1;  // query groups [g0, g1) of this block (the whole head unless split)
  // Q fragments of this wave's first two 16-query groups are requested before K/V are staged, so
  // their latency hides under the staging instead of stalling each group's first MFMA
  vec8<T> qpre[2][G::NKS];
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const int grp = g0 + ((sl & 1) ? (sl + 1) * NW - 1 - wave : sl * NW + wave);
    if (grp < ng) load_reg_frags<T, HD>(qpre[sl], Qg, ld, grp * 16 + qc, S, lane);
  }
  // ---- stage K and V of the keys visible to this block: 8 chunks in flight per thread per round
  {
    constexpr int U = 4;
    const int nch = SPB * G::CH;
    for (int c0 = tid; c0 < nch; c0 += U * NT) {
      short8 kv[U], vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = c0 + u * NT;
        const int r = i / G::CH, c = i % G::CH;
        if (i < nch && r < S) {
          kv[u] = *reinterpret_cast<const short8*>(Kg + (int64_t)r * ld + c * 8);
          vv[u] = *reinterpret_cast<const short8*>(Vg + (int64_t)r * ld + c * 8);
        } else {
          kv[u] = short8{0, 0, 0, 0, 0, 0, 0, 0};
          vv[u] = short8{0, 0, 0, 0, 0, 0, 0, 0};
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = c0 + u * NT;
        if (i < nch) {
          const int r = i / G::CH, c = i % G::CH;
          *reinterpret_cast<short8*>(Ks + r * G::RS + c * 16) = kv[u];
          *reinterpret_cast<short8*>(Vs + r * G::TRS + c * 16) = vv[u];
        }
      }
    }
    if (G::HDP != HD) {
      constexpr int PADC = (G::HDP - HD) / 8;
      for (int i = tid; i < SPB * PADC; i += NT) {
        const int r = i / PADC, c = HD / 8 + i % PADC;
        *reinterpret_cast<short8*>(Ks + r * G::RS + c * 16) = short8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  }
  __syncthreads();

  T* Og = out + (int64_t)b * S * D + h * HD;
  for (int slot = 0;; ++slot) {
    const int grp = g0 + ((slot & 1) ? (slot + 1) * NW - 1 - wave : slot * NW + wave);  // snake order
    if (slot * NW >= ng - g0) break;
    if (grp >= ng) continue;
    const int q0 = grp * 16, myq = q0 + qc;
    vec8<T> qf[G::NKS];
    if (slot < 2) {
#pragma unroll
      for (int s = 0; s < G::NKS; ++s) qf[s] = slot == 0 ? qpre[0][s] : qpre[1][s];
    } else {
      load_reg_frags<T, HD>(qf, Qg, ld, myq, S, lane);
    }
    float m = -INFINITY, l = 0.f;
    float4_ o[G::NOT];
#pragma unroll
    for (int i = 0; i < G::NOT; ++i) o[i] = float4_{0.f, 0.f, 0.f, 0.f};
    const int kend = min(q0 + 16, klen);
    const int nkt = (kend + BKV - 1) / BKV;
    // one key tile; DIAG (compile-time) = the per-element causal / key-length mask.  Only a group's
    // LAST key tile can reach past its queries or the key length, so the others run the mask-free
    // instantiation (a runtime `diag` flag made hipcc emit one scalar branch per score element)
    auto ktile = [&](const int kt, auto diagc) {
      constexpr bool diag = decltype(diagc)::value;
      const int k0 = kt * BKV;
      float4_ st[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        st[t] = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < G::NKS; ++s)
          st[t] = mfma16(ld_frag<T>(Ks + (k0 + t * 16 + qc) * G::RS + (4 * s + g) * 16), qf[s], st[t]);
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = st[t][r] * c2;
          if constexpr (diag) {
            const int key = k0 + t * 16 + g * 4 + r;
            if (key > myq || key >= klen) v = -INFINITY;
          }
          st[t][r] = v;
          tmax = fmaxf(tmax, v);
        }
      tmax = xor16_max(tmax);
      tmax = xor32_max(tmax);
      const bool resc = __any(tmax > m + 8.f);
      float alpha = 1.f;
      if (resc) {
        const float mnew = fmaxf(m, tmax);
        alpha = (m == -INFINITY) ? 0.f : fast_exp2(m - mnew);
        m = mnew;
      }
      vec8<T> pf[2];
      float psum = 0.f;
      uint32_t kbits[2] = {0u, 0u};  // this lane's keep nibbles, placed at their record bits
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        bool kp[4] = {true, true, true, true};
        if (thr != 0) {
          const uint64_t i0 = ((uint64_t)bh * S + myq) * S + k0 + t * 16 + g * 4;
          if (hze) mift_keep4_hm(seed, hm0, i0, thr, kp);  // block-uniform (i0 even when S is)
          else mift_keep4(seed, i0, thr, kp);
          const uint32_t nib = (uint32_t)kp[0] | ((uint32_t)kp[1] << 1) | ((uint32_t)kp[2] << 2) | ((uint32_t)kp[3] << 3);
          kbits[t >> 1] |= nib << ((t & 1) * 16 + g * 4);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float pv = (m == -INFINITY) ? 0.f : fast_exp2(st[t][r] - m);
          psum += pv;
          if (thr != 0) pv = kp[r] ? pv * inv_keep : 0.f;
          pf[t >> 1][(t & 1) * 4 + r] = (T)pv;
        }
      }
      if (dmask != nullptr) {
        // KEEP BITS: record element kt*4 + t of query myq holds keys k0 + 16t + 0..15 (bit j <-> key
        // k0 + 16t + j); the four g-lanes of a query each own one nibble of every element
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          kbits[h2] = xor16_or(kbits[h2]);
          kbits[h2] = xor32_or(kbits[h2]);
        }
        if (g == 0 && myq < S)
          *reinterpret_cast<uint2*>(dmask + ((int64_t)bh * S + myq) * NR + kt * 4) = make_uint2(kbits[0], kbits[1]);
      }
      l = l * alpha + psum;
      if (resc) {
        if constexpr (OT) {
#pragma unroll
          for (int i = 0; i < G::NOT; ++i) o[i] *= alpha;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float ar = __shfl(alpha, g * 4 + r, 64);
#pragma unroll
            for (int i = 0; i < G::NOT; ++i) o[i][r] *= ar;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < G::NOT; ++i)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const vec8<T> vf = tr_frag<T>(Vs, G::TRS, k0 + 32 * s2, i * 16, lane);
          o[i] = OT ? mfma16(vf, pf[s2], o[i]) : mfma16(pf[s2], vf, o[i]);
        }
    };
    for (int kt = 0; kt + 1 < nkt; ++kt) ktile(kt, std::false_type{});
    if (nkt > 0) ktile(nkt - 1, std::true_type{});
    l = xor16_add(l);
    l = xor32_add(l);
    const float inv_l = l > 0.f ? 1.f / l : 0.f;
    if (g == 0 && myq < S) lse[(int64_t)bh * S + myq] = (l > 0.f) ? (m + log2f(l)) * LN2 : -INFINITY;
    if constexpr (OT) {
      if (myq < S) {
#pragma unroll
        for (int i = 0; i < G::NOT; ++i) {
          float v4[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v4[r] = o[i][r] * inv_l;
          store4<T>(Og + (int64_t)myq * D + i * 16 + g * 4, v4);
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float il = __shfl(inv_l, g * 4 + r, 64);
        const int q = q0 + g * 4 + r;
        if (q < S) {
#pragma unroll
          for (int i = 0; i < G::NOT; ++i) Og[(int64_t)q * D + i * 16 + qc] = (T)(o[i][r] * il);
        }
      }
    }
  }
}

// ============================ backward: dQ (+D) =============================
template <typename T, int HD>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const T* __restrict__ qkv, const T* __restrict__ o,
                                                          const T* __restrict__ dout, const float* __restrict__ lse,
                                                          float* __restrict__ Dv, T* __restrict__ dqkv,
                                                          const int* __restrict__ kv_len, int B, int S, int H,
                                                          float scale, uint64_t seed, const int64_t* __restrict__ sstep, uint32_t thr,
                                                          float inv_keep, int xcd) {
  seed = mift_seed(seed, sstep);
  using G = Geo<HD>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ks = smem;                                 // K rows, b128 image (A of S^T)
  char* Vs = smem + G::ROW_BYTES;                  // V rows, b128 image (A of dP^T)
  char* Kt = smem + 2 * G::ROW_BYTES;              // K rows, tr image (B of dQ)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on it
  const int g = lane >> 4, qc = lane & 15;
  const int nqt = (S + BQ - 1) / BQ;
  const int bid = attn_block_id(xcd);
  const int qt = nqt - 1 - (bid % nqt);
  const int bh = bid / nqt;
  const int b = bh / H, h = bh % H;
  const int D = H * HD;
  const int64_t ld = 3LL * D;
  const T* Qg = qkv + (int64_t)b * S * ld + h * HD;
  const T* Kg = Qg + D;
  const T* Vg = Qg + 2 * D;
  const T* dOg = dout + (int64_t)b * S * D + h * HD;
  const T* Og = o + (int64_t)b * S * D + h * HD;
  const int klen = kv_len ? kv_len[b] : S;
  MIFT_ASSERT(klen >= 0 && klen <= S);
  const int q0 = qt * BQ + wave * 16;
  const int myq = q0 + qc;
  const float c2 = scale * LOG2E;

  vec8<T> qf[G::NKS], df[G::NKS];
  load_reg_frags<T, HD>(qf, Qg, ld, myq, S, lane);
  load_reg_frags<T, HD>(df, dOg, D, myq, S, lane);
  // D = rowsum(dO ∘ O) for this lane's query (fused attn_bwd_pre)
  float Dq = 0.f;
  {
    vec8<T> of[G::NKS];
    load_reg_frags<T, HD>(of, Og, D, myq, S, lane);
#pragma unroll
    for (int s = 0; s < G::NKS; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) Dq += (float)of[s][e] * (float)df[s][e];
    Dq = xor16_add(Dq);
    Dq = xor32_add(Dq);
    if (g == 0 && myq < S) Dv[(int64_t)bh * S + myq] = Dq;
  }
  const float lse2 = myq < S ? lse[(int64_t)bh * S + myq] * LOG2E : 0.f;
  zero_row_pad<HD>(Ks, tid);
  zero_row_pad<HD>(Vs, tid);

  float4_ dq[G::NOT];
#pragma unroll
  for (int i = 0; i < G::NOT; ++i) dq[i] = float4_{0.f, 0.f, 0.f, 0.f};

  const int kend = min((qt + 1) * BQ, klen);
  const int nkt = (kend + BKV - 1) / BKV;
  TileRegs<HD> kr, vr;
  if (nkt > 0) {
    kr.load(Kg, ld, 0, S, tid);
    vr.load(Vg, ld, 0, S, tid);
  }
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * BKV;
    __syncthreads();
    kr.store(Ks, G::RS, tid);
    kr.store(Kt, G::TRS, tid);
    vr.store(Vs, G::RS, tid);
    __syncthreads();
    if (kt + 1 < nkt) {
      kr.load(Kg, ld, k0 + BKV, S, tid);
      vr.load(Vg, ld, k0 + BKV, S, tid);
    }
    vec8<T> dsf[2];
    const bool diag = (k0 + BKV > q0) || (k0 + BKV > klen);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float4_ sa = float4_{0.f, 0.f, 0.f, 0.f}, pa = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < G::NKS; ++s) {
        sa = mfma16(ld_frag<T>(Ks + (t * 16 + qc) * G::RS + (4 * s + g) * 16), qf[s], sa);
        pa = mfma16(ld_frag<T>(Vs + (t * 16 + qc) * G::RS + (4 * s + g) * 16), df[s], pa);
      }
      bool kp[4] = {true, true, true, true};
      if (thr != 0) {
        const uint64_t i0 = ((uint64_t)bh * S + myq) * S + k0 + t * 16 + g * 4;
        if ((uint64_t)B * H * S * S < (1ull << 33) && !(i0 & 1)) mift_keep4_hm(seed, mift_hmix(seed, 0), i0, thr, kp);
        else mift_keep4(seed, i0, thr, kp);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float p = fast_exp2(sa[r] * c2 - lse2);
        if (diag) {  // wave-uniform: interior tiles skip the per-element causal / padding mask
          const int key = k0 + t * 16 + g * 4 + r;
          if (key > myq || key >= klen) p = 0.f;
        }
        float dp = pa[r];
        if (thr != 0) dp = kp[r] ? dp * inv_keep : 0.f;
        dsf[t >> 1][(t & 1) * 4 + r] = (T)(p * (dp - Dq));
      }
    }
#pragma unroll
    for (int i = 0; i < G::NOT; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) dq[i] = mfma16(dsf[s2], tr_frag<T>(Kt, G::TRS, 32 * s2, i * 16, lane), dq[i]);
  }
  T* dQg = dqkv + (int64_t)b * S * ld + h * HD;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = q0 + g * 4 + r;
    if (q < S) {
#pragma unroll
      for (int i = 0; i < G::NOT; ++i) dQg[(int64_t)q * ld + i * 16 + qc] = (T)(dq[i][r] * scale);
    }
  }
}

// ========================== backward: dK, dV ===============================
template <typename T, int HD, int OCC = (HD <= 64 ? 3 : 2)>
__global__ __launch_bounds__(256, OCC) void attn_bwd_dkdv_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                            const float* __restrict__ lse, const float* __restrict__ Dv,
                                                            T* __restrict__ dqkv, const int* __restrict__ kv_len,
                                                            int B, int S, int H, float scale, uint64_t seed,
                                                            const int64_t* __restrict__ sstep, uint32_t thr, float inv_keep,
                                                            int xcd) {
  seed = mift_seed(seed, sstep);
  using G = Geo<HD>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Qs = smem;                                   // Q rows b128 image (A of S)
  char* dOs = smem + G::ROW_BYTES;                   // dO rows b128 image (A of dP)
  char* Qt = smem + 2 * G::ROW_BYTES;                // Q rows tr image (B of dK)
  char* dOt = Qt + G::TR_BYTES;                      // dO rows tr image (B of dV)
  float* lse_s = reinterpret_cast<float*>(dOt + G::TR_BYTES);
  float* D_s = lse_s + 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on it
  const int g = lane >> 4, kc = lane & 15;
  const int nkt = (S + BKV - 1) / BKV;
  const int bid = attn_block_id(xcd);
  const int kt = bid % nkt;
  const int bh = bid / nkt;
  const int b = bh / H, h = bh % H;
  const int D = H * HD;
  const int64_t ld = 3LL * D;
  const T* Qg = qkv + (int64_t)b * S * ld + h * HD;
  const T* Kg = Qg + D;
  const T* Vg = Qg + 2 * D;
  const T* dOg = dout + (int64_t)b * S * D + h * HD;
  const int klen = kv_len ? kv_len[b] : S;
  MIFT_ASSERT(klen >= 0 && klen <= S);
  const int k0 = kt * BKV + wave * 16;
  const int mykey = k0 + kc;
  const float c2 = scale * LOG2E;

  vec8<T> kf[G::NKS], vf[G::NKS];
  load_reg_frags<T, HD>(kf, Kg, ld, mykey, S, lane);
  load_reg_frags<T, HD>(vf, Vg, ld, mykey, S, lane);
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
  const int qt0 = active ? kt : nqt;
  TileRegs<HD> qr, dr;
  if (qt0 < nqt) {
    qr.load(Qg, ld, qt0 * BQ, S, tid);
    dr.load(dOg, D, qt0 * BQ, S, tid);
  }
  for (int qt = qt0; qt < nqt; ++qt) {
    const int qb = qt * BQ;
    __syncthreads();
    qr.store(Qs, G::RS, tid);
    qr.store(Qt, G::TRS, tid);
    dr.store(dOs, G::RS, tid);
    dr.store(dOt, G::TRS, tid);
    if (tid < 64) {
      const int q = min(qb + tid, S - 1);
      lse_s[tid] = lse[(int64_t)bh * S + q] * LOG2E;
      D_s[tid] = Dv[(int64_t)bh * S + q];
    }
    __syncthreads();
    if (qt + 1 < nqt) {
      qr.load(Qg, ld, qb + BQ, S, tid);
      dr.load(dOg, D, qb + BQ, S, tid);
    }
    vec8<T> pf[2], dsf[2];
    // wave-uniform: every query of the tile sees every key of this wave (no causal / length mask)
    const bool interior = qb >= k0 + 15 && qb + BQ <= S && k0 + 16 <= klen;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float4_ sa = float4_{0.f, 0.f, 0.f, 0.f}, pa = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < G::NKS; ++s) {
        sa = mfma16(ld_frag<T>(Qs + (t * 16 + kc) * G::RS + (4 * s + g) * 16), kf[s], sa);
        pa = mfma16(ld_frag<T>(dOs + (t * 16 + kc) * G::RS + (4 * s + g) * 16), vf[s], pa);
      }
      // acc layout: row = query t*16 + g*4 + r, col = key kc.  Dropout bits:
      // keys (kc, kc^1) share one hash pair per query, so the even-key lane
      // hashes queries r=0,1 and the odd-key lane r=2,3, then they swap.
      uint32_t hb[4] = {0, 0, 0, 0};
      if (thr != 0) {
        const int odd = kc & 1;
        const int qa = min(qb + t * 16 + g * 4 + 2 * odd, S - 1);
        const uint64_t p0 = (((uint64_t)bh * S + qa) * S + mykey) >> 1;
        const uint64_t p1 = (((uint64_t)bh * S + min(qa + 1, S - 1)) * S + mykey) >> 1;
        uint32_t h0, h1;
        if ((uint64_t)B * H * S * S < (1ull << 33)) {  // high words 0: hoisted hash (bit-identical)
          const uint32_t hm = mift_hmix(seed, 0);
          h0 = mift_hash_lo(seed, hm, (uint32_t)p0);
          h1 = mift_hash_lo(seed, hm, (uint32_t)p1);
        } else {
          h0 = mift_hash_pair(seed, p0);
          h1 = mift_hash_pair(seed, p1);
        }
        const uint32_t o0 = __shfl_xor(h0, 1, 64), o1 = __shfl_xor(h1, 1, 64);
        hb[0] = odd ? o0 : h0;
        hb[1] = odd ? o1 : h1;
        hb[2] = odd ? h0 : o0;
        hb[3] = odd ? h1 : o1;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = t * 16 + g * 4 + r;
        const int q = qb + ql;
        bool valid = true;
        float p = fast_exp2(sa[r] * c2 - lse_s[ql]);
        if (!interior) {
          valid = q < S && mykey <= q && mykey < klen;
          if (!valid) p = 0.f;
        }
        float pd = p, dp = pa[r];
        if (thr != 0) {
          const uint32_t bits = (S & 1) ? mift_bits16(seed, ((uint64_t)bh * S + q) * S + mykey)
                                        : ((hb[r] >> ((mykey & 1) << 4)) & 0xFFFFu);
          const bool kp = valid && bits >= thr;
          pd = kp ? p * inv_keep : 0.f;
          dp = kp ? dp * inv_keep : 0.f;
        }
        pf[t >> 1][(t & 1) * 4 + r] = (T)pd;
        dsf[t >> 1][(t & 1) * 4 + r] = (T)(p * (dp - D_s[ql]));
      }
    }
#pragma unroll
    for (int i = 0; i < G::NOT; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        dv[i] = mfma16(pf[s2], tr_frag<T>(dOt, G::TRS, 32 * s2, i * 16, lane), dv[i]);
        dk[i] = mfma16(dsf[s2], tr_frag<T>(Qt, G::TRS, 32 * s2, i * 16, lane), dk[i]);
      }
  }
  T* dKg = dqkv + (int64_t)b * S * ld + D + h * HD;
  T* dVg = dKg + D;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int key = k0 + g * 4 + r;
    if (key < S) {
#pragma unroll
      for (int i = 0; i < G::NOT; ++i) {
        dKg[(int64_t)key * ld + i * 16 + kc] = (T)(dk[i][r] * scale);
        dVg[(int64_t)key * ld + i * 16 + kc] = (T)dv[i][r];
      }
    }
  }
}

// ================= backward, whole sequence in LDS (short S) =================
// Same structure as attn_fwd_seq_kernel: one block of NW waves per (batch, head), the operand
// rows of the whole sequence staged once in a single b128 image per tensor (the transposed
// B-operand reads use ds_read_b64_tr_b16 on that same image: correct for any 8-B-aligned row
// stride, a few bank conflicts instead of a second image), groups in snake order.
template <typename T, int HD>
MIFT_HD void stage_rows(char* img, const T* src, int64_t ld, int S, int SP, int tid, int nt) {
  using G = Geo<HD>;
  constexpr int U = 4;
  const int nch = SP * G::CH;
  for (int c0 = tid; c0 < nch; c0 += U * nt) {
    short8 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = c0 + u * nt;
      const int r = i / G::CH, c = i % G::CH;
      v[u] = (i < nch && r < S) ? *reinterpret_cast<const short8*>(src + (int64_t)r * ld + c * 8)
                                : short8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = c0 + u * nt;
      if (i < nch) *reinterpret_cast<short8*>(img + (i / G::CH) * G::RS + (i % G::CH) * 16) = v[u];
    }
  }
  if (G::HDP != HD) {
    constexpr int PADC = (G::HDP - HD) / 8;
    for (int i = tid; i < SP * PADC; i += nt)
      *reinterpret_cast<short8*>(img + (i / PADC) * G::RS + (HD / 8 + i % PADC) * 16) = short8{0, 0, 0, 0, 0, 0, 0, 0};
  }
}

template <typename T, int HD, int NW>
__global__ __launch_bounds__(NW * 64, HD <= 80 ? 4 : 2) void attn_bwd_dq_seq_kernel(const T* __restrict__ qkv, const T* __restrict__ o,
                                                                 const T* __restrict__ dout, const float* __restrict__ lse,
                                                                 float* __restrict__ Dv, T* __restrict__ dqkv,
                                                                 const int* __restrict__ kv_len, int B, int S, int H,
                                                                 float scale, uint64_t seed,
                                                                 const int64_t* __restrict__ sstep, uint32_t thr,
                                                                 float inv_keep, const uint16_t* __restrict__ dmask,
                                                                 SeqSplit split) {
  seed = mift_seed(seed, sstep);
  using G = Geo<HD>;
  constexpr int NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int SP = (S + BKV - 1) / BKV * BKV;
  constexpr int PADOFF = G::HDP * 2;      // row padding [PADOFF, RS) = 32 B per row of each image
  static_assert(G::RS - PADOFF == 32, "32-B row padding");
  char* Ks = smem;                        // K rows (A of S^T; tr-read B of dQ)
  char* Vs = smem + (size_t)SP * G::RS;   // V rows (A of dP^T)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, qc = lane & 15;
  int bh, g0, g1;
  seq_block(split, (S + 15) / 16, bh, g0, g1);
  const int SPB = min(SP, (16 * g1 + BKV - 1) / BKV * BKV);  // keys this block's queries can see
  const int b = bh / H, h = bh % H;
  const int D = H * HD;
  const int64_t ld = 3LL * D;
  const T* Qg = qkv + (int64_t)b * S * ld + h * HD;
  const T* Kg = Qg + D;
  const T* Vg = Qg + 2 * D;
  const T* dOg = dout + (int64_t)b * S * D + h * HD;
  const T* Og = o + (int64_t)b * S * D + h * HD;
  const int klen = kv_len ? kv_len[b] : S;
  MIFT_ASSERT(klen >= 0 && klen <= S);
  const float c2 = scale * LOG2E;
  const bool hze = (uint64_t)B * H * S * S < (1ull << 33) && S % 2 == 0;  // hoisted hash, even i0
  const uint32_t hm0 = mift_hmix(seed, 0);
  const int ng = g1;  // query groups [g0, g1) of this block (the whole head unless split)
  stage_rows<T, HD>(Ks, Kg, ld, S, SPB, tid, NT);
  stage_rows<T, HD>(Vs, Vg, ld, S, SPB, tid, NT);
  // keep-bit records of the forward (KEEP BITS): query q's record goes to the row-q padding, 8-B
  // words 0..3 (64-key tiles 0..3) in the K image, 4..7 in the V image (this block's queries only;
  // the records keep the full-head width NW4 = SP / 64)
  const int NW4 = SP / 64;
  const bool mk = dmask != nullptr;
  if (mk) {
    MIFT_ASSERT(NW4 <= 8);
    const int qa = 16 * g0, qb = min(S, 16 * g1);
    for (int i = qa * NW4 + tid; i < qb * NW4; i += NT) {
      const int q = i / NW4, w = i % NW4;
      const uint2 v = *reinterpret_cast<const uint2*>(dmask + ((int64_t)bh * S + q) * (NW4 * 4) + w * 4);
      *reinterpret_cast<uint2*>((w < 4 ? Ks : Vs) + (size_t)q * G::RS + PADOFF + (w & 3) * 8) = v;
    }
  }
  __syncthreads();
  T* dQg = dqkv + (int64_t)b * S * ld + h * HD;
  for (int slot = 0;; ++slot) {
    const int grp = g0 + ((slot & 1) ? (slot + 1) * NW - 1 - wave : slot * NW + wave);
    if (slot * NW >= ng - g0) break;
    if (grp >= ng) continue;
    const int q0 = grp * 16, myq = q0 + qc;
    vec8<T> qf[G::NKS], df[G::NKS];
    float Dq = 0.f;
    {
      vec8<T> of[G::NKS];
      load_reg_frags<T, HD>(qf, Qg, ld, myq, S, lane);
      load_reg_frags<T, HD>(df, dOg, D, myq, S, lane);
      load_reg_frags<T, HD>(of, Og, D, myq, S, lane);
#pragma unroll
      for (int s = 0; s < G::NKS; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) Dq += (float)of[s][e] * (float)df[s][e];
      Dq = xor16_add(Dq);
      Dq = xor32_add(Dq);
      if (g == 0 && myq < S) Dv[(int64_t)bh * S + myq] = Dq;
    }
    const float lse2 = myq < S ? lse[(int64_t)bh * S + myq] * LOG2E : 0.f;
    float4_ dq[G::NOT];
#pragma unroll
    for (int i = 0; i < G::NOT; ++i) dq[i] = float4_{0.f, 0.f, 0.f, 0.f};
    const int kend = min(q0 + 16, klen);
    const int nkt = (kend + BKV - 1) / BKV;
    // compile-time causal / key-length mask: only the last key tile of a group needs it (as forward)
    auto ktile = [&](const int kt, auto diagc) {
      constexpr bool diag = decltype(diagc)::value;
      const int k0 = kt * BKV;
      vec8<T> dsf[2];
      uint2 kw = make_uint2(0u, 0u);
      if (mk) kw = *reinterpret_cast<const uint2*>((kt < 4 ? Ks : Vs) + (size_t)min(myq, S - 1) * G::RS + PADOFF + (kt & 3) * 8);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float4_ sa = float4_{0.f, 0.f, 0.f, 0.f}, pa = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < G::NKS; ++s) {
          sa = mfma16(ld_frag<T>(Ks + (k0 + t * 16 + qc) * G::RS + (4 * s + g) * 16), qf[s], sa);
          pa = mfma16(ld_frag<T>(Vs + (k0 + t * 16 + qc) * G::RS + (4 * s + g) * 16), df[s], pa);
        }
        bool kp[4] = {true, true, true, true};
        if (mk) {
          const uint32_t e = ((t < 2 ? kw.x : kw.y) >> ((t & 1) * 16 + g * 4)) & 0xFu;
#pragma unroll
          for (int r = 0; r < 4; ++r) kp[r] = (e >> r) & 1u;
        } else if (thr != 0) {
          const uint64_t i0 = ((uint64_t)bh * S + myq) * S + k0 + t * 16 + g * 4;
          if (hze) mift_keep4_hm(seed, hm0, i0, thr, kp);  // block-uniform (i0 even when S is)
          else mift_keep4(seed, i0, thr, kp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float pr = fast_exp2(sa[r] * c2 - lse2);
          if constexpr (diag) {
            const int key = k0 + t * 16 + g * 4 + r;
            if (key > myq || key >= klen) pr = 0.f;
          }
          float dp = pa[r];
          if (thr != 0) dp = kp[r] ? dp * inv_keep : 0.f;
          dsf[t >> 1][(t & 1) * 4 + r] = (T)(pr * (dp - Dq));
        }
      }
#pragma unroll
      for (int i = 0; i < G::NOT; ++i)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) dq[i] = mfma16(dsf[s2], tr_frag<T>(Ks, G::RS, k0 + 32 * s2, i * 16, lane), dq[i]);
    };
    for (int kt = 0; kt + 1 < nkt; ++kt) ktile(kt, std::false_type{});
    if (nkt > 0) ktile(nkt - 1, std::true_type{});
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + g * 4 + r;
      if (q < S) {
#pragma unroll
        for (int i = 0; i < G::NOT; ++i) dQg[(int64_t)q * ld + i * 16 + qc] = (T)(dq[i][r] * scale);
      }
    }
  }
}

template <typename T, int HD, int NW>
__global__ __launch_bounds__(NW * 64, HD <= 64 ? 4 : 2) void attn_bwd_dkdv_seq_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                                   const float* __restrict__ lse,
                                                                   const float* __restrict__ Dv, T* __restrict__ dqkv,
                                                                   const int* __restrict__ kv_len, int B, int S, int H,
                                                                   float scale, uint64_t seed,
                                                                   const int64_t* __restrict__ sstep, uint32_t thr,
                                                                   float inv_keep, const uint16_t* __restrict__ dmask,
                                                                   SeqSplit split) {
  seed = mift_seed(seed, sstep);
  using G = Geo<HD>;
  constexpr int NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int SP = (S + BKV - 1) / BKV * BKV;
  char* Qs = smem;                          // Q rows (A of S; tr-read B of dK); lse·log2e in the row padding
  char* dOs = smem + (size_t)SP * G::RS;    // dO rows (A of dP; tr-read B of dV); D in the row padding
  constexpr int PADOFF = G::HDP * 2;        // first padding byte of a row (RS - HDP*2 >= 32)
  static_assert(G::RS - PADOFF >= 32, "32-B row padding");
  // Byte x of row q's 32-B padding sits at (x + 16·((q >> 2) & 1)) mod 32: the two half-wave lane
  // groups of a padding read address rows q and q + 4 (g = 0, 1), whose rows are a multiple of
  // 128 B apart, so unrotated they hit the same bank with different addresses (2-way on every lse /
  // D / keep-bit read: 3.1 M conflict cycles per distilgpt2 dispatch); rotated by 16 B
  // the two groups use disjoint banks.
  auto pad = [&](char* img, int q, int x) { return img + (size_t)q * G::RS + PADOFF + ((x + 16 * ((q >> 2) & 1)) & 31); };
  auto lse_at = [&](int q) { return *reinterpret_cast<const float*>(pad(Qs, q, 0)); };
  auto D_at = [&](int q) { return *reinterpret_cast<const float*>(pad(dOs, q, 0)); };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, kc = lane & 15;
  int bh, g0, g1;
  seq_block(split, (S + 15) / 16, bh, g0, g1);  // key groups [g0, g1) of head bh
  const int QA = (16 * g0) / BQ * BQ;            // first query row any of them visits (causal)
  const int b = bh / H, h = bh % H;
  const int D = H * HD;
  const int64_t ld = 3LL * D;
  const T* Qg = qkv + (int64_t)b * S * ld + h * HD;
  const T* Kg = Qg + D;
  const T* Vg = Qg + 2 * D;
  const T* dOg = dout + (int64_t)b * S * D + h * HD;
  const int klen = kv_len ? kv_len[b] : S;
  MIFT_ASSERT(klen >= 0 && klen <= S);
  const float c2 = scale * LOG2E;
  const int ng = g1;
  // rows [QA, SP) of the Q / dO images (stage_rows from the offset row keeps the image row = query)
  stage_rows<T, HD>(Qs + (size_t)QA * G::RS, Qg + (int64_t)QA * ld, ld, S - QA, SP - QA, tid, NT);
  stage_rows<T, HD>(dOs + (size_t)QA * G::RS, dOg + (int64_t)QA * D, D, S - QA, SP - QA, tid, NT);
  for (int i = QA + tid; i < SP; i += NT) {
    const int q = min(i, S - 1);
    *reinterpret_cast<float*>(pad(Qs, i, 0)) = lse[(int64_t)bh * S + q] * LOG2E;
    *reinterpret_cast<float*>(pad(dOs, i, 0)) = Dv[(int64_t)bh * S + q];
  }
  // keep-bit records of the forward (KEEP BITS), element e of query q after the lse (e < 14) or the
  // D (e >= 14) float of row q: 28 B of padding per image row
  const int NR = SP / 16;
  const bool mk = dmask != nullptr;
  auto rec_at = [&](int q, int e) -> char* { return e < 14 ? pad(Qs, q, 4 + e * 2) : pad(dOs, q, 4 + (e - 14) * 2); };
  if (mk) {
    MIFT_ASSERT(NR <= 28);
    for (int i = QA * (NR / 4) + tid; i < S * (NR / 4); i += NT) {
      const int q = i / (NR / 4), w = i % (NR / 4);
      const uint2 v = *reinterpret_cast<const uint2*>(dmask + ((int64_t)bh * S + q) * NR + w * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<uint16_t*>(rec_at(q, w * 4 + j)) = (uint16_t)(((j < 2 ? v.x : v.y) >> ((j & 1) * 16)) & 0xFFFFu);
    }
  }
  __syncthreads();
  T* dKg = dqkv + (int64_t)b * S * ld + D + h * HD;
  T* dVg = dKg + D;
  const bool hz = (uint64_t)B * H * S * S < (1ull << 33);
  const uint32_t hm0 = mift_hmix(seed, 0);
  for (int slot = 0;; ++slot) {
    const int grp = g0 + ((slot & 1) ? (slot + 1) * NW - 1 - wave : slot * NW + wave);
    if (slot * NW >= ng - g0) break;
    if (grp >= ng) continue;
    const int k0 = grp * 16, mykey = k0 + kc;
    vec8<T> kf[G::NKS], vf[G::NKS];
    load_reg_frags<T, HD>(kf, Kg, ld, mykey, S, lane);
    load_reg_frags<T, HD>(vf, Vg, ld, mykey, S, lane);
    float4_ dk[G::NOT], dv[G::NOT];
#pragma unroll
    for (int i = 0; i < G::NOT; ++i) {
      dk[i] = float4_{0.f, 0.f, 0.f, 0.f};
      dv[i] = float4_{0.f, 0.f, 0.f, 0.f};
    }
    // query tiles of 64 starting at the tile holding this group's first key (causal)
    const int qt0 = k0 < klen ? k0 / BQ : SP / BQ;
    for (int qb = qt0 * BQ; qb < S; qb += BQ) {
      vec8<T> pf[2], dsf[2];
      const bool interior = qb >= k0 + 15 && qb + BQ <= S && k0 + 16 <= klen;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float4_ sa = float4_{0.f, 0.f, 0.f, 0.f}, pa = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < G::NKS; ++s) {
          sa = mfma16(ld_frag<T>(Qs + (qb + t * 16 + kc) * G::RS + (4 * s + g) * 16), kf[s], sa);
          pa = mfma16(ld_frag<T>(dOs + (qb + t * 16 + kc) * G::RS + (4 * s + g) * 16), vf[s], pa);
        }
        uint32_t hb[4] = {0, 0, 0, 0};
        if (mk) {
          // keep bit of (query, mykey): element grp = k0 / 16 of the query's record, bit kc
#pragma unroll
          for (int r = 0; r < 4; ++r)
            hb[r] = *reinterpret_cast<const uint16_t*>(rec_at(min(qb + t * 16 + g * 4 + r, S - 1), grp));
        } else if (thr != 0) {
          const int odd = kc & 1;
          const int qa = min(qb + t * 16 + g * 4 + 2 * odd, S - 1);
          const uint64_t p0 = (((uint64_t)bh * S + qa) * S + mykey) >> 1;
          const uint64_t p1 = (((uint64_t)bh * S + min(qa + 1, S - 1)) * S + mykey) >> 1;
          uint32_t h0, h1;
          if (hz) {
            h0 = mift_hash_lo(seed, hm0, (uint32_t)p0);
            h1 = mift_hash_lo(seed, hm0, (uint32_t)p1);
          } else {
            h0 = mift_hash_pair(seed, p0);
            h1 = mift_hash_pair(seed, p1);
          }
          const uint32_t o0 = __shfl_xor(h0, 1, 64), o1 = __shfl_xor(h1, 1, 64);
          hb[0] = odd ? o0 : h0;
          hb[1] = odd ? o1 : h1;
          hb[2] = odd ? h0 : o0;
          hb[3] = odd ? h1 : o1;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = qb + t * 16 + g * 4 + r;
          bool valid = true;
          float pr = fast_exp2(sa[r] * c2 - lse_at(ql));
          if (!interior) {
            valid = ql < S && mykey <= ql && mykey < klen;
            if (!valid) pr = 0.f;
          }
          float pd = pr, dp = pa[r];
          if (thr != 0) {
            bool kp;
            if (mk) {
              kp = valid && ((hb[r] >> kc) & 1u);
            } else {
              const uint32_t bits = (S & 1) ? mift_bits16(seed, ((uint64_t)bh * S + ql) * S + mykey)
                                            : ((hb[r] >> ((mykey & 1) << 4)) & 0xFFFFu);
              kp = valid && bits >= thr;
            }
            pd = kp ? pr * inv_keep : 0.f;
            dp = kp ? dp * inv_keep : 0.f;
          }
          pf[t >> 1][(t & 1) * 4 + r] = (T)pd;
          dsf[t >> 1][(t & 1) * 4 + r] = (T)(pr * (dp - D_at(ql)));
        }
      }
#pragma unroll
      for (int i = 0; i < G::NOT; ++i)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          dv[i] = mfma16(pf[s2], tr_frag<T>(dOs, G::RS, qb + 32 * s2, i * 16, lane), dv[i]);
          dk[i] = mfma16(dsf[s2], tr_frag<T>(Qs, G::RS, qb + 32 * s2, i * 16, lane), dk[i]);
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = k0 + g * 4 + r;
      if (key < S) {
#pragma unroll
        for (int i = 0; i < G::NOT; ++i) {
          dKg[(int64_t)key * ld + i * 16 + kc] = (T)(dk[i][r] * scale);
          dVg[(int64_t)key * ld + i * 16 + kc] = (T)dv[i][r];
        }
      }
    }
  }
}

// (A 32x32x16 forward with 32 queries per wave, "v2", was measured slower than this one on every
// model shape in rounds 3 and 5 — profiles/r3/bench_attn_v1_v2.txt, profiles/r5/bench_attn_fwd_v1_v2_xcd.json —
// and removed in round 6.)
template <typename T, int HD>
void fwd_launch(const at::Tensor& qkv, at::Tensor& o, at::Tensor& lse, const int* kvl, int B, int S, int H, float scale,
                uint64_t seed, uint32_t thr, float inv_keep, hipStream_t st, uint16_t* dmask) {
  using G = Geo<HD>;
  // query groups per wave (MIFT_ATTN_QG=1|2).  QG = 2 halves LDS bytes per MFMA but needs
  // 193 VGPRs (2 waves/SIMD vs 3) and measured slower on MI355X (tools/bench_attn.py: OPT-2.7B
  // fwd 75.2 vs 69.9 us, distilgpt2 41.0 vs 32.1 us, OPT-6.7B 243 vs 152 us): default 1
  static const int qg = [] { const char* e = getenv("MIFT_ATTN_QG"); return e ? atoi(e) : 1; }();
  const int seq_env = attn_seq_mode();
  const int smem = G::ROW_BYTES + G::TR_BYTES;
  // whole-sequence kernel when K and V of one head fit in LDS next to another block's (two
  // blocks per CU) and there are enough heads to fill the chip with one block per head
  const int SP = (S + BKV - 1) / BKV * BKV;
  const int seq_smem = SP * seq_row_bytes<HD>();
  const bool seq = seq_env && 2 * seq_smem <= 160 * 1024 && (B * H >= 256 || seq_env == 2);
  // transposed-output P·V (read per call: A/B): on for the whole-sequence kernel (distilgpt2 fwd 23.3 ->
  // 22.8 us), off for the tiled one (OPT-2.7B 49.2 vs 49.9 us, OPT-6.7B 115.9 vs 118.5;
  // profiles/r5/bench_attn_ot_xcd.jsonl)
  const char* ote = getenv("MIFT_ATTN_OT");
  const bool ot = ote ? atoi(ote) != 0 : seq;
  if (seq) {
    auto kern = ot ? attn_fwd_seq_kernel<T, HD, 8, true> : attn_fwd_seq_kernel<T, HD, 8, false>;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)attn_fwd_seq_kernel<T, HD, 8, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      (void)hipFuncSetAttribute((const void*)attn_fwd_seq_kernel<T, HD, 8, false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      attr = true;
    }
    int nblk = B * H;
    const SeqSplit split = seq_split_plan(B * H, S, num_cus_attn(), nblk);
    hipLaunchKernelGGL(kern, dim3(nblk), dim3(512), seq_smem, st, (const T*)qkv.data_ptr(), (T*)o.data_ptr(),
                       lse.data_ptr<float>(), kvl, B, S, H, scale, seed, mift_seed_step(), thr, inv_keep,
                       thr != 0 ? dmask : nullptr, split);
    return;
  }
  if (qg == 2) {
    const int nqt = (S + 2 * BQ - 1) / (2 * BQ);
    hipLaunchKernelGGL((attn_fwd_kernel<T, HD, 2>), dim3(B * H * nqt), dim3(256), smem, st, (const T*)qkv.data_ptr(),
                       (T*)o.data_ptr(), lse.data_ptr<float>(), kvl, B, S, H, scale, seed, mift_seed_step(), thr,
                       inv_keep, attn_xcd_env());
  } else {
    const int nqt = (S + BQ - 1) / BQ;
    auto k1 = ot ? attn_fwd_kernel<T, HD, 1, true> : attn_fwd_kernel<T, HD, 1, false>;
    hipLaunchKernelGGL(k1, dim3(B * H * nqt), dim3(256), smem, st, (const T*)qkv.data_ptr(),
                       (T*)o.data_ptr(), lse.data_ptr<float>(), kvl, B, S, H, scale, seed, mift_seed_step(), thr,
                       inv_keep, attn_xcd_env());
  }
}

template <typename T, int HD>
void bwd_launch(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& o, const at::Tensor& lse,
                at::Tensor& Dv, at::Tensor& dqkv, const int* kvl, int B, int S, int H, float scale, uint64_t seed,
                uint32_t thr, float inv_keep, hipStream_t st, const uint16_t* dmask) {
  using G = Geo<HD>;
  const int seq_env = attn_seq_mode();
  const int SP = (S + BKV - 1) / BKV * BKV;
  const int seq_dq = 2 * SP * G::RS, seq_kv = 2 * SP * G::RS;  // dkdv: lse / D live in the row padding
  if (seq_env && 2 * seq_kv <= 160 * 1024 && (B * H >= 256 || seq_env == 2)) {  // whole sequence in LDS, 2 blocks per CU
    auto kq = attn_bwd_dq_seq_kernel<T, HD, 8>;
    auto kk = attn_bwd_dkdv_seq_kernel<T, HD, 8>;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)kq, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      (void)hipFuncSetAttribute((const void*)kk, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      attr = true;
    }
    int nblk = B * H;
    const SeqSplit split = seq_split_plan(B * H, S, num_cus_attn(), nblk);
    hipLaunchKernelGGL(kq, dim3(nblk), dim3(512), seq_dq, st, (const T*)qkv.data_ptr(), (const T*)o.data_ptr(),
                       (const T*)dout.data_ptr(), lse.data_ptr<float>(), Dv.data_ptr<float>(), (T*)dqkv.data_ptr(),
                       kvl, B, S, H, scale, seed, mift_seed_step(), thr, inv_keep, thr != 0 ? dmask : nullptr, split);
    int nblk_kv = B * H;
    const SeqSplit split_kv = seq_split_plan_kv(B * H, S, num_cus_attn(), nblk_kv);
    hipLaunchKernelGGL(kk, dim3(nblk_kv), dim3(512), seq_kv, st, (const T*)qkv.data_ptr(), (const T*)dout.data_ptr(),
                       lse.data_ptr<float>(), Dv.data_ptr<float>(), (T*)dqkv.data_ptr(), kvl, B, S, H, scale, seed,
                       mift_seed_step(), thr, inv_keep, thr != 0 ? dmask : nullptr, split_kv);
    return;
  }
  const int nqt = (S + BQ - 1) / BQ, nkt = (S + BKV - 1) / BKV;
  const int smem_dq = 2 * G::ROW_BYTES + G::TR_BYTES;
  hipLaunchKernelGGL((attn_bwd_dq_kernel<T, HD>), dim3(B * H * nqt), dim3(256), smem_dq, st, (const T*)qkv.data_ptr(),
                     (const T*)o.data_ptr(), (const T*)dout.data_ptr(), lse.data_ptr<float>(),
                     Dv.data_ptr<float>(), (T*)dqkv.data_ptr(), kvl, B, S, H, scale, seed, mift_seed_step(), thr, inv_keep,
                     attn_xcd_env());
  const int smem_kv = 2 * G::ROW_BYTES + 2 * G::TR_BYTES + 2 * 64 * 4;
  // minimum waves per SIMD of the tiled dK/dV kernel (MIFT_ATTN_DKDV_OCC, read per call: A/B).  With the
  // round-3 bound (HD <= 64 ? 3 : 1) hd 128 took 268 registers — one wave per SIMD, below the two its LDS
  // allows; two: OPT-6.7B attention backward 629 -> 428 us (137 -> 201 TF/s), OPT-2.7B 184 -> 171 us;
  // three spills (1084 / 230 us) (profiles/r4/bench_attn_dkdv_occupancy.txt)
  const char* oe = getenv("MIFT_ATTN_DKDV_OCC");
  const int occ = oe ? atoi(oe) : 0;
  auto kv = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(B * H * nkt), dim3(256), smem_kv, st, (const T*)qkv.data_ptr(),
                       (const T*)dout.data_ptr(), lse.data_ptr<float>(), Dv.data_ptr<float>(), (T*)dqkv.data_ptr(),
                       kvl, B, S, H, scale, seed, mift_seed_step(), thr, inv_keep, attn_xcd_env());
  };
  if (occ == 2) kv(attn_bwd_dkdv_kernel<T, HD, 2>);
  else if (occ == 3) kv(attn_bwd_dkdv_kernel<T, HD, 3>);
  else kv(attn_bwd_dkdv_kernel<T, HD>);
}

}  // namespace

// KEEP BITS: with attention dropout on the whole-sequence path, the forward records every keep
// decision it draws (1 bit per (query, key) of the causal tiles it visits: [B*H, S, SP/16] uint16,
// element e of query q = keys 16e..16e+15, 3 MB per distilgpt2 layer) and the backward kernels
// read the bits instead of re-hashing: the hash is drawn once per element instead of three times.
// The bits ARE the hash's decisions, so the masks stay bit-identical to the counter-hash contract
// (common.h) and to the tiled / CPU paths, which keep hashing.
namespace {
int64_t keep_bits_elems(int64_t B, int64_t S, int64_t H, int64_t HD, double p) {
  if (p <= 0.0) return 0;
  const int64_t SP = (S + BKV - 1) / BKV * BKV;
  int64_t row = 0;
  switch (HD) {
    case 32: row = seq_row_bytes<32>(); break;
    case 64: row = seq_row_bytes<64>(); break;
    case 80: row = seq_row_bytes<80>(); break;
    case 128: row = seq_row_bytes<128>(); break;
    default: return 0;
  }
  const int mode = attn_seq_mode();
  if (!(mode && 2 * SP * row <= 160 * 1024 && (B * H >= 256 || mode == 2))) return 0;  // tiled path: no record
  return B * H * S * (SP / 16);
}
}  // namespace

std::vector<at::Tensor> mift_attn_fwd_impl(const at::Tensor& qkv, int64_t B, int64_t S, int64_t H, int64_t HD,
                                           double scale, double p, int64_t seed, const c10::optional<at::Tensor>& kv_len,
                                           bool want_bits);

std::vector<at::Tensor> mift_attn_fwd(const at::Tensor& qkv, int64_t B, int64_t S, int64_t H, int64_t HD, double scale,
                                      double p, int64_t seed, const c10::optional<at::Tensor>& kv_len) {
  return mift_attn_fwd_impl(qkv, B, S, H, HD, scale, p, seed, kv_len, false);
}

std::vector<at::Tensor> mift_attn_fwd_bits(const at::Tensor& qkv, int64_t B, int64_t S, int64_t H, int64_t HD,
                                           double scale, double p, int64_t seed,
                                           const c10::optional<at::Tensor>& kv_len) {
  return mift_attn_fwd_impl(qkv, B, S, H, HD, scale, p, seed, kv_len, true);
}

std::vector<at::Tensor> mift_attn_fwd_impl(const at::Tensor& qkv, int64_t B, int64_t S, int64_t H, int64_t HD,
                                           double scale, double p, int64_t seed, const c10::optional<at::Tensor>& kv_len,
                                           bool want_bits) {
  TORCH_CHECK(qkv.is_cuda() && qkv.is_contiguous() && (qkv.scalar_type() == at::kBFloat16 || qkv.scalar_type() == at::kHalf),
              "attn: bf16/fp16 contiguous qkv");
  TORCH_CHECK(qkv.numel() == B * S * 3 * H * HD, "attn: qkv shape");
  auto o = at::empty({B * S, H * HD}, qkv.options());
  auto lse = at::empty({B, H, S}, qkv.options().dtype(at::kFloat));
  const int* kvl = nullptr;
  if (kv_len) {
    TORCH_CHECK(kv_len->scalar_type() == at::kInt && kv_len->numel() == B, "attn: kv_len int32 [B]");
    kvl = kv_len->data_ptr<int>();
  }
  const int64_t nbits = want_bits ? keep_bits_elems(B, S, H, HD, p) : 0;
  auto bits = at::empty({nbits}, qkv.options().dtype(at::kShort));
  if (B * S == 0) return {o, lse, bits};
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const uint32_t thr = mift_thr16(p);
  const float inv_keep = p > 0 ? mift_inv_keep(p) : 1.f;
  const bool half = qkv.scalar_type() == at::kHalf;
  uint16_t* bp = nbits > 0 ? reinterpret_cast<uint16_t*>(bits.data_ptr()) : nullptr;
#define MIFT_FWD(D)                                                                                             \
  case D:                                                                                                       \
    if (half) fwd_launch<fp16, D>(qkv, o, lse, kvl, B, S, H, (float)scale, (uint64_t)seed, thr, inv_keep, st, bp); \
    else fwd_launch<bf16, D>(qkv, o, lse, kvl, B, S, H, (float)scale, (uint64_t)seed, thr, inv_keep, st, bp);      \
    break;
  switch (HD) {
    MIFT_FWD(64) MIFT_FWD(80) MIFT_FWD(128) MIFT_FWD(32)
    default: TORCH_CHECK(false, "attn: unsupported head dim ", HD);
#undef MIFT_FWD
  }
  if (want_bits) return {o, lse, bits};
  return {o, lse};
}

at::Tensor mift_attn_bwd_bits(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& o, const at::Tensor& lse,
                              int64_t B, int64_t S, int64_t H, int64_t HD, double scale, double p, int64_t seed,
                              const c10::optional<at::Tensor>& kv_len, const c10::optional<at::Tensor>& bits);

at::Tensor mift_attn_bwd(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& o, const at::Tensor& lse,
                         int64_t B, int64_t S, int64_t H, int64_t HD, double scale, double p, int64_t seed,
                         const c10::optional<at::Tensor>& kv_len) {
  return mift_attn_bwd_bits(dout, qkv, o, lse, B, S, H, HD, scale, p, seed, kv_len, c10::nullopt);
}

at::Tensor mift_attn_bwd_bits(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& o, const at::Tensor& lse,
                              int64_t B, int64_t S, int64_t H, int64_t HD, double scale, double p, int64_t seed,
                              const c10::optional<at::Tensor>& kv_len, const c10::optional<at::Tensor>& bits) {
  TORCH_CHECK(dout.is_contiguous() && o.is_contiguous(), "attn_bwd: contiguous");
  auto dqkv = at::empty_like(qkv);
  auto Dv = at::empty({B, H, S}, qkv.options().dtype(at::kFloat));
  if (B * S == 0) return dqkv;
  const int* kvl = kv_len ? kv_len->data_ptr<int>() : nullptr;
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const uint32_t thr = mift_thr16(p);
  const float inv_keep = p > 0 ? mift_inv_keep(p) : 1.f;
  TORCH_CHECK(dout.scalar_type() == qkv.scalar_type() && o.scalar_type() == qkv.scalar_type(), "attn_bwd: dtype");
  const bool half = qkv.scalar_type() == at::kHalf;
  // the forward's keep-bit record is used only when it exists for THIS launch geometry (the
  // backward takes the whole-sequence path exactly when the forward did); otherwise re-hash
  const uint16_t* bp = nullptr;
  if (bits && bits->numel() > 0) {
    TORCH_CHECK(bits->is_cuda() && bits->scalar_type() == at::kShort && bits->is_contiguous(), "attn_bwd: keep bits");
    if (bits->numel() == keep_bits_elems(B, S, H, HD, p)) bp = reinterpret_cast<const uint16_t*>(bits->data_ptr());
  }
#define MIFT_BWD(D)                                                                                          \
  case D:                                                                                                    \
    if (half) bwd_launch<fp16, D>(dout, qkv, o, lse, Dv, dqkv, kvl, B, S, H, (float)scale, (uint64_t)seed, thr, \
                                  inv_keep, st, bp);                                                         \
    else bwd_launch<bf16, D>(dout, qkv, o, lse, Dv, dqkv, kvl, B, S, H, (float)scale, (uint64_t)seed, thr,      \
                             inv_keep, st, bp);                                                              \
    break;
  switch (HD) {
    MIFT_BWD(64) MIFT_BWD(80) MIFT_BWD(128) MIFT_BWD(32)
    default: TORCH_CHECK(false, "attn_bwd: unsupported head dim ", HD);
#undef MIFT_BWD
  }
  return dqkv;
}
