// K1/K2: bf16/fp16 MFMA GEMM "NT" with fused epilogues.
//
//   C[M,N] = epi( A[M,K] · B[N,K]^T  (+ A2[M,32] · B2[N,32]^T) )
//
// Both operands are K-contiguous ("NT"), the layout the gfx950 MFMA
// fragments want: a 16x16x32 A or B fragment is 8 consecutive K elements of
// one row = one 16-byte ds_read_b128.  Frozen base weights are stored once
// per orientation (W as [out,in] for forward, W^T as [in,out] for dgrad),
// so forward and dgrad are both this kernel (see mift/models/layers.py).
//
// The optional A2/B2 pair is the LoRA "K-extension": with
// T = s·dropout(X)·A^T (rank r<=32, zero padded to 32 columns) and
// B2 = B (padded to [N,32]), one extra MFMA K-step adds the low-rank update
// s·dropout(X)·A^T·B^T to the same accumulators as X·W^T.  In the dgrad the
// extension is kept separate and added under the LoRA-input dropout mask.
//
// Main loop (gfx950): NWM x NWN waves, block tile BM x BN x 64, each wave
// owns (BM/NWM) x (BN/NWN) as 16x16 MFMA tiles (mfma_f32_16x16x32).
// Global->LDS staging by global_load_lds_dwordx4 (no VGPR round trip) into
// an NSTAGE-deep ring of XOR-swizzled images (16-B chunk c of row r stored at
// chunk c ^ (r & 7): the ds_read_b128 fragment reads of rows r0..r0+15 (r0 % 8 == 0) cover all 16
// slots of a 256-B bank row per 16-lane group, i.e. conflict-free by the §LDS bank rule — the PMC
// conflicts of round 2 came from the epilogue's C-tile image, see CTile below);
// swizzle applied on the per-lane global SOURCE address because the LDS-DMA
// destination is lane-linear, guide rule 21).  NSTAGE-1 tiles are in flight:
// each K step waits with a COUNTED s_waitcnt vmcnt (never 0 in steady state)
// and a raw s_barrier, so the LDS-DMA of the next tiles overlaps the MFMAs
// (guide §5 "Pipelining across barriers"; __syncthreads would drain it).
// MFMA operands are swapped (A-slot = B tile) so accumulators hold four
// consecutive output columns per lane (8-byte epilogue writes).
//
// Epilogue (two phases): accumulators (+bias, +masked LoRA ext) -> 16-bit
// tile in LDS, then every thread streams 8 consecutive columns (16-B
// loads/stores): pre-add, pre-activation output, activation (gelu_new / relu
// / gelu_erf) or activation-backward (dZ = dY ⊙ act'(aux)), dropout (counter
// hash, common.h) and residual add.
//
// Block order is XCD-aware (bijective remap, guide T1): blocks that share
// an XCD (b, b+8, ...) walk the N tiles of the same A row panel.
#include "common.h"
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

// This file is compiled as four translation units (gemm.hip = part 0, gemm_p1/p2/p3.hip): each defines
// MIFT_GEMM_PART and instantiates only its own kernels, so the ~80 kernel instantiations compile in
// parallel and an edit to one tile family rebuilds one small object.
//   part 0: gemm_nt entry, tiles 1-6 / 64x64, the skinny decode GEMMs, gemm_ln*
//   part 1: the 256x256 tiles (8: phased 8-wave loop, 10: 4-wave loop)
//   part 2: the 128-row ring tiles 7 (128x96) and 9 (128x192)
//   part 3: the fused LM head (forward, persistent forward, dgrad)
#ifndef MIFT_GEMM_PART
#define MIFT_GEMM_PART 0
#endif

// tile launchers of parts 1 / 2 (ep: this header's EpiArgs, by address; a2 / b2: 16-bit [.., 32])
void mift_gemm_part1(int tile, bool half, const at::Tensor& a, const at::Tensor& b, at::Tensor& c, const void* a2,
                     const void* b2, int M, int N, int K, const void* ep, hipStream_t st);
void mift_gemm_part2(int tile, bool half, const at::Tensor& a, const at::Tensor& b, at::Tensor& c, const void* a2,
                     const void* b2, int M, int N, int K, const void* ep, hipStream_t st);

namespace {

enum Act : int {
  ACT_NONE = 0,
  ACT_GELU_TANH = 1,
  ACT_RELU = 2,
  ACT_GELU_ERF = 3,
  ACT_GELU_TANH_BWD = 4,  // out = acc * gelu_tanh'(aux)
  ACT_RELU_BWD = 5,       // out = acc * (aux > 0)
  ACT_GELU_ERF_BWD = 6,
};

// Fused LM head + cross-entropy (EPI 1 / 2 below; host: mift_lmhead_fwd / mift_lmhead_dgrad).
//   forward  (EPI 1, phased 256x256 tile): z = x·Wᵀ stays in registers; per (row, 256-column tile j)
//            the epilogue writes E = exp(z - m_j) (16-bit, <= 1), the tile max m_j and
//            s_j = Σ_tile E, and the fp32 logit of the row's label.  Logits are never stored.
//   loss     (lmhead_lse_kernel): lse = log Σ_j s_j·exp(m_j), loss = lse - z_label.
//   backward (EPI 2, phased 256x256 tile, split-K): dlogits = g·(E·exp(m_j - lse) - onehot)
//            is never materialised: dX = g·(Σ_j exp(m_j - lse)·E_j·W_j - W[label]); the per-row,
//            per-column-tile factors are applied flash-attention style, rescaling the
//            accumulator at every 256-column group boundary; the one-hot part and g are applied
//            in the split-K reduction (lmhead_reduce_kernel).
struct LmArgs {
  const int64_t* labels;  // [M] (ignore_index / out of range -> no target)
  int V;                  // real vocabulary (columns >= V are padding)
  float2* stats;          // [M][ntn] (m_j, s_j)
  float* zlab;            // [M] fp32 logit of the label
  // backward
  const float* lse;       // [M]
  const float* gscale;    // device scalar: upstream grad (x loss scale / tokens)
  int ntn;                // column tiles of the forward (= groups of the backward)
  int gpc;                // groups per split-K chunk
  float* partial;         // [S][M][N] fp32 split-K slabs
  int dbg;                // MIFT_LM_DBG (diagnostics only): bit 0 = skip the E store, bit 2 = no FULL-tile epilogue
  int shift;              // > 0: labels are the UNSHIFTED [B*S] ids, S = shift (see lm_label)
  int64_t ignore;         // >= 0: this id is no target (OPT ignores its pad id, a real vocabulary entry)
};

// Target of row `row`: with shift = S the labels tensor holds the unshifted ids and row r's target
// is ids[r + 1] within its sequence (none for a sequence's last position) — the causal-LM shift done
// in the kernels instead of by two extra tensor ops per step.
MIFT_HD int64_t lm_label(const int64_t* labels, int row, int shift, int64_t ignore) {
  const int64_t l = shift <= 0 ? labels[row] : (row % shift == shift - 1) ? (int64_t)-1 : labels[row + 1];
  return l == ignore ? (int64_t)-1 : l;
}

struct EpiArgs {
  LmArgs lm;
  const void* bias;  // [N] (T or float)
  int bias_f32;
  const void* aux;   // [M,N] T (pre-activation for *_BWD)
  void* preact;      // [M,N] T (store z before activation)
  const void* residual;  // [M,N] T: out = residual + dropout(act(z))
  int act;
  uint64_t seed;
  uint32_t thr;      // dropout threshold (0 = no dropout)
  float inv_keep;
  float alpha;       // acc scale
  const float* alpha_ptr;  // optional device-side extra scale (e.g. upstream grad / loss scale)
  const void* pre_add;     // [M,N] T added to z before the activation
  uint32_t ext_thr;        // != 0: K-extension product is dropout-masked (LoRA input-dropout backward)
  uint64_t ext_seed;
  float ext_inv_keep;
  const int64_t* sstep;    // device micro-step for graph-replayed dropout seeds (common.h mift_seed)
  int group_m;             // tile raster: 0 = row panels (n fastest); g > 0 = groups of g row panels, m fastest
  // LoRA input projection of the OUTPUT (T = s·drop(out)·Aᵀ for the next layer's adapter, e.g. GPT-2
  // mlp.c_proj's input f = gelu(c_fc(x))): pw = A32s [32, N] (s baked in), the first prow rows
  // non-zero; each tile's partial over its BN columns goes to the fp32 slab pws [ntn][M][16|32]
  // (deterministic), proj_reduce_kernel sums the slabs in order into pout [M, 32] x palpha.
  const void* pw;
  int prow;
  uint32_t pthr;
  uint64_t pseed;
  float* pws;
  void* pout;
  float palpha;
  // ReLU sign bits [M][N/8] (bit e of byte (row, col/8) = stored output (row, col + e) > 0): written by an
  // ACT_RELU epilogue, read by ACT_RELU_BWD in place of the 16-bit aux (1/16 of its bytes)
  uint8_t* sbits;
  int pfg;        // 256x256 epilogue: operands requested per group of 4 chunks (MIFT_EPI_PFG, default 1)
  int ntc;        // non-temporal C stores (outputs >= 96 MiB; MIFT_EPI_NT forces)
  // diagnostics (tools/gemm_stamps.py): per block, wave 0's s_memtime at [0] entry, [1] main loop
  // started (prologue done), [2] main loop done, [3] C tile in LDS, [4] exit; s_memrealtime at [6] / [7]
  long long* stamps;
  int staged;     // interior tiles: feature-staged epilogue phase 2 (MIFT_EPI_STAGED, default 1)
  int hoist;      // dropout-mask hashes with the hoisted high-word mix (output < 2^33 elements; MIFT_EPI_HOIST)
  int ext_lds;    // NSTAGE >= 2 tiles: K-extension operands staged into LDS during the last k-tile (MIFT_EXT_LDS)
};

// Tile t (after the XCD remap, consecutive t share an XCD) -> (row tile, column tile).  With g > 0
// the tiles run in groups of g row panels with the row index fastest: the ~32 blocks an XCD holds at
// once cover g row panels x 32/g column tiles, so each B (weight) tile is fetched once per group
// instead of once per row panel.  The LM head (N = 50304, 197 column tiles) fetched its 77 MB
// weight 32x from HBM in row-panel order (TCC_EA0_RDREQ 2.5x hipBLASLt's, tools/pmc_lmhead.sh).
MIFT_HD void raster(int t, int ntm, int ntn, int g, int& tm, int& tn) {
  if (g <= 1) {
    tm = t / ntn;
    tn = t % ntn;
    return;
  }
  const int per = g * ntn, grp = t / per, first = grp * g;
  const int gs = min(ntm - first, g), r = t - grp * per;
  tm = first + r % gs;
  tn = r / gs;
}

// Split-K tail (second launch of a hybrid data-parallel + split-K GEMM): the
// ragged last wave of tiles [tile0, tile0 + ntiles) is cut into gx k-chunks per
// tile, one block per chunk.  Chunk blocks store fp32 partials and release a
// per-tile counter; the last-chunk block acquires it (agent scope: chunks may
// sit on different XCDs / L2s), reduces, runs the normal fused epilogue and
// re-arms the counter.  It only waits for lower-index blocks, which the
// in-order dispatcher started earlier, so it cannot deadlock even when RCCL
// kernels hold some CUs.
struct SkArgs {
  int enabled;
  int tile0, ntiles, gx;  // gx = k-splits per tile
  float* ws;   // [ntiles * gx][BM*BN] fp32 partial slots (one per block)
  int* flags;  // [ntiles] arrival counters, zero on entry and on exit
};

template <typename T>
using frag_t = typename std::conditional<std::is_same<T, bf16>::value, bf16x8, fp16x8>::type;

template <typename T>
MIFT_HD float4_ mfma16(frag_t<T> a, frag_t<T> b, float4_ c) {
  if constexpr (std::is_same<T, bf16>::value)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

MIFT_HD float apply_act(int act, float z, float aux) {
  switch (act) {
    case ACT_GELU_TANH: return gelu_tanh(z);
    case ACT_RELU: return fmaxf(z, 0.f);
    case ACT_GELU_ERF: return gelu_erf(z);
    case ACT_GELU_TANH_BWD: return z * gelu_tanh_grad(aux);
    case ACT_RELU_BWD: return aux > 0.f ? z : 0.f;
    case ACT_GELU_ERF_BWD: return z * gelu_erf_grad(aux);
    default: return z;
  }
}

constexpr int BK = 64;
constexpr int ROWB = BK * 2;  // bytes per LDS row (128)
constexpr int LM_GW = 25;     // LM-head dgrad: groups (forward column tiles) per LDS window of tile maxima (25: the
                              // distilgpt2 chunks of 25 groups take one window, OPT's of 50 two)

// s_waitcnt vmcnt(n) with a compile-time n (0..63)
template <int N>
MIFT_HD void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- building blocks of the 4-wave 256x256 schedule (mainloop4 below) ----
// Every instruction of that loop is a volatile asm statement, so hipcc keeps them in the written
// order: the interleave of MFMAs with LDS reads and LDS-DMA issues IS the schedule.  hipcc neither
// counts these loads nor pads their hazards (guide §5.7): the loop waits with its own counted
// s_waitcnt and keeps >= 8 MFMAs between an MFMA's last read of a fragment register and the
// ds_read that overwrites it.
typedef int srd_t __attribute__((ext_vector_type(4)));  // buffer resource descriptor (4 SGPRs)

template <int N, typename F, int... I>
MIFT_HD void static_for_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
// f(integral_constant<0>) ... f(integral_constant<N-1>), unrolled at compile time
template <int N, typename F>
MIFT_HD void static_for(F&& f) {
  static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}
// LDS byte address of a pointer into the dynamic shared segment
MIFT_HD uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}
// 16-B LDS read; the caller waits (s_waitcnt lgkmcnt) before the first use
template <int OFF, typename F>
MIFT_HD void lds_rd(F& dst, uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset is 16-bit");
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(OFF));
}
// acc += b·a, accumulator pinned to AGPRs (256 accumulators per lane: the builtin form let the
// register allocator shuttle copies between the two files, round 3)
template <typename T>
MIFT_HD void mfma_acc(float4_& c, frag_t<T> b, frag_t<T> a) {
  if constexpr (std::is_same<T, bf16>::value)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
  else
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
}
// acc = b·a (first k-step of a tile: no zero fill of the 256 accumulators)
template <typename T>
MIFT_HD void mfma_acc0(float4_& c, frag_t<T> b, frag_t<T> a) {
  if constexpr (std::is_same<T, bf16>::value)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(b), "v"(a));
  else
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(c) : "v"(b), "v"(a));
}
// one 1-KiB LDS-DMA piece: 16 B per lane from srd base + voff to LDS [lds, lds + 1024).  M0 is
// compiler-reserved: set and restored inside the statement (guide §5.7 item "M0")
MIFT_HD void dma16(uint32_t voff, srd_t srd, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(srd), "s"(lds)
      : "memory");
}
template <int N>
MIFT_HD void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
MIFT_HD void sbarrier() { asm volatile("s_barrier" ::: "memory"); }
// >= 32 wait states: MFMA result -> VALU reader, and VALU write -> MFMA srcC (loop entry / exit)
MIFT_HD void mfma_fence() { asm volatile("s_nop 15\n\ts_nop 15" ::: "memory"); }
// empty statement that "rewrites" every accumulator: placed next to mfma_fence it keeps the
// compiler's own reads / writes of acc on their side of the fence (data dependence)
template <int TM, int TN>
MIFT_HD void pin_acc(float4_ (&acc)[TM][TN]) {
  static_assert(TN == 8, "pin_acc: 8 accumulators per statement");
#pragma unroll
  for (int i = 0; i < TM; ++i)
    asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]), "+a"(acc[i][4]),
                 "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
}

// ---- C-tile staging image in LDS (epilogue phase 1 -> phase 2) ----
// Unit = 8 bytes (4 16-bit elements).  Row r's unit u is stored at unit u ^ sw(r) of a row of CLDU
// units.  Phase 1 writes one unit per lane (ds_write_b64: 16-lane groups, bank = dword % 32; the
// 16 lanes of a group hold rows r0..r0+15 of ONE logical unit); phase 2 reads 16 B = units
// (2k, 2k+1) per lane (ds_read_b128, bank = dword % 64), which the XOR keeps adjacent (swapped
// when sw(r) is odd).  BN % 64 == 0: CLDU = BN/4 (whole 128-B bank rows) and sw(r) = r & 15 —
// conflict-free for both phases.  BN = 96 (12 chunks per row, so a phase-2 lane group straddles
// rows): CLDU = 40 and a 32-row permutation table found by an exhaustive bank model of both phases
// (lane groups per MI355X_MICROARCH.md §LDS; the model reproduces the PMC count of the plain
// layout exactly, 192 conflict cycles per block) -> 0 on writes, 32 cycles per block on reads.
// The round-2 BN+8 padding was 2-way on every phase-1 write (PMC: 1.08 M conflict cycles per
// 128x192 dispatch, 12.9 M per LM-head forward).
template <int BN>
struct CTile {
  static constexpr int CLDU = BN % 64 == 0 ? BN / 4 : 40;
  static constexpr int CLD = CLDU * 4;  // elements
  static_assert(BN % 64 == 0 || BN == 96, "C-tile swizzle: BN % 64 == 0 or BN == 96");
  static MIFT_HD int sw(int row) {
    if constexpr (BN % 64 == 0) {
      return row & 15;
    } else {
      const uint64_t t = (row & 16) ? 0xe8fb5163d9ac2074ull : 0xdcfa34028eb97156ull;
      return (int)((t >> ((row & 15) * 4)) & 15);
    }
  }
  // element offset of the 4 elements at (row, col), col % 4 == 0
  static MIFT_HD int off4(int row, int col) { return row * CLD + (((col >> 2) ^ sw(row)) << 2); }
  // the 8 elements at (row, c8), c8 % 8 == 0
  static MIFT_HD short8 read8(const void* cs, int row, int c8) {
    const int x = sw(row);
    const short8 v = *reinterpret_cast<const short8*>(reinterpret_cast<const short*>(cs) + row * CLD +
                                                       ((((c8 >> 2) ^ x) & ~1) << 2));
    return (x & 1) ? short8{v[4], v[5], v[6], v[7], v[0], v[1], v[2], v[3]} : v;
  }
  // inverse of read8 (the half swap is an involution)
  static MIFT_HD void write8(void* cs, int row, int c8, short8 v) {
    const int x = sw(row);
    *reinterpret_cast<short8*>(reinterpret_cast<short*>(cs) + row * CLD + ((((c8 >> 2) ^ x) & ~1) << 2)) =
        (x & 1) ? short8{v[4], v[5], v[6], v[7], v[0], v[1], v[2], v[3]} : v;
  }
};

// wait until at most N stages of LDS-DMA pieces are outstanding: PS_HI pieces per stage on waves
// < NHI, PS_LO on the rest (the stage's pieces need not split evenly over the waves)
template <int N, int PS_HI, int PS_LO, int NHI>
MIFT_HD void wait_stages(int wave) {
  if constexpr (PS_HI == PS_LO) {
    wait_vmcnt<N * PS_HI>();
  } else {
    if (wave < NHI) wait_vmcnt<N * PS_HI>();
    else wait_vmcnt<N * PS_LO>();
  }
}

// KB: k-tile depth, 64 (128-B LDS rows, 16-B chunk c of row r at slot c ^ (r & 7)) or 32 (64-B rows:
// four rows share a 256-B bank row, chunk c of row r at slot c ^ ((r >> 2) & 3) — the 16 rows of a
// fragment read then cover the 16 slots of a bank row once, conflict-free as for KB = 64).  KB = 32
// keeps the LDS of a 2-stage KB = 64 ring but holds 4 half-depth stages: three k-tiles in flight
// instead of one for the K = 768 shapes whose main loop waits on LDS-DMA latency.
// waves per SIMD a tile's LDS footprint allows (launch_gemm's SMEM): the register budget the compiler must
// respect so that the blocks the LDS admits can actually co-reside (e.g. 128x192: two 8-wave blocks = 4
// waves per SIMD = 128 VGPRs; without the bound a richer epilogue silently halves the occupancy)
template <int BM, int BN, int NWM, int NWN, int NSTAGE, int KB>
constexpr int gemm_waves_per_eu() {
  constexpr int NT = NWM * NWN * 64;
  constexpr int RING = (NSTAGE <= 1 ? 2 : NSTAGE) * (BM + BN) * KB * 2;
  constexpr int CLDU = BN % 64 == 0 ? BN / 4 : 40;
  constexpr int EPI_BYTES = BM * CLDU * 4 * 2;
  constexpr int SMEM = RING > EPI_BYTES ? RING : EPI_BYTES;
  constexpr int BPC = (160 * 1024 / SMEM) < (2048 / NT) ? (160 * 1024 / SMEM) : (2048 / NT);
  constexpr int W = (BPC > 0 ? BPC : 1) * (NT / 64) / 4;
  return W > 0 ? W : 1;
}

template <typename T, int BM, int BN, int NWM, int NWN, int NSTAGE, bool SKM, int EPI = 0, int KB = 64>
__global__ __launch_bounds__(NWM* NWN * 64, (gemm_waves_per_eu<BM, BN, NWM, NWN, NSTAGE, KB>())) void gemm_nt_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                                T* __restrict__ C, const T* __restrict__ A2,
                                                                const T* __restrict__ B2, int M, int N, int K,
                                                                int lda, int ldb, int ldc, EpiArgs ep, SkArgs sk) {
  constexpr int NW = NWM * NWN;
  constexpr int NT = NW * 64;
  constexpr int WM = BM / NWM, WN = BN / NWN;  // wave tile
  constexpr int TM = WM / 16, TN = WN / 16;    // MFMA tiles per wave
  static_assert(KB == 64 || (KB == 32 && NSTAGE > 0 && EPI == 0), "KB = 32: ring pipeline, plain GEMM only");
  constexpr int KBY = KB * 2;       // bytes per LDS row
  constexpr int RPP = 1024 / KBY;   // rows per 1-KiB LDS-DMA piece
  constexpr int CPR = KB / 8;       // 16-B chunks per row
  constexpr int A_BYTES = BM * KBY, B_BYTES = BN * KBY;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int A_INSTR = BM / RPP, B_INSTR = BN / RPP;  // 1-KiB LDS-DMA pieces per stage
  constexpr bool EVEN = A_INSTR % NW == 0 && B_INSTR % NW == 0;
  constexpr int P_ALL = A_INSTR + B_INSTR;
  // vmcnt units per stage: PS_HI on waves < NHI, PS_LO on the others (all equal when EVEN)
  constexpr int PS_LO = P_ALL / NW, NHI = P_ALL % NW, PS_HI = PS_LO + (NHI ? 1 : 0);
  auto swz = [](int r) { return KB == 64 ? (r & 7) : ((r >> 2) & 3); };
  constexpr int NBUF = NSTAGE <= 1 ? 2 : NSTAGE;  // NSTAGE 0 / 1 = phased / 4-wave schedule on 2 buffers
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (ep.sstep != nullptr) {
    ep.seed = mift_seed(ep.seed, ep.sstep);
    ep.ext_seed = mift_seed(ep.ext_seed, ep.sstep);
    ep.pseed = mift_seed(ep.pseed, ep.sstep);
  }

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / NWN, wn = wave % NWN;
  auto stamp = [&](int i) {
    if (ep.stamps != nullptr && tid == 0)
      ep.stamps[(size_t)blockIdx.x * 8 + i] =
          i >= 6 ? (long long)__builtin_amdgcn_s_memrealtime() : (long long)__builtin_amdgcn_s_memtime();
  };
  stamp(0);
  stamp(6);

  const int ntm = (M + BM - 1) / BM, ntn = (N + BN - 1) / BN;
  int m0 = 0, n0 = 0;

  // per-lane staging coordinates: lane -> (row in the piece, phys chunk) (lane-linear LDS-DMA destination)
  const int srow = lane / CPR, spc = lane % CPR;
  auto stage = [&](int buf, int k0) {
    char* base = smem + buf * STAGE_BYTES;
    if constexpr (EVEN) {
#pragma unroll
      for (int ii = 0; ii < A_INSTR / NW; ++ii) {
        const int i = wave + ii * NW;
        const int r = i * RPP + srow;
        const int lc = spc ^ swz(r);
        const int gr = min(m0 + r, M - 1);
        __builtin_amdgcn_global_load_lds((const void*)(A + (size_t)gr * lda + k0 + lc * 8),
                                         (void*)(base + i * 1024), 16, 0, 0);
      }
#pragma unroll
      for (int ii = 0; ii < B_INSTR / NW; ++ii) {
        const int i = wave + ii * NW;
        const int r = i * RPP + srow;
        const int lc = spc ^ swz(r);
        const int gr = min(n0 + r, N - 1);
        __builtin_amdgcn_global_load_lds((const void*)(B + (size_t)gr * ldb + k0 + lc * 8),
                                         (void*)(base + A_BYTES + i * 1024), 16, 0, 0);
      }
    } else {
      // pieces 0 .. P_ALL-1 (A then B) round-robin over the waves (wave-uniform branches)
#pragma unroll
      for (int ii = 0; ii < PS_HI; ++ii) {
        const int i = wave + ii * NW;
        if (i < P_ALL) {
          const bool isa = i < A_INSTR;
          const int pi = isa ? i : i - A_INSTR;
          const int r = pi * RPP + srow;
          const int lc = spc ^ swz(r);
          const T* src = isa ? A + (size_t)min(m0 + r, M - 1) * lda : B + (size_t)min(n0 + r, N - 1) * ldb;
          __builtin_amdgcn_global_load_lds((const void*)(src + k0 + lc * 8), (void*)(base + i * 1024), 16, 0, 0);
        }
      }
    }
  };

  float4_ acc[TM][TN];
  const int fr = lane & 15;  // fragment row
  const int fq = lane >> 4;  // k sub-chunk (0..3)

  // LoRA K-extension operands (A2 [M, 32], B2 [N, 32]: 64-B rows) of this tile staged into a free ring
  // buffer by LDS-DMA during the last k-tile, so the epilogue reads them from LDS instead of waiting a
  // global round trip after the main loop (epilogue phase 1 with the extension +1.2k-2.0k -> +0.5k-0.8k
  // cycles per block, profiles/r6/gemm_stamps_dgpt_ext_{global,lds}.txt; distilgpt2 step 4.680 -> 4.666 ms
  // same-process, step_ab_dgpt_ext_lds.json).  1-KiB pieces of 16 rows; lane -> (row 16p + lane/4, physical 16-B chunk lane%4) holding
  // logical chunk phys ^ ((row >> 2) & 3), so a fragment read (16 rows, one logical chunk) spreads
  // over all 64 banks.
  constexpr int EXT_PA = BM / 16, EXT_PB = BN / 16;
  int ext_buf = -1;  // ring buffer holding the staged K-extension operands (-1: not staged)
  // The bias row of the tile rides along (one 1-KiB piece after the extension rows, bytes
  // [n0·esz, n0·esz + 1024) of the bias; lanes past the end re-read its last 16 B, which only feed
  // columns >= N): phase 1 read it from global after the main loop, +0.8k-1.5k cycles per block.
  constexpr int EXT_BIAS_OFF = (BM + BN) * 64;
  const int besz = ep.bias_f32 ? 4 : 2;
  const bool bias_lds = ep.bias != nullptr && ((size_t)N * besz) % 16 == 0 && BN * 4 <= 1024;
  auto stage_ext = [&](int buf) {
    char* base = smem + buf * STAGE_BYTES;
    const int row = lane >> 2, phys = lane & 3;
    if (A2 != nullptr) {
      for (int p = wave; p < EXT_PA + EXT_PB; p += NW) {  // wave-uniform
        const bool isa = p < EXT_PA;
        const int r = (isa ? p : p - EXT_PA) * 16 + row;
        const int lc = phys ^ ((r >> 2) & 3);
        const T* src = isa ? A2 + (size_t)min(m0 + r, M - 1) * 32 : B2 + (size_t)min(n0 + r, N - 1) * 32;
        __builtin_amdgcn_global_load_lds((const void*)(src + lc * 8), (void*)(base + p * 1024), 16, 0, 0);
      }
    }
    if (bias_lds && wave == NW - 1) {
      const size_t off = min((size_t)n0 * besz + (size_t)lane * 16, (size_t)N * besz - 16);
      __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const char*>(ep.bias) + off),
                                       (void*)(base + EXT_BIAS_OFF), 16, 0, 0);
    }
  };
  static_assert(NSTAGE < 2 || (BM % 16 == 0 && BN % 16 == 0 && (BM + BN) * 64 + 1024 <= STAGE_BYTES),
                "K-extension / bias staging: 16-row pieces and the bias piece fit one ring buffer");

  // acc = sum over k-tiles [kb, ke) of the (m0, n0) tile; extl: stage the K-extension operands too
  auto mainloop = [&](int kb, int ke, bool extl = false) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = float4_{0.f, 0.f, 0.f, 0.f};
    const int nk = ke - kb;
    // prologue: NBUF-1 tiles in flight
#pragma unroll
    for (int s = 0; s < NBUF - 1; ++s)
      if (s < nk) stage(s, (kb + s) * KB);
    for (int kt = 0; kt < nk; ++kt) {
      // tile kt landed <=> at most (#tiles issued after kt) * (pieces per stage) outstanding:
      // min(NBUF - 2, nk - 1 - kt) tiles were issued after it (counted, never drained to 0 early)
      if constexpr (NBUF >= 4) {
        const int after = min(NBUF - 2, nk - 1 - kt);
        if (after >= 2) wait_stages<2, PS_HI, PS_LO, NHI>(wave);
        else if (after == 1) wait_stages<1, PS_HI, PS_LO, NHI>(wave);
        else wait_vmcnt<0>();
        static_assert(NBUF <= 4 && 2 * PS_HI < 64, "deeper rings need more wait cases");
      } else if constexpr (NBUF == 3) {
        if (kt + 1 < nk) wait_stages<1, PS_HI, PS_LO, NHI>(wave);
        else wait_vmcnt<0>();
      } else {
        wait_vmcnt<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // everyone's pieces of kt landed; everyone done reading kt-1
      asm volatile("" ::: "memory");  // no LDS access may move above the barrier
      if (kt + NBUF - 1 < nk) stage((kt + NBUF - 1) % NBUF, (kb + kt + NBUF - 1) * KB);
      else if (extl && kt == nk - 1) {  // that buffer held tile kt-1, read by everyone before the barrier
        ext_buf = (kt + NBUF - 1) % NBUF;
        stage_ext(ext_buf);
      }
      const char* As = smem + (kt % NBUF) * STAGE_BYTES;
      const char* Bs = As + A_BYTES;
#pragma unroll
      for (int kk = 0; kk < KB / 32; ++kk) {
        const int lc = kk * 4 + fq;
        frag_t<T> af[TM], bfv[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int r = wm * WM + i * 16 + fr;
          af[i] = *reinterpret_cast<const frag_t<T>*>(As + r * KBY + ((lc ^ swz(r)) << 4));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = wn * WN + j * 16 + fr;
          bfv[j] = *reinterpret_cast<const frag_t<T>*>(Bs + r * KBY + ((lc ^ swz(r)) << 4));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<T>(bfv[j], af[i], acc[i][j]);
      }
    }
  };

  // ---- phased schedule (NSTAGE == 0): 256x256 tile, 2x4 waves of 128x64, BK = 64 ----
  // Each k-tile is 4 phases, one output quadrant (64x32 of the wave tile, 16 MFMAs) each:
  //   ph0 (q 0,0): ds_read A rows 0-63 (8) + B cols 0-31 (4)   | LDS-DMA A half 0 of tile kt+1
  //   ph1 (q 0,1): ds_read B cols 32-63 (4)                     | LDS-DMA A half 1 of tile kt+1
  //   ph2 (q 1,1): ds_read A rows 64-127 (8)                    |
  //   ph3 (q 1,0): (A, B from registers)                        | LDS-DMA B halves of tile kt+2,
  //                                                               counted vmcnt(4) retires tile kt+1
  // phase = {reads, DMA issue, [wait]} -> s_barrier -> MFMA cluster (setprio 1) -> s_barrier.
  // Wave row 1 (waves 4-7) runs one barrier behind row 0, so on every SIMD one wave is in its
  // MFMA cluster while its partner issues reads / DMA (guide §5 "256² 8-phase template").
  // Buffer hazards (two buffers, tile t in buffer t&1): a region is restaged >= 2 phases after
  // its last ds_read (B of tile kt read last in ph1 -> B(kt+2) in ph3; A of tile kt-1 read last
  // in its ph2 -> A(kt+1) in ph0/ph1), and read >= 1 phase after the wait that retires it.
  // acc += sum over k-tiles [kb, ke); hook(kt) runs at the top of every k-tile (before its reads)
  auto mainloop8 = [&](int kb, int ke, auto&& hook) {
   if constexpr (NSTAGE == 0) {
    static_assert(BM == 256 && BN == 256 && NWM == 2 && NWN == 4, "phased loop: 256x256 tile, 2x4 waves");
    const int nk = ke - kb;
    // half h (rows 128h..128h+127) of operand o (0 = A, 1 = B) of k-tile t -> buffer t & 1
    auto stage_half = [&](int t, int o, int h) {
      char* base = smem + (t & 1) * STAGE_BYTES + o * A_BYTES;
      const T* G = o ? B : A;
      const int ld = o ? ldb : lda;
      const int rmax = (o ? N : M) - 1;
      const int r00 = o ? n0 : m0;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = 16 * h + wave + 8 * ii;
        const int r = i * 8 + srow;
        const int gr = min(r00 + r, rmax);
        const void* src = (const void*)(G + (size_t)gr * ld + (kb + t) * BK + (spc ^ (r & 7)) * 8);
        __builtin_amdgcn_global_load_lds(src, (void*)(base + i * 1024), 16, 0, 0);
      }
    };
    const int arow = wm * WM + fr, brow = wn * WN + fr;
    const int sw0 = (fq ^ (fr & 7)) << 4, sw1 = ((4 + fq) ^ (fr & 7)) << 4;
    frag_t<T> af[4][2], bq[4][2];
    auto rd = [&](const char* p) { return *reinterpret_cast<const frag_t<T>*>(p); };
    auto cluster = [&](int qi, int qj) {
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[qi * 4 + i][qj * 2 + j] = mfma16<T>(bq[qj * 2 + j][kk], af[i][kk], acc[qi * 4 + i][qj * 2 + j]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };

    stage_half(0, 0, 0);
    stage_half(0, 0, 1);
    stage_half(0, 1, 0);
    stage_half(0, 1, 1);
    if (nk > 1) {
      stage_half(1, 1, 0);
      stage_half(1, 1, 1);
      wait_vmcnt<4>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();  // stagger the wave rows by one barrier
    asm volatile("" ::: "memory");
    for (int kt = 0; kt < nk; ++kt) {
      hook(kt);
      const char* As = smem + (kt & 1) * STAGE_BYTES;
      const char* Bs = As + A_BYTES;
      // ph0
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i][0] = rd(As + (arow + i * 16) * ROWB + sw0);
        af[i][1] = rd(As + (arow + i * 16) * ROWB + sw1);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bq[j][0] = rd(Bs + (brow + j * 16) * ROWB + sw0);
        bq[j][1] = rd(Bs + (brow + j * 16) * ROWB + sw1);
      }
      if (kt + 1 < nk) stage_half(kt + 1, 0, 0);
      cluster(0, 0);
      // ph1
#pragma unroll
      for (int j = 2; j < 4; ++j) {
        bq[j][0] = rd(Bs + (brow + j * 16) * ROWB + sw0);
        bq[j][1] = rd(Bs + (brow + j * 16) * ROWB + sw1);
      }
      if (kt + 1 < nk) stage_half(kt + 1, 0, 1);
      cluster(0, 1);
      // ph2
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i][0] = rd(As + (arow + (i + 4) * 16) * ROWB + sw0);
        af[i][1] = rd(As + (arow + (i + 4) * 16) * ROWB + sw1);
      }
      cluster(1, 1);
      // ph3
      if (kt + 2 < nk) {
        stage_half(kt + 2, 1, 0);
        stage_half(kt + 2, 1, 1);
        wait_vmcnt<4>();
      } else {
        wait_vmcnt<0>();
      }
      cluster(1, 0);
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();  // re-align the rows (equal barrier counts)
   }
  };

  // ---- 4-wave schedule (NSTAGE == 1): 256x256 tile, 2x2 waves = ONE wave per SIMD owning a 128x128
  // quadrant (8x8 MFMA 16x16x32 tiles, 256 accumulators per lane in AGPRs), BK = 64, two LDS buffers.
  // The issue order of the library's own MT256x256x64 kernel for these shapes (hipBLASLt
  // Custom_Cijk_Alik_Bljk_HHS_BH_MT256x256x64_MI16x16x1, llvm-objdump of the local gfx950 code object:
  // one buffer_load…lds or ds_read_b128 between consecutive MFMAs, 3 barriers per k-tile), re-expressed
  // here in our own LDS image (XOR-swizzled rows, not the library's padding):
  //   * the fragments of a k-tile are double-buffered in registers by k-half (F0 = k 0-31, F1 = 32-63,
  //     8 A + 8 B fragments each = 128 VGPRs): F1 of tile kt is read during the MFMAs on F0, F0 of tile
  //     kt+1 during the MFMAs on F1, so every LDS read hides behind 8+ MFMAs;
  //   * because tile kt's LDS image is fully in registers a third of the way into k-tile kt, its buffer is
  //     restaged THEN with tile kt+2 — B once every wave's B reads retired (barrier 1, MFMA 17), A after
  //     barrier 2 (MFMA 51) — so each piece has ~1.3 k-tiles (~2.6k cycles) to land, where the round-3
  //     4-wave loop restaged one k-tile ahead behind a vmcnt(0) and lost to the phased loop;
  //   * the 16 LDS-DMA pieces of a k-tile are spread one per two MFMAs (not issued in a burst);
  //   * one counted vmcnt(16) + barrier (MFMA 87) publishes tile kt+1 before its F0 reads.
  // Hazards: B(kt) is overwritten only after barrier 1 of k-tile kt, which every wave passes after
  // lgkmcnt(0) retired its F1 B reads of tile kt (its F0 B reads retired at the end of k-tile kt-1);
  // A likewise at barrier 2; tile kt+1 is read only after the vmcnt + barrier that retires every wave's
  // pieces of it.  Fragment registers are overwritten >= 9 MFMAs after their last MFMA read.
  auto mainloop4 = [&](int kb, int ke) {
   if constexpr (NSTAGE == 1) {
    static_assert(BM == 256 && BN == 256 && NWM == 2 && NWN == 2 && KB == 64, "4-wave loop: 256x256x64, 2x2 waves");
    static_assert(TM == 8 && TN == 8 && A_BYTES == 32768 && STAGE_BYTES == 65536, "4-wave loop layout");
    const int nk = ke - kb;
    const uint32_t lds0 = lds_addr(smem);
    // LDS-DMA sources: wave w stages pieces w + 4·ii (ii < 8) of each operand; piece i = rows 8i..8i+7,
    // lane -> (row 8i + srow, physical chunk spc) reads logical chunk spc ^ (row & 7) = spc ^ srow.
    // Per-lane byte offsets from the tile's row origin (rows past the matrix clamped, as stage()).
    const int lc = spc ^ srow;
    uint32_t voA[8], voB[8];
#pragma unroll
    for (int ii = 0; ii < 8; ++ii) {
      const int r = (wave + 4 * ii) * 8 + srow;
      voA[ii] = (uint32_t)(min(m0 + r, M - 1) - m0) * (uint32_t)(lda * 2) + (uint32_t)(lc * 16);
      voB[ii] = (uint32_t)(min(n0 + r, N - 1) - n0) * (uint32_t)(ldb * 2) + (uint32_t)(lc * 16);
    }
    const uint64_t gA = (uint64_t)(uintptr_t)(A + (size_t)m0 * lda + (size_t)kb * BK);
    const uint64_t gB = (uint64_t)(uintptr_t)(B + (size_t)n0 * ldb + (size_t)kb * BK);
    // raw buffer descriptor of k-tile t's operand columns (num_records 2^32-1: the offsets above are
    // always in range; host-checked to fit 32 bits)
    auto srd = [](uint64_t g, int t) {
      const uint64_t a = g + (uint64_t)t * (BK * 2);
      srd_t s;
      s[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
      s[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
      s[2] = -1;
      s[3] = 0x00020000;
      return s;
    };
    const uint32_t ldsw = lds0 + (uint32_t)wave * 1024;  // + buffer·64K + operand·32K + ii·4K
    // LDS read addresses of a lane's fragments: row wm·128 + 16i + fr (A) / wn·128 + 16j + fr (B) at
    // logical chunk 4h + fq; fragment i / j adds the immediate offset 2048·i
    const uint32_t rA = lds0 + (uint32_t)((wm * 128 + fr) * ROWB), rB = rA + A_BYTES + (uint32_t)((wn - wm) * 128 * ROWB);
    const uint32_t cq0 = (uint32_t)((fq ^ (fr & 7)) << 4), cq1 = (uint32_t)(((4 + fq) ^ (fr & 7)) << 4);
    frag_t<T> fa[2][8], fb[2][8];

    auto stage_tile = [&](int t) {  // prologue form: B then A pieces of tile t into buffer t & 1
      const srd_t sa = srd(gA, t), sb = srd(gB, t);
      const uint32_t d = ldsw + (uint32_t)(t & 1) * STAGE_BYTES;
      static_for<8>([&](auto c) { dma16(voB[c], sb, d + A_BYTES + c * 4096); });
      static_for<8>([&](auto c) { dma16(voA[c], sa, d + c * 4096); });
    };
    // 16 fragment reads of k-half h of the tile in buffer b, issued inline
    auto read_half = [&](int b, auto hc) {
      constexpr int h = decltype(hc)::value;
      const uint32_t o = (uint32_t)b * STAGE_BYTES + (h ? cq1 : cq0);
      static_for<8>([&](auto c) { lds_rd<c * 2048>(fb[h][c], rB + o); });
      static_for<8>([&](auto c) { lds_rd<c * 2048>(fa[h][c], rA + o); });
    };

    // one k-tile: MODE 0 = steady state (restages tile kt+2), 1 = next-to-last (no restage), 2 = last
    // (no next tile); FIRST: the first k-step writes the accumulators (no zero fill)
    auto body = [&](int kt, auto modec, auto firstc) {
      constexpr int MODE = decltype(modec)::value;
      constexpr bool FIRST = decltype(firstc)::value;
      const uint32_t cur = (uint32_t)(kt & 1) * STAGE_BYTES, nxt = (uint32_t)((kt + 1) & 1) * STAGE_BYTES;
      const uint32_t aB1 = rB + cur + cq1, aA1 = rA + cur + cq1;  // F1 of tile kt
      const uint32_t aB0 = rB + nxt + cq0, aA0 = rA + nxt + cq0;  // F0 of tile kt+1
      srd_t sa{}, sb{};
      if constexpr (MODE == 0) {
        sa = srd(gA, kt + 2);
        sb = srd(gB, kt + 2);
      }
      const uint32_t dA = ldsw + cur, dB = dA + A_BYTES;  // tile kt+2 goes where tile kt was
      static_for<128>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        constexpr int h = m / 64, i = (m % 64) / 8, j = m % 8;
        if constexpr (m == 64) wait_lgkm<0>();  // F1 in registers
        if constexpr (FIRST && h == 0) mfma_acc0<T>(acc[i][j], fb[0][j], fa[0][i]);
        else mfma_acc<T>(acc[i][j], fb[h][j], fa[h][i]);
        if constexpr (MODE == 0) {
          if constexpr (m <= 15 && m % 2 == 1) lds_rd<(m / 2) * 2048>(fb[1][m / 2], aB1);
          if constexpr (m == 17) { wait_lgkm<0>(); sbarrier(); }  // every wave's B reads of tile kt retired
          if constexpr (m >= 19 && m <= 49 && m % 2 == 1) {
            constexpr int s = (m - 19) / 2;
            if constexpr (s % 2 == 0) lds_rd<(s / 2) * 2048>(fa[1][s / 2], aA1);
            else dma16(voB[s / 2], sb, dB + (s / 2) * 4096);
          }
          if constexpr (m == 51) { wait_lgkm<0>(); sbarrier(); }  // ... and A reads
          if constexpr (m >= 53 && m <= 67 && m % 2 == 1) dma16(voA[(m - 53) / 2], sa, dA + ((m - 53) / 2) * 4096);
          if constexpr (m == 87) { wait_vmcnt<16>(); sbarrier(); }  // tile kt+1 landed (16 newer pieces)
        } else {
          if constexpr (m <= 31 && m % 2 == 1) {
            constexpr int s = m / 2;
            if constexpr (s < 8) lds_rd<s * 2048>(fb[1][s], aB1);
            else lds_rd<(s - 8) * 2048>(fa[1][s - 8], aA1);
          }
          if constexpr (MODE == 1 && m == 87) { wait_vmcnt<0>(); sbarrier(); }
        }
        if constexpr (MODE != 2 && m >= 89 && m <= 119 && m % 2 == 1) {
          constexpr int s = (m - 89) / 2;
          if constexpr (s < 8) lds_rd<s * 2048>(fb[0][s], aB0);
          else lds_rd<(s - 8) * 2048>(fa[0][s - 8], aA0);
        }
      });
      if constexpr (MODE != 2) wait_lgkm<0>();  // F0 of tile kt+1 in registers
    };

    // prologue: tiles 0 and 1 in flight, tile 0 published, its F0 read
    stage_tile(0);
    if (nk > 1) {
      stage_tile(1);
      wait_vmcnt<16>();
    } else {
      wait_vmcnt<0>();
    }
    sbarrier();
    read_half(0, std::integral_constant<int, 0>{});
    wait_lgkm<0>();
    stamp(1);
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using TF = std::true_type;
    using FF = std::false_type;
    if (nk >= 3) {
      body(0, I0{}, TF{});
      for (int kt = 1; kt < nk - 2; ++kt) body(kt, I0{}, FF{});
      body(nk - 2, I1{}, FF{});
      body(nk - 1, I2{}, FF{});
    } else if (nk == 2) {
      body(0, I1{}, TF{});
      body(1, I2{}, FF{});
    } else {
      body(0, I2{}, TF{});
    }
    mfma_fence();  // last MFMA -> the epilogue's accumulator reads
    pin_acc<TM, TN>(acc);
   }
  };

  // fused epilogue of the (m0, n0) tile from acc (+ LoRA K-extension)
  auto epilogue = [&]() {
    // ---- LoRA K-extension: one extra K=32 step from global (A2[M,32], B2[N,32]) ----
    frag_t<T> af2[TM], bf2[TN];
    const bool ext = A2 != nullptr;
    float bpre[TN][4];  // the tile's bias columns, read from the staged piece before the ring is reused
    const bool bias_pre = bias_lds && ext_buf >= 0;
    if (ext_buf >= 0) {  // staged by the main loop's last k-tile (NSTAGE >= 2 data-parallel tiles)
      wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave's pieces landed
      asm volatile("" ::: "memory");
    }
    if (bias_pre) {
      const char* bb = smem + ext_buf * STAGE_BYTES + EXT_BIAS_OFF;
  #pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WN + j * 16 + fq * 4;
        if (ep.bias_f32) {
          const float4 t4 = *reinterpret_cast<const float4*>(bb + col * 4);
          bpre[j][0] = t4.x; bpre[j][1] = t4.y; bpre[j][2] = t4.z; bpre[j][3] = t4.w;
        } else {
          load4<T>(reinterpret_cast<const T*>(bb) + col, bpre[j]);
        }
      }
    }
    if (ext && ext_buf >= 0) {
      const char* eb = smem + ext_buf * STAGE_BYTES;
  #pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WM + i * 16 + fr;
        af2[i] = *reinterpret_cast<const frag_t<T>*>(eb + r * 64 + ((fq ^ ((r >> 2) & 3)) << 4));
      }
  #pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WN + j * 16 + fr;
        bf2[j] = *reinterpret_cast<const frag_t<T>*>(eb + BM * 64 + r * 64 + ((fq ^ ((r >> 2) & 3)) << 4));
      }
    } else if (ext) {
  #pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = min(m0 + wm * WM + i * 16 + fr, M - 1);
        af2[i] = *reinterpret_cast<const frag_t<T>*>(A2 + (size_t)r * 32 + fq * 8);
      }
  #pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = min(n0 + wn * WN + j * 16 + fr, N - 1);
        bf2[j] = *reinterpret_cast<const frag_t<T>*>(B2 + (size_t)r * 32 + fq * 8);
      }
    }
    if (ext) {
      if (ep.ext_thr == 0) {
  #pragma unroll
        for (int i = 0; i < TM; ++i)
  #pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<T>(bf2[j], af2[i], acc[i][j]);
      }
    }
    const bool ext_masked = ext && ep.ext_thr != 0;

    // ---- epilogue phase 1: accumulators -> LDS tile (one 8-byte write per 16x16 tile) ----
    __syncthreads();  // staging ring is reused for the C tile
    T* Cs = reinterpret_cast<T*>(smem);
    using CT = CTile<BN>;
    const float alpha = ep.alpha_ptr != nullptr ? ep.alpha * ep.alpha_ptr[0] : ep.alpha;
    // acc (+bias, + the dropout-masked K-extension) of fragment column j -> C tile; MASKED is a
    // compile-time split so the common unmasked body stays a short straight-line block (the 4-wave
    // tile unrolls 64 fragments: the masked hash inlined into each cost it 36k cycles of I-cache-bound
    // code per tile, tools/gemm_stamps.py)
    const uint32_t ehm = mift_hmix(ep.ext_seed, 0);
    auto phase1 = [&](auto maskedc) {
      constexpr bool MASKED = decltype(maskedc)::value;
  #pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WN + j * 16 + fq * 4;
        float bv[4] = {0.f, 0.f, 0.f, 0.f};
        if (bias_pre) {
          if (n0 + col < N) {
  #pragma unroll
            for (int e = 0; e < 4; ++e) bv[e] = bpre[j][e];
          }
        } else if (ep.bias != nullptr && n0 + col < N) {
          if (ep.bias_f32) {
            float4 t4 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(ep.bias) + n0 + col);
            bv[0] = t4.x; bv[1] = t4.y; bv[2] = t4.z; bv[3] = t4.w;
          } else {
            load4<T>(reinterpret_cast<const T*>(ep.bias) + n0 + col, bv);
          }
        }
  #pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * WM + i * 16 + fr;
          float z[4];
  #pragma unroll
          for (int e = 0; e < 4; ++e) z[e] = acc[i][j][e] * alpha + bv[e];
          if (MASKED || (NSTAGE != 1 && ext_masked)) {
            float4_ xt = mfma16<T>(bf2[j], af2[i], float4_{0.f, 0.f, 0.f, 0.f});
            bool kp[4];
            // pair index < 2^32 (host-checked): one hoisted high-word mix, no branches.  Not on the
            // 4-wave tile: the extra live value there pushed its 256 pinned accumulators out of the
            // AGPRs (256 -> 65, copies around every MFMA: OPT step 79 -> 514 ms; build.py checks)
            if (NSTAGE != 1 && ep.hoist)
              mift_keep4_hm(ep.ext_seed, ehm, (uint64_t)(m0 + row) * N + n0 + col, ep.ext_thr, kp);
            else
              mift_keep4(ep.ext_seed, (uint64_t)(m0 + row) * N + n0 + col, ep.ext_thr, kp);
  #pragma unroll
            for (int e = 0; e < 4; ++e) z[e] += kp[e] ? xt[e] * ep.ext_inv_keep : 0.f;
          }
          store4<T>(Cs + CT::off4(row, col), z);
        }
      }
    };
    if constexpr (NSTAGE == 1) {
      if (ext_masked) phase1(std::true_type{});
      else phase1(std::false_type{});
    } else {
      phase1(std::false_type{});  // (the runtime ext_masked test inside, as before)
    }
    __syncthreads();
    stamp(3);

    // ---- epilogue phase 2: 8 columns per thread, 16-B vector I/O, whole rows ----
    // The global operands of ALL this thread's chunks (activation aux, residual) are loaded up
    // front (acc is dead here), so their HBM latency is paid once per tile rather than once per
    // chunk behind the previous chunk's store; loads are unconditional from clamped addresses
    // (no per-chunk branch around a load: guide §5 "Projection GEMM" item 4(c)).
    constexpr int VPR = BN / 8;
    constexpr int ITER = BM * VPR / NT;
    static_assert((BM * VPR) % NT == 0, "epilogue chunks must split evenly over the threads");
    // (an up-front operand prefetch for all chunks, MIFT_EPI_PREFETCH, measured +1.5 % on the distilgpt2
    // step and +2..5 % on the 256x256 tile, rounds 2 / 5, and was removed in round 6; interior tiles
    // take the staged form below)
    constexpr bool PF_OK = ITER <= 8;
    // one 8-column chunk: (aux, res) come prefetched when have_aux / have_res
    auto chunk = [&](int it, bool have_aux, short8 auxv, bool have_res, short8 resv, int sbp) {
      const int v = tid + it * NT;
      const int row = v / VPR, c8 = (v % VPR) * 8;
      const int gr = m0 + row, gc = n0 + c8;
      if (gr >= M || gc >= N) return;
      float z[8];
      unpack8<T>(CT::read8(Cs, row, c8), z);
      const size_t off = (size_t)gr * ldc + gc;
      const bool full = gc + 8 <= N;
      if (ep.pre_add != nullptr) {
        float pa[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (full) load8<T>(reinterpret_cast<const T*>(ep.pre_add) + off, pa);
        else for (int e = 0; e < N - gc; ++e) pa[e] = (float)reinterpret_cast<const T*>(ep.pre_add)[off + e];
  #pragma unroll
        for (int e = 0; e < 8; ++e) z[e] += pa[e];
      }
      if (ep.preact != nullptr) {
        if (full) store8<T>(reinterpret_cast<T*>(ep.preact) + off, z);
        else for (int e = 0; e < N - gc; ++e) reinterpret_cast<T*>(ep.preact)[off + e] = (T)z[e];
      }
      if (ep.act == ACT_RELU_BWD && ep.aux == nullptr && ep.sbits != nullptr) {
        const uint32_t sb = sbp >= 0 ? (uint32_t)sbp : ep.sbits[(size_t)gr * (N >> 3) + (gc >> 3)];
  #pragma unroll
        for (int e = 0; e < 8; ++e) z[e] = (sb >> e) & 1u ? z[e] : 0.f;
      } else if (ep.act != ACT_NONE) {
        float ax[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (ep.aux != nullptr) {
          if (full && have_aux) unpack8<T>(auxv, ax);
          else if (full) load8<T>(reinterpret_cast<const T*>(ep.aux) + off, ax);
          else for (int e = 0; e < N - gc; ++e) ax[e] = (float)reinterpret_cast<const T*>(ep.aux)[off + e];
        }
        // one uniform branch per 8 elements (not a switch per element)
        switch (ep.act) {
          case ACT_GELU_TANH:
  #pragma unroll
            for (int e = 0; e < 8; ++e) z[e] = gelu_tanh(z[e]);
            break;
          case ACT_GELU_TANH_BWD:
  #pragma unroll
            for (int e = 0; e < 8; ++e) z[e] *= gelu_tanh_grad(ax[e]);
            break;
          case ACT_RELU:
  #pragma unroll
            for (int e = 0; e < 8; ++e) z[e] = fmaxf(z[e], 0.f);
            break;
          case ACT_RELU_BWD:
  #pragma unroll
            for (int e = 0; e < 8; ++e) z[e] = ax[e] > 0.f ? z[e] : 0.f;
            break;
          default:
  #pragma unroll
            for (int e = 0; e < 8; ++e) z[e] = apply_act(ep.act, z[e], ax[e]);
        }
      }
      if (ep.thr != 0) {
        bool kp[8];
        mift_keep8(ep.seed, (uint64_t)gr * N + gc, ep.thr, kp);
  #pragma unroll
        for (int e = 0; e < 8; ++e) z[e] = kp[e] ? z[e] * ep.inv_keep : 0.f;
      }
      if (ep.residual != nullptr) {
        float rv[8];
        if (full && have_res) unpack8<T>(resv, rv);
        else if (full) load8<T>(reinterpret_cast<const T*>(ep.residual) + off, rv);
        else for (int e = 0; e < N - gc; ++e) rv[e] = (float)reinterpret_cast<const T*>(ep.residual)[off + e];
  #pragma unroll
        for (int e = 0; e < 8; ++e) z[e] += rv[e];
      }
      if (ep.pws != nullptr) {  // the rounded output, in place of z, for the projection phase
        short8 o;
  #pragma unroll
        for (int e = 0; e < 8; ++e) { T t = (T)z[e]; short h; __builtin_memcpy(&h, &t, 2); o[e] = h; }
        CT::write8(Cs, row, c8, o);
      }
      if (ep.sbits != nullptr && ep.act == ACT_RELU) {  // N % 8 == 0 (host): every chunk is full
        uint32_t sb = 0;
  #pragma unroll
        for (int e = 0; e < 8; ++e) sb |= ((float)(T)z[e] > 0.f ? 1u : 0u) << e;
        ep.sbits[(size_t)gr * (N >> 3) + (gc >> 3)] = (uint8_t)sb;
      }
      if (ep.lm.dbg & 1) return;  // diagnostics: MIFT_LM_DBG bit 0 skips the C store
      if (full && ep.ntc) {  // MIFT_EPI_NT=1 (A/B): non-temporal C stores
        short8 o;
  #pragma unroll
        for (int e = 0; e < 8; ++e) { T t = (T)z[e]; short h; __builtin_memcpy(&h, &t, 2); o[e] = h; }
        __builtin_nontemporal_store(o, reinterpret_cast<short8*>(C + off));
      } else if (full) store8<T>(C + off, z);
      else for (int e = 0; e < N - gc; ++e) C[off + e] = (T)z[e];
    };
    // ---- epilogue phase 3 (ep.pws): partial T = drop(out tile) · pw[:, n0 : n0+BN]ᵀ over this
    // tile's columns, MFMA 16x16x32 from the C tile in LDS (read8 = one A fragment), one 16-row
    // stripe per wave; the LoRA-input dropout mask of element (row, col) is the consumer's
    // (index row·N + col, as lora_proj / lora_wgrad / the dgrad K-extension regenerate it).
    auto proj_phase = [&]() {
      // every chunk's output is in the C tile: an LDS-only barrier (phase 2's global stores may stay in
      // flight; measured neutral against __syncthreads() at OPT's shapes, profiles/r5/bench_opt_epilogue_pfg.json)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int fr = lane & 15, g = lane >> 4;
      const uint32_t hm0 = mift_hmix(ep.pseed, 0);
      const bool hz = (uint64_t)M * N < (1ull << 33);
      const int PW = ep.prow <= 16 ? 16 : 32;
      float* slab = ep.pws + (size_t)(n0 / BN) * M * PW;
      // the pw fragments depend on (s, j, lane) only: loaded once for all of the wave's row stripes
      // (they were re-requested per stripe, one dependent L2 round trip each)
      short8 pwv[BN / 32][2];
  #pragma unroll
      for (int s = 0; s < BN / 32; ++s) {
        const int gc = n0 + s * 32 + g * 8;
  #pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int wr = j * 16 + fr;
          pwv[s][j] = (j * 16 < ep.prow && wr < ep.prow && gc < N)
                          ? *reinterpret_cast<const short8*>(reinterpret_cast<const T*>(ep.pw) + (size_t)wr * N + gc)
                          : short8{0, 0, 0, 0, 0, 0, 0, 0};
        }
      }
      for (int rt = wave; rt < BM / 16; rt += NW) {
        const int row = rt * 16 + fr, gr = m0 + row;
        float4_ pacc[2] = {float4_{0.f, 0.f, 0.f, 0.f}, float4_{0.f, 0.f, 0.f, 0.f}};
  #pragma unroll
        for (int s = 0; s < BN / 32; ++s) {
          const int c = s * 32 + g * 8, gc = n0 + c;
          short8 av = CT::read8(Cs, row, c);
          if (gr >= M || gc >= N) av = short8{0, 0, 0, 0, 0, 0, 0, 0};
          if (ep.pthr != 0) {
            uint32_t w[4], km[4];
            __builtin_memcpy(w, &av, 16);
            mift_andmask8(ep.pseed, hm0, hz, (uint64_t)gr * N + gc, ep.pthr, km);
  #pragma unroll
            for (int e = 0; e < 4; ++e) w[e] &= km[e];
            __builtin_memcpy(&av, w, 16);
          }
          frag_t<T> af;
          __builtin_memcpy(&af, &av, 16);
  #pragma unroll
          for (int j = 0; j < 2; ++j) {
            if (j * 16 >= ep.prow) break;  // uniform: rows >= prow of pw are zero
            frag_t<T> bf;
            __builtin_memcpy(&bf, &pwv[s][j], 16);
            pacc[j] = mfma16<T>(bf, af, pacc[j]);  // lane: out[row fr][16j + 4g .. +3]
          }
        }
        if (gr < M) {
  #pragma unroll
          for (int j = 0; j < 2; ++j)
            if (j * 16 < PW) *reinterpret_cast<float4_*>(slab + (size_t)gr * PW + j * 16 + 4 * g) = pacc[j];
        }
      }
    };
    // 4-wave tile (32 chunks per thread, one wave per SIMD): chunks in groups of G, each epilogue
    // feature applied to the whole group before the next (one uniform branch per feature and group,
    // the group's loads in flight together) — the per-chunk form ran each chunk's LDS read -> operand
    // loads -> store as one dependent chain (40k cycles per tile).  Interior tiles only (no bounds
    // tests); same arithmetic and rounding points as chunk().
    auto staged = [&]() {
     {
      // group size: 8 chunks where registers allow; the 8-wave 128-row tiles (two blocks per CU,
      // <= 128 VGPRs) take groups of 3 / 4
      constexpr int G = ITER >= 8 ? (NW == 8 && BM == 128 ? 4 : 8) : (ITER % 3 == 0 ? 3 : ITER);
      static_assert(ITER % G == 0, "chunk groups");
      const T* pre_add = reinterpret_cast<const T*>(ep.pre_add);
      const T* auxp = reinterpret_cast<const T*>(ep.aux);
      const T* resp = reinterpret_cast<const T*>(ep.residual);
      const bool sb_bwd = ep.act == ACT_RELU_BWD && ep.aux == nullptr && ep.sbits != nullptr;
      const uint32_t dhm = mift_hmix(ep.seed, 0);
      for (int g0 = 0; g0 < ITER; g0 += G) {
        int row[G], c8[G];
        size_t off[G];
        float z[G][8];
  #pragma unroll
        for (int k = 0; k < G; ++k) {
          const int v = tid + (g0 + k) * NT;
          row[k] = v / VPR;
          c8[k] = (v % VPR) * 8;
          off[k] = (size_t)(m0 + row[k]) * ldc + n0 + c8[k];
          unpack8<T>(CT::read8(Cs, row[k], c8[k]), z[k]);
        }
        if (pre_add != nullptr) {
          short8 pa[G];
  #pragma unroll
          for (int k = 0; k < G; ++k) pa[k] = *reinterpret_cast<const short8*>(pre_add + off[k]);
  #pragma unroll
          for (int k = 0; k < G; ++k) {
            float t[8];
            unpack8<T>(pa[k], t);
  #pragma unroll
            for (int e = 0; e < 8; ++e) z[k][e] += t[e];
          }
        }
        if (ep.preact != nullptr) {
  #pragma unroll
          for (int k = 0; k < G; ++k) store8<T>(reinterpret_cast<T*>(ep.preact) + off[k], z[k]);
        }
        if (sb_bwd) {
          uint32_t sb[G];
  #pragma unroll
          for (int k = 0; k < G; ++k) sb[k] = ep.sbits[(size_t)(m0 + row[k]) * (N >> 3) + ((n0 + c8[k]) >> 3)];
  #pragma unroll
          for (int k = 0; k < G; ++k)
  #pragma unroll
            for (int e = 0; e < 8; ++e) z[k][e] = (sb[k] >> e) & 1u ? z[k][e] : 0.f;
        } else if (ep.act != ACT_NONE) {
          float ax[G][8];
          if (auxp != nullptr) {
            short8 av[G];
  #pragma unroll
            for (int k = 0; k < G; ++k) av[k] = *reinterpret_cast<const short8*>(auxp + off[k]);
  #pragma unroll
            for (int k = 0; k < G; ++k) unpack8<T>(av[k], ax[k]);
          } else {
  #pragma unroll
            for (int k = 0; k < G; ++k)
  #pragma unroll
              for (int e = 0; e < 8; ++e) ax[k][e] = 0.f;
          }
          switch (ep.act) {
            case ACT_GELU_TANH:
  #pragma unroll
              for (int k = 0; k < G; ++k)
  #pragma unroll
                for (int e = 0; e < 8; ++e) z[k][e] = gelu_tanh(z[k][e]);
              break;
            case ACT_GELU_TANH_BWD:
  #pragma unroll
              for (int k = 0; k < G; ++k)
  #pragma unroll
                for (int e = 0; e < 8; ++e) z[k][e] *= gelu_tanh_grad(ax[k][e]);
              break;
            case ACT_RELU:
  #pragma unroll
              for (int k = 0; k < G; ++k)
  #pragma unroll
                for (int e = 0; e < 8; ++e) z[k][e] = fmaxf(z[k][e], 0.f);
              break;
            case ACT_RELU_BWD:
  #pragma unroll
              for (int k = 0; k < G; ++k)
  #pragma unroll
                for (int e = 0; e < 8; ++e) z[k][e] = ax[k][e] > 0.f ? z[k][e] : 0.f;
              break;
            default:
  #pragma unroll
              for (int k = 0; k < G; ++k)
  #pragma unroll
                for (int e = 0; e < 8; ++e) z[k][e] = apply_act(ep.act, z[k][e], ax[k][e]);
          }
        }
        if (ep.thr != 0) {
  #pragma unroll
          for (int k = 0; k < G; ++k) {
            bool kp[8];
            if (NSTAGE != 1 && ep.hoist) {  // the 4 pairs' hashes from the hoisted high-word mix
              const uint32_t lo = (uint32_t)(((uint64_t)(m0 + row[k]) * N + n0 + c8[k]) >> 1);
  #pragma unroll
              for (int e = 0; e < 8; e += 2) {
                const uint32_t h = mift_hash_lo(ep.seed, dhm, lo + (e >> 1));
                kp[e] = (h & 0xFFFFu) >= ep.thr;
                kp[e + 1] = (h >> 16) >= ep.thr;
              }
            } else {
              mift_keep8(ep.seed, (uint64_t)(m0 + row[k]) * N + n0 + c8[k], ep.thr, kp);
            }
  #pragma unroll
            for (int e = 0; e < 8; ++e) z[k][e] = kp[e] ? z[k][e] * ep.inv_keep : 0.f;
          }
        }
        if (resp != nullptr) {
          short8 rv[G];
  #pragma unroll
          for (int k = 0; k < G; ++k) rv[k] = *reinterpret_cast<const short8*>(resp + off[k]);
  #pragma unroll
          for (int k = 0; k < G; ++k) {
            float t[8];
            unpack8<T>(rv[k], t);
  #pragma unroll
            for (int e = 0; e < 8; ++e) z[k][e] += t[e];
          }
        }
        short8 o[G];
  #pragma unroll
        for (int k = 0; k < G; ++k)
  #pragma unroll
          for (int e = 0; e < 8; ++e) { T t = (T)z[k][e]; short h; __builtin_memcpy(&h, &t, 2); o[k][e] = h; }
        if (ep.pws != nullptr) {
  #pragma unroll
          for (int k = 0; k < G; ++k) CT::write8(Cs, row[k], c8[k], o[k]);
        }
        if (ep.sbits != nullptr && ep.act == ACT_RELU) {
  #pragma unroll
          for (int k = 0; k < G; ++k) {
            uint32_t sb = 0;
  #pragma unroll
            for (int e = 0; e < 8; ++e) sb |= ((float)(T)z[k][e] > 0.f ? 1u : 0u) << e;
            ep.sbits[(size_t)(m0 + row[k]) * (N >> 3) + ((n0 + c8[k]) >> 3)] = (uint8_t)sb;
          }
        }
        if (ep.lm.dbg & 1) continue;
        if (ep.ntc) {
  #pragma unroll
          for (int k = 0; k < G; ++k) __builtin_nontemporal_store(o[k], reinterpret_cast<short8*>(C + off[k]));
        } else {
  #pragma unroll
          for (int k = 0; k < G; ++k) *reinterpret_cast<short8*>(C + off[k]) = o[k];
        }
      }
     }
    };
    // interior tiles: the staged form (every tile; MIFT_EPI_STAGED=0 keeps the per-chunk form, A/B)
    if (ep.staged && m0 + BM <= M && n0 + BN <= N) {
      staged();
      if (ep.pws != nullptr) proj_phase();
      return;
    }
    if constexpr (PF_OK) {
      for (int it = 0; it < ITER; ++it) chunk(it, false, short8{}, false, short8{}, -1);
    } else {
      // 256x256 (16 chunks per thread, one block per CU: no second block hides a chunk's operand round
      // trip, ~1 us from HBM, paid 16 times per tile in the rolled loop — OPT's residual-dropout
      // epilogues cost +51..62 us per GEMM at micro-batch 48): groups of 4 chunks request their aux /
      // residual / sign-bit operands together, one round trip per group.  MIFT_EPI_PFG=0: per chunk (A/B)
      constexpr int G = 4;
      static_assert(ITER % G == 0, "chunk groups");
      const bool g_aux = ep.pfg && ep.aux != nullptr && ep.act != ACT_NONE && N >= 8;
      const bool g_res = ep.pfg && ep.residual != nullptr && N >= 8;
      const bool g_sb = ep.pfg && ep.sbits != nullptr && ep.act == ACT_RELU_BWD && ep.aux == nullptr;
      for (int g0 = 0; g0 < ITER; g0 += G) {
        short8 av[G], rv[G];
        int bv[G];
  #pragma unroll
        for (int k = 0; k < G; ++k) {
          const int v = tid + (g0 + k) * NT;
          const int gr = min(m0 + v / VPR, M - 1), gc = min(n0 + (v % VPR) * 8, N - 8);
          const size_t o = (size_t)gr * ldc + gc;
          av[k] = g_aux ? *reinterpret_cast<const short8*>(reinterpret_cast<const T*>(ep.aux) + o) : short8{};
          rv[k] = g_res ? *reinterpret_cast<const short8*>(reinterpret_cast<const T*>(ep.residual) + o) : short8{};
          bv[k] = g_sb ? (int)ep.sbits[(size_t)gr * (N >> 3) + (gc >> 3)] : -1;
        }
  #pragma unroll
        for (int k = 0; k < G; ++k) chunk(g0 + k, g_aux, av[k], g_res, rv[k], bv[k]);
      }
    }
    if (ep.pws != nullptr) proj_phase();
  };

  // ---- EPI 1: LM-head forward epilogue (see LmArgs).  The 16-bit E tile is staged in LDS
  // (the ring is reused) and written out as whole-row 16-B chunks: storing it straight from the
  // accumulator layout (32-B row pieces per lane group) cost ~140 us of the 820 us distilgpt2 head
  // (tools/diag_lmhead.py), the coalesced copy-out hides under the next tiles' main loops like the
  // plain GEMM's.  Two [NW][WM] row-partial arrays (max, sum) behind the C tile exchange the NWN
  // waves' partials of a row.
  auto lm_fwd_epilogue = [&]() {
    const LmArgs& lm = ep.lm;
    using CT = CTile<BN>;
    constexpr int CLD = CT::CLD;
    __syncthreads();  // every wave is done reading the staging ring
    T* Cs = reinterpret_cast<T*>(smem);
    float* redm = reinterpret_cast<float*>(smem + BM * CLD * sizeof(T));
    float* reds = redm + NW * WM;
    const int V = lm.V;
    constexpr float L2E = 1.4426950408889634f;
    // labels first: their load latency hides under the max pass (they are consumed after a barrier)
    // the block's row targets go to LDS (read after the max-pass barrier): requested first so their
    // latency hides under the max pass, and no registers held across it (the kernel sits at 256)
    int* labs = reinterpret_cast<int*>(reds + NW * WM);
    if (tid < BM) {
      const int64_t l = lm_label(lm.labels, min(m0 + tid, M - 1), lm.shift, lm.ignore);
      labs[tid] = (l >= 0 && l < V) ? (int)l : -1;
    }
    // Two instantiations of the exp epilogue: every column tile but the last is FULL (no padding
    // columns), and there it needs no per-element bounds selects; the label's logit is picked by
    // selects across the row's column tiles and stored once per row fragment (one divergent store
    // per i instead of one exec-mask branch per (i, j)).
    const bool dbg_raw = (lm.dbg & 2) != 0;
    auto exp_pass = [&](auto fullc) {
      constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        float m = -INFINITY;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = n0 + wn * WN + j * 16 + fq * 4;
#pragma unroll
          for (int e = 0; e < 4; ++e) m = (FULL || col + e < V) ? fmaxf(m, acc[i][j][e]) : m;
        }
        m = xor16_max(m);
        m = xor32_max(m);
        if (fq == 0) redm[wave * WM + i * 16 + fr] = m;
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        float m = -INFINITY;
#pragma unroll
        for (int w = 0; w < NWN; ++w) m = fmaxf(m, redm[(wm * NWN + w) * WM + i * 16 + fr]);
        if (m == -INFINITY) m = 0.f;  // tile entirely beyond V (cannot happen for V_pad - V < BN)
        const int lrow = wm * WM + i * 16 + fr;
        const int row = m0 + lrow;
        const int lab = row < M ? labs[lrow] : -1;
        const float mb = m * L2E;
        float s = 0.f, zl = 0.f;
        bool hit = false;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int lcol = wn * WN + j * 16 + fq * 4;
          const int col = n0 + lcol;
          float ev[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            ev[e] = dbg_raw ? acc[i][j][e]
                    : (FULL || col + e < V) ? __builtin_amdgcn_exp2f(__builtin_fmaf(acc[i][j][e], L2E, -mb)) : 0.f;
            s += ev[e];
          }
          const int d = lab - col;  // static selects: a runtime vector index would go to scratch
          const float4_ a4 = acc[i][j];
          const float v = d == 0 ? a4[0] : d == 1 ? a4[1] : d == 2 ? a4[2] : a4[3];
          const bool h = d >= 0 && d < 4;
          zl = h ? v : zl;
          hit = hit || h;
          store4<T>(Cs + CT::off4(lrow, lcol), ev);
        }
        if (hit) lm.zlab[row] = zl;
        s = xor16_add(s);
        s = xor32_add(s);
        if (fq == 0) reds[wave * WM + i * 16 + fr] = s;
      }
    };
    if (n0 + BN <= V && !(lm.dbg & 4)) exp_pass(std::true_type{});  // block-uniform; dbg bit 2: A/B
    else exp_pass(std::false_type{});
    __syncthreads();
    if (tid < BM) {  // one thread per block row: combine the NWN wave partials
      const int wr = tid / WM, rr = tid % WM;
      const int row = m0 + tid;
      float m = -INFINITY, s = 0.f;
#pragma unroll
      for (int w = 0; w < NWN; ++w) {
        m = fmaxf(m, redm[(wr * NWN + w) * WM + rr]);
        s += reds[(wr * NWN + w) * WM + rr];
      }
      if (m == -INFINITY) m = 0.f;
      if (row < M) lm.stats[(size_t)row * lm.ntn + n0 / BN] = make_float2(m, s);
    }
    if (lm.dbg & 1) return;
    constexpr int VPR = BN / 8;
    static_assert((BM * VPR) % NT == 0, "E copy-out chunks must split evenly over the threads");
#pragma unroll 4
    for (int it = 0; it < BM * VPR / NT; ++it) {
      const int v = tid + it * NT;
      const int r = v / VPR, c8 = (v % VPR) * 8;
      const int gr = m0 + r, gc = n0 + c8;
      if (gr < M && gc < N) {
        const short8 ev = CT::read8(Cs, r, c8);
        *reinterpret_cast<short8*>(C + (size_t)gr * ldc + gc) = ev;
      }
    }
  };

  const int nk_all = K / KB;
  if constexpr (EPI == 1) {
    static_assert(NSTAGE == 0, "LM-head forward runs on the phased 256x256 tile");
    // one block per tile: a persistent loop over tiles (E stores draining under the next tile's main
    // loop) measured 2-3 % faster in isolation but pushed the kernel past 256 VGPRs into scratch
    // spills; with the row targets in LDS the one-tile kernel needs 220 and no spills
    const int nblk = ntm * ntn;
    {
      const int t0 = blockIdx.x;
      int bid = t0;
      {
        const int q = nblk / 8, r = nblk % 8;
        const int xcd = bid % 8, loc = bid / 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
      }
      {
        int tm, tn;
        raster(bid, ntm, ntn, ep.group_m, tm, tn);
        m0 = tm * BM;
        n0 = tn * BN;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = float4_{0.f, 0.f, 0.f, 0.f};
      mainloop8(0, nk_all, [](int) {});
      lm_fwd_epilogue();
    }
    return;
  } else if constexpr (EPI == 2) {
    // ---- LM-head dgrad on the phased 256x256 tile.  A = E [M, V_pad], B = Wᵀ [N, V_pad].
    // Each group of GK k-tiles is one forward column tile j whose E is relative to its own max
    // m_j.  Flash-style, acc is kept relative to a per-row reference ref: at every group start
    // acc *= exp(ref - ref'), ref' = max(m_j, ref - 60) (the clamp bounds acc's growth by e^60;
    // a tile more than 60 below the running reference contributes < e^-60 of the row, so adding
    // it at the clamped reference errs by < e^-60 relative), and the chunk's result is
    // acc·exp(ref - lse).  Block -> (tile, split-K chunk of gpc groups); the reduction kernel
    // sums the chunks, subtracts W[label] and applies the upstream gradient.
    static_assert(NSTAGE == 0, "LM-head dgrad runs on the phased 256x256 tile");
    const LmArgs& lm = ep.lm;
    const int S = (lm.ntn + lm.gpc - 1) / lm.gpc;
    const int tl = blockIdx.x / S, cidx = blockIdx.x % S;
    m0 = (tl / ntn) * BM;
    n0 = (tl % ntn) * BN;
    const int g0 = cidx * lm.gpc, g1 = min(lm.ntn, g0 + lm.gpc);
    constexpr int GK = 256 / BK;
    constexpr int cstride = LM_GW | 1;  // odd stride: the 16 rows of a fragment hit 16 banks
    float* ms = reinterpret_cast<float*>(smem + 2 * STAGE_BYTES);  // [BM][cstride] tile maxima, behind the ring
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = float4_{0.f, 0.f, 0.f, 0.f};
    float ref[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) ref[i] = -INFINITY;
    for (int w0 = g0; w0 < g1; w0 += LM_GW) {
      const int w1 = min(g1, w0 + LM_GW), nw = w1 - w0;
      __syncthreads();  // the previous window's readers are done
      // each thread requests PB window entries before their LDS writes (a per-row loop waited for
      // each row's load in turn: 16 round trips per window; all 13 at once spill the accumulators),
      // element i = (row i / LM_GW, group i % LM_GW); the odd stride keeps the fragment-row reads
      // conflict-free
      constexpr int PER = (BM * LM_GW + NT - 1) / NT, PB = 5;
#pragma unroll 1
      for (int u0 = 0; u0 < PER; u0 += PB) {
        float wv[PB];
#pragma unroll
        for (int u = 0; u < PB; ++u) {
          const int i = tid + (u0 + u) * NT, r = i / LM_GW, g = i % LM_GW;
          wv[u] = (i < BM * LM_GW && g < nw) ? lm.stats[(size_t)min(m0 + r, M - 1) * lm.ntn + w0 + g].x : 0.f;
        }
#pragma unroll
        for (int u = 0; u < PB; ++u) {
          const int i = tid + (u0 + u) * NT;
          if (i < BM * LM_GW) ms[(i / LM_GW) * cstride + i % LM_GW] = wv[u];
        }
      }
      __syncthreads();
      mainloop8(w0 * GK, min(nk_all, w1 * GK), [&](int kt) {
        const int gk = w0 * GK + kt;
        if (gk % GK != 0) return;
        if (lm.dbg & 8) return;  // diagnostics (MIFT_LM_DBG bit 3): no rescale — wrong numbers, timing only
        const int g = gk / GK - w0;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const float m = ms[(wm * WM + i * 16 + fr) * cstride + g];
          const float rn = fmaxf(m, ref[i] - 60.f);
          const float f = __expf(ref[i] - rn);  // 0 on the first group (acc is 0 there)
          ref[i] = rn;
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] *= f;
        }
      });
    }
    float* dst = lm.partial + (size_t)cidx * M * N;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = m0 + wm * WM + i * 16 + fr;
      if (row >= M) continue;
      const float fac = __expf(ref[i] - lm.lse[row]);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * WN + j * 16 + fq * 4;
        if (col < N) *reinterpret_cast<float4_*>(dst + (size_t)row * N + col) = acc[i][j] * fac;
      }
    }
    return;
  } else if constexpr (!SKM) {
    // ---- data-parallel tile, XCD-aware bijective block remap (T1) ----
    const int nblk = gridDim.x;  // tiles [0, gridDim.x) (all of them unless stream-K takes the tail)
    int bid = blockIdx.x;
    {
      const int q = nblk / 8, r = nblk % 8;
      const int xcd = bid % 8, loc = bid / 8;
      bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
    }
    {
      int tm, tn;
      raster(bid, ntm, ntn, ep.group_m, tm, tn);
      m0 = tm * BM;
      n0 = tn * BN;
    }
    if constexpr (NSTAGE == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = float4_{0.f, 0.f, 0.f, 0.f};
      mainloop8(0, nk_all, [](int) {});
    } else if constexpr (NSTAGE == 1) {
      mainloop4(0, nk_all);
    } else {
      mainloop(0, nk_all, (A2 != nullptr || bias_lds) && ep.ext_lds);
    }
    stamp(2);
    epilogue();
    stamp(4);
    stamp(7);
    return;
  } else {
    // ---- split-K tail (separate instantiation: its bookkeeping must not cost the DP kernel
    // registers).  Block b handles k-chunk (b % S) of tile tile0 + b / S; the block holding a
    // tile's LAST chunk finishes it after the lower-index chunk blocks (dispatched before it,
    // running concurrently: no cycles, next to no waiting) released their fp32 partials.
    const int S = sk.gx;
    const int tl = blockIdx.x / S, cidx = blockIdx.x % S;
    const int tile = sk.tile0 + tl;
    {
      int tm, tn;
      raster(tile, ntm, ntn, ep.group_m, tm, tn);  // same raster as the data-parallel launch
      m0 = tm * BM;
      n0 = tn * BN;
    }
    mainloop((int)((long)cidx * nk_all / S), (int)((long)(cidx + 1) * nk_all / S));
    constexpr int SLOT = TM * TN * NT;  // float4 per partial tile
    if (cidx < S - 1) {
      float4_* dst = reinterpret_cast<float4_*>(sk.ws) + (size_t)blockIdx.x * SLOT;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) dst[(i * TN + j) * NT + tid] = acc[i][j];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(sk.flags + tl, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (tid == 0) {
      while (__hip_atomic_load(sk.flags + tl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < S - 1)
        __builtin_amdgcn_s_sleep(2);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(sk.flags + tl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    for (int c = 1; c < S; ++c) {
      const float4_* src = reinterpret_cast<const float4_*>(sk.ws) + (size_t)(blockIdx.x - c) * SLOT;
      // in groups of 4 float4: keeps the scheduler from hoisting all TM*TN loads at once
      // (a second accumulator-sized register set -> spills on the 256x256 tile)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] += src[(i * TN + j) * NT + tid];
          if (((i * TN + j) & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
    }
    epilogue();
  }  // SKM
}

// ---- persistent fused LM-head forward (EPI 1's arithmetic; default, MIFT_LM_PERSIST=0: the one-tile kernel) ----
// The distilgpt2 head is 6,304 tiles of 256x256 at K = 768: 12 k-tiles of main loop per tile, after which
// the one-tile kernel runs its epilogue (row maxima, exp, E store) and its block exits; the next block's
// prologue then refills the ring from nothing.  Here one 512-thread block per CU
// walks the tiles xb, xb + G, ... (G = grid, xb = XCD-remapped block id: the 32 blocks sharing an XCD
// take 32 consecutive tile slots, as the one-tile launch placed them) as ONE continuous k-tile stream:
// the phased 4-phase schedule of mainloop8 issues k-tile g+1's A halves and g+2's B halves whatever tile
// they belong to, so when a tile's last k-tile retires, the next tile's first k-tile is already in LDS
// and its second in flight while the epilogue runs.  The epilogue keeps E out of LDS (the ring is busy
// with the next tile): each lane packs its 4-column fragments to 16 bits and one v_permlane16_swap per
// dword pairs lanes l / l^16 so every lane holds 8 consecutive columns -> one 16-B store per lane and
// row-fragment pair (16 rows x 64 contiguous bytes per instruction, whole 128-B lines per wave).  Only
// the cross-wave row maxima / sums and the row targets go through a 9 KiB LDS side area behind the
// ring; its barriers are raw s_barriers (a __syncthreads would drain the in-flight LDS-DMA and E stores).
template <typename T>
__global__ __launch_bounds__(512) void lmhead_fwd_persist_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                                  T* __restrict__ E, int M, int N, int K, int lda,
                                                                  int ldb, int lde, LmArgs lm, int ntiles, int group_m) {
  constexpr int BM = 256, BN = 256, NWN = 4, NW = 8, WM = 128, WN = 64, TM = 8, TN = 4;
  constexpr int A_BYTES = BM * ROWB, STAGE_BYTES = (BM + BN) * ROWB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* redm = reinterpret_cast<float*>(smem + 2 * STAGE_BYTES);  // [NW][WM] wave row maxima
  float* reds = redm + NW * WM;                                     // [NW][WM] wave row sums
  // raw label ids of rows m0 .. m0 + 383 (3 KiB: the unshifted ids need row + 1), brought in by LDS-DMA
  // at the tile's first k-tile: a plain global load used in the epilogue would make hipcc wait
  // vmcnt(0) there, draining the next tile's in-flight ring DMA (guide §5 "Pipelining across barriers")
  int64_t* ids = reinterpret_cast<int64_t*>(reds + NW * WM);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / NWN, wn = wave % NWN;
  const int fr = lane & 15, fq = lane >> 4;
  const int srow = lane >> 3, spc = lane & 7;
  const int ntm = (M + BM - 1) / BM, ntn = (N + BN - 1) / BN;
  const int nk = K / BK;  // >= 2 (host-checked)
  const int G = gridDim.x;
  int xb;
  {
    const int q = G / 8, r = G % 8, xcd = blockIdx.x % 8, loc = blockIdx.x / 8;
    xb = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  }
  const int ntl = (ntiles - xb + G - 1) / G;  // G <= ntiles: every block owns >= 1 tile
  const int total = ntl * nk;
  auto coords = [&](int j, int& m0, int& n0) {
    int tm, tn;
    raster(j * G + xb, ntm, ntn, group_m, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
  };
  auto stage_half = [&](int buf, int m0, int n0, int kt, int o, int h) {
    char* base = smem + buf * STAGE_BYTES + o * A_BYTES;
    const T* Gp = o ? B : A;
    const int ld = o ? ldb : lda;
    const int rmax = (o ? N : M) - 1;
    const int r00 = o ? n0 : m0;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      const int i = 16 * h + wave + 8 * ii;
      const int r = i * 8 + srow;
      const int gr = min(r00 + r, rmax);
      __builtin_amdgcn_global_load_lds((const void*)(Gp + (size_t)gr * ld + kt * BK + (spc ^ (r & 7)) * 8),
                                       (void*)(base + i * 1024), 16, 0, 0);
    }
  };
  float4_ acc[TM][TN];
  frag_t<T> af[4][2], bq[4][2];
  auto rd = [&](const char* p) { return *reinterpret_cast<const frag_t<T>*>(p); };
  auto cluster = [&](int qi, int qj) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qi * 4 + i][qj * 2 + j] = mfma16<T>(bq[qj * 2 + j][kk], af[i][kk], acc[qi * 4 + i][qj * 2 + j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto raw_barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  constexpr float L2E = 1.4426950408889634f;
  auto pack2 = [](float a, float b) {
    T ta = (T)a, tb = (T)b;
    unsigned short ua, ub;
    __builtin_memcpy(&ua, &ta, 2);
    __builtin_memcpy(&ub, &tb, 2);
    return (unsigned)ua | ((unsigned)ub << 16);
  };
  // tile (m0, n0) epilogue from acc: E = exp(z - m_row,tile) 16-bit, (m, s) stats, the label's fp32 logit
  auto epilogue = [&](int m0, int n0, auto fullc) {
    constexpr bool FULL = decltype(fullc)::value;
    const int V = lm.V;
    // lm_label on the LDS copy of the ids (rows m0 + r, r < BM; the copy starts at row m0)
    auto label_of = [&](int lrow) {
      const int row = m0 + lrow;
      if (row >= M) return -1;
      const int64_t l = lm.shift <= 0 ? ids[lrow] : (row % lm.shift == lm.shift - 1) ? (int64_t)-1 : ids[lrow + 1];
      return (l == lm.ignore || l < 0 || l >= V) ? -1 : (int)l;
    };
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float m = -INFINITY;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * WN + j * 16 + fq * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) m = (FULL || col + e < V) ? fmaxf(m, acc[i][j][e]) : m;
      }
      m = xor16_max(m);
      m = xor32_max(m);
      if (fq == 0) redm[wave * WM + i * 16 + fr] = m;
    }
    raw_barrier();
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float m = -INFINITY;
#pragma unroll
      for (int w = 0; w < NWN; ++w) m = fmaxf(m, redm[(wm * NWN + w) * WM + i * 16 + fr]);
      if (m == -INFINITY) m = 0.f;
      const int lrow = wm * WM + i * 16 + fr;
      const int row = m0 + lrow;
      const int lab = label_of(lrow);
      const float mb = m * L2E;
      float s = 0.f, zl = 0.f;
      bool hit = false;
      unsigned pk[TN][2];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * WN + j * 16 + fq * 4;
        float ev[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ev[e] = (FULL || col + e < V) ? __builtin_amdgcn_exp2f(__builtin_fmaf(acc[i][j][e], L2E, -mb)) : 0.f;
          s += ev[e];
        }
        const int d = lab - col;
        const float4_ a4 = acc[i][j];
        const float v = d == 0 ? a4[0] : d == 1 ? a4[1] : d == 2 ? a4[2] : a4[3];
        const bool h = d >= 0 && d < 4;
        zl = h ? v : zl;
        hit = hit || h;
        pk[j][0] = pack2(ev[0], ev[1]);
        pk[j][1] = pack2(ev[2], ev[3]);
      }
      if (hit && row < M) lm.zlab[row] = zl;
      s = xor16_add(s);
      s = xor32_add(s);
      if (fq == 0) reds[wave * WM + i * 16 + fr] = s;
      // lanes l (row quarter fq even) and l ^ 16 trade fragments: fq even ends with columns
      // 32p + 8(fq>>1) .. +7, fq odd with 32p + 16 + 8(fq>>1) .. +7 of the wave's 64
#pragma unroll
      for (int p = 0; p < TN / 2; ++p) {
        const auto r0 = __builtin_amdgcn_permlane16_swap(pk[2 * p][0], pk[2 * p + 1][0], false, false);
        const auto r1 = __builtin_amdgcn_permlane16_swap(pk[2 * p][1], pk[2 * p + 1][1], false, false);
        const int c0 = n0 + wn * WN + (2 * p + (fq & 1)) * 16 + (fq >> 1) * 8;
        if (!(lm.dbg & 1) && row < M && (FULL || c0 < N)) {
          const v4u32 val = {(unsigned)r0[0], (unsigned)r1[0], (unsigned)r0[1], (unsigned)r1[1]};
          *reinterpret_cast<v4u32*>(E + (size_t)row * lde + c0) = val;
        }
      }
    }
    raw_barrier();
    if (tid < BM) {  // one thread per block row: the NWN waves' partials of the row
      const int wr = tid / WM, rr = tid % WM;
      float m = -INFINITY, s = 0.f;
#pragma unroll
      for (int w = 0; w < NWN; ++w) {
        m = fmaxf(m, redm[(wr * NWN + w) * WM + rr]);
        s += reds[(wr * NWN + w) * WM + rr];
      }
      if (m == -INFINITY) m = 0.f;
      if (m0 + tid < M) lm.stats[(size_t)(m0 + tid) * lm.ntn + n0 / BN] = make_float2(m, s);
    }
  };

  // waves 0-2: one 1-KiB LDS-DMA each of ids[m0 + 128w .. +127] (rows clamped in range)
  auto stage_ids = [&](int m0) {
    if (wave < 3) {
      const int r = min(m0 + wave * 128 + lane * 2, M - 2);  // M even (host-checked): r even, 16-B aligned
      __builtin_amdgcn_global_load_lds((const void*)(lm.labels + r), (void*)(ids + wave * 128), 16, 0, 0);
    }
  };
  int m0, n0, nm0 = 0, nn0 = 0;
  coords(0, m0, n0);
  if (ntl > 1) coords(1, nm0, nn0);
  stage_ids(m0);
  stage_half(0, m0, n0, 0, 0, 0);
  stage_half(0, m0, n0, 0, 0, 1);
  stage_half(0, m0, n0, 0, 1, 0);
  stage_half(0, m0, n0, 0, 1, 1);
  if (total > 1) {
    stage_half(1, m0, n0, 1, 1, 0);
    stage_half(1, m0, n0, 1, 1, 1);
    wait_vmcnt<4>();
  } else {
    wait_vmcnt<0>();
  }
  __builtin_amdgcn_s_barrier();
  if (wm == 1) __builtin_amdgcn_s_barrier();  // stagger the wave rows by one barrier (mainloop8)
  asm volatile("" ::: "memory");
  const int arow = wm * WM + fr, brow = wn * WN + fr;
  const int sw0 = (fq ^ (fr & 7)) << 4, sw1 = ((4 + fq) ^ (fr & 7)) << 4;
  // early: the previous epilogue already issued this tile's k-tile 1 A halves (then FULL-tile epilogues
  // leave 16 E stores per lane younger than them, which the first ph3 wait need not drain)
  int early = 0;  // 0 none, 1 issued (wait conservatively), 2 issued behind a FULL epilogue's 16 stores
  for (int j = 0; j < ntl; ++j) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < TN; ++q) acc[i][q] = float4_{0.f, 0.f, 0.f, 0.f};
    if (j > 0) stage_ids(m0);  // older than every ring DMA waited for below: landed by the first ph3
    for (int kt = 0; kt < nk; ++kt) {
      const int g = j * nk + kt;
      const char* As = smem + (g & 1) * STAGE_BYTES;
      const char* Bs = As + A_BYTES;
      // k-tiles g+1 / g+2: this tile's or (wrapping past its last k-tile) the next tile's
      const bool w1 = kt + 1 >= nk, w2 = kt + 2 >= nk;
      const int k1 = w1 ? kt + 1 - nk : kt + 1, k2 = w2 ? kt + 2 - nk : kt + 2;
      const int m1 = w1 ? nm0 : m0, n1 = w1 ? nn0 : n0, m2 = w2 ? nm0 : m0, n2 = w2 ? nn0 : n0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i][0] = rd(As + (arow + i * 16) * ROWB + sw0);
        af[i][1] = rd(As + (arow + i * 16) * ROWB + sw1);
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        bq[q][0] = rd(Bs + (brow + q * 16) * ROWB + sw0);
        bq[q][1] = rd(Bs + (brow + q * 16) * ROWB + sw1);
      }
      const bool pre = kt == 0 && early != 0;  // block-uniform
      if (g + 1 < total && !pre) stage_half((g + 1) & 1, m1, n1, k1, 0, 0);
      cluster(0, 0);
#pragma unroll
      for (int q = 2; q < 4; ++q) {
        bq[q][0] = rd(Bs + (brow + q * 16) * ROWB + sw0);
        bq[q][1] = rd(Bs + (brow + q * 16) * ROWB + sw1);
      }
      if (g + 1 < total && !pre) stage_half((g + 1) & 1, m1, n1, k1, 0, 1);
      cluster(0, 1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i][0] = rd(As + (arow + (i + 4) * 16) * ROWB + sw0);
        af[i][1] = rd(As + (arow + (i + 4) * 16) * ROWB + sw1);
      }
      cluster(1, 1);
      if (g + 2 < total) {
        stage_half(g & 1, m2, n2, k2, 1, 0);
        stage_half(g & 1, m2, n2, k2, 1, 1);
        // retire k-tile g+1 (A, B): all but the 4 B(g+2) pieces — and, right after a FULL epilogue that
        // issued k-tile g+1's A early, all but those 4 and the 16 younger E stores per lane
        if (kt == 0 && early == 2) wait_vmcnt<20>();
        else wait_vmcnt<4>();
      } else {
        wait_vmcnt<0>();
      }
      cluster(1, 0);
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();  // re-align the wave rows for the epilogue's barriers
    asm volatile("" ::: "memory");
    // k-tile g+2 = the next tile's k-tile 1: its A halves go to the buffer whose A region every wave
    // finished reading in the last k-tile's ph2 (before the barrier above) — issued now, ahead of the
    // epilogue's stores, so the next tile's first ph3 wait does not also wait for those stores
    {
      const int g = j * nk + nk - 1;
      early = 0;
      if (g + 2 < total) {
        const int k2 = 1 - (nk == 1);
        stage_half(g & 1, nm0, nn0, k2, 0, 0);
        stage_half(g & 1, nm0, nn0, k2, 0, 1);
        early = 1;
      }
    }
    const bool full = n0 + BN <= lm.V && !(lm.dbg & 4);  // block-uniform
    if (full) epilogue(m0, n0, std::true_type{});
    else epilogue(m0, n0, std::false_type{});
    if (early && full && !(lm.dbg & 1)) early = 2;
    if (wm == 1 && j + 1 < ntl) __builtin_amdgcn_s_barrier();  // re-stagger for the next tile
    asm volatile("" ::: "memory");
    m0 = nm0;
    n0 = nn0;
    if (j + 2 < ntl) coords(j + 2, nm0, nn0);
  }
}

int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
  }();
  return n;
}

// persistent, self-re-arming stream-K tile counters (zeroed once; finishers reset theirs)
int* sk_flags(int n) {
  static at::Tensor flags;
  if (!flags.defined() || flags.numel() < n)
    flags = at::zeros({std::max<int64_t>(n, 1 << 16)}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA));
  return flags.data_ptr<int>();
}

int sk_mode_env() {
  static int v = [] { const char* e = getenv("MIFT_GEMM_SK"); return e ? atoi(e) : -1; }();
  return v;  // -1 auto, 0 off, 1 force
}

// tile raster group (EpiArgs::group_m): MIFT_GEMM_GROUP (read per call, A/B-able) or the default
int gemm_group_m(int N) {
  if (const char* e = getenv("MIFT_GEMM_GROUP")) return atoi(e);
  return N >= 8192 ? 4 : 0;
}

// out[m, 0:32] = alpha · Σ_t slab[t][m][0:PW] (columns >= PW zero): the per-column-tile partials of
// the epilogue projection, summed in tile order.  4 outputs per thread (every thread of a 16-wide slab
// loads: the 8-per-thread form idled half of them), 8 tiles' loads requested before their adds (the
// rolled loop paid one dependent round trip per tile: 27.5 us for OPT fc1's 63 MB of slabs at mb 48)
template <typename T>
__global__ __launch_bounds__(256) void proj_reduce_kernel(const float* __restrict__ slab, int ntn, int M, int PW,
                                                          float alpha, T* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (row, 4-column group)
  if (i >= (int64_t)M * 8) return;
  const int m = (int)(i >> 3), c4 = (int)(i & 7) * 4;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  if (c4 < PW) {
    const float* p = slab + (size_t)m * PW + c4;
    const size_t ts = (size_t)M * PW;
    int t = 0;
    for (; t + 8 <= ntn; t += 8) {
      float4 a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = *reinterpret_cast<const float4*>(p + (size_t)(t + u) * ts);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[0] += a[u].x; v[1] += a[u].y; v[2] += a[u].z; v[3] += a[u].w;
      }
    }
    for (; t < ntn; ++t) {
      const float4 a = *reinterpret_cast<const float4*>(p + (size_t)t * ts);
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
    }
  }
  float o[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = v[e] * alpha;
  store4<T>(out + (size_t)m * 32 + c4, o);
}

template <typename T, int BM, int BN, int NWM, int NWN, int NSTAGE, int KB = 64>
void launch_gemm(const at::Tensor& a, const at::Tensor& b, at::Tensor& c, const T* a2, const T* b2, int M, int N,
                 int K, const EpiArgs& ep, hipStream_t st) {
  constexpr int STAGE_BYTES = (BM + BN) * KB * 2;
  constexpr int EPI_BYTES = BM * CTile<BN>::CLD * 2;
  constexpr int RING = (NSTAGE <= 1 ? 2 : NSTAGE) * STAGE_BYTES;
  constexpr int SMEM = RING > EPI_BYTES ? RING : EPI_BYTES;
  constexpr int NT = NWM * NWN * 64;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  const int nblk = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  // the 256x256 tile has no register headroom for the split-K fixup (it would spill): DP only
  constexpr bool HAS_SK = BM * BN <= 256 * 128;
  auto kern = gemm_nt_kernel<T, BM, BN, NWM, NWN, NSTAGE, false, 0, KB>;
  auto kern_sk = gemm_nt_kernel<T, BM, BN, NWM, NWN, NSTAGE, HAS_SK, 0, KB>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    (void)hipFuncSetAttribute((const void*)kern_sk, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr_set = true;
  }
  // hybrid data-parallel + split-K tail: full waves of tiles run data-parallel; a ragged last
  // wave of rem tiles (< ~85 % of the resident slots) is split S ways along K so it fills the
  // chip: time ~ ceil(rem*S/G)/S tile-times instead of 1 (S chosen on that model + fixup cost)
  constexpr int BPC = (160 * 1024 / SMEM) < (2048 / NT) ? (160 * 1024 / SMEM) : (2048 / NT);
  const int G = num_cus() * (BPC > 0 ? BPC : 1);
  const int rem = nblk % G;
  int sk_tiles = 0, S = 1;
  const int mode = sk_mode_env();
  if (HAS_SK && mode != 0 && rem != 0 && (mode == 1 || rem * 100 < G * 85)) {
    double best = 1.0;
    // chunks of >= 16 k-tiles: below that the fp32 partial round trip costs more than the
    // balanced wave saves (measured: K=768 GEMMs lost 2-4x with 3-k-tile chunks)
    for (int s = 2; s <= 8 && K / s >= 1024; ++s) {
      const double cost = (double)((rem * s + G - 1) / G) / s + 0.03 * (s - 1);
      if (cost < best - 1e-9) { best = cost; S = s; }
    }
    if (S > 1) sk_tiles = rem;
  }
  const int dp_tiles = nblk - sk_tiles;
  SkArgs sk{};
  EpiArgs epx = ep;  // + the projection slab, sized by this tile's BN
  at::Tensor slab;
  const int ntn = (N + BN - 1) / BN, PW = ep.prow <= 16 ? 16 : 32;
  if (ep.pw != nullptr) {
    slab = at::empty({(int64_t)ntn * M * PW}, a.options().dtype(at::kFloat));
    epx.pws = slab.data_ptr<float>();
  }
  const T* A = (const T*)a.data_ptr();
  const T* Bp = (const T*)b.data_ptr();
  T* Cp = (T*)c.data_ptr();
  if (dp_tiles > 0)
    hipLaunchKernelGGL(kern, dim3(dp_tiles), dim3(NT), SMEM, st, A, Bp, Cp, a2, b2, M, N, K, (int)a.stride(0),
                       (int)b.stride(0), (int)c.stride(0), epx, sk);
  if (sk_tiles > 0) {
    auto ws = at::empty({(int64_t)sk_tiles * S * BM * BN}, a.options().dtype(at::kFloat));
    sk.enabled = 1;
    sk.tile0 = dp_tiles;
    sk.ntiles = sk_tiles;
    sk.gx = S;
    sk.ws = ws.data_ptr<float>();
    sk.flags = sk_flags(sk_tiles);
    hipLaunchKernelGGL(kern_sk, dim3(sk_tiles * S), dim3(NT), SMEM, st, A, Bp, Cp, a2, b2, M, N, K, (int)a.stride(0),
                       (int)b.stride(0), (int)c.stride(0), epx, sk);
  }
  if (ep.pw != nullptr)
    hipLaunchKernelGGL(proj_reduce_kernel<T>, dim3((unsigned)(((int64_t)M * 8 + 255) / 256)), dim3(256), 0, st,
                       (const float*)epx.pws, ntn, M, PW, ep.palpha, (T*)ep.pout);
}

// ---- skinny GEMM (M <= 64 rows: greedy decode, one token per sequence) ----
// The tiled kernels cover M = 64 with ONE row of 64x64 tiles: 12-48 blocks for the distilgpt2 decode
// shapes, each running the whole K loop as a chain of dependent tile loads on one CU (8.7 us for
// 64x2304x768, whose 3.5 MB of weights are 0.45 us of HBM).  Here a block owns BN output columns for
// all (<= 64) rows and its NW waves take interleaved 32-deep K steps, loading their MFMA fragments
// straight from global memory (no LDS staging: the 64 activation rows are L2-resident and shared by
// every block, each weight row is read once) with several k-steps of loads in flight.  The NW partial
// tiles are summed through LDS in wave order (deterministic), then the gemm_nt epilogue runs on 8-column
// chunks: bias, LoRA K-extension (one more k-step), pre-add, pre-activation store, forward activation,
// residual, and the next adapter's input projection as per-column-tile fp32 slabs (proj_reduce_kernel).
// Not for dropout (training) or activation-backward epilogues: those keep the tiled kernels.
// LNM = 1: A is the raw residual stream and the block applies LayerNorm(A; lnw, lnb, eps) on the fly —
// row statistics first (two-pass, as ln_fwd8_kernel), then every A fragment normalised and rounded
// to 16 bits before its MFMA: the decode step's separate LN launches (13 per distilgpt2 step) go away.
// LNM = 2: the LayerNorm folded into the weights (B = γ∘W rounded, lfc1 = row sums of B, lfc2 = W·β +
// bias, fp32): the MFMAs run on the raw A fragments as soon as they land, the same two-pass row
// statistics are taken from those registers while the matrix pipe works, and the epilogue applies
// out = rstd·(acc − mean·lfc1) + lfc2 — no normalisation pass and no statistics barrier between the
// loads and the first MFMA (the LNM = 1 chain cost 4-5 us per decode projection over the plain GEMM).
template <typename T, int BN, int NW, int LNM>
__global__ __launch_bounds__(NW * 64) void gemm_skinny_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                              T* __restrict__ C, const T* __restrict__ A2,
                                                              const T* __restrict__ B2, int M, int N, int K, int lda,
                                                              int ldb, int ldc, EpiArgs ep, const T* __restrict__ lnw,
                                                              const T* __restrict__ lnb, float eps, int ksplit,
                                                              float* __restrict__ kws, unsigned* __restrict__ kflags,
                                                              int pfe, const float* __restrict__ lfc1,
                                                              const float* __restrict__ lfc2) {
  constexpr bool LNP = LNM != 0;
  constexpr int NT = BN / 16;  // 16-column MFMA tiles per block
  constexpr int RLD = BN + 4;  // LDS row pitch (floats) of the partial tiles
  // dynamic LDS: the NW partial tiles, then (projection epilogue only) the rounded output tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  auto red = reinterpret_cast<float(*)[64][RLD]>(smem);
  auto ot = reinterpret_cast<float(*)[BN + 1]>(smem + (size_t)NW * 64 * RLD * 4);
  __shared__ float lred[LNP ? 2 : 1][LNP ? NW : 1][64];  // per-wave row partials: sum, then sum of squares
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  // ksplit > 1 (long K, e.g. fc2's 3072): the ksplit blocks of a column tile take equal k ranges and the
  // last to arrive sums their fp32 partials in split order before the epilogue (write-through partials,
  // one counter per tile: common.h mift_group_arrival)
  const int tile = blockIdx.x / ksplit, sidx = blockIdx.x - tile * ksplit;
  const int n0 = tile * BN;
  float4_ acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = float4_{0.f, 0.f, 0.f, 0.f};
  const T* ap[4];
  const T* bp[NT];
#pragma unroll
  for (int i = 0; i < 4; ++i) ap[i] = A + (size_t)min(i * 16 + fr, M - 1) * lda + fq * 8;
#pragma unroll
  for (int j = 0; j < NT; ++j) bp[j] = B + (size_t)min(n0 + j * 16 + fr, N - 1) * ldb + fq * 8;
  const int kper = K / 32 / ksplit, kb0 = sidx * kper, nks = kb0 + kper;
  // epilogue operands of this thread's output chunk (one chunk per thread when 64 x BN / 8 <= threads)
  // requested before the K loop: their latency hides under it instead of following the reduction
  // barrier as one more dependent round trip (the decode step is a chain of such short kernels)
  constexpr int CPR = BN / 8;  // 8-column chunks per row
  constexpr bool PFE = 64 * CPR <= NW * 64;
  short8 pf_bias = short8{0, 0, 0, 0, 0, 0, 0, 0}, pf_res = pf_bias;
  const bool pf_b = PFE && pfe && ep.bias != nullptr && !ep.bias_f32;
  const bool pf_r = PFE && pfe && ep.residual != nullptr;
  float4 pf_f1[2] = {}, pf_f2[2] = {};  // LNM = 2: this thread's chunk of lfc1 / lfc2
  if constexpr (PFE) {
    const int row = tid / CPR, c8 = (tid % CPR) * 8;
    if (tid < 64 * CPR && row < M && n0 + c8 < N) {
      if (pf_b) pf_bias = *reinterpret_cast<const short8*>(reinterpret_cast<const T*>(ep.bias) + n0 + c8);
      if (pf_r)
        pf_res = *reinterpret_cast<const short8*>(reinterpret_cast<const T*>(ep.residual) + (size_t)row * ldc + n0 + c8);
      if constexpr (LNM == 2) {
        pf_f1[0] = *reinterpret_cast<const float4*>(lfc1 + n0 + c8);
        pf_f1[1] = *reinterpret_cast<const float4*>(lfc1 + n0 + c8 + 4);
        pf_f2[0] = *reinterpret_cast<const float4*>(lfc2 + n0 + c8);
        pf_f2[1] = *reinterpret_cast<const float4*>(lfc2 + n0 + c8 + 4);
      }
    }
  }
  if constexpr (LNP) {
    // LayerNorm prologue (K <= 1024: at most KSM k-steps per wave).  All of the wave's fragments are
    // loaded first; the row statistics come from THOSE registers — per-lane partial sums over the
    // wave's k-columns, the 4 k-groups of a row reduced by two lane shuffles, the NW waves through
    // LDS — two-pass (mean, then squared deviations) as ln_fwd8_kernel; then every fragment is
    // normalised in place before its MFMA.  The first form re-read whole rows for the statistics,
    // one dependent load round more (12.7-13.8 us vs 6.2 us for the same GEMM without LN).
    constexpr int KSM = (1024 / 32 + NW - 1) / NW;
    constexpr int KW = LNM == 1 ? KSM : 1;
    frag_t<T> afs[KSM][4], bfs[KSM][NT];
    float wv[KW][8], bv[KW][8];
#pragma unroll
    for (int kk = 0; kk < KSM; ++kk) {
      const int ks = w + kk * NW;
      if (ks < nks) {  // wave-uniform
        const int k = ks * 32;
#pragma unroll
        for (int i = 0; i < 4; ++i) afs[kk][i] = *reinterpret_cast<const frag_t<T>*>(ap[i] + k);
#pragma unroll
        for (int j = 0; j < NT; ++j) bfs[kk][j] = *reinterpret_cast<const frag_t<T>*>(bp[j] + k);
        if constexpr (LNM == 1) {
          load8<T>(lnw + k + fq * 8, wv[kk]);
          load8<T>(lnb + k + fq * 8, bv[kk]);
        }
      }
    }
    if constexpr (LNM == 2) {  // the products first: raw A against the folded weights
#pragma unroll
      for (int kk = 0; kk < KSM; ++kk) {
        if (w + kk * NW >= nks) break;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = mfma16<T>(bfs[kk][j], afs[kk][i], acc[i][j]);
      }
    }
    float mean[4], rstd[4];
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      float ps[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KSM; ++kk) {
        if (w + kk * NW >= nks) break;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          short8 raw;
          __builtin_memcpy(&raw, &afs[kk][i], 16);
          float x[8];
          unpack8<T>(raw, x);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = pass == 0 ? x[e] : x[e] - mean[i];
            ps[i] += pass == 0 ? d : d * d;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ps[i] = xor16_add(ps[i]);
        ps[i] = xor32_add(ps[i]);
      }
      if (fq == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) lred[pass][w][i * 16 + fr] = ps[i];
      }
      if (LNM == 2 && pass == 1) break;  // the squares are published by the partial-tile barrier below
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float t = 0.f;
#pragma unroll
        for (int v = 0; v < NW; ++v) t += lred[pass][v][i * 16 + fr];
        if (pass == 0) mean[i] = t / K;
        else rstd[i] = rsqrtf(t / K + eps);
      }
    }
    if constexpr (LNM == 1) {
#pragma unroll
      for (int kk = 0; kk < KSM; ++kk) {
        if (w + kk * NW >= nks) break;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          short8 raw;
          __builtin_memcpy(&raw, &afs[kk][i], 16);
          float x[8];
          unpack8<T>(raw, x);
          short8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const T t = (T)((x[e] - mean[i]) * rstd[i] * wv[kk][e] + bv[kk][e]);
            short h;
            __builtin_memcpy(&h, &t, 2);
            o[e] = h;
          }
          frag_t<T> af;
          __builtin_memcpy(&af, &o, 16);
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = mfma16<T>(bfs[kk][j], af, acc[i][j]);
        }
      }
    }
  } else {
    // swapped products (weights first): lane holds out[row i*16 + fr][cols j*16 + 4 fq .. +3]
#pragma unroll 4
    for (int ks = kb0 + w; ks < nks; ks += NW) {
      const int k = ks * 32;
      frag_t<T> af[4], bf[NT];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const frag_t<T>*>(ap[i] + k);
#pragma unroll
      for (int j = 0; j < NT; ++j) bf[j] = *reinterpret_cast<const frag_t<T>*>(bp[j] + k);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma16<T>(bf[j], af[i], acc[i][j]);
    }
  }
  if (A2 != nullptr && w == NW - 1 && sidx == ksplit - 1) {  // LoRA K-extension: one more k-step
    frag_t<T> af2[4], bf2[NT];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      af2[i] = *reinterpret_cast<const frag_t<T>*>(A2 + (size_t)min(i * 16 + fr, M - 1) * 32 + fq * 8);
#pragma unroll
    for (int j = 0; j < NT; ++j)
      bf2[j] = *reinterpret_cast<const frag_t<T>*>(B2 + (size_t)min(n0 + j * 16 + fr, N - 1) * 32 + fq * 8);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = mfma16<T>(bf2[j], af2[i], acc[i][j]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
      *reinterpret_cast<float4_*>(&red[w][i * 16 + fr][j * 16 + 4 * fq]) = acc[i][j];
  __syncthreads();
  const float alpha = ep.alpha_ptr != nullptr ? ep.alpha * ep.alpha_ptr[0] : ep.alpha;
  // pf: (row, c8) is this thread's prefetched chunk (ch == tid)
  auto finish = [&](int row, int c8, float* z, bool pf) {
    const int gn = n0 + c8;
    if constexpr (LNM == 2) {  // out = rstd·(acc − mean·lfc1) + lfc2, the statistics summed in wave order
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int v = 0; v < NW; ++v) {
        sm += lred[0][v][row];
        sq += lred[1][v][row];
      }
      const float mu = sm / K, rs = rsqrtf(sq / K + eps);
      float f1[8], f2[8];
      if (pf) {
        __builtin_memcpy(f1, pf_f1, 32);
        __builtin_memcpy(f2, pf_f2, 32);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          f1[e] = lfc1[gn + e];
          f2[e] = lfc2[gn + e];
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) z[e] = rs * (z[e] - mu * f1[e]) + f2[e];
    }
    float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (pf && pf_b) {
      unpack8<T>(pf_bias, bv);
    } else if (ep.bias != nullptr) {
      if (ep.bias_f32) {
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[e] = reinterpret_cast<const float*>(ep.bias)[gn + e];
      } else {
        load8<T>(reinterpret_cast<const T*>(ep.bias) + gn, bv);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) z[e] = (float)(T)(z[e] * alpha + bv[e]);  // the tiled path's 16-bit C tile
    const size_t off = (size_t)row * ldc + gn;
    if (ep.pre_add != nullptr) {
      float pa[8];
      load8<T>(reinterpret_cast<const T*>(ep.pre_add) + off, pa);
#pragma unroll
      for (int e = 0; e < 8; ++e) z[e] += pa[e];
    }
    if (ep.preact != nullptr) store8<T>(reinterpret_cast<T*>(ep.preact) + off, z);
    if (ep.act != ACT_NONE) {
#pragma unroll
      for (int e = 0; e < 8; ++e) z[e] = apply_act(ep.act, z[e], 0.f);
    }
    if (ep.residual != nullptr) {
      float rv[8];
      if (pf && pf_r) unpack8<T>(pf_res, rv);
      else load8<T>(reinterpret_cast<const T*>(ep.residual) + off, rv);
#pragma unroll
      for (int e = 0; e < 8; ++e) z[e] += rv[e];
    }
    store8<T>(C + off, z);
    if (ep.pws != nullptr) {
#pragma unroll
      for (int e = 0; e < 8; ++e) ot[row][c8 + e] = (float)(T)z[e];
    }
  };
  for (int ch = tid; ch < 64 * CPR; ch += NW * 64) {
    const int row = ch / CPR, c8 = (ch % CPR) * 8;
    if (row >= M || n0 + c8 >= N) continue;
    float z[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) z[e] = 0.f;
#pragma unroll
    for (int v = 0; v < NW; ++v) {
      const float4 p0 = *reinterpret_cast<const float4*>(&red[v][row][c8]);
      const float4 p1 = *reinterpret_cast<const float4*>(&red[v][row][c8 + 4]);
      z[0] += p0.x; z[1] += p0.y; z[2] += p0.z; z[3] += p0.w;
      z[4] += p1.x; z[5] += p1.y; z[6] += p1.z; z[7] += p1.w;
    }
    if (ksplit > 1) {
      float* dst = kws + (((size_t)tile * ksplit + sidx) * 64 + row) * BN + c8;
#pragma unroll
      for (int e = 0; e < 8; ++e) mift_st_sc1(dst + e, z[e]);
      continue;
    }
    finish(row, c8, z, PFE && ch == tid);
  }
  if (ksplit > 1) {
    __shared__ int klast;
    if (!mift_group_arrival(kflags + tile, (unsigned)ksplit, &klast)) return;
    for (int ch = tid; ch < 64 * CPR; ch += NW * 64) {
      const int row = ch / CPR, c8 = (ch % CPR) * 8;
      if (row >= M || n0 + c8 >= N) continue;
      float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int q = 0; q < ksplit; ++q) {
        const float* src = kws + (((size_t)tile * ksplit + q) * 64 + row) * BN + c8;
        const float4 p0 = *reinterpret_cast<const float4*>(src);
        const float4 p1 = *reinterpret_cast<const float4*>(src + 4);
        z[0] += p0.x; z[1] += p0.y; z[2] += p0.z; z[3] += p0.w;
        z[4] += p1.x; z[5] += p1.y; z[6] += p1.z; z[7] += p1.w;
      }
      finish(row, c8, z, PFE && ch == tid);
    }
  }
  if (ep.pws == nullptr) return;  // block-uniform
  // next adapter's input projection over this block's columns: slab[blockIdx][row][j]
  __syncthreads();
  const int PW = ep.prow <= 16 ? 16 : 32;
  float* slab = ep.pws + (size_t)tile * M * PW;
  const T* pw = reinterpret_cast<const T*>(ep.pw);
  for (int idx = tid; idx < M * PW; idx += NW * 64) {
    const int r = idx / PW, j = idx % PW;
    float s = 0.f;
    if (j < ep.prow) {
#pragma unroll
      for (int c = 0; c < BN; ++c) s += ot[r][c] * (float)pw[(size_t)j * N + n0 + c];
    }
    slab[(size_t)r * PW + j] = s;
  }
}

// persistent per-column-tile arrival counters of the skinny kernel's K split (zeroed once, re-armed
// by each tile's last arriver; stream-ordered users; first allocated by an eager call)
unsigned* skinny_flags(int n) {
  static at::Tensor flags;
  if (!flags.defined() || flags.numel() < n)
    flags = at::zeros({std::max<int64_t>(n, 1 << 12)}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA));
  return reinterpret_cast<unsigned*>(flags.data_ptr<int>());
}

template <typename T, int BN, int NW>
void launch_skinny(const at::Tensor& a, const at::Tensor& b, at::Tensor& c, const T* a2, const T* b2, int M, int N,
                   int K, const EpiArgs& ep, hipStream_t st, const T* lnw = nullptr, const T* lnb = nullptr,
                   float eps = 0.f, int ksplit = 1, const float* lfc1 = nullptr, const float* lfc2 = nullptr) {
  const int nb = (N + BN - 1) / BN;
  at::Tensor kwsb;
  float* kws = nullptr;
  unsigned* kflags = nullptr;
  if (ksplit > 1) {
    kwsb = at::empty({(int64_t)nb * ksplit * 64 * BN}, a.options().dtype(at::kFloat));
    kws = kwsb.data_ptr<float>();
    kflags = skinny_flags(nb);
  }
  EpiArgs epx = ep;
  at::Tensor slab;
  const int PW = ep.prow <= 16 ? 16 : 32;
  if (ep.pw != nullptr) {
    slab = at::empty({(int64_t)nb * M * PW}, a.options().dtype(at::kFloat));
    epx.pws = slab.data_ptr<float>();
  }
  constexpr int RED = NW * 64 * (BN + 4) * 4, OT = 64 * (BN + 1) * 4;
  static_assert(RED + OT <= 160 * 1024, "LDS budget");
  // epilogue-operand prefetch (MIFT_SKINNY_PF=0: off; read per call, A/B)
  const char* pfs = getenv("MIFT_SKINNY_PF");
  const int pfe = pfs ? atoi(pfs) : 1;
  const int smem = RED + (ep.pw != nullptr ? OT : 0);
  static bool attr = false;
  if (!attr) {
    if constexpr (BN == 16 && NW == 8) {
      (void)hipFuncSetAttribute((const void*)gemm_skinny_kernel<T, BN, NW, 1>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, RED + OT);
      (void)hipFuncSetAttribute((const void*)gemm_skinny_kernel<T, BN, NW, 2>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, RED + OT);
    }
    (void)hipFuncSetAttribute((const void*)gemm_skinny_kernel<T, BN, NW, 0>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, RED + OT);
    attr = true;
  }
  if (lnw != nullptr || lfc1 != nullptr) {
    // the LN prologue / folded LN holds a wave's whole K range in registers: the 16-column, 8-wave form only
    if constexpr (BN == 16 && NW == 8) {
      auto kern = lfc1 != nullptr ? gemm_skinny_kernel<T, BN, NW, 2> : gemm_skinny_kernel<T, BN, NW, 1>;
      hipLaunchKernelGGL(kern, dim3(nb), dim3(NW * 64), smem, st, (const T*)a.data_ptr(), (const T*)b.data_ptr(),
                         (T*)c.data_ptr(), a2, b2, M, N, K, (int)a.stride(0), (int)b.stride(0), (int)c.stride(0), epx,
                         lnw, lnb, eps, 1, (float*)nullptr, (unsigned*)nullptr, pfe, lfc1, lfc2);
    } else {
      TORCH_CHECK(false, "gemm_skinny: LN prologue needs the 16-column 8-wave form");
    }
  } else {
    hipLaunchKernelGGL((gemm_skinny_kernel<T, BN, NW, 0>), dim3(nb * ksplit), dim3(NW * 64), smem, st,
                       (const T*)a.data_ptr(), (const T*)b.data_ptr(), (T*)c.data_ptr(), a2, b2, M, N, K,
                       (int)a.stride(0), (int)b.stride(0), (int)c.stride(0), epx, (const T*)nullptr,
                       (const T*)nullptr, 0.f, ksplit, kws, kflags, pfe, (const float*)nullptr, (const float*)nullptr);
  }
  if (ep.pw != nullptr)
    hipLaunchKernelGGL(proj_reduce_kernel<T>, dim3((unsigned)(((int64_t)M * 8 + 255) / 256)), dim3(256), 0, st,
                       (const float*)epx.pws, nb, M, PW, ep.palpha, (T*)ep.pout);
}

// the skinny kernel applies: a forward epilogue without dropout on <= 64 rows (MIFT_GEMM_SKINNY=0: off)
bool skinny_ok(int M, int N, int K, const EpiArgs& ep) {
  static const int env = [] { const char* e = getenv("MIFT_GEMM_SKINNY"); return e ? atoi(e) : 1; }();
  if (!env || M > 64 || N % 16 != 0) return false;
  if (N > 4096 ? (K > 1024 || N % 64 != 0 || env < 2) : (K > 4096 || (K > 1024 && (K / 32) % ((K + 1023) / 1024)))) return false;
  if (ep.thr != 0 || ep.ext_thr != 0 || ep.aux != nullptr || ep.sbits != nullptr || ep.lm.dbg != 0) return false;
  if (ep.act != ACT_NONE && ep.act != ACT_GELU_TANH && ep.act != ACT_RELU && ep.act != ACT_GELU_ERF) return false;
  if (ep.pw != nullptr && ep.pthr != 0) return false;
  return true;
}

// Tile configurations (tile id -> geometry):
//   1: 256x128, 8 waves (4x2), 3-stage ring (144 KiB, 1 block/CU)  — large N
//   2: 128x64,  4 waves (2x2), 3-stage ring (72 KiB, 2 blocks/CU)  — N ~ 768
//   3: 128x128, 4 waves (2x2), 2-stage ring (64 KiB, 2 blocks/CU)
//   4: 64x64,   4 waves (2x2), 3-stage ring (48 KiB)               — tiny problems
//   5: 256x256, 8 waves (2x4), 2-stage ring (128 KiB; C tile 132 KiB) — halves L2->CU bytes/MAC vs 128x128
//   6: 128x256, 8 waves (2x4), 2-stage ring (96 KiB)
//   7: 128x96,  4 waves (2x2, wave tile 64x48), 2-stage ring (56 KiB, 2 blocks/CU) — balances
//      ragged waves: N=768 gives 512 tiles = exactly one wave of 2x256 slots (128x128: 384)
//   8: 256x256, 8 waves (2x4), phased schedule (mainloop8: 4 phases per k-tile, staggered wave
//      rows, counted vmcnt across barriers, setprio MFMA clusters)
//   9: 128x192, 8 waves (2x4, wave tile 64x48), 2-stage ring (80 KiB -> two blocks = 16 waves per
//      CU): the wide-N distilgpt2 shapes (N = 2304 / 3072, K = 768) ran 20-25 % faster than 128x96 /
//      128x128 (c_fc fwd 52.6 vs 63.5 us, c_attn fwd 37.2 vs 48.9, c_proj dgrad 62.3 vs 75.7);
//      with fewer than two tiles per CU (N = 768) it lost up to 2x.  Deeper rings (3-4 stages, one
//      block per CU) lost 30-50 % on every distilgpt2 shape (tools/bench_kernels.py --only dgpt).
template <typename T>
void dispatch_tile(const at::Tensor& a, const at::Tensor& b, at::Tensor& c, const T* a2, const T* b2, int M, int N,
                   int K, const EpiArgs& ep, hipStream_t st, int tile) {
  if (tile == 0 && skinny_ok(M, N, K, ep)) {
    // decode-sized problems: 16-column blocks of 8 waves (48-192 blocks at the distilgpt2 shapes:
    // c_attn 8.7 -> 5.9 us, c_fc 8.7 -> 6.9).  Every block streams its rows' K range through its CU, so
    // long K is split over (K + 1023) / 1024 blocks per column tile, reduced by the last to arrive
    // (fc2, K = 3072: one block per tile ran 16 us on 8 or 16 waves vs 14 on the 64x64 split-K path);
    // wide N (the LM head: 32-column blocks 32 us, 64-column 26.7, vs 17.7-19.5 on 128x128 tiles) stays
    // tiled unless MIFT_GEMM_SKINNY=2 (A/B; profiles/r4/decode_skinny_trace.txt, decode_skinny2_trace.txt)
    if (N > 4096) launch_skinny<T, 64, 4>(a, b, c, a2, b2, M, N, K, ep, st);
    else launch_skinny<T, 16, 8>(a, b, c, a2, b2, M, N, K, ep, st, nullptr, nullptr, 0.f, (K + 1023) / 1024);
    return;
  }
  if (tile == 0) {
    // auto, from tools/bench_kernels.py on MI355X (profiles/bench_gemm_tiles_sk.json):
    //  * the phased 256x256 kernel (tile 8) wins with >= half a chip-wave of 256x256 tiles at
    //    K >= 1024 (OPT-2.7B every GEMM at M = 4096: +10..30 % over tiles 5/6 in isolation,
    //    profiles/bench_gemm_p8.json) or with very many tiles;
    //  * long-K problems with few 256x256 tiles (M = 2048, N = 2560, K >= 4096) run 128x256 +
    //    the split-K ragged-wave tail;
    //  * distilgpt2-scale problems (K = 768, N <= 3072) keep 128x128 / 128x96: at 1.1-1.5 waves of
    //    256x256 tiles with a gelu/pre-activation epilogue tile 8 ran 10-20 % slower end to end.
    const long n256 = (long)((M + 255) / 256) * ((N + 255) / 256);
    const long t128 = (long)((M + 127) / 128) * ((N + 127) / 128);
    const long t96 = (long)((M + 127) / 128) * ((N + 95) / 96);
    if ((K >= 1024 && n256 >= 128) || n256 >= 2048) {
      // the 4-wave loop (tile 10) beats the phased 8-wave one on plain and bias / ReLU / gelu / LoRA
      // K-extension epilogues (OPT layer GEMMs 1-7 % plain, qkv / fc1 forward 7-11 % at M 2048-4096),
      // but one wave per SIMD cannot hide the dependent hash chains of a dropout mask: with a residual
      // dropout or a masked K-extension tile 8 stays faster (out / fc2 / dgrads, 4-19 %;
      // profiles/r6/bench_gemm4_epilogues.json).  MIFT_GEMM_T10=0 / 1 forces either (read per call, A/B)
      const char* e = getenv("MIFT_GEMM_T10");
      const bool hashes = ep.thr != 0 || ep.ext_thr != 0;
      tile = (e ? atoi(e) != 0 : !hashes) ? 10 : 8;
    }
    // one chip-wave of 128x96 tiles (1-2 per CU): the OPT micro-batch-4 shapes (M = 2048, N = 2560)
    // ran 20-30 % faster than on the 128x256 split-K / 128x128 tiles (fc2 fwd 167 -> 122 us, qkv dgrad
    // 134 -> 94, out proj 50 -> 40; profiles/r4/bench_tiles_opt_pp_microbatch.json); the distilgpt2
    // N = 768 GEMMs on the 8-wave 128x192 tile instead: step 4.634 -> 4.838 ms (profiles/r6)
    else if (t96 >= num_cus() && t96 <= 2L * num_cus()) tile = 7;
    else if (K >= 4096 && t128 >= 128) tile = 6;
    else if (N % 192 == 0 && (long)((M + 127) / 128) * (N / 192) >= 2L * num_cus()) tile = 9;
    else if (t128 >= 64) {
      tile = 3;
      // 128x96 when its whole-wave count x tile area beats 128x128's (5 % per-tile
      // efficiency handicap for the smaller tile)
      if (N % 96 == 0) {
        const long G = 2L * num_cus();
        const long t96 = (long)((M + 127) / 128) * (N / 96);
        if ((t96 + G - 1) / G * 3 * 105 < (t128 + G - 1) / G * 4 * 100) tile = 7;
      }
    } else tile = 4;
  }
  constexpr bool HALF = std::is_same<T, fp16>::value;
  switch (tile) {
    case 1: launch_gemm<T, 256, 128, 4, 2, 3>(a, b, c, a2, b2, M, N, K, ep, st); break;
    case 2: launch_gemm<T, 128, 64, 2, 2, 3>(a, b, c, a2, b2, M, N, K, ep, st); break;
    case 3: launch_gemm<T, 128, 128, 2, 2, 2>(a, b, c, a2, b2, M, N, K, ep, st); break;
    case 5: launch_gemm<T, 256, 256, 2, 4, 2>(a, b, c, a2, b2, M, N, K, ep, st); break;
    case 6: launch_gemm<T, 128, 256, 2, 4, 2>(a, b, c, a2, b2, M, N, K, ep, st); break;
    case 7:
    case 9: mift_gemm_part2(tile, HALF, a, b, c, a2, b2, M, N, K, &ep, st); break;
    case 8:
    case 10: mift_gemm_part1(tile, HALF, a, b, c, a2, b2, M, N, K, &ep, st); break;
    default: launch_gemm<T, 64, 64, 2, 2, 3>(a, b, c, a2, b2, M, N, K, ep, st); break;
  }
}

#if MIFT_GEMM_PART == 1
template <typename T>
void part1_tiles(int tile, const at::Tensor& a, const at::Tensor& b, at::Tensor& c, const T* a2, const T* b2, int M,
                 int N, int K, const EpiArgs& ep, hipStream_t st) {
  // tile 10: the 4-wave loop addresses its operands with 32-bit buffer offsets (else: tile 8)
  if (tile == 10 && (uint64_t)M * a.stride(0) * 2 < (1ull << 32) && (uint64_t)N * b.stride(0) * 2 < (1ull << 32))
    launch_gemm<T, 256, 256, 2, 2, 1>(a, b, c, a2, b2, M, N, K, ep, st);
  else
    launch_gemm<T, 256, 256, 2, 4, 0>(a, b, c, a2, b2, M, N, K, ep, st);
}
#endif
#if MIFT_GEMM_PART == 2
template <typename T>
void part2_tiles(int tile, const at::Tensor& a, const at::Tensor& b, at::Tensor& c, const T* a2, const T* b2, int M,
                 int N, int K, const EpiArgs& ep, hipStream_t st) {
  if (tile == 7) launch_gemm<T, 128, 96, 2, 2, 2>(a, b, c, a2, b2, M, N, K, ep, st);
  else launch_gemm<T, 128, 192, 2, 4, 2>(a, b, c, a2, b2, M, N, K, ep, st);
}
#endif

// ---- LM head: loss from the forward's tile statistics (one wave per row) ----
// Wave w of block b takes rows (b·4 + w) + k·(4·grid), k < rpw.  total != nullptr: also the summed
// loss — per-block partials (the wave sums in row order, then waves in order), the last block to
// arrive sums them in block order: deterministic, and no separate reduction launch.  The grid is
// capped (rpw rows per wave) so few blocks arrive.
__global__ __launch_bounds__(256) void lmhead_lse_kernel(const float2* __restrict__ stats, int ntn,
                                                         const float* __restrict__ zlab,
                                                         const int64_t* __restrict__ labels, int V, int M, int shift,
                                                         int64_t ignore, int rpw, float* __restrict__ lse,
                                                         float* __restrict__ loss, float* __restrict__ part,
                                                         unsigned* __restrict__ counter, float* __restrict__ total) {
  __shared__ float wl[4];
  __shared__ float red[4];
  __shared__ int flag;
  const int lane = threadIdx.x & 63;
  const int rstride = 4 * gridDim.x;
  float lsum = 0.f;
  for (int k = 0; k < rpw; ++k) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6) + k * rstride;
    if (row >= M) break;  // wave-uniform
    const float2* st = stats + (size_t)row * ntn;
    // the row's target and label logit requested with its stats (not after the reduction)
    const int64_t lab = lm_label(labels, row, shift, ignore);
    const float zl = zlab[row];  // written for rows with a target, read only for those
    float m = -INFINITY, s = 0.f;
    constexpr int JL = 4;  // a row's stats in registers when ntn <= 256: ONE memory round trip per row
    if (ntn <= 64 * JL) {  // (the loops below waited for every load in turn)
      float2 v[JL];
#pragma unroll
      for (int u = 0; u < JL; ++u) v[u] = lane + 64 * u < ntn ? st[lane + 64 * u] : make_float2(-INFINITY, 0.f);
#pragma unroll
      for (int u = 0; u < JL; ++u) m = fmaxf(m, v[u].x);
      m = wave_max(m);
#pragma unroll
      for (int u = 0; u < JL; ++u)  // same per-lane order as the loop form: bit-identical
        if (lane + 64 * u < ntn) s += v[u].y * __expf(v[u].x - m);
    } else {
      for (int j = lane; j < ntn; j += 64) m = fmaxf(m, st[j].x);
      m = wave_max(m);
      for (int j = lane; j < ntn; j += 64) s += st[j].y * __expf(st[j].x - m);
    }
    s = wave_sum(s);
    if (lane == 0) {
      const float l = m + __logf(s);
      lse[row] = l;
      const float lrow = (lab >= 0 && lab < V) ? l - zl : 0.f;
      loss[row] = lrow;
      lsum += lrow;
    }
  }
  if (total == nullptr) return;  // block-uniform
  if (lane == 0) wl[threadIdx.x >> 6] = lsum;
  __syncthreads();
  if (threadIdx.x == 0) mift_st_sc1(&part[blockIdx.x], ((wl[0] + wl[1]) + wl[2]) + wl[3]);
  if (!mift_last_block_arrival(counter, &flag)) return;
  float t = 0.f;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += 256) t += part[i];
  t = block_sum<4>(t, red);
  if (threadIdx.x == 0) total[0] = t;
}

// ---- LM head: sum the split-K slabs, subtract g·W[label] (the one-hot part of dlogits) ----
template <typename T>
__global__ __launch_bounds__(256) void lmhead_reduce_kernel(const float* __restrict__ partial, int S, int M, int N,
                                                            const T* __restrict__ w, int ldw,
                                                            const int64_t* __restrict__ labels, int V, int shift,
                                                            int64_t ignore, const float* __restrict__ gscale,
                                                            const float* __restrict__ gmul, T* __restrict__ out) {
  const size_t v = (size_t)blockIdx.x * 256 + threadIdx.x;  // one 8-column chunk
  const int cpr = N / 8;
  if (v >= (size_t)M * cpr) return;
  const int row = (int)(v / cpr), c8 = (int)(v % cpr) * 8;
  float acc[8];
  {
    const float4* p = reinterpret_cast<const float4*>(partial + (size_t)row * N + c8);
    float4 a = p[0], b = p[1];
    acc[0] = a.x; acc[1] = a.y; acc[2] = a.z; acc[3] = a.w; acc[4] = b.x; acc[5] = b.y; acc[6] = b.z; acc[7] = b.w;
  }
  for (int s = 1; s < S; ++s) {
    const float4* p = reinterpret_cast<const float4*>(partial + ((size_t)s * M + row) * N + c8);
    float4 a = p[0], b = p[1];
    acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w; acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
  }
  const int64_t lab = lm_label(labels, row, shift, ignore);
  if (lab >= 0 && lab < V) {  // dX = g·(softmax·W - W[label]); rows without a target get 0
    float wv[8];
    load8<T>(w + (size_t)lab * ldw + c8, wv);
    // g = upstream grad [x gmul: 1/tokens of a replayed step, multiplied here instead of by a
    // separate scalar kernel; the same fp32 product, so eager and replayed steps agree bitwise]
    const float g = gmul ? gscale[0] * gmul[0] : gscale[0];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = g * (acc[e] - wv[e]);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  }
  store8<T>(out + (size_t)row * N + c8, acc);
}

template <typename T>
std::vector<at::Tensor> lmhead_fwd_impl(const at::Tensor& a, const at::Tensor& w, const at::Tensor& labels, int V,
                                        int shift, int64_t ignore, const c10::optional<at::Tensor>& ws) {
  const int M = a.size(0), K = a.size(1), N = w.size(0);
  constexpr int BM = 256, BN = 256;
  const int ntm = (M + BM - 1) / BM, ntn = (N + BN - 1) / BN;
  auto E = at::empty({M, N}, a.options());
  auto f32 = a.options().dtype(at::kFloat);
  auto stats = at::empty({M, ntn, 2}, f32);
  auto zlab = at::empty({M}, f32);  // written for every row with a target; read only for those
  auto lse = at::empty({M}, f32);
  auto loss = at::empty({M}, f32);
  EpiArgs ep{};
  ep.alpha = 1.f;
  ep.lm.labels = labels.data_ptr<int64_t>();
  ep.lm.V = V;
  ep.lm.stats = reinterpret_cast<float2*>(stats.data_ptr<float>());
  ep.lm.zlab = zlab.data_ptr<float>();
  ep.lm.ntn = ntn;
  ep.lm.shift = shift;
  ep.lm.ignore = ignore;
  if (const char* d = getenv("MIFT_LM_DBG")) ep.lm.dbg = atoi(d);
  {
    // tile raster of the head: the 32 blocks an XCD runs at once cover g row panels x 32/g vocab tiles,
    // so each W tile is fetched from the Infinity Cache once per g row panels (row-panel order, g = 1,
    // fetched 2.5 GB per distilgpt2 forward: FETCH_SIZE, profiles/r5/pmc_roofline_distilgpt2_step.txt);
    // persistent kernel measured g = 4 best at K = 768 in isolation (648 vs 714 us), g = 8 at K = 2560
    // (1381 vs 1491) (profiles/r5/bench_lm_persist.jsonl); inside the distilgpt2 step g = 3 is best
    // (4.630 vs 4.649 / 4.660 / 4.731 ms for g = 2 / 4 / 1, profiles/r6/step_ab_dgpt_lm_group*.json).
    // MIFT_LM_GROUP (per call) overrides.
    const char* g = getenv("MIFT_LM_GROUP");
    ep.group_m = g ? atoi(g) : (K <= 1024 ? 3 : 8);
  }
  SkArgs sk{};
  // staging ring (128 KiB) reused for the E tile + the two row-partial arrays
  constexpr int SMEM = std::max(2 * (BM + BN) * ROWB, BM * CTile<BN>::CLD * 2 + 2 * 8 * (BM / 2) * 4 + BM * 4);
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  // persistent kernel: the ring + the row-partial side area (E never staged in LDS)
  constexpr int SMEM_P = 2 * (BM + BN) * ROWB + 2 * 8 * (BM / 2) * 4 + 384 * 8;  // + the ids copy
  static_assert(SMEM_P <= 160 * 1024, "LDS budget");
  auto kern = gemm_nt_kernel<T, BM, BN, 2, 4, 0, false, 1>;
  auto kernp = lmhead_fwd_persist_kernel<T>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    (void)hipFuncSetAttribute((const void*)kernp, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM_P);
    attr = true;
  }
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const int grid = ntm * ntn;
  // persistent kernel at K <= 1024 (12 k-tiles per tile at distilgpt2's K = 768: the per-tile prologue
  // and epilogue are a large share; 664 vs 723 us), the one-tile kernel above (OPT K = 2560: 40 k-tiles
  // per tile, 1350 vs 1394 us with the raster group of both) — profiles/r5/bench_lm_persist_v2.jsonl.
  // MIFT_LM_PERSIST=0/1 forces either (read per call: A/B-able).  Even M: the ids copy moves 16-B pairs.
  const char* pe = getenv("MIFT_LM_PERSIST");
  const bool persist = (pe ? atoi(pe) != 0 : K <= 1024) && K / BK >= 2 && M >= 2 && M % 2 == 0;
  if (persist) {
    const int G = std::min(grid, num_cus());  // one 512-thread, 137 KiB block per CU
    hipLaunchKernelGGL(kernp, dim3(G), dim3(512), SMEM_P, st, (const T*)a.data_ptr(), (const T*)w.data_ptr(),
                       (T*)E.data_ptr(), M, N, K, (int)a.stride(0), (int)w.stride(0), N, ep.lm, grid, ep.group_m);
  } else {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(512), SMEM, st, (const T*)a.data_ptr(), (const T*)w.data_ptr(),
                       (T*)E.data_ptr(), nullptr, nullptr, M, N, K, (int)a.stride(0), (int)w.stride(0), N, ep, sk);
  }
  // ~4 blocks per CU (2 rows per wave at distilgpt2's M = 8192): the rows of a wave are a dependent
  // chain of stats loads, so fewer, fatter blocks ran slower (512 blocks of 4 rows per wave: 19 us vs
  // 9.4 us for one row per wave), while the two-level arrival counters keep 1024 arrivals cheap
  const int rows4 = (M + 3) / 4;
  const int rpw = (rows4 + 4 * num_cus() - 1) / (4 * num_cus());
  const int lgrid = (rows4 + rpw - 1) / rpw;
  at::Tensor total, part;
  if (ws) {
    total = at::empty({1}, f32);
    part = at::empty({lgrid}, f32);
  }
  hipLaunchKernelGGL(lmhead_lse_kernel, dim3(lgrid), dim3(256), 0, st,
                     reinterpret_cast<const float2*>(stats.data_ptr<float>()), ntn, zlab.data_ptr<float>(),
                     labels.data_ptr<int64_t>(), V, M, shift, ignore, rpw, lse.data_ptr<float>(), loss.data_ptr<float>(),
                     ws ? part.data_ptr<float>() : nullptr,
                     ws ? reinterpret_cast<unsigned*>(ws->data_ptr<int>()) : nullptr,
                     ws ? total.data_ptr<float>() : nullptr);
  if (ws) return {E, stats, lse, loss, zlab, total};
  return {E, stats, lse, loss, zlab};
}

template <typename T>
at::Tensor lmhead_dgrad_impl(const at::Tensor& E, const at::Tensor& wt, const at::Tensor& w, const at::Tensor& labels,
                             int V, const at::Tensor& stats, const at::Tensor& lse, const at::Tensor& gscale, int shift,
                             int64_t ignore, const c10::optional<at::Tensor>& gmul) {
  const int M = E.size(0), K = E.size(1), N = wt.size(0);
  const int ntn_f = stats.size(1);
  constexpr int BM = 256, BN = 256;
  constexpr int STAGE_BYTES = (BM + BN) * ROWB;
  constexpr int SMEM = 2 * STAGE_BYTES + BM * (LM_GW | 1) * 4;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  // split the vocabulary so the grid is a whole number of chip waves (one block per CU), >= 3 waves
  const int cus = num_cus();
  int S = std::max(1, std::min(ntn_f, (3 * cus + tiles - 1) / tiles));
  if (const char* e = getenv("MIFT_LM_SPLIT")) S = std::max(1, std::min(ntn_f, atoi(e)));  // A/B knob, per call
  const int gpc = (ntn_f + S - 1) / S;
  S = (ntn_f + gpc - 1) / gpc;
  auto partial = at::empty({S, M, N}, E.options().dtype(at::kFloat));
  EpiArgs ep{};
  ep.alpha = 1.f;
  ep.lm.labels = labels.data_ptr<int64_t>();
  ep.lm.V = V;
  ep.lm.stats = reinterpret_cast<float2*>(const_cast<float*>(stats.data_ptr<float>()));
  ep.lm.lse = lse.data_ptr<float>();
  ep.lm.gscale = gscale.data_ptr<float>();
  ep.lm.ntn = ntn_f;
  ep.lm.gpc = gpc;
  ep.lm.partial = partial.data_ptr<float>();
  ep.lm.shift = shift;
  ep.lm.ignore = ignore;
  SkArgs sk{};
  auto kern2 = gemm_nt_kernel<T, BM, BN, 2, 4, 0, false, 2>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern2, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr = true;
  }
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  auto out = at::empty({M, N}, E.options());
  // (an in-launch reduction by each tile's last chunk block was bit-identical but slower — head 1.42 ->
  // 1.59 ms, profiles/r4/lmhead_in_launch_reduction_rejected.txt — and was removed in round 6)
  hipLaunchKernelGGL(kern2, dim3(tiles * S), dim3(512), SMEM, st, (const T*)E.data_ptr(), (const T*)wt.data_ptr(),
                     (T*)nullptr, nullptr, nullptr, M, N, K, (int)E.stride(0), (int)wt.stride(0), N, ep, sk);
  const size_t chunks = (size_t)M * (N / 8);
  hipLaunchKernelGGL(lmhead_reduce_kernel<T>, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, st,
                     partial.data_ptr<float>(), S, M, N, (const T*)w.data_ptr(), (int)w.stride(0),
                     labels.data_ptr<int64_t>(), V, shift, ignore, gscale.data_ptr<float>(),
                     gmul ? gmul->data_ptr<float>() : nullptr, (T*)out.data_ptr());
  return out;
}

}  // namespace

#if MIFT_GEMM_PART == 1
void mift_gemm_part1(int tile, bool half, const at::Tensor& a, const at::Tensor& b, at::Tensor& c, const void* a2,
                     const void* b2, int M, int N, int K, const void* ep, hipStream_t st) {
  const EpiArgs& e = *static_cast<const EpiArgs*>(ep);
  if (half) part1_tiles<fp16>(tile, a, b, c, (const fp16*)a2, (const fp16*)b2, M, N, K, e, st);
  else part1_tiles<bf16>(tile, a, b, c, (const bf16*)a2, (const bf16*)b2, M, N, K, e, st);
}
#endif
#if MIFT_GEMM_PART == 2
void mift_gemm_part2(int tile, bool half, const at::Tensor& a, const at::Tensor& b, at::Tensor& c, const void* a2,
                     const void* b2, int M, int N, int K, const void* ep, hipStream_t st) {
  const EpiArgs& e = *static_cast<const EpiArgs*>(ep);
  if (half) part2_tiles<fp16>(tile, a, b, c, (const fp16*)a2, (const fp16*)b2, M, N, K, e, st);
  else part2_tiles<bf16>(tile, a, b, c, (const bf16*)a2, (const bf16*)b2, M, N, K, e, st);
}
#endif

#if MIFT_GEMM_PART == 3
// Fused LM head + cross-entropy forward: a = LN(h) [M,K], w = tied embedding [V_pad,K],
// labels [M] int64 (ignore -> any value outside [0, V)): the targets themselves (shift = 0), or the
// unshifted ids of sequences of length shift (row r's target = ids[r + 1] inside its sequence).
// -> (E [M,V_pad] = exp(z - m_tile) 16-bit, stats [M, V_pad/256, 2] (m, s), lse [M], loss [M], zlab [M]
//     [, total [1] = Σ loss, when `ws` (an int32 zero-initialised arrival counter) is given]).
// ignore >= 0: that id is no target.
std::vector<at::Tensor> mift_lmhead_fwd(const at::Tensor& a, const at::Tensor& w, const at::Tensor& labels, int64_t V,
                                        int64_t shift, int64_t ignore, const c10::optional<at::Tensor>& ws) {
  TORCH_CHECK(a.is_cuda() && w.is_cuda() && labels.is_cuda(), "lmhead_fwd: GPU tensors");
  TORCH_CHECK(a.dim() == 2 && w.dim() == 2 && a.size(1) == w.size(1), "lmhead_fwd: a [M,K], w [V_pad,K]");
  TORCH_CHECK(a.stride(1) == 1 && w.stride(1) == 1 && a.size(1) % 64 == 0, "lmhead_fwd: K-contiguous, K % 64 == 0");
  TORCH_CHECK(a.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "lmhead_fwd: 16-B aligned rows");
  TORCH_CHECK(w.size(0) % 8 == 0 && V <= w.size(0) && w.size(0) - V < 256, "lmhead_fwd: V_pad % 8, V_pad - V < 256");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous() && labels.numel() == a.size(0),
              "lmhead_fwd: int64 labels [M]");
  TORCH_CHECK(shift >= 0 && (shift == 0 || a.size(0) % shift == 0), "lmhead_fwd: rows must be whole sequences");
  TORCH_CHECK(a.scalar_type() == w.scalar_type(), "lmhead_fwd: dtype mismatch");
  TORCH_CHECK(!ws || (ws->is_cuda() && ws->scalar_type() == at::kInt && ws->numel() >= MIFT_ARRIVE_INTS),
              "lmhead_fwd: ws int32[arrive_ints]");
  if (a.scalar_type() == at::kBFloat16) return lmhead_fwd_impl<bf16>(a, w, labels, (int)V, (int)shift, ignore, ws);
  TORCH_CHECK(a.scalar_type() == at::kHalf, "lmhead_fwd: bf16/fp16");
  return lmhead_fwd_impl<fp16>(a, w, labels, (int)V, (int)shift, ignore, ws);
}

// Backward of the fused head: dX [M,N] = g·(softmax - onehot)·W without materialising dlogits.
// E / stats / lse from mift_lmhead_fwd; wt = Wᵀ [N, V_pad] (K-contiguous), w = W [V_pad, N];
// gscale: 1-element fp32 device tensor (upstream gradient, e.g. loss_scale / tokens), times the
// optional 1-element fp32 gmul.
at::Tensor mift_lmhead_dgrad(const at::Tensor& E, const at::Tensor& wt, const at::Tensor& w, const at::Tensor& labels,
                             int64_t V, const at::Tensor& stats, const at::Tensor& lse, const at::Tensor& gscale,
                             int64_t shift, int64_t ignore, const c10::optional<at::Tensor>& gmul) {
  TORCH_CHECK(E.is_cuda() && wt.is_cuda() && w.is_cuda(), "lmhead_dgrad: GPU tensors");
  TORCH_CHECK(E.dim() == 2 && wt.dim() == 2 && wt.size(1) == E.size(1), "lmhead_dgrad: E [M,V_pad], wt [N,V_pad]");
  TORCH_CHECK(E.stride(1) == 1 && wt.stride(1) == 1 && E.size(1) % 64 == 0, "lmhead_dgrad: V_pad % 64 == 0");
  TORCH_CHECK(E.is_contiguous() && wt.stride(0) % 8 == 0, "lmhead_dgrad: layouts");
  TORCH_CHECK(w.size(0) >= V && w.size(1) == wt.size(0) && w.stride(1) == 1 && w.stride(0) % 8 == 0,
              "lmhead_dgrad: w [V_pad, N]");
  TORCH_CHECK(wt.size(0) % 8 == 0, "lmhead_dgrad: N % 8 == 0");
  TORCH_CHECK(stats.dim() == 3 && stats.size(0) == E.size(0) && stats.size(2) == 2 && stats.is_contiguous() &&
                  stats.size(1) * 256 >= E.size(1),
              "lmhead_dgrad: stats [M, ntn, 2]");
  TORCH_CHECK(lse.numel() == E.size(0) && gscale.numel() >= 1 && gscale.scalar_type() == at::kFloat,
              "lmhead_dgrad: lse [M], fp32 gscale");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == E.size(0), "lmhead_dgrad: labels");
  TORCH_CHECK(!gmul || (gmul->is_cuda() && gmul->scalar_type() == at::kFloat && gmul->numel() >= 1),
              "lmhead_dgrad: gmul fp32[1]");
  if (E.scalar_type() == at::kBFloat16)
    return lmhead_dgrad_impl<bf16>(E, wt, w, labels, (int)V, stats, lse, gscale, (int)shift, ignore, gmul);
  TORCH_CHECK(E.scalar_type() == at::kHalf, "lmhead_dgrad: bf16/fp16");
  return lmhead_dgrad_impl<fp16>(E, wt, w, labels, (int)V, stats, lse, gscale, (int)shift, ignore, gmul);
}

#endif  // MIFT_GEMM_PART == 3

#if MIFT_GEMM_PART == 0
// diagnostics: every later gemm_nt launch records per-block cycle stamps into buf (int64 [blocks, 8]),
// None turns it off (tools/gemm_stamps.py)
static long long* g_gemm_stamps = nullptr;
void mift_gemm_set_stamps(const c10::optional<at::Tensor>& buf) {
  TORCH_CHECK(!buf || (buf->is_cuda() && buf->scalar_type() == at::kLong && buf->is_contiguous()),
              "gemm_set_stamps: int64 GPU buffer");
  g_gemm_stamps = buf ? reinterpret_cast<long long*>(buf->data_ptr<int64_t>()) : nullptr;
}

// out = epi(a @ b^T [+ a2 @ b2^T]).  a:[M,K], b:[N,K] (K-contiguous, K%64==0).
std::vector<at::Tensor> mift_gemm_nt(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& bias,
                                     const c10::optional<at::Tensor>& a2, const c10::optional<at::Tensor>& b2,
                                     int64_t act, const c10::optional<at::Tensor>& aux,
                                     const c10::optional<at::Tensor>& residual, double dropout_p, int64_t seed,
                                     bool want_preact, double alpha, const c10::optional<at::Tensor>& out,
                                     int64_t tile, const c10::optional<at::Tensor>& alpha_t,
                                     const c10::optional<at::Tensor>& pre_add, double ext_p, int64_t ext_seed,
                                     const c10::optional<at::Tensor>& proj_w, int64_t proj_rows, double proj_p,
                                     int64_t proj_seed, double proj_alpha, const c10::optional<at::Tensor>& sbits) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda(), "gemm_nt: GPU tensors required");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2, "gemm_nt: 2-D operands");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1, "gemm_nt: K must be contiguous");
  TORCH_CHECK(a.scalar_type() == b.scalar_type(), "gemm_nt: dtype mismatch");
  const int M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "gemm_nt: K mismatch");
  TORCH_CHECK(K % 64 == 0, "gemm_nt: K must be a multiple of 64, got ", K);
  TORCH_CHECK(N % 4 == 0, "gemm_nt: N must be a multiple of 4, got ", N);
  TORCH_CHECK((a.stride(0) % 8) == 0 && (b.stride(0) % 8) == 0, "gemm_nt: row strides must be 16-B aligned");
  at::Tensor c = out ? *out : at::empty({M, N}, a.options());
  TORCH_CHECK(c.size(0) == M && c.size(1) == N && c.stride(1) == 1 && c.stride(0) % 8 == 0, "gemm_nt: bad out");
  EpiArgs ep{};
  ep.bias = nullptr;
  if (bias) {
    TORCH_CHECK(bias->numel() == N, "gemm_nt: bias size");
    ep.bias = bias->data_ptr();
    ep.bias_f32 = bias->scalar_type() == at::kFloat;
  }
  if (a2) {
    TORCH_CHECK(b2.has_value(), "gemm_nt: a2 needs b2");
    TORCH_CHECK(a2->size(0) == M && a2->size(1) == 32 && a2->is_contiguous(), "gemm_nt: a2 must be [M,32]");
    TORCH_CHECK(b2->size(0) == N && b2->size(1) == 32 && b2->is_contiguous(), "gemm_nt: b2 must be [N,32]");
  }
  ep.act = (int)act;
  ep.aux = nullptr;
  if (aux) {
    TORCH_CHECK(aux->size(0) == M && aux->size(1) == N && aux->stride(0) == c.stride(0) && aux->stride(1) == 1,
                "gemm_nt: aux layout must match out");
    ep.aux = aux->data_ptr();
  }
  at::Tensor pre;
  ep.preact = nullptr;
  if (want_preact) {
    TORCH_CHECK(c.stride(0) == N, "gemm_nt: preact output needs a dense out");
    pre = at::empty({M, N}, a.options());
    ep.preact = pre.data_ptr();
  }
  ep.residual = nullptr;
  if (residual) {
    TORCH_CHECK(residual->size(0) == M && residual->size(1) == N && residual->stride(0) == c.stride(0),
                "gemm_nt: residual layout must match out");
    ep.residual = residual->data_ptr();
  }
  ep.seed = (uint64_t)seed;
  ep.thr = mift_thr16(dropout_p);
  ep.inv_keep = dropout_p > 0 ? mift_inv_keep(dropout_p) : 1.f;
  ep.alpha = (float)alpha;
  ep.alpha_ptr = nullptr;
  if (alpha_t) {
    TORCH_CHECK(alpha_t->scalar_type() == at::kFloat && alpha_t->is_cuda(), "gemm_nt: alpha_t fp32 GPU");
    ep.alpha_ptr = alpha_t->data_ptr<float>();
  }
  ep.ext_thr = mift_thr16(ext_p);
  ep.ext_seed = (uint64_t)ext_seed;
  ep.ext_inv_keep = ext_p > 0 ? mift_inv_keep(ext_p) : 1.f;
  ep.sstep = mift_seed_step();
  ep.group_m = gemm_group_m(N);
  {
    const char* e = getenv("MIFT_EPI_PFG");  // read per call (A/B)
    ep.pfg = e ? atoi(e) : 1;
    // non-temporal C stores for large outputs (OPT-2.7B mb 48, every output 126-503 MB: 4-block step
    // 302.9 -> 300.7 ms); the distilgpt2 outputs (<= 50 MB) are re-read from the Infinity Cache by the
    // next kernel (4.872 -> 4.904 ms with NT stores), so the default is by size (profiles/r5/
    // step_ab_opt_nt*.json, step_ab_dgpt_nt.json).  MIFT_EPI_NT=0 / 1 forces (A/B)
    // threshold at the Infinity Cache size (256 MiB): a smaller output can still be re-read from it by
    // the next kernel, which NT stores would give up (the 96 MiB form measured +0.7 % on the
    // mb-48 step, inside the box spread: its gain came from the 503 MB fc1 / fc2-dgrad outputs)
    const char* n = getenv("MIFT_EPI_NT");
    ep.ntc = n ? atoi(n) : ((int64_t)M * N * (int64_t)a.element_size() >= (256ll << 20) ? 1 : 0);
  }
  if (const char* d = getenv("MIFT_LM_DBG")) ep.lm.dbg = atoi(d);  // diagnostics (bit 0: no C store)
  ep.pre_add = nullptr;
  if (pre_add) {
    TORCH_CHECK(pre_add->size(0) == M && pre_add->size(1) == N && pre_add->stride(0) == c.stride(0) &&
                    pre_add->scalar_type() == a.scalar_type(),
                "gemm_nt: pre_add layout must match out");
    ep.pre_add = pre_add->data_ptr();
  }
  at::Tensor proj;
  if (proj_w) {  // T = s·drop(out)·Aᵀ of the next adapter, from the epilogue (EpiArgs::pw)
    TORCH_CHECK(proj_w->is_contiguous() && proj_w->size(0) == 32 && proj_w->size(1) == N &&
                    proj_w->scalar_type() == a.scalar_type(),
                "gemm_nt: proj_w must be [32, N] contiguous, same dtype");
    TORCH_CHECK(proj_rows >= 1 && proj_rows <= 32 && N % 32 == 0, "gemm_nt: proj rows in [1, 32], N % 32 == 0");
    proj = at::empty({M, 32}, a.options());
    ep.pw = proj_w->data_ptr();
    ep.prow = (int)proj_rows;
    ep.pthr = mift_thr16(proj_p);
    ep.pseed = (uint64_t)proj_seed;
    ep.pout = proj.data_ptr();
    ep.palpha = (float)proj_alpha * (proj_p > 0 ? mift_inv_keep(proj_p) : 1.f);
  }
  ep.stamps = g_gemm_stamps;
  {
    const char* e = getenv("MIFT_EPI_STAGED");  // read per call (A/B)
    ep.staged = e ? atoi(e) : 1;
    const char* h = getenv("MIFT_EPI_HOIST");   // read per call (A/B); needs M·N < 2^33
    ep.hoist = (h ? atoi(h) : 1) && (uint64_t)M * N < (1ull << 33);
    const char* x = getenv("MIFT_EXT_LDS");     // read per call (A/B)
    ep.ext_lds = x ? atoi(x) : 1;
  }
  ep.sbits = nullptr;
  if (sbits) {  // ReLU sign bits: written (act = relu) or read in place of aux (act = relu backward)
    TORCH_CHECK((act == ACT_RELU || (act == ACT_RELU_BWD && !aux)) && N % 8 == 0 && sbits->is_cuda() &&
                    sbits->scalar_type() == at::kByte && sbits->is_contiguous() && sbits->size(0) == M &&
                    sbits->size(1) == N / 8,
                "gemm_nt: sbits must be uint8 [M, N/8] with act relu / relu-bwd (no aux), N % 8 == 0");
    ep.sbits = sbits->data_ptr<uint8_t>();
  }
  if (M == 0 || N == 0) return {c, pre, proj};
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  if (a.scalar_type() == at::kBFloat16) {
    dispatch_tile<bf16>(a, b, c, a2 ? (const bf16*)a2->data_ptr() : nullptr, b2 ? (const bf16*)b2->data_ptr() : nullptr,
                        M, N, K, ep, st, (int)tile);
  } else if (a.scalar_type() == at::kHalf) {
    dispatch_tile<fp16>(a, b, c, a2 ? (const fp16*)a2->data_ptr() : nullptr, b2 ? (const fp16*)b2->data_ptr() : nullptr,
                        M, N, K, ep, st, (int)tile);
  } else {
    TORCH_CHECK(false, "gemm_nt: bf16/fp16 only");
  }
  return {c, pre, proj};
}

// out [M, N] = act(LayerNorm(x) · wᵀ + bias) for M <= 64 (decode): the skinny kernel with its LN prologue
// (no normalised copy of x, no LN launch).  The caller checks mift_gemm_ln_ok (else LN + gemm_nt).
bool mift_gemm_ln_ok(int64_t M, int64_t N, int64_t K) { return M >= 1 && M <= 64 && N % 16 == 0 && N <= 4096 &&
                                                               K % 64 == 0 && K <= 1024; }

// out [M, N] = act(rstd·(x·wfᵀ − mean·c1) + c2) = act(LayerNorm(x; γ, β) · wᵀ + bias) with wf = γ∘w (x's
// dtype), c1 = row sums of wf and c2 = w·β + bias (fp32 [N]) prepared once by the caller
// (mift.ops.fused._ln_fold): the skinny kernel's LNM = 2 form (decode projections, M <= 64).
at::Tensor mift_gemm_ln_fold(const at::Tensor& x, const at::Tensor& wf, const at::Tensor& c1, const at::Tensor& c2,
                             double eps, int64_t act) {
  TORCH_CHECK(x.is_cuda() && wf.is_cuda() && x.dim() == 2 && wf.dim() == 2 && x.size(1) == wf.size(1),
              "gemm_ln_fold: x [M,K], wf [N,K]");
  TORCH_CHECK(x.stride(1) == 1 && wf.stride(1) == 1 && x.stride(0) % 8 == 0 && wf.stride(0) % 8 == 0,
              "gemm_ln_fold: layouts");
  const int M = x.size(0), K = x.size(1), N = wf.size(0);
  TORCH_CHECK(x.scalar_type() == wf.scalar_type(), "gemm_ln_fold: wf of x's dtype");
  TORCH_CHECK(c1.scalar_type() == at::kFloat && c2.scalar_type() == at::kFloat && c1.is_contiguous() &&
                  c2.is_contiguous() && c1.numel() == N && c2.numel() == N,
              "gemm_ln_fold: c1 / c2 fp32 [N]");
  TORCH_CHECK(mift_gemm_ln_ok(M, N, K), "gemm_ln_fold: M <= 64, N % 16 == 0, N <= 4096, K % 64 == 0, K <= 1024");
  TORCH_CHECK(act == ACT_NONE || act == ACT_GELU_TANH || act == ACT_RELU || act == ACT_GELU_ERF,
              "gemm_ln_fold: forward act");
  at::Tensor c = at::empty({M, N}, x.options());
  EpiArgs ep{};
  ep.alpha = 1.f;
  ep.act = (int)act;
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  if (x.scalar_type() == at::kBFloat16)
    launch_skinny<bf16, 16, 8>(x, wf, c, nullptr, nullptr, M, N, K, ep, st, nullptr, nullptr, (float)eps, 1,
                               c1.data_ptr<float>(), c2.data_ptr<float>());
  else {
    TORCH_CHECK(x.scalar_type() == at::kHalf, "gemm_ln_fold: bf16/fp16");
    launch_skinny<fp16, 16, 8>(x, wf, c, nullptr, nullptr, M, N, K, ep, st, nullptr, nullptr, (float)eps, 1,
                               c1.data_ptr<float>(), c2.data_ptr<float>());
  }
  return c;
}

std::vector<at::Tensor> mift_gemm_ln(const at::Tensor& x, const at::Tensor& ln_w, const at::Tensor& ln_b, double eps,
                                     const at::Tensor& w, const c10::optional<at::Tensor>& bias, int64_t act,
                                     bool want_preact) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "gemm_ln: x [M,K], w [N,K]");
  TORCH_CHECK(x.stride(1) == 1 && w.stride(1) == 1 && x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "gemm_ln: layouts");
  TORCH_CHECK(x.scalar_type() == w.scalar_type() && ln_w.scalar_type() == x.scalar_type() &&
                  ln_b.scalar_type() == x.scalar_type() && ln_w.numel() == x.size(1) && ln_b.numel() == x.size(1) &&
                  ln_w.is_contiguous() && ln_b.is_contiguous(),
              "gemm_ln: LN weights of x's dtype, [K]");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(mift_gemm_ln_ok(M, N, K), "gemm_ln: M <= 64, N % 16 == 0, N <= 4096, K % 64 == 0, K <= 1024");
  TORCH_CHECK(act == ACT_NONE || act == ACT_GELU_TANH || act == ACT_RELU || act == ACT_GELU_ERF, "gemm_ln: forward act");
  at::Tensor c = at::empty({M, N}, x.options());
  at::Tensor pre;
  EpiArgs ep{};
  ep.alpha = 1.f;
  ep.act = (int)act;
  if (bias) {
    TORCH_CHECK(bias->numel() == N, "gemm_ln: bias size");
    ep.bias = bias->data_ptr();
    ep.bias_f32 = bias->scalar_type() == at::kFloat;
  }
  if (want_preact) {
    pre = at::empty({M, N}, x.options());
    ep.preact = pre.data_ptr();
  }
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  if (x.scalar_type() == at::kBFloat16)
    launch_skinny<bf16, 16, 8>(x, w, c, nullptr, nullptr, M, N, K, ep, st, (const bf16*)ln_w.data_ptr(),
                               (const bf16*)ln_b.data_ptr(), (float)eps);
  else {
    TORCH_CHECK(x.scalar_type() == at::kHalf, "gemm_ln: bf16/fp16");
    launch_skinny<fp16, 16, 8>(x, w, c, nullptr, nullptr, M, N, K, ep, st, (const fp16*)ln_w.data_ptr(),
                               (const fp16*)ln_b.data_ptr(), (float)eps);
  }
  return {c, pre};
}
#endif  // MIFT_GEMM_PART == 0
