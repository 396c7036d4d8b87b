// Shared device helpers for the mift gfx950 kernels.
//
// Conventions (all kernels):
//   * wave64: lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
//   * 16-bit element types are clang's native __bf16 / _Float16 (gfx950 has
//     hardware converts: v_cvt_pk_bf16_f32), accumulation is always fp32;
//   * dropout masks are counter-based (no mask tensors are stored): element
//     `idx` of a call with seed `s` is kept iff mift_hash(s, idx) >= thr,
//     thr = p * 2^32.  mift.ops.reference re-implements the same hash in
//     torch so CPU tests reproduce the GPU mask bit for bit, and recompute
//     (activation checkpointing) regenerates identical masks.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#define MIFT_HD __device__ __forceinline__

// Device-side bounds / shape checks: compiled only into the debug build (`python -m mift.build
// --debug` -> _C_debug.so, -DMIFT_DEBUG=1); a failing check prints the site and traps, so the
// faulting kernel is named by the fault itself (no GPU ASan on this pool).
#if defined(MIFT_DEBUG) && MIFT_DEBUG
#define MIFT_ASSERT(cond)                                                               \
  do {                                                                                  \
    if (!(cond)) {                                                                      \
      printf("MIFT_ASSERT %s:%d: %s (block %d thread %d)\n", __FILE__, __LINE__, #cond, \
             (int)blockIdx.x, (int)threadIdx.x);                                        \
      __builtin_trap();                                                                 \
    }                                                                                   \
  } while (0)
#else
#define MIFT_ASSERT(cond) \
  do {                    \
  } while (0)
#endif

// Graph-replayable dropout seeds.  mift.models.layers.seed_for(base, step, site) =
// fin(base*C1 + step*C2 + site*C3) with fin(x) = (x ^ x>>31) & (2^63-1).  Eager launches pass
// the finished seed and sstep == nullptr.  Under hipGraph capture (mift.train.graph) the host
// passes pre = base*C1 + site*C3 and sstep -> a device int64 micro-step counter, so every
// replay of the same captured kernels draws the masks of a new micro-step, bit-identical to
// the eager path.  Kernels take `seed, sstep` and call mift_seed once at entry.
__device__ __forceinline__ uint64_t mift_seed(uint64_t s, const int64_t* sstep) {
  if (sstep == nullptr) return s;
  uint64_t x = s + (uint64_t)(*sstep) * 0xBF58476D1CE4E5B9ull;
  x ^= x >> 31;
  return x & 0x7FFFFFFFFFFFFFFFull;
}
// host: the device micro-step counter bound by mift._C.set_seed_step (nullptr = eager)
const int64_t* mift_seed_step();

// host: deterministic reductions — no float atomics in any gradient reduction, so a
// step's results are bit-identical run to run.  On by default; MIFT_DETERMINISTIC=0 opts out.
inline bool mift_deterministic() {
  const char* e = getenv("MIFT_DETERMINISTIC");
  return e == nullptr || e[0] != '0';
}

typedef __bf16 bf16;
typedef _Float16 fp16;

typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4_ __attribute__((ext_vector_type(4)));
typedef float float4_ __attribute__((ext_vector_type(4)));
typedef unsigned v4u32 __attribute__((ext_vector_type(4)));
typedef float float16_ __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 fp16x8 __attribute__((ext_vector_type(8)));

template <typename T> MIFT_HD float to_f32(T x) { return (float)x; }
template <typename T> MIFT_HD T from_f32(float x) { return (T)x; }

// Counter-based dropout RNG (32-bit ops only: 64-bit multiplies are
// emulated on CDNA and made the old splitmix64 mask VALU-bound).
// One 32-bit hash per element PAIR (idx >> 1); element idx uses the low
// (even idx) or high (odd idx) 16 bits; keep iff bits >= thr16 where
// thr16 = round(p * 65536).  Unbiased rescale: inv_keep = 65536/(65536-thr16).
MIFT_HD uint32_t mix32(uint32_t x) {  // "lowbias32" finaliser
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
MIFT_HD uint32_t mift_hash_pair(uint64_t seed, uint64_t pair) {
  const uint32_t lo = (uint32_t)pair, hi = (uint32_t)(pair >> 32);
  return mix32((lo * 0x9E3779B9U) ^ mix32(hi ^ (uint32_t)(seed >> 32)) ^ (uint32_t)seed);
}
// Hoisted form of mift_hash_pair: hm = mix32(hi ^ seed_hi) depends only on the
// pair's high word, which is 0 for every tensor below 2^33 elements -> a kernel
// computes it once (mift_hmix(seed, 0)) and pays 3 instead of 5 multiplies per
// pair.  Bit-identical to mift_hash_pair for pairs with that high word.
MIFT_HD uint32_t mift_hmix(uint64_t seed, uint32_t hi) { return mix32(hi ^ (uint32_t)(seed >> 32)); }
MIFT_HD uint32_t mift_hash_lo(uint64_t seed, uint32_t hm, uint32_t lo) {
  return mix32((lo * 0x9E3779B9U) ^ hm ^ (uint32_t)seed);
}
MIFT_HD uint32_t mift_bits16(uint64_t seed, uint64_t idx) {
  return (mift_hash_pair(seed, idx >> 1) >> ((idx & 1) << 4)) & 0xFFFFu;
}
MIFT_HD bool mift_keep(uint64_t seed, uint64_t idx, uint32_t thr) { return mift_bits16(seed, idx) >= thr; }
// 8 consecutive elements: 4 hashes when idx0 is even (the common case).
MIFT_HD void mift_keep8(uint64_t seed, uint64_t idx0, uint32_t thr, bool* k) {
  const uint32_t lo0 = (uint32_t)(idx0 >> 1);
  if ((idx0 & 1) == 0 && lo0 <= 0xFFFFFFFCu) {
    // the 4 pairs share their high word: one hoisted mix (14 instead of 20 multiplies)
    const uint32_t hm = mift_hmix(seed, (uint32_t)(idx0 >> 33));
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const uint32_t h = mift_hash_lo(seed, hm, lo0 + (e >> 1));
      k[e] = (h & 0xFFFFu) >= thr;
      k[e + 1] = (h >> 16) >= thr;
    }
  } else if ((idx0 & 1) == 0) {
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const uint32_t h = mift_hash_pair(seed, (idx0 + e) >> 1);
      k[e] = (h & 0xFFFFu) >= thr;
      k[e + 1] = (h >> 16) >= thr;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) k[e] = mift_keep(seed, idx0 + e, thr);
  }
}

#ifndef __HIP_DEVICE_COMPILE__
#include <algorithm>
#endif
static inline uint32_t mift_thr16(double p) {
  if (p <= 0.0) return 0u;
  double t = p * 65536.0 + 0.5;
  return (uint32_t)(t > 65536.0 ? 65536.0 : t);
}
static inline float mift_inv_keep(double p) {
  const uint32_t t = mift_thr16(p);
  return t >= 65536u ? 0.f : (float)(65536.0 / (65536.0 - (double)t));
}

// GPT-2 "gelu_new" (tanh approximation) and its derivative, in the sigmoid form
//   0.5·x·(1 + tanh(u)) = x·σ(2u),  u = k0·(x + k1·x³)
// = x / (1 + 2^(x·(c0 + c1·x²))): one v_exp_f32 + one v_rcp_f32 + 4 FMA-class ops
// (the tanh form needed an extra divide/negate chain; the MLP GEMM epilogues apply it to
// 25 M elements per layer, where it was the dominant VALU cost).  Saturates correctly:
// x -> -inf gives 2^+inf = inf -> σ = 0; x -> +inf gives σ = 1.
MIFT_HD float gelu_sig(float x, float x2) {
  constexpr float c0 = -2.3022081983f;    // -2·k0·log2(e)
  constexpr float c1 = -0.1029432396f;    // c0·k1
  const float e = __builtin_amdgcn_exp2f(x * __builtin_fmaf(c1, x2, c0));
  return __builtin_amdgcn_rcpf(1.f + e);
}
MIFT_HD float fast_tanh(float u) { return 1.f - __fdividef(2.f, 1.f + __expf(2.f * u)); }
MIFT_HD float gelu_tanh(float x) { return x * gelu_sig(x, x * x); }
MIFT_HD float gelu_tanh_grad(float x) {
  // d/dx x·σ(2u) = σ + x·σ(1-σ)·2u',  2u' = 2k0·(1 + 3k1·x²)
  constexpr float c2 = 1.5957691216057308f, c3 = 0.2140644488f;  // 2k0, 6·k0·k1
  const float x2 = x * x;
  const float s = gelu_sig(x, x2);
  return __builtin_fmaf(x * s * (1.f - s), __builtin_fmaf(c3, x2, c2), s);
}
MIFT_HD float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
MIFT_HD float gelu_erf_grad(float x) {
  float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// Lanes l and l ^ 16 (l ^ 32) combined through gfx950's v_permlane16_swap (v_permlane32_swap): a VALU
// exchange, where __shfl_xor at these distances is a ds_bpermute_b32 LDS round trip plus its lgkmcnt
// wait.  The swap of a register with itself leaves {own, partner} in the two results (in a
// lane-dependent order); max / + / | are commutative, so the results equal the __shfl_xor forms bit
// for bit.
MIFT_HD float xor16_max(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
MIFT_HD float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
MIFT_HD float xor16_add(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
MIFT_HD float xor32_add(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
MIFT_HD uint32_t xor16_or(uint32_t x) {
  const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  return (uint32_t)r[0] | (uint32_t)r[1];
}
MIFT_HD uint32_t xor32_or(uint32_t x) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return (uint32_t)r[0] | (uint32_t)r[1];
}

// wave64 reductions (DPP/shuffle handled by the compiler for __shfl_xor).
MIFT_HD float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
MIFT_HD float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blocks of NW waves; `scratch` needs NW floats of LDS.
template <int NW>
MIFT_HD float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (NW == 1) return v;
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) r += scratch[i];
  return r;
}

// In-launch cross-workgroup hand-off ("last block done"), the write-through form of the MI355X
// guide's Guideline 16: each block stores the values it hands off with mift_st_sc1 (sc1 stores go
// through the XCD's L2 to memory: no release fence, which would write back the whole L2 from every
// block — a per-thread __threadfence() here took lmhead_lse from 9 to 139 us and the optimizer stats
// from 14 to 28 us, profiles/r4/step_timeline_fence_per_thread.txt), waits for them, and calls this.
// It returns true in every thread of the block that arrives LAST; that block's lane 0 has taken an
// agent-scope acquire, so plain loads of the handed-off values after it are fresh.  Arrivals are
// counted in two levels — 8 group counters (block index mod 8), then one top counter taken by
// each group's last block: same-address agent atomics serialise at the memory side, and 2048
// blocks on one counter cost lmhead_lse ~24 us (profiles/r4/step_timeline_sc1_one_counter.txt).
// `counters` = MIFT_ARRIVE_INTS zero-initialised ints (each counter on a 128-B line of its own),
// reset by the arrivers; launches sharing them must be stream-ordered.
MIFT_HD void mift_st_sc1(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
MIFT_HD void mift_st_sc1(float2* p, float2 v) {
  const unsigned long long bits =
      (unsigned long long)__float_as_uint(v.x) | ((unsigned long long)__float_as_uint(v.y) << 32);
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The same hand-off for a group of n blocks sharing one counter (e.g. the K-splits of one output
// tile): true in every thread of the group's n-th arriving block, which has taken the acquire.
MIFT_HD bool mift_group_arrival(unsigned* counter, unsigned n, int* flag_lds) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int last = 0;
    if (__hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n - 1) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      last = 1;
    }
    *flag_lds = last;
  }
  __syncthreads();
  return *flag_lds != 0;
}

constexpr int MIFT_ARRIVE_INTS = 9 * 32;
// 16-B write-through store: a buffer store with the sc1 bit (aux 16) at byte offset `off` of the
// buffer at `base` (wave-uniform), for hand-offs of tiles (the dword stores of mift_st_sc1 cost ~6x
// per byte).
MIFT_HD void mift_st16_sc1(float* base, uint32_t off, float4_ v) {
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  v4u32 u;
  __builtin_memcpy(&u, &v, 16);
  __builtin_amdgcn_raw_buffer_store_b128(u, rsrc, (int)off, 0, 16);
}

MIFT_HD bool mift_last_block_arrival(unsigned* counters, int* flag_lds) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through stores are done
  __syncthreads();                                    // ... and every other wave's
  if (threadIdx.x == 0) {
    const unsigned nb = gridDim.x, g = blockIdx.x & 7u;
    const unsigned ng = nb < 8u ? nb : 8u, gsize = (nb - g + 7u) >> 3;
    unsigned* gc = counters + 32 * g;
    unsigned* top = counters + 32 * 8;
    int last = 0;
    if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
      __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1) {
        __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = 1;
      }
    }
    *flag_lds = last;
  }
  __syncthreads();
  return *flag_lds != 0;
}

// 8 packed 16-bit elements -> fp32
template <typename T>
MIFT_HD void unpack8(short8 v, float* out) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    short s = v[i];
    T t;
    __builtin_memcpy(&t, &s, 2);
    out[i] = (float)t;
  }
}

// Vector load/store of 8 elements (16 B per lane for 16-bit types, Guideline 13).
template <typename T>
MIFT_HD void load8(const T* p, float* out) {
  if constexpr (sizeof(T) == 4) {
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
    out[4] = b.x; out[5] = b.y; out[6] = b.z; out[7] = b.w;
  } else {
    short8 v = *reinterpret_cast<const short8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      short s = v[i];
      T t;
      __builtin_memcpy(&t, &s, 2);
      out[i] = (float)t;
    }
  }
}
template <typename T>
MIFT_HD void store8(T* p, const float* in) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(in[0], in[1], in[2], in[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(in[4], in[5], in[6], in[7]);
  } else {
    short8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      T t = (T)in[i];
      short s;
      __builtin_memcpy(&s, &t, 2);
      v[i] = s;
    }
    *reinterpret_cast<short8*>(p) = v;
  }
}

// 4 elements (8 B for 16-bit types).
template <typename T>
MIFT_HD void load4(const T* p, float* out) {
  if constexpr (sizeof(T) == 4) {
    float4 a = *reinterpret_cast<const float4*>(p);
    out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
  } else {
    short4_ v = *reinterpret_cast<const short4_*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      short s = v[i];
      T t;
      __builtin_memcpy(&t, &s, 2);
      out[i] = (float)t;
    }
  }
}
template <typename T>
MIFT_HD void store4(T* p, const float* in) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(in[0], in[1], in[2], in[3]);
  } else {
    short4_ v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      T t = (T)in[i];
      short s;
      __builtin_memcpy(&s, &t, 2);
      v[i] = s;
    }
    *reinterpret_cast<short4_*>(p) = v;
  }
}
// keep bits of idx0..idx0+3 (idx0 even, all pairs with high word matching hm)
MIFT_HD void mift_keep4_hm(uint64_t seed, uint32_t hm, uint64_t idx0, uint32_t thr, bool* k) {
  const uint32_t lo = (uint32_t)(idx0 >> 1);
  const uint32_t h0 = mift_hash_lo(seed, hm, lo), h1 = mift_hash_lo(seed, hm, lo + 1);
  k[0] = (h0 & 0xFFFFu) >= thr; k[1] = (h0 >> 16) >= thr;
  k[2] = (h1 & 0xFFFFu) >= thr; k[3] = (h1 >> 16) >= thr;
}
// AND-masks of 8 consecutive packed 16-bit values at element idx0 (even): w[e] keeps element pair
// (2e, 2e+1) as 0x0000FFFF / 0xFFFF0000 halves.  Same keep decisions as mift_keep8; for kernels that
// apply the 1/(1-p) scale once to an fp32 accumulator instead of per element (hz: the pair index's
// high word is 0, hm0 = mift_hmix(seed, 0) hoisted by the caller).
MIFT_HD void mift_andmask8(uint64_t seed, uint32_t hm0, bool hz, uint64_t idx0, uint32_t thr, uint32_t* w) {
  const uint64_t pr = idx0 >> 1;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t h = hz ? mift_hash_lo(seed, hm0, (uint32_t)pr + e) : mift_hash_pair(seed, pr + e);
    w[e] = ((h & 0xFFFFu) >= thr ? 0x0000FFFFu : 0u) | ((h >> 16) >= thr ? 0xFFFF0000u : 0u);
  }
}
// bare v_exp_f32 (no denormal range handling; softmax inputs are <= 0 or -inf)
MIFT_HD float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

MIFT_HD void mift_keep4(uint64_t seed, uint64_t idx0, uint32_t thr, bool* k) {
  const uint32_t lo0 = (uint32_t)(idx0 >> 1);
  if ((idx0 & 1) == 0 && lo0 != 0xFFFFFFFFu) {
    // the two pairs share their high word: one hoisted mix (6 instead of 10 multiplies), bit-identical
    const uint32_t hm = mift_hmix(seed, (uint32_t)(idx0 >> 33));
    const uint32_t h0 = mift_hash_lo(seed, hm, lo0), h1 = mift_hash_lo(seed, hm, lo0 + 1);
    k[0] = (h0 & 0xFFFFu) >= thr; k[1] = (h0 >> 16) >= thr;
    k[2] = (h1 & 0xFFFFu) >= thr; k[3] = (h1 >> 16) >= thr;
  } else if ((idx0 & 1) == 0) {
    const uint32_t h0 = mift_hash_pair(seed, idx0 >> 1), h1 = mift_hash_pair(seed, (idx0 >> 1) + 1);
    k[0] = (h0 & 0xFFFFu) >= thr; k[1] = (h0 >> 16) >= thr;
    k[2] = (h1 & 0xFFFFu) >= thr; k[3] = (h1 >> 16) >= thr;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) k[e] = mift_keep(seed, idx0 + e, thr);
  }
}

#define MIFT_CHECK_HIP(expr)                                                        \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    TORCH_CHECK(_e == hipSuccess, "HIP error: ", hipGetErrorString(_e), " at ", #expr); \
  } while (0)
