// K12: single-token decode attention over a KV cache (greedy generation).
//
// Reference: HF ``generate(max_new_tokens=16)`` on distilgpt2 in the lab probe
// (`run_labs45_tiny_final.sbatch:80-82`) — each decode step is a
// forward over the KV cache.
//
// One 256-thread workgroup per (batch row, head).  The step's fused qkv row
// [B, 3*H*HD] (straight from the qkv GEMM) supplies q and the NEW k/v, which
// are (a) appended to the cache at position t and (b) used directly for key t
// (never re-read from the cache inside this launch).  Cache layout
// [B, H, Tmax, HD] keeps one head's keys contiguous, so the score pass is one
// thread per key with 16-B row loads and the P·V pass maps threads to
// (head-dim lane, key group) so each wave reads whole V rows coalesced.
// Padding, two layouts: left padding — keys < start[b] are masked (HF left-padded batched
// generate); or a prompt GAP — the prefill ran the prompts right-aligned to position 0 through the
// flash kernel (kv_len = prompt length), so row b's cache holds its prompt at [0, plen[b]) and the
// generated tokens from gend on: keys in [plen[b], gend) are masked.
// Decode is HBM/latency bound (B·H·t·HD·2·2 bytes per layer): no MFMA.
#include "common.h"
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

namespace {

template <typename T, int HD>
__global__ __launch_bounds__(256) void decode_attn_kernel(const T* __restrict__ qkv, T* __restrict__ kc,
                                                          T* __restrict__ vc, T* __restrict__ out,
                                                          const int* __restrict__ start,
                                                          const int* __restrict__ plen, int gend, int H, int Tmax,
                                                          int t_arg, const int* __restrict__ t_dev, float scale) {
  // t_dev: the position lives on the device (graph-replayed decode steps advance it in-graph)
  const int t = t_dev ? t_dev[0] : t_arg;
  constexpr int G = 256 / HD;  // key groups in the P·V pass
  constexpr int NC = HD / 8;   // 16-B pieces per K / V row
  extern __shared__ float sm[];
  float* qs = sm;              // [HD]
  float* red = qs + HD;        // [G*HD] (also used for the block reductions)
  T* vs = reinterpret_cast<T*>(red + G * HD);  // [256][HD]: V rows of keys 0..255 (16-B aligned)
  float* sc = reinterpret_cast<float*>(vs + 256 * HD);  // [t+1]
  const int bh = blockIdx.x, b = bh / H, h = bh % H, tid = threadIdx.x;
  const int64_t ld = 3LL * H * HD;
  const T* qg = qkv + (int64_t)b * ld + h * HD;
  const T* kg = qg + (int64_t)H * HD;
  const T* vg = qg + 2LL * H * HD;
  T* kcb = kc + (int64_t)bh * Tmax * HD;
  T* vcb = vc + (int64_t)bh * Tmax * HD;
  const int s0 = start ? start[b] : 0;
  const int g0 = plen ? plen[b] : gend;  // masked gap [g0, gend)
  // Every global read of keys 0..255 is issued here, before the first barrier: thread j holds key j's
  // K row in registers and stages its V row in LDS, so a short context (every decode step of the
  // distilgpt2 probe) pays one memory latency instead of three dependent ones (q -> K rows -> V rows).
  // Key t (the new token) comes from the qkv row, never from the cache written in this launch.
  const int j0 = tid;
  const bool live0 = j0 <= t && j0 >= s0 && (j0 < g0 || j0 >= gend);
  short8 kr[NC];
  if (live0) {
    const T* krow = (j0 == t) ? kg : kcb + (int64_t)j0 * HD;
    const T* vrow = (j0 == t) ? vg : vcb + (int64_t)j0 * HD;
#pragma unroll
    for (int c = 0; c < NC; ++c) kr[c] = *reinterpret_cast<const short8*>(krow + c * 8);
#pragma unroll
    for (int c = 0; c < NC; ++c)
      *reinterpret_cast<short8*>(vs + j0 * HD + c * 8) = *reinterpret_cast<const short8*>(vrow + c * 8);
  }
  for (int i = tid; i < HD; i += 256) {
    qs[i] = (float)qg[i] * scale;
    kcb[(int64_t)t * HD + i] = kg[i];
    vcb[(int64_t)t * HD + i] = vg[i];
  }
  __syncthreads();
  float mx = -INFINITY;
  for (int j = tid; j <= t; j += 256) {
    float s = -INFINITY;
    if (j >= s0 && (j < g0 || j >= gend)) {
      s = 0.f;
      if (j == j0) {  // the prefetched row
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          float kv[8];
          unpack8<T>(kr[c], kv);
#pragma unroll
          for (int e = 0; e < 8; ++e) s += qs[c * 8 + e] * kv[e];
        }
      } else {
        const T* krow = (j == t) ? kg : kcb + (int64_t)j * HD;
#pragma unroll
        for (int c = 0; c < HD; c += 8) {
          float kv[8];
          load8<T>(krow + c, kv);
#pragma unroll
          for (int e = 0; e < 8; ++e) s += qs[c + e] * kv[e];
        }
      }
    }
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  const int lane = tid & 63, w = tid >> 6;
  if (lane == 0) red[w] = mx;
  __syncthreads();
  const float M = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int j = tid; j <= t; j += 256) {
    const float p = sc[j] == -INFINITY ? 0.f : __expf(sc[j] - M);
    sc[j] = p;
    sum += p;
  }
  sum = wave_sum(sum);
  if (lane == 0) red[w] = sum;
  __syncthreads();
  const float inv = 1.f / (red[0] + red[1] + red[2] + red[3]);
  __syncthreads();
  const int d = tid % HD, g = tid / HD;
  float acc = 0.f;
  if (g < G) {
    for (int j = s0 + g; j <= t; j += G) {
      if (j >= g0 && j < gend) continue;  // gap keys: p = 0, their V rows are never read
      const float vj = j < 256 ? (float)vs[j * HD + d]
                               : (float)((j == t) ? vg : vcb + (int64_t)j * HD)[d];
      acc += sc[j] * vj;
    }
    red[g * HD + d] = acc;
  }
  __syncthreads();
  if (g == 0) {
    float o = 0.f;
#pragma unroll
    for (int k = 0; k < G; ++k) o += red[k * HD + d];
    out[(int64_t)b * H * HD + h * HD + d] = (T)(o * inv);
  }
}

template <typename T, int HD>
void launch(const at::Tensor& qkv, at::Tensor& kc, at::Tensor& vc, at::Tensor& out, const int* start, const int* plen,
            int gend, int B, int H, int Tmax, int t, const int* t_dev, float scale, hipStream_t st) {
  constexpr int G = 256 / HD;
  // q, the reduction scratch, the staged V rows of keys 0..255, then the score buffer for keys [0, t]
  // (a device-side t is only bounded by the cache)
  const size_t smem = (size_t)(HD + G * HD) * sizeof(float) + (size_t)256 * HD * sizeof(T) +
                      (size_t)(t_dev ? Tmax : t + 1) * sizeof(float);
  static bool attr = false;
  if (!attr) {  // up to ~130 KB at HD 128 with a device-side position
    (void)hipFuncSetAttribute((const void*)decode_attn_kernel<T, HD>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((decode_attn_kernel<T, HD>), dim3(B * H), dim3(256), smem, st, (const T*)qkv.data_ptr(),
                     (T*)kc.data_ptr(), (T*)vc.data_ptr(), (T*)out.data_ptr(), start, plen, gend, H, Tmax, t, t_dev,
                     scale);
}

}  // namespace

// qkv [B, 3*H*HD]; kc/vc [B, H, Tmax, HD] (row t written); start [B] int32 or None; plen [B] int32 or
// None with gend: keys in [plen[b], gend) masked -> o [B, H*HD].  t_dev: optional int32 [1] device
// tensor holding the position (t is then only the host-side lower bound; the caller keeps
// gend <= t_dev < Tmax — graph-replayed decode steps advance it in-graph, infer/generate.py).
at::Tensor mift_decode_attn(const at::Tensor& qkv, at::Tensor& kc, at::Tensor& vc, int64_t t, double scale,
                            const c10::optional<at::Tensor>& start, const c10::optional<at::Tensor>& plen,
                            int64_t gend, const c10::optional<at::Tensor>& t_dev) {
  TORCH_CHECK(qkv.is_cuda() && qkv.is_contiguous() && qkv.dim() == 2, "decode_attn: qkv [B, 3*H*HD] contiguous");
  TORCH_CHECK(kc.is_contiguous() && vc.is_contiguous() && kc.dim() == 4 && kc.sizes() == vc.sizes(),
              "decode_attn: caches [B,H,Tmax,HD]");
  TORCH_CHECK(kc.scalar_type() == qkv.scalar_type() && vc.scalar_type() == qkv.scalar_type(), "decode_attn: dtype");
  const int B = kc.size(0), H = kc.size(1), Tmax = kc.size(2), HD = kc.size(3);
  TORCH_CHECK(qkv.size(0) == B && qkv.size(1) == 3LL * H * HD, "decode_attn: qkv/cache shape mismatch");
  const int* td = nullptr;
  if (t_dev && t_dev->defined()) {
    TORCH_CHECK(t_dev->is_cuda() && t_dev->scalar_type() == at::kInt && t_dev->numel() == 1,
                "decode_attn: t_dev int32 [1] GPU tensor");
    TORCH_CHECK(Tmax <= 16384, "decode_attn: cache too long for the LDS score buffer");
    td = t_dev->data_ptr<int>();
  }
  TORCH_CHECK(t >= 0 && t < Tmax, "decode_attn: position ", t, " outside cache of ", Tmax);
  TORCH_CHECK(t < 16384, "decode_attn: context too long for the LDS score buffer");
  const int* sp = nullptr;
  if (start) {
    TORCH_CHECK(start->scalar_type() == at::kInt && start->numel() == B && start->is_cuda(), "decode_attn: start");
    sp = start->data_ptr<int>();
  }
  const int* pl = nullptr;
  if (plen) {
    TORCH_CHECK(plen->scalar_type() == at::kInt && plen->numel() == B && plen->is_cuda(), "decode_attn: plen");
    TORCH_CHECK(gend >= 0 && gend <= t, "decode_attn: gap end must be <= t");
    pl = plen->data_ptr<int>();
  }
  auto out = at::empty({B, H * HD}, qkv.options());
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  const bool half = qkv.scalar_type() == at::kHalf;
  TORCH_CHECK(half || qkv.scalar_type() == at::kBFloat16, "decode_attn: bf16/fp16");
#define MIFT_DEC(D)                                                                        \
  case D:                                                                                  \
    if (half) launch<fp16, D>(qkv, kc, vc, out, sp, pl, (int)gend, B, H, Tmax, (int)t, td, (float)scale, st); \
    else launch<bf16, D>(qkv, kc, vc, out, sp, pl, (int)gend, B, H, Tmax, (int)t, td, (float)scale, st);      \
    break;
  switch (HD) {
    MIFT_DEC(32) MIFT_DEC(64) MIFT_DEC(80) MIFT_DEC(128)
    default: TORCH_CHECK(false, "decode_attn: unsupported head dim ", HD);
  }
#undef MIFT_DEC
  return out;
}

namespace {

// ---- greedy decode step tail: ONE launch for what was ~12 small torch kernels per step ----
// Per row b (one block): next = argmax(logits[b, :V]) — the first index of the maximum, NaN counting
// as maximal (torch.argmax); a finished row emits pad; out[b, col[b]] = token; done[b] |= token == eos
// (eos >= 0); the next step's input ids[b] = done ? fill : token; col, pos advance; block 0 advances
// the cache position t.  16-B logit loads (row stride % 8 == 0), scalar tail.
// Order-preserving integer key of a logit: NaN maximal (torch.argmax), -0 == +0, otherwise the float
// order.  The first version compared (value, index) with early returns for the NaN cases; hipcc kept
// them as two divergent branches per element (decode_tail 13.8 us for 64 x 50257 logits): integer keys
// compile to compares and selects only.
MIFT_HD int argmax_key(float v) {
  const int b = __float_as_int(v);
  const int k = b >= 0 ? b : b ^ 0x7fffffff;
  return v != v ? 0x7fffffff : (v == 0.f ? 0 : k);
}

template <typename T, int NTH>
__global__ __launch_bounds__(NTH) void decode_tail_kernel(const T* __restrict__ logits, int64_t ldl, int V,
                                                          bool* __restrict__ done, int64_t* __restrict__ ids,
                                                          int64_t* __restrict__ out, int max_new,
                                                          int64_t* __restrict__ col, int64_t* __restrict__ pos,
                                                          int* __restrict__ t, int64_t fill, int64_t pad, int64_t eos) {
  // each thread's chunks loaded in batches of UN before any compare (one load in flight per thread
  // was a chain of dependent loads); a thread visits its elements in increasing index order, so a
  // strictly greater key keeps the first maximum; lanes and waves then tie-break on the index
  constexpr int UN = 8;
  __shared__ int sk[NTH / 64];
  __shared__ int si[NTH / 64];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const T* row = logits + (int64_t)b * ldl;
  int bk = (int)0x80000000, bi = 0x7fffffff;
  const int nv = V / 8;
  // this row's bookkeeping inputs, requested before the scan (consumed by thread 0 at the end)
  bool d0 = false;
  int64_t c = 0, p0 = 0;
  int t0 = 0;
  if (tid == 0) {
    d0 = done[b];
    c = col[b];
    p0 = pos[b];
    if (b == 0) t0 = t[0];
  }
  for (int c0 = tid; c0 < nv; c0 += NTH * UN) {
    short8 v[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int ch = min(c0 + u * NTH, nv - 1);  // clamped: a repeated chunk never wins (not greater)
      v[u] = *reinterpret_cast<const short8*>(row + (int64_t)ch * 8);
    }
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      float f[8];
      unpack8<T>(v[u], f);
      const int base = min(c0 + u * NTH, nv - 1) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = argmax_key(f[e]);
        const bool gt = k > bk;
        bk = gt ? k : bk;
        bi = gt ? base + e : bi;
      }
    }
  }
  for (int j = nv * 8 + tid; j < V; j += NTH) {
    const int k = argmax_key((float)row[j]);
    const bool gt = k > bk;
    bk = gt ? k : bk;
    bi = gt ? j : bi;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int ok = __shfl_xor(bk, o, 64), oi = __shfl_xor(bi, o, 64);
    const bool bt = ok > bk || (ok == bk && oi < bi);
    bk = bt ? ok : bk;
    bi = bt ? oi : bi;
  }
  if (lane == 0) { sk[w] = bk; si[w] = bi; }
  __syncthreads();
  if (tid == 0) {
#pragma unroll
    for (int q = 1; q < NTH / 64; ++q) {
      const bool bt = sk[q] > bk || (sk[q] == bk && si[q] < bi);
      bk = bt ? sk[q] : bk;
      bi = bt ? si[q] : bi;
    }
    const int64_t tok = d0 ? pad : (int64_t)bi;
    if (c >= 0 && c < max_new) out[(int64_t)b * max_new + c] = tok;
    const bool d = d0 || (eos >= 0 && tok == eos);
    done[b] = d;
    ids[b] = d ? fill : tok;
    col[b] = c + 1;
    pos[b] = p0 + 1;
    if (b == 0) t[0] = t0 + 1;
  }
}

}  // namespace

void mift_decode_tail(const at::Tensor& logits, int64_t V, at::Tensor& done, at::Tensor& ids, at::Tensor& out,
                      at::Tensor& col, at::Tensor& pos, at::Tensor& t, int64_t fill, int64_t pad, int64_t eos) {
  const int64_t B = logits.size(0);
  TORCH_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1 && logits.size(1) >= V,
              "decode_tail: logits [B, >= V], unit column stride");
  TORCH_CHECK(logits.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(logits.data_ptr()) % 16 == 0,
              "decode_tail: 16-B aligned logit rows");
  TORCH_CHECK(done.scalar_type() == at::kBool && done.numel() == B && done.is_contiguous(), "decode_tail: done [B] bool");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.numel() == B && ids.is_contiguous(), "decode_tail: ids [B] int64");
  TORCH_CHECK(out.scalar_type() == at::kLong && out.dim() == 2 && out.size(0) == B && out.is_contiguous(),
              "decode_tail: out [B, max_new] int64");
  TORCH_CHECK(col.scalar_type() == at::kLong && col.numel() == B && col.is_contiguous(), "decode_tail: col [B] int64");
  TORCH_CHECK(pos.scalar_type() == at::kLong && pos.numel() == B && pos.is_contiguous(), "decode_tail: pos [B] int64");
  TORCH_CHECK(t.scalar_type() == at::kInt && t.numel() >= 1, "decode_tail: t int32[1]");
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  auto launch = [&](auto tag) {
    using T = decltype(tag);
    // block size: MIFT_TAIL_NTH (A/B, read per call) — 256 / 512 / 1024 threads per row
    const char* e = getenv("MIFT_TAIL_NTH");
    const int nth = e ? atoi(e) : 1024;
    auto go = [&](auto kern, int threads) {
      kern<<<(unsigned)B, threads, 0, st>>>(
          reinterpret_cast<const T*>(logits.data_ptr()), logits.stride(0), (int)V, done.data_ptr<bool>(),
          ids.data_ptr<int64_t>(), out.data_ptr<int64_t>(), (int)out.size(1), col.data_ptr<int64_t>(),
          pos.data_ptr<int64_t>(), t.data_ptr<int>(), fill, pad, eos);
    };
    if (nth == 256) go(decode_tail_kernel<T, 256>, 256);
    else if (nth == 512) go(decode_tail_kernel<T, 512>, 512);
    else go(decode_tail_kernel<T, 1024>, 1024);
  };
  if (logits.scalar_type() == at::kBFloat16) launch(bf16{});
  else {
    TORCH_CHECK(logits.scalar_type() == at::kHalf, "decode_tail: bf16 / fp16 logits");
    launch(fp16{});
  }
}

namespace {

// ---- prefill: the prompt's K / V rows into the caches, both in one launch ----
// qkv [B*S, 3*H*HD] (row b*S + s), caches [B, H, Tmax, HD]: rows [0, S) of every (b, h).  One thread
// per 16-B piece of the destination; replaces two strided torch copies per layer.
template <typename T>
__global__ __launch_bounds__(256) void kv_store_kernel(const T* __restrict__ qkv, T* __restrict__ kc,
                                                       T* __restrict__ vc, int B, int S, int H, int HD, int Tmax) {
  const int npc = HD / 8;  // pieces per row
  const int64_t per = (int64_t)B * H * S * npc;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= 2 * per) return;
  const bool isv = i >= per;
  int64_t r = isv ? i - per : i;
  const int c = (int)(r % npc);
  r /= npc;
  const int s = (int)(r % S);
  r /= S;
  const int h = (int)(r % H);
  const int b = (int)(r / H);
  const int64_t d = (int64_t)H * HD;
  const T* src = qkv + ((int64_t)b * S + s) * 3 * d + (isv ? 2 : 1) * d + (int64_t)h * HD + c * 8;
  T* dst = (isv ? vc : kc) + (((int64_t)b * H + h) * Tmax + s) * HD + c * 8;
  *reinterpret_cast<short8*>(dst) = *reinterpret_cast<const short8*>(src);
}

}  // namespace

// qkv [B*S, 3*H*HD] -> kc / vc [B, H, Tmax, HD] rows [0, S)
void mift_kv_store(const at::Tensor& qkv, at::Tensor& kc, at::Tensor& vc, int64_t S) {
  TORCH_CHECK(qkv.is_cuda() && qkv.is_contiguous() && qkv.dim() == 2, "kv_store: qkv [B*S, 3*H*HD] contiguous");
  TORCH_CHECK(kc.is_contiguous() && vc.is_contiguous() && kc.dim() == 4 && kc.sizes() == vc.sizes(),
              "kv_store: caches [B,H,Tmax,HD]");
  TORCH_CHECK(kc.scalar_type() == qkv.scalar_type() && vc.scalar_type() == qkv.scalar_type(), "kv_store: dtype");
  const int B = kc.size(0), H = kc.size(1), Tmax = kc.size(2), HD = kc.size(3);
  TORCH_CHECK(S >= 1 && S <= Tmax && qkv.size(0) == (int64_t)B * S && qkv.size(1) == 3LL * H * HD,
              "kv_store: shapes");
  TORCH_CHECK(HD % 8 == 0, "kv_store: head dim % 8");
  const int64_t n = 2LL * B * H * S * (HD / 8);
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  auto go = [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(kv_store_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       (const T*)qkv.data_ptr(), (T*)kc.data_ptr(), (T*)vc.data_ptr(), B, (int)S, H, HD, Tmax);
  };
  if (qkv.scalar_type() == at::kBFloat16) go(bf16{});
  else {
    TORCH_CHECK(qkv.scalar_type() == at::kHalf, "kv_store: bf16 / fp16");
    go(fp16{});
  }
}
