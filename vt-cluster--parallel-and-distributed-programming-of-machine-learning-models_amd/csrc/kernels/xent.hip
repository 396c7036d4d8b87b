// K7: causal-LM cross-entropy over [M, V] logits with the gradient produced
// in the same launch (the loss is the graph's last node, so dL/dlogits is
// known at forward time).
//
// One 256-thread block per row: pass 1 = online (max, sum-exp) over the row
// with 16-B loads; pass 2 = overwrite the row in place with
// softmax - onehot(label) (unscaled; the LM-head dgrad GEMM applies the
// upstream gradient / loss scale through its device-side alpha).  Rows
// whose label == ignore_index get loss 0 and a zero gradient row; padded
// vocabulary columns [V, ldV) are written as zeros so the dgrad GEMM over
// the padded K dimension is exact.
// Reference semantics: HF shifted CE with ignore_index=-100 (GPT-2) /
// pad id (OPT OPTHead, P2/finetune_lora_opt_pp.py:143-152).
#include "common.h"
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

namespace {

template <typename T>
__global__ __launch_bounds__(256) void xent_kernel(T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                   float* __restrict__ loss, float* __restrict__ lse_out, int V,
                                                   int ldV, int64_t ignore_index, int write_grad) {
  __shared__ float sm[8], ss[8];
  const int row = blockIdx.x;
  T* x = logits + (int64_t)row * ldV;
  const int tid = threadIdx.x;
  float m = -INFINITY, s = 0.f;
  const int Vv = V & ~7;
  for (int c = tid * 8; c < Vv; c += 256 * 8) {
    float v[8];
    load8<T>(x + c, v);
    float lm = v[0];
#pragma unroll
    for (int e = 1; e < 8; ++e) lm = fmaxf(lm, v[e]);
    float nm = fmaxf(m, lm);
    float acc = s * __expf(m - nm);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += __expf(v[e] - nm);
    m = nm;
    s = acc;
  }
  for (int c = Vv + tid; c < V; c += 256) {
    float v = (float)x[c];
    float nm = fmaxf(m, v);
    s = s * __expf(m - nm) + __expf(v - nm);
    m = nm;
  }
  // block combine of (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  const int lane = tid & 63, w = tid >> 6;
  if (lane == 0) { sm[w] = m; ss[w] = s; }
  __syncthreads();
  float M = sm[0];
  for (int i = 1; i < 4; ++i) M = fmaxf(M, sm[i]);
  float Ssum = 0.f;
  for (int i = 0; i < 4; ++i) Ssum += ss[i] * __expf(sm[i] - M);
  const float lse = M + __logf(Ssum);
  const int64_t lab = labels[row];
  const bool valid = lab != ignore_index && lab >= 0 && lab < V;
  if (tid == 0) {
    float xl = valid ? (float)x[lab] : 0.f;
    loss[row] = valid ? (lse - xl) : 0.f;
    if (lse_out) lse_out[row] = lse;
  }
  if (!write_grad) return;
  __syncthreads();  // everyone has read x[lab] before it is overwritten
  for (int c = tid * 8; c < ldV; c += 256 * 8) {
    float v[8];
    if (c + 8 <= Vv) {
      load8<T>(x + c, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float p = valid ? __expf(v[e] - lse) : 0.f;
        if (valid && c + e == lab) p -= 1.f;
        v[e] = p;
      }
      store8<T>(x + c, v);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        int cc = c + e;
        if (cc >= ldV) break;
        float p = 0.f;
        if (cc < V && valid) {
          p = __expf((float)x[cc] - lse);
          if (cc == lab) p -= 1.f;
        }
        x[cc] = (T)p;
      }
    }
  }
}

// Single-pass variant: the row lives in registers (NV 16-B vectors per
// thread, 512 threads -> rows up to NV*4096 wide), so HBM traffic is one read
// + one write of the logits (the 2-pass kernel above reads twice).
template <typename T, int NV>
__global__ __launch_bounds__(512) void xent_reg_kernel(T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       float* __restrict__ loss, float* __restrict__ lse_out, int V,
                                                       int ldV, int64_t ignore_index, int write_grad) {
  __shared__ float red[8];
  __shared__ float lab_logit;
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  T* x = logits + (int64_t)row * ldV;
  short8 v[NV];
  float m = -INFINITY;
  // Only the chunk holding column V-1 needs the per-element `< V` test; every
  // other chunk takes the branch-free path (keeps the ALU work per logit near
  // its floor of ~2 exp + ~10 ops).
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 512 + tid) * 8;
    if (c < ldV) {
      v[k] = *reinterpret_cast<const short8*>(x + c);
      float f[8];
      load8<T>(reinterpret_cast<const T*>(&v[k]), f);
      if (c + 8 <= V) {
#pragma unroll
        for (int e = 0; e < 8; ++e) m = fmaxf(m, f[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (c + e < V) m = fmaxf(m, f[e]);
      }
    }
  }
  const int64_t lab = labels[row];
  const bool valid = lab != ignore_index && lab >= 0 && lab < V;
  if (tid == 0) lab_logit = valid ? (float)x[lab] : 0.f;
  m = wave_max(m);
  if (lane == 0) red[w] = m;
  __syncthreads();
  float M = red[0];
#pragma unroll
  for (int i = 1; i < 8; ++i) M = fmaxf(M, red[i]);
  __syncthreads();
  // exp(f - M) = exp2(f*log2e - M*log2e): one FMA feeding v_exp_f32
  constexpr float L2E = 1.4426950408889634f;
  const float Ml = M * L2E;
  // Pass 2 overwrites each register vector with e = exp(f - M) rounded to T
  // (zero past V), so pass 3 is one multiply by 1/S per logit instead of a
  // second FMA + v_exp (softmax rel. error <= 2^-8, below the bf16 output's).
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 512 + tid) * 8;
    if (c < ldV) {
      float f[8];
      load8<T>(reinterpret_cast<const T*>(&v[k]), f);
      if (c + 8 <= V) {
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = __builtin_amdgcn_exp2f(fmaf(f[e], L2E, -Ml));
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = (c + e < V) ? __builtin_amdgcn_exp2f(fmaf(f[e], L2E, -Ml)) : 0.f;
      }
      short8 pk;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s += f[e];
        T t = (T)f[e];
        short sh;
        __builtin_memcpy(&sh, &t, 2);
        pk[e] = sh;
      }
      v[k] = pk;
    }
  }
  s = wave_sum(s);
  if (lane == 0) red[w] = s;
  __syncthreads();
  float S = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) S += red[i];
  const float lse = M + __logf(S);
  if (tid == 0) {
    loss[row] = valid ? (lse - lab_logit) : 0.f;
    if (lse_out) lse_out[row] = lse;
  }
  if (!write_grad) return;
  const float inv_s = valid ? 1.f / S : 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 512 + tid) * 8;
    if (c < ldV) {
      float f[8];
      load8<T>(reinterpret_cast<const T*>(&v[k]), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= inv_s;
      const unsigned d = (unsigned)(lab - c);
      if (valid && d < 8u) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if ((unsigned)e == d) f[e] -= 1.f;
      }
      store8<T>(x + c, f);
    }
  }
}

// NV = register vectors per thread (row width <= NV*4096); the exact-fit
// instantiations cover GPT-2 (50304 padded -> 13) and OPT (50272 -> 13).
template <typename T>
void xent_reg_launch(at::Tensor& logits, const at::Tensor& lab, at::Tensor& loss, at::Tensor& lse, int V, int ldV,
                     int nv, int64_t ignore_index, bool write_grad, int M, hipStream_t st) {
  T* x = reinterpret_cast<T*>(logits.data_ptr());
  const int64_t* l = lab.data_ptr<int64_t>();
  float* lo = loss.data_ptr<float>();
  float* ls = lse.data_ptr<float>();
  const int wg = write_grad ? 1 : 0;
#define XR(N) xent_reg_kernel<T, N><<<M, 512, 0, st>>>(x, l, lo, ls, V, ldV, ignore_index, wg)
  if (nv <= 1) XR(1);
  else if (nv <= 2) XR(2);
  else if (nv <= 4) XR(4);
  else if (nv <= 8) XR(8);
  else if (nv <= 12) XR(12);
  else if (nv == 13) XR(13);
  else XR(16);
#undef XR
}

}  // namespace

// logits [M, ldV] (modified in place into dlogits when write_grad) -> (loss[M], lse[M])
std::vector<at::Tensor> mift_xent_fwd_bwd(at::Tensor& logits, const at::Tensor& labels, int64_t V,
                                          int64_t ignore_index, bool write_grad) {
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "xent: 2-D row-major logits");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == logits.size(0), "xent: labels");
  const int M = logits.size(0), ldV = logits.stride(0);
  TORCH_CHECK(ldV % 8 == 0 && V <= logits.size(1), "xent: ldV % 8");
  auto loss = at::empty({M}, logits.options().dtype(at::kFloat));
  auto lse = at::empty({M}, logits.options().dtype(at::kFloat));
  if (M == 0) return {loss, lse};
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  auto lab = labels.contiguous();
  const int nv = (ldV + 4095) / 4096;
  const bool is_bf = logits.scalar_type() == at::kBFloat16, is_h = logits.scalar_type() == at::kHalf;
  if ((is_bf || is_h) && nv <= 16) {
    if (is_bf) xent_reg_launch<bf16>(logits, lab, loss, lse, (int)V, ldV, nv, ignore_index, write_grad, M, st);
    else xent_reg_launch<fp16>(logits, lab, loss, lse, (int)V, ldV, nv, ignore_index, write_grad, M, st);
    return {loss, lse};
  }
  if (logits.scalar_type() == at::kBFloat16)
    xent_kernel<bf16><<<M, 256, 0, st>>>((bf16*)logits.data_ptr(), lab.data_ptr<int64_t>(), loss.data_ptr<float>(),
                                         lse.data_ptr<float>(), (int)V, ldV, ignore_index, write_grad ? 1 : 0);
  else if (logits.scalar_type() == at::kHalf)
    xent_kernel<fp16><<<M, 256, 0, st>>>((fp16*)logits.data_ptr(), lab.data_ptr<int64_t>(), loss.data_ptr<float>(),
                                         lse.data_ptr<float>(), (int)V, ldV, ignore_index, write_grad ? 1 : 0);
  else
    xent_kernel<float><<<M, 256, 0, st>>>((float*)logits.data_ptr(), lab.data_ptr<int64_t>(), loss.data_ptr<float>(),
                                          lse.data_ptr<float>(), (int)V, ldV, ignore_index, write_grad ? 1 : 0);
  return {loss, lse};
}
