// Throughput of the dropout counter hash (common.h mift_hash_lo: 3 x 32-bit multiplies per pair)
// vs a 24-bit-multiply candidate, one thread per pair, 64 pairs per thread, keep-count reduced.
//   hipcc --offload-arch=gfx950 -O3 tools/hip/hash_bench.hip -o /tmp/hash_bench && /tmp/hash_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
__device__ __forceinline__ uint32_t h_cur(uint32_t s0, uint32_t hm, uint32_t lo) {
  return mix32((lo * 0x9E3779B9U) ^ hm ^ s0);
}
__device__ __forceinline__ uint32_t mad24(uint32_t a, uint32_t b, uint32_t c) { return __umul24(a, b) + c; }
__device__ __forceinline__ uint32_t h_new(uint32_t s0, uint32_t s1, uint32_t lo) {
  uint32_t x = lo ^ s0;
  x ^= x >> 16; x = mad24(x, 0x9E3779u, s1);
  x ^= x >> 15; x = mad24(x, 0x2C1B3Cu, 0x7F4A7C15u);
  x ^= x >> 13; x = mad24(x, 0x297A2Du, 0x165667B1u);
  x ^= x >> 16;
  return x;
}
template <int V>
__global__ void k(uint32_t s0, uint32_t s1, uint32_t thr, unsigned* out, int iters) {
  uint32_t lo = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned cnt = 0;
  for (int i = 0; i < iters; ++i) {
    uint32_t h = V == 0 ? h_cur(s0, s1, lo + i * 7919u) : h_new(s0, s1, lo + i * 7919u);
    cnt += ((h & 0xFFFFu) >= thr) + ((h >> 16) >= thr);
  }
  atomicAdd(out, cnt);
}
int main() {
  unsigned* d; (void)hipMalloc(&d, 8); (void)hipMemset(d, 0, 8);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int blocks = 256 * 32, threads = 256, iters = 256;
  for (int rep = 0; rep < 3; ++rep)
    for (int v = 0; v < 2; ++v) {
      hipEventRecord(a);
      if (v == 0) k<0><<<blocks, threads>>>(0x1234567u, 0x89abcdefu, 6554, d, iters);
      else k<1><<<blocks, threads>>>(0x1234567u, 0x89abcdefu, 6554, d, iters);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      double pairs = (double)blocks * threads * iters;
      unsigned h; hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost); hipMemset(d, 0, 8);
      printf("%s: %.3f ms  %.1f G elements/s  keep=%.4f\n", v == 0 ? "mul32 hash" : "mul24 hash", ms,
             2 * pairs / ms / 1e6, h / (2 * pairs));
    }
  return 0;
}
