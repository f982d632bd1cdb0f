// Infinity-Cache (MALL) warm-up of a weight range ahead of its GEMM.
//
// Batch-1 decode leaves HBM idle while latency-bound kernels run (the attention +
// split combine of a layer: ~13 us of a ~90 us layer). A concurrent launch on a
// side stream (forked after the QKV GEMM, joined before the O GEMM) reads the next
// projections' weights once so the 256 MiB memory-side cache holds them when the
// GEMM streams them. Every load is a 16-B non-temporal load (the XCD L2s keep the
// activations); the values feed one XOR that is stored only under a condition no
// launch meets, so the loads cannot be removed. Opt-in (XGS_MALL_PREFETCH).
#include "common.h"

namespace xgk {

__global__ void __launch_bounds__(256) mall_prefetch_kernel(const uint4* __restrict__ p, int64_t n16,
                                                            uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {  // four 16-B loads in flight per lane
    const uint4 a = ld16_nt(p + i), b = ld16_nt(p + i + stride);
    const uint4 c = ld16_nt(p + i + 2 * stride), d = ld16_nt(p + i + 3 * stride);
    acc ^= a.x ^ b.y ^ c.z ^ d.w;
  }
  for (; i < n16; i += stride) acc ^= ld16_nt(p + i).x;
  if (acc == 0x9E3779B9u && threadIdx.x == 0xFFFF) sink[0] = acc;  // never: keeps the loads
}

void mall_prefetch(const void* p, int64_t bytes, int blocks, uint32_t* sink, hipStream_t st) {
  const int64_t n16 = bytes / 16;
  if (n16 <= 0 || blocks <= 0) return;
  hipLaunchKernelGGL(mall_prefetch_kernel, dim3(blocks), dim3(256), 0, st, static_cast<const uint4*>(p), n16, sink);
}

}  // namespace xgk
