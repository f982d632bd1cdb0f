// K2 + K4: rotary embedding fused with the paged KV-cache append.
//
// Input is the QKV GEMM output row [q (Hq*D) | k (Hkv*D) | v (Hkv*D)] of each
// token. In one pass per token:
//   * q is rotated in place (attention reads it straight from the QKV buffer,
//     no copy);
//   * k is rotated and scattered into the paged K cache at slot_mapping[t];
//   * v is scattered into the paged V cache.
// Rotation is the Llama "rotate_half" form on (x[d], x[d+D/2]) pairs with a
// precomputed fp32 [max_pos, D] table = [cos | sin] (Appendix B: never compute
// trig on device). Every access is 16 B per lane: a work item is 8 pairs.
// Cache layout: [num_blocks, Hkv, block_size, D] -- a (page, kv-head) is one
// contiguous block_size*D run, which is what the attention kernels stream.
// slot_mapping < 0 marks padding tokens (CUDA-graph-style padded decode batch)
// that must not write the cache.
#include "common.h"

namespace xgk {

template <int D>
__global__ void __launch_bounds__(256) rope_cache_kernel(uint16_t* __restrict__ qkv, int64_t row_stride,
                                                         const int32_t* __restrict__ positions,
                                                         const float* __restrict__ cos_sin,
                                                         uint16_t* __restrict__ k_cache,
                                                         uint16_t* __restrict__ v_cache,
                                                         const int32_t* __restrict__ slot_mapping, int Hq,
                                                         int Hkv, int block_size, int apply_rope) {
  constexpr int HALF = D / 2;
  constexpr int CPH = HALF / 8;  // rope work items per head
  constexpr int VPH = D / 8;     // copy work items per head
  const int t = blockIdx.x;
  uint16_t* row = qkv + static_cast<int64_t>(t) * row_stride;
  const int slot = slot_mapping[t];
  const int64_t page = slot >= 0 ? slot / block_size : 0;
  const int off = slot >= 0 ? slot % block_size : 0;
  const int pos = positions[t];
  const float* cs = cos_sin + static_cast<int64_t>(pos) * D;
  const int n_rope = (Hq + Hkv) * CPH;
  const int n_all = n_rope + Hkv * VPH;
  for (int it = threadIdx.x; it < n_all; it += blockDim.x) {
    if (it < n_rope) {
      const int h = it / CPH, c = it % CPH;
      uint16_t* base = row + h * D;
      float a[8], b[8];
      unpack8(ld16(base + c * 8), a);
      unpack8(ld16(base + HALF + c * 8), b);
      if (apply_rope) {
        const float4 c0 = *reinterpret_cast<const float4*>(cs + c * 8);
        const float4 c1 = *reinterpret_cast<const float4*>(cs + c * 8 + 4);
        const float4 s0 = *reinterpret_cast<const float4*>(cs + HALF + c * 8);
        const float4 s1 = *reinterpret_cast<const float4*>(cs + HALF + c * 8 + 4);
        const float cv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float x1 = a[i], x2 = b[i];
          a[i] = x1 * cv[i] - x2 * sv[i];
          b[i] = x2 * cv[i] + x1 * sv[i];
        }
      }
      const uint4 pa = pack8(a), pb = pack8(b);
      if (h < Hq) {
        if (apply_rope) {
          st16(base + c * 8, pa);
          st16(base + HALF + c * 8, pb);
        }
      } else if (slot >= 0) {
        const int kh = h - Hq;
        uint16_t* dst = k_cache + ((page * Hkv + kh) * block_size + off) * D;
        st16(dst + c * 8, pa);
        st16(dst + HALF + c * 8, pb);
      }
    } else if (slot >= 0) {
      const int j = it - n_rope;
      const int kh = j / VPH, c = j % VPH;
      const uint16_t* src = row + (Hq + Hkv + kh) * D + c * 8;
      uint16_t* dst = v_cache + ((page * Hkv + kh) * block_size + off) * D + c * 8;
      st16(dst, ld16(src));
    }
  }
}

int rope_cache(uint16_t* qkv, int64_t row_stride, const int32_t* positions, const float* cos_sin,
               uint16_t* k_cache, uint16_t* v_cache, const int32_t* slot_mapping, int T, int Hq, int Hkv,
               int D, int block_size, int apply_rope, hipStream_t st) {
  if (T <= 0) return 0;
  dim3 g(T), b(256);
  switch (D) {
    case 64:
      hipLaunchKernelGGL(rope_cache_kernel<64>, g, b, 0, st, qkv, row_stride, positions, cos_sin, k_cache,
                         v_cache, slot_mapping, Hq, Hkv, block_size, apply_rope);
      return 0;
    case 128:
      hipLaunchKernelGGL(rope_cache_kernel<128>, g, b, 0, st, qkv, row_stride, positions, cos_sin, k_cache,
                         v_cache, slot_mapping, Hq, Hkv, block_size, apply_rope);
      return 0;
    default:
      return -1;
  }
}

}  // namespace xgk
