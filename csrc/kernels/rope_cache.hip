// K2 + K4: rotary embedding fused with the paged KV-cache append.
//
// Input is the QKV projection of each token, either as a bf16 row
// [q (Hq*D) | k (Hkv*D) | v (Hkv*D)] or as the fp32 split-K partial sums of the
// decode skinny GEMM ([S, T, (Hq+2Hkv)*D], reduced here in the prologue). In
// one pass per token:
//   * q is rotated and written to q_out (in place for the bf16 input, so
//     attention reads it straight from the QKV buffer);
//   * k is rotated and scattered into the paged K cache at slot_mapping[t];
//   * v is scattered into the paged V cache.
// Rotation is the Llama "rotate_half" form on (x[d], x[d+D/2]) pairs with a
// precomputed fp32 [max_pos, D] table = [cos | sin] (Appendix B: never compute
// trig on device). Every access is 16 B per lane: a work item is 8 pairs.
// Cache layout: [num_blocks, Hkv, block_size, D] -- a (page, kv-head) is one
// contiguous block_size*D run, which is what the attention kernels stream.
// slot_mapping < 0 marks padding tokens (graph-padded decode batch) that must
// not write the cache.
#include "common.h"

namespace xgk {

struct QkvSrc {
  const uint16_t* row_bf16;  // bf16 QKV buffer (or null)
  int64_t row_stride;
  const float* part;         // fp32 partials [S, T, width] (or null)
  int S, T, width;
};

// SP > 0: exactly SP partials (all loads issued before the adds -- a runtime
// trip count would serialise them into S dependent L2 round trips);
// SP == 0: runtime S; SP < 0: bf16 row source.
template <int SP>
__device__ __forceinline__ void qkv_load8(const QkvSrc& src, int t, int col, float* f) {
  if constexpr (SP < 0) {
    unpack8(ld16(src.row_bf16 + static_cast<int64_t>(t) * src.row_stride + col), f);
  } else if constexpr (SP == 0) {
    for (int i = 0; i < 8; ++i) f[i] = 0.f;
    for (int s = 0; s < src.S; ++s) {
      const float* p = src.part + (static_cast<int64_t>(s) * src.T + t) * src.width + col;
      const float4 a = *reinterpret_cast<const float4*>(p);
      const float4 b = *reinterpret_cast<const float4*>(p + 4);
      f[0] += a.x; f[1] += a.y; f[2] += a.z; f[3] += a.w;
      f[4] += b.x; f[5] += b.y; f[6] += b.z; f[7] += b.w;
    }
  } else {
    float4 a[SP], b[SP];
#pragma unroll
    for (int s = 0; s < SP; ++s) {
      const float* p = src.part + (static_cast<int64_t>(s) * src.T + t) * src.width + col;
      a[s] = *reinterpret_cast<const float4*>(p);
      b[s] = *reinterpret_cast<const float4*>(p + 4);
    }
    for (int i = 0; i < 8; ++i) f[i] = 0.f;
#pragma unroll
    for (int s = 0; s < SP; ++s) {
      f[0] += a[s].x; f[1] += a[s].y; f[2] += a[s].z; f[3] += a[s].w;
      f[4] += b[s].x; f[5] += b[s].y; f[6] += b[s].z; f[7] += b[s].w;
    }
  }
}

constexpr int ROPE_THREADS = 128;

// grid (T, ceil(items / ROPE_THREADS)): one work item per thread, so a decode
// batch of 64 tokens still spreads over ~256 workgroups.
template <int D, int SP>
__global__ void __launch_bounds__(ROPE_THREADS) rope_cache_kernel(QkvSrc src, uint16_t* __restrict__ q_out, int64_t q_stride,
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
  const int slot = slot_mapping[t];
  const int64_t page = slot >= 0 ? slot / block_size : 0;
  const int off = slot >= 0 ? slot % block_size : 0;
  const int pos = positions[t];
  const float* cs = cos_sin + static_cast<int64_t>(pos) * D;
  const int n_rope = (Hq + Hkv) * CPH;
  const int n_all = n_rope + Hkv * VPH;
  const bool inplace_q = SP < 0 && q_out == src.row_bf16;
  const int it = blockIdx.y * ROPE_THREADS + threadIdx.x;
  if (it >= n_all) return;
  {
    if (it < n_rope) {
      const int h = it / CPH, c = it % CPH;
      if (h >= Hq && slot < 0) return;
      if (h < Hq && inplace_q && !apply_rope) return;
      float a[8], b[8];
      qkv_load8<SP>(src, t, h * D + c * 8, a);
      qkv_load8<SP>(src, t, h * D + HALF + c * 8, b);
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
        uint16_t* qd = q_out + static_cast<int64_t>(t) * q_stride + h * D;
        st16(qd + c * 8, pa);
        st16(qd + HALF + c * 8, pb);
      } else {
        const int kh = h - Hq;
        uint16_t* dst = k_cache + ((page * Hkv + kh) * block_size + off) * D;
        st16(dst + c * 8, pa);
        st16(dst + HALF + c * 8, pb);
      }
    } else if (slot >= 0) {
      const int j = it - n_rope;
      const int kh = j / VPH, c = j % VPH;
      uint16_t* dst = v_cache + ((page * Hkv + kh) * block_size + off) * D + c * 8;
      if constexpr (SP >= 0) {
        float f[8];
        qkv_load8<SP>(src, t, (Hq + Hkv + kh) * D + c * 8, f);
        st16(dst, pack8(f));
      } else {
        st16(dst, ld16(src.row_bf16 + static_cast<int64_t>(t) * src.row_stride + (Hq + Hkv + kh) * D + c * 8));
      }
    }
  }
}

template <int D, int SP>
static void launch_rope_t(dim3 g, QkvSrc src, uint16_t* q_out, int64_t q_stride, const int32_t* positions,
                          const float* cos_sin, uint16_t* k_cache, uint16_t* v_cache, const int32_t* slot_mapping,
                          int Hq, int Hkv, int block_size, int apply_rope, hipStream_t st) {
  hipLaunchKernelGGL((rope_cache_kernel<D, SP>), g, dim3(ROPE_THREADS), 0, st, src, q_out, q_stride, positions,
                     cos_sin, k_cache, v_cache, slot_mapping, Hq, Hkv, block_size, apply_rope);
}

template <int D>
static void launch_rope_d(dim3 g, QkvSrc src, uint16_t* q_out, int64_t q_stride, const int32_t* positions,
                          const float* cos_sin, uint16_t* k_cache, uint16_t* v_cache, const int32_t* slot_mapping,
                          int Hq, int Hkv, int block_size, int apply_rope, hipStream_t st) {
#define XGK_ROPE(SPV) launch_rope_t<D, SPV>(g, src, q_out, q_stride, positions, cos_sin, k_cache, v_cache, \
                                           slot_mapping, Hq, Hkv, block_size, apply_rope, st)
  if (src.part == nullptr) XGK_ROPE(-1);
  else if (src.S == 1) XGK_ROPE(1);
  else if (src.S == 2) XGK_ROPE(2);
  else if (src.S == 4) XGK_ROPE(4);
  else if (src.S == 8) XGK_ROPE(8);
  else XGK_ROPE(0);
#undef XGK_ROPE
}

static int launch_rope(QkvSrc src, uint16_t* q_out, int64_t q_stride, const int32_t* positions, const float* cos_sin,
                       uint16_t* k_cache, uint16_t* v_cache, const int32_t* slot_mapping, int T, int Hq, int Hkv,
                       int D, int block_size, int apply_rope, hipStream_t st) {
  if (T <= 0) return 0;
  if (D != 64 && D != 128) return -1;
  const int items = (Hq + Hkv) * (D / 16) + Hkv * (D / 8);
  dim3 g(T, (items + ROPE_THREADS - 1) / ROPE_THREADS);
  if (D == 64)
    launch_rope_d<64>(g, src, q_out, q_stride, positions, cos_sin, k_cache, v_cache, slot_mapping, Hq, Hkv,
                      block_size, apply_rope, st);
  else
    launch_rope_d<128>(g, src, q_out, q_stride, positions, cos_sin, k_cache, v_cache, slot_mapping, Hq, Hkv,
                       block_size, apply_rope, st);
  return 0;
}

int rope_cache(uint16_t* qkv, int64_t row_stride, const int32_t* positions, const float* cos_sin,
               uint16_t* k_cache, uint16_t* v_cache, const int32_t* slot_mapping, int T, int Hq, int Hkv,
               int D, int block_size, int apply_rope, hipStream_t st) {
  QkvSrc src{qkv, row_stride, nullptr, 0, 0, 0};
  return launch_rope(src, qkv, row_stride, positions, cos_sin, k_cache, v_cache, slot_mapping, T, Hq, Hkv, D,
                     block_size, apply_rope, st);
}

int rope_cache_partials(const float* part, int S, uint16_t* q_out, int64_t q_stride, const int32_t* positions,
                        const float* cos_sin, uint16_t* k_cache, uint16_t* v_cache, const int32_t* slot_mapping,
                        int T, int Hq, int Hkv, int D, int block_size, int apply_rope, hipStream_t st) {
  QkvSrc src{nullptr, 0, part, S, T, (Hq + 2 * Hkv) * D};
  return launch_rope(src, q_out, q_stride, positions, cos_sin, k_cache, v_cache, slot_mapping, T, Hq, Hkv, D,
                     block_size, apply_rope, st);
}

}  // namespace xgk
