// K1: RMSNorm and fused residual-add + RMSNorm (Llama/Mixtral), LayerNorm (GPT-2).
//
// One workgroup per token row. The row is read ONCE with 16-byte loads and kept
// in registers (VPT chunks of 8 bf16 per thread), reduced with a wave64 xor
// butterfly + a 4-entry LDS step, then scaled and written with 16-byte stores.
// The fused variant reads x and residual, writes the new residual (bf16) and
// the normalised output in the same pass, so the residual stream is touched
// exactly once per sub-layer.
#include "common.h"

namespace xgk {

template <int VPT, bool FUSED>
__global__ void __launch_bounds__(256) rmsnorm_kernel(const uint16_t* __restrict__ x,
                                                      uint16_t* __restrict__ residual,
                                                      const uint16_t* __restrict__ w,
                                                      uint16_t* __restrict__ out, int H, float eps,
                                                      int64_t x_stride, int64_t out_stride) {
  __shared__ float red[8];
  const int row = blockIdx.x;
  const int nchunk = H >> 3;
  const uint16_t* xr = x + row * x_stride;
  uint16_t* rr = FUSED ? residual + static_cast<int64_t>(row) * H : nullptr;
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = threadIdx.x + k * blockDim.x;
    if (c < nchunk) {
      unpack8(ld16(xr + c * 8), v[k]);
      if constexpr (FUSED) {
        float r[8];
        unpack8(ld16(rr + c * 8), r);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[k][i] += r[i];
        // The residual stream is kept in bf16; normalise the rounded value so
        // every consumer of the residual sees the same numbers.
        uint4 pk = pack8(v[k]);
        st16(rr + c * 8, pk);
        unpack8(pk, v[k]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[k][i] * v[k][i];
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / static_cast<float>(H) + eps);
  uint16_t* orow = out + row * out_stride;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = threadIdx.x + k * blockDim.x;
    if (c < nchunk) {
      float wf[8], o[8];
      unpack8(ld16(w + c * 8), wf);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = v[k][i] * inv * wf[i];
      st16(orow + c * 8, pack8(o));
    }
  }
}

// LayerNorm with bias (GPT-2). Same structure, two moments.
template <int VPT>
__global__ void __launch_bounds__(256) layernorm_kernel(const uint16_t* __restrict__ x,
                                                        const uint16_t* __restrict__ w,
                                                        const uint16_t* __restrict__ b,
                                                        uint16_t* __restrict__ out, int H, float eps) {
  __shared__ float red[8];
  const int row = blockIdx.x;
  const int nchunk = H >> 3;
  const uint16_t* xr = x + static_cast<int64_t>(row) * H;
  float v[VPT][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = threadIdx.x + k * blockDim.x;
    if (c < nchunk) {
      unpack8(ld16(xr + c * 8), v[k]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[k][i];
    }
  }
  const float mean = block_sum(s, red) / H;
  float s2 = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = threadIdx.x + k * blockDim.x;
    if (c < nchunk)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float d = v[k][i] - mean;
        s2 += d * d;
      }
  }
  const float inv = rsqrtf(block_sum(s2, red) / H + eps);
  uint16_t* orow = out + static_cast<int64_t>(row) * H;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = threadIdx.x + k * blockDim.x;
    if (c < nchunk) {
      float wf[8], bf[8], o[8];
      unpack8(ld16(w + c * 8), wf);
      unpack8(ld16(b + c * 8), bf);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[k][i] - mean) * inv * wf[i] + bf[i];
      st16(orow + c * 8, pack8(o));
    }
  }
}

static int pick_threads(int nchunk, int& vpt) {
  int threads = nchunk >= 256 ? 256 : ((nchunk + 63) / 64) * 64;
  vpt = (nchunk + threads - 1) / threads;
  vpt = vpt <= 1 ? 1 : vpt <= 2 ? 2 : vpt <= 4 ? 4 : 8;
  return threads;
}

template <bool FUSED>
static void launch_rms(const uint16_t* x, uint16_t* res, const uint16_t* w, uint16_t* out, int T, int H,
                       float eps, int64_t xs, int64_t os, hipStream_t st) {
  int vpt;
  int thr = pick_threads(H / 8, vpt);
  dim3 g(T), b(thr);
  switch (vpt) {
    case 1: hipLaunchKernelGGL((rmsnorm_kernel<1, FUSED>), g, b, 0, st, x, res, w, out, H, eps, xs, os); break;
    case 2: hipLaunchKernelGGL((rmsnorm_kernel<2, FUSED>), g, b, 0, st, x, res, w, out, H, eps, xs, os); break;
    case 4: hipLaunchKernelGGL((rmsnorm_kernel<4, FUSED>), g, b, 0, st, x, res, w, out, H, eps, xs, os); break;
    default: hipLaunchKernelGGL((rmsnorm_kernel<8, FUSED>), g, b, 0, st, x, res, w, out, H, eps, xs, os); break;
  }
}

void rmsnorm(const uint16_t* x, const uint16_t* w, uint16_t* out, int T, int H, float eps, int64_t xs,
             int64_t os, hipStream_t st) {
  if (T > 0) launch_rms<false>(x, nullptr, w, out, T, H, eps, xs, os, st);
}

void fused_add_rmsnorm(const uint16_t* x, uint16_t* res, const uint16_t* w, uint16_t* out, int T, int H,
                       float eps, hipStream_t st) {
  if (T > 0) launch_rms<true>(x, res, w, out, T, H, eps, H, H, st);
}

// Per-row sum of squares (fp32) of bf16 [T, H] rows: the RMSNorm statistic the
// fused decode GEMMs apply as an epilogue row scale (layer 0's input).
__global__ void __launch_bounds__(256) row_sumsq_kernel(const uint16_t* __restrict__ x, float* __restrict__ ss,
                                                        int H) {
  __shared__ float red[8];
  const uint16_t* xr = x + static_cast<int64_t>(blockIdx.x) * H;
  float s = 0.f;
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) {
    float v[8];
    unpack8(ld16(xr + c * 8), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i] * v[i];
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) ss[blockIdx.x] = s;
}

void row_sumsq(const uint16_t* x, int T, int H, float* ss, hipStream_t st) {
  if (T > 0) hipLaunchKernelGGL(row_sumsq_kernel, dim3(T), dim3(256), 0, st, x, ss, H);
}

// K7: token-embedding gather, out[t] = table[ids[t]] (bf16 rows, 16 B per lane),
// optionally with the row's sum of squares (ss != nullptr: the fused decode
// layer's first RMSNorm statistic -- one launch instead of gather + row_sumsq).
// Ids outside [0, V) produce a zero row (never an out-of-bounds read).
__global__ void __launch_bounds__(256) embed_gather_kernel(const int32_t* __restrict__ ids,
                                                           const uint16_t* __restrict__ table,
                                                           uint16_t* __restrict__ out, float* __restrict__ ss, int H,
                                                           int V) {
  __shared__ float red[8];
  const int t = blockIdx.x;
  const int id = ids[t];
  const bool ok = id >= 0 && id < V;
  const uint16_t* src = table + static_cast<int64_t>(ok ? id : 0) * H;
  uint16_t* dst = out + static_cast<int64_t>(t) * H;
  float s = 0.f;
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) {
    uint4 v = ok ? ld16(src + c * 8) : make_uint4(0u, 0u, 0u, 0u);
    st16(dst + c * 8, v);
    if (ss != nullptr) {
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += f[i] * f[i];
    }
  }
  if (ss != nullptr) {
    s = block_sum(s, red);
    if (threadIdx.x == 0) ss[t] = s;
  }
}

void embed_gather(const int32_t* ids, int T, const uint16_t* table, int V, int H, uint16_t* out, float* ss,
                  hipStream_t st) {
  if (T > 0) hipLaunchKernelGGL(embed_gather_kernel, dim3(T), dim3(H >= 2048 ? 256 : 128), 0, st, ids, table, out, ss,
                                H, V);
}

void layernorm(const uint16_t* x, const uint16_t* w, const uint16_t* b, uint16_t* out, int T, int H,
               float eps, hipStream_t st) {
  if (T <= 0) return;
  int vpt;
  int thr = pick_threads(H / 8, vpt);
  dim3 g(T), blk(thr);
  switch (vpt) {
    case 1: hipLaunchKernelGGL(layernorm_kernel<1>, g, blk, 0, st, x, w, b, out, H, eps); break;
    case 2: hipLaunchKernelGGL(layernorm_kernel<2>, g, blk, 0, st, x, w, b, out, H, eps); break;
    case 4: hipLaunchKernelGGL(layernorm_kernel<4>, g, blk, 0, st, x, w, b, out, H, eps); break;
    default: hipLaunchKernelGGL(layernorm_kernel<8>, g, blk, 0, st, x, w, b, out, H, eps); break;
  }
}

}  // namespace xgk
