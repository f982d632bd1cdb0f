// K3: SiLU-gate (SwiGLU) and GELU-tanh (GPT-2 "gelu_new").
//
// silu_and_mul reads the fused gate_up GEMM output [T, 2F] (gate | up halves)
// and writes silu(gate) * up as [T, F]: one pass, 16-byte loads/stores, fp32 math.
// The grid is a flat grid-stride loop capped at 8 blocks/CU (Guideline 11).
#include "common.h"

namespace xgk {

// interleave16 != 0: the row is laid out in blocks of 16 as [g0..g15 u0..u15 g16..]
// (the layout the decode skinny GEMM's fused SiLU epilogue needs).
__global__ void __launch_bounds__(256) silu_and_mul_kernel(const uint16_t* __restrict__ in,
                                                           uint16_t* __restrict__ out, int T, int F,
                                                           int interleave16) {
  const int fc = F >> 3;  // chunks of 8 per row
  const int64_t total = static_cast<int64_t>(T) * fc;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t t = i / fc;
    const int c = static_cast<int>(i - t * fc);
    const uint16_t* row = in + t * 2 * F;
    const int f = c * 8;
    const int gi = interleave16 ? (f >> 4) * 32 + (f & 15) : f;
    const int ui = interleave16 ? gi + 16 : F + f;
    float g[8], u[8], o[8];
    unpack8(ld16(row + gi), g);
    unpack8(ld16(row + ui), u);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = g[k] / (1.f + __expf(-g[k])) * u[k];
    st16(out + t * F + c * 8, pack8(o));
  }
}

__global__ void __launch_bounds__(256) gelu_tanh_kernel(const uint16_t* __restrict__ in,
                                                        uint16_t* __restrict__ out, int64_t n8) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n8;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    float x[8], o[8];
    unpack8(ld16(in + i * 8), x);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float v = x[k];
      const float inner = 0.7978845608028654f * (v + 0.044715f * v * v * v);
      o[k] = 0.5f * v * (1.f + tanhf(inner));
    }
    st16(out + i * 8, pack8(o));
  }
}

static int grid_for(int64_t work) {
  int64_t g = (work + 255) / 256;
  return static_cast<int>(g < 2048 ? (g > 0 ? g : 1) : 2048);
}

void silu_and_mul(const uint16_t* in, uint16_t* out, int T, int F, int interleave16, hipStream_t st) {
  if (T <= 0) return;
  hipLaunchKernelGGL(silu_and_mul_kernel, dim3(grid_for(static_cast<int64_t>(T) * (F / 8))), dim3(256), 0,
                     st, in, out, T, F, interleave16);
}

void gelu_tanh(const uint16_t* in, uint16_t* out, int64_t n, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gelu_tanh_kernel, dim3(grid_for(n / 8)), dim3(256), 0, st, in, out, n / 8);
}

}  // namespace xgk
