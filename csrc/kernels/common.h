// Shared device helpers for the gfx950 (CDNA4) kernels.
//
// Conventions used by every kernel in csrc/kernels:
//   * wave64 everywhere (lane = threadIdx.x & 63), block sizes multiples of 64;
//   * bf16 is carried as raw uint16_t / packed in 16-byte vectors and converted
//     with shifts (bf16 -> f32) and the v_cvt_pk_bf16_f32 that a plain __bf16
//     cast lowers to (f32 -> bf16, RNE, NaN-preserving);
//   * every global access on a hot path is 16 B per lane (Guideline 13);
//   * kernels take raw device pointers + a hipStream_t; the host wrappers in
//     ops.cpp do shape checks before launch.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xgk {

typedef __attribute__((ext_vector_type(8))) short bf16x8_t;   // MFMA A/B fragment (16x16x32)
typedef __attribute__((ext_vector_type(4))) short bf16x4_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;     // MFMA C/D (16x16)
typedef __attribute__((ext_vector_type(16))) float f32x16_t;   // MFMA C/D (32x32)
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4_t;

struct alignas(16) u16x8 { uint16_t v[8]; };
struct alignas(8) u16x4 { uint16_t v[4]; };

__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float(static_cast<uint32_t>(u) << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, b);
}

typedef __bf16 bf16x2v_t __attribute__((ext_vector_type(2)));
typedef float f32x2v_t __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 pair (a low) in ONE v_cvt_pk_bf16_f32 (round to nearest
// even, as f2bf); the scalar-cast form compiled to two converts + shift + or
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2v_t{a, b}, bf16x2v_t));
}

__device__ __forceinline__ uint4 ld16(const void* p) { return *reinterpret_cast<const uint4*>(p); }

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
// non-temporal 16-B load: for weights streamed once per step (guide: nt-weights)
__device__ __forceinline__ uint4 ld16_nt(const void* p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void st16(void* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }

__device__ __forceinline__ void unpack8(uint4 v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2(f[0], f[1]);
  v.y = pack2(f[2], f[3]);
  v.z = pack2(f[4], f[5]);
  v.w = pack2(f[6], f[7]);
  return v;
}

// ---- wave / block reductions (wave64) -------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum; `red` must hold >= blockDim.x/64 floats. All threads get the result.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  __syncthreads();
  return t;
}

__device__ __forceinline__ bf16x4_t lds_read_tr16(const uint16_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(p));
#else
  return bf16x4_t{};
#endif
}

__device__ __forceinline__ f32x4_t mfma16x16x32(bf16x8_t a, bf16x8_t b, f32x4_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
#else
  return c;
#endif
}

__device__ __forceinline__ bf16x8_t as_frag(uint4 v) { return __builtin_bit_cast(bf16x8_t, v); }

}  // namespace xgk

#define XGK_CHECK_LAUNCH() (void)hipGetLastError()
