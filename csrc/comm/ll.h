// Push ("LL") protocol lines shared by the custom all-reduce kernels
// (custom_allreduce.hip) and the GEMM epilogue that all-reduces in its own launch
// (gemm_m64g.hip GG_AR). Protocol description: custom_allreduce.hip, "Push".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../kernels/common.h"

namespace xgk {

constexpr int CAR_MAX_RANKS = 8;

struct LLLine {
  uint32_t d0, f0, d1, f1;
};

__device__ __forceinline__ void ll_store(uint8_t* dst, uint32_t d0, uint32_t d1, uint32_t gen) {
  u32x4_t v = {d0, gen, d1, gen};
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4_t*>(dst));
}

// Poll `n` lines at src (stride 16 B) until every flag equals gen; returns the
// payload words. Timeouts as car_wait (ctl[0] error counter, ctl[1] limit).
template <int N>
__device__ __forceinline__ bool ll_recv(const uint8_t* src, uint32_t gen, uint32_t* ctl, uint32_t (&d)[2 * N]) {
  uint32_t got = 0;  // bit i: line i has arrived
  uint64_t t0 = 0, limit = 0;
  uint32_t spins = 0;
  while (true) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if (got & (1u << i)) continue;
      // volatile: one real 16-B load per poll (a plain load may be hoisted out of the
      // spin and served from a register forever)
      typedef __attribute__((address_space(1))) const volatile u32x4_t gvec_t;
      const u32x4_t v = *(gvec_t*)(src + 16 * i);
      if (v[1] == gen && v[3] == gen) {
        d[2 * i] = v[0];
        d[2 * i + 1] = v[2];
        got |= 1u << i;
      }
    }
    if (got == (1u << N) - 1) return true;
    if (spins == 0) {
      if (__hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
      limit = __hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t0 = wall_clock64();
    }
    if ((++spins & 63) == 0) {
      if (__hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
      if (wall_clock64() - t0 > limit) {
        atomicAdd(ctl, 1u);
        return false;
      }
    }
  }
}

// Poll one line from each of the sources in `need` (bit r: source r, line at
// base + r * stride) until every one carries `gen`; all pending polls of a round are
// issued before any is tested, so the sources cost one memory round trip together
// instead of one each. d[r] = the two payload words of source r. Timeouts as ll_recv.
__device__ __forceinline__ bool ll_recv_multi(const uint8_t* base, int64_t stride, uint32_t need, uint32_t gen,
                                              uint32_t* ctl, uint32_t (&d)[CAR_MAX_RANKS][2]) {
  uint64_t t0 = 0, limit = 0;
  uint32_t spins = 0;
  typedef __attribute__((address_space(1))) const volatile u32x4_t gvec_t;
  while (need) {
    u32x4_t v[CAR_MAX_RANKS];
#pragma unroll
    for (int r = 0; r < CAR_MAX_RANKS; ++r)
      if (need & (1u << r)) v[r] = *(gvec_t*)(base + r * stride);
#pragma unroll
    for (int r = 0; r < CAR_MAX_RANKS; ++r)
      if ((need & (1u << r)) && v[r][1] == gen && v[r][3] == gen) {
        d[r][0] = v[r][0];
        d[r][1] = v[r][2];
        need &= ~(1u << r);
      }
    if (!need) return true;
    if (spins == 0) {
      if (__hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
      limit = __hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t0 = wall_clock64();
    }
    if ((++spins & 63) == 0) {
      if (__hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
      if (wall_clock64() - t0 > limit) {
        atomicAdd(ctl, 1u);
        return false;
      }
    }
  }
  return true;
}

}  // namespace xgk
