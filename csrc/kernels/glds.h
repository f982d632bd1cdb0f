// LDS-DMA pipeline helpers shared by the MFMA GEMMs (gemm_m64g.hip, gemm_tile.hip):
//   * global_load_lds_dwordx4 issued from inline asm -- hipcc's waitcnt pass does
//     not see it (with the builtin it serialises the DMAs of different slots:
//     vmcnt(0) between them and before every fragment read), so completion is
//     tracked ONLY by the explicit counted waits; "memory" keeps the compiler
//     from moving LDS reads across them. The LDS base goes in through a "{m0}"
//     operand, so the compiler writes M0 itself (no clobbered reserved register,
//     which hipcc flags as undefined behaviour); the s_nop 0 at the head of the
//     statement is the M0-write -> LDS-DMA wait state, which the hazard
//     recognizer does not insert in front of inline asm (cdna_hip_programming.md §5.7);
//   * counted s_waitcnt vmcnt(N) and a raw s_barrier (never __syncthreads inside
//     a pipelined loop: its fence drains the DMA queue);
//   * the write-through (sc1) 16-B store of in-launch hand-offs (Guideline 16 R1).
#pragma once

#include "common.h"

namespace xgk {

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)(lds_base))));
  asm volatile(
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :
      : "v"(src), "{m0}"(lds)
      : "memory");
#endif
}

// non-temporal weight stream (read once per step: keeps the activations in L2)
__device__ __forceinline__ void glds16_nt(const void* src, void* lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)(lds_base))));
  asm volatile(
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off nt"
      :
      : "v"(src), "{m0}"(lds)
      : "memory");
#endif
}

// device-coherent (sc1) LDS-DMA: reads data another workgroup of the same launch
// published with write-through stores, past this XCD's possibly stale L2 lines
__device__ __forceinline__ void glds16_sc1(const void* src, void* lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)(lds_base))));
  asm volatile(
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off sc1"
      :
      : "v"(src), "{m0}"(lds)
      : "memory");
#endif
}

// s_waitcnt vmcnt(N) (expcnt, lgkmcnt left at max)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#endif
}

__device__ __forceinline__ void raw_barrier() {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_barrier" ::: "memory");
#endif
}

// Write-through (sc1) 16-B store: visible chip-wide once the storing wave's vmcnt
// drains, so a hand-off ticket after it needs no release fence. Not counted by
// hipcc: the caller's explicit vmcnt(0) covers it; s_nop 1 keeps the next
// instruction from overwriting the data registers before the store reads them.
__device__ __forceinline__ void st16_sc1(float* p, f32x4_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
#endif
}

// 8-B and 4-B write-through stores (same contract as st16_sc1)
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;
__device__ __forceinline__ void st8_sc1(void* p, uint2 v) {
#if defined(__HIP_DEVICE_COMPILE__)
  const u32x2_t w = {v.x, v.y};
  asm volatile("global_store_dwordx2 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
#endif
}
__device__ __forceinline__ void st16u_sc1(void* p, uint4 v) {
#if defined(__HIP_DEVICE_COMPILE__)
  const u32x4_t w = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
#endif
}
__device__ __forceinline__ void st4_sc1(float* p, float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("global_store_dword %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
#endif
}

}  // namespace xgk
