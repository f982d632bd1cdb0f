// LDS-DMA streaming probe (diagnostics for the persistent decode kernel's loader):
// one workgroup per CU, ONE wave issuing global_load_lds_dwordx4 (1 KiB per
// instruction) into an LDS ring, keeping DEPTH instructions in flight with counted
// vmcnt waits. Each workgroup streams its own contiguous slice of a large buffer
// (the loader's access pattern). Prints GB/s per CU and chip TB/s per depth, for
// 1 and 2 loader waves per workgroup.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/dma_probe bench/dma_probe.hip && /tmp/dma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void glds16_nt(const void* src, void* lds_base) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)(lds_base))));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt" : : "v"(src), "s"(lds) : "memory");
}

template <int DEPTH, int LOADERS>
__global__ void __launch_bounds__(256, 1) probe(const uint8_t* __restrict__ buf, int64_t lines_per_wg, int* sink) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave >= LOADERS) return;
  const uint8_t* base = buf + static_cast<int64_t>(blockIdx.x) * lines_per_wg * 1024 + lane * 16;
  uint8_t* ring = smem + wave * 64 * 1024;
  int rp = 0;
  for (int64_t j = wave; j < lines_per_wg; j += LOADERS) {
    glds16_nt(base + j * 1024, ring + rp * 1024);
    rp = (rp + 1) & 63;
    if ((j / LOADERS & 7) == 7) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH - 8) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0 && smem[wave * 64 * 1024 + 5] == 123) sink[0] = 1;
}

template <int DEPTH, int LOADERS>
int run(const uint8_t* buf, int64_t lines, int ncu, int* sink) {
  hipFuncSetAttribute(reinterpret_cast<const void*>(probe<DEPTH, LOADERS>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      160 * 1024);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int it = 0; it < 3; ++it) {
    hipEventRecord(a);
    hipLaunchKernelGGL((probe<DEPTH, LOADERS>), dim3(ncu), dim3(256), LOADERS * 64 * 1024, 0, buf, lines, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    if (it == 2)
      printf("{\"depth\": %d, \"loaders\": %d, \"MB_per_cu\": %.1f, \"us\": %.1f, \"GBps_per_cu\": %.1f, \"chip_TBps\": %.2f}\n",
             DEPTH, LOADERS, lines / 1024.0, ms * 1000, lines * 1024.0 / (ms * 1e6), ncu * lines * 1024.0 / (ms * 1e9));
  }
  return 0;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int64_t lines = 16 * 1024;  // 16 MiB per CU, 4 GiB total
  uint8_t* buf;
  int* sink;
  CHECK(hipMalloc(&buf, static_cast<size_t>(ncu) * lines * 1024));
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMemset(buf, 1, static_cast<size_t>(ncu) * lines * 1024));
  run<16, 1>(buf, lines, ncu, sink);
  run<32, 1>(buf, lines, ncu, sink);
  run<48, 1>(buf, lines, ncu, sink);
  run<56, 1>(buf, lines, ncu, sink);
  run<32, 2>(buf, lines, ncu, sink);
  run<56, 2>(buf, lines, ncu, sink);
  CHECK(hipDeviceSynchronize());
  return 0;
}
