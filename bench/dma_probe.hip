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
#include <vector>

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

// The persistent kernel's pattern: per layer four weight matrices (separate
// allocations, Llama-3-8B shapes), each workgroup streaming its contiguous row slice
// of each in turn (all workgroups in the same matrix at the same time).
template <int LOADERS>
__global__ void __launch_bounds__(256, 1) probe_model(const uint8_t* const* __restrict__ mats, const int64_t* __restrict__ slice,
                                                     int nmat, int* sink) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave >= LOADERS) return;
  uint8_t* ring = smem + wave * 64 * 1024;
  int rp = 0, n = 0;
  for (int m = 0; m < nmat; ++m) {
    const int64_t lines = slice[m & 3];
    const uint8_t* base = mats[m] + static_cast<int64_t>(blockIdx.x) * lines * 1024 + lane * 16;
    for (int64_t j = wave; j < lines; j += LOADERS) {
      glds16_nt(base + j * 1024, ring + rp * 1024);
      rp = (rp + 1) & 63;
      if ((++n & 7) == 0) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0 && smem[wave * 64 * 1024 + 5] == 123) sink[0] = 1;
}

template <int LOADERS>
int run_model(int ncu, int* sink) {
  const int L = 32;
  const int64_t rows[4] = {6144, 4096, 28672, 4096}, kk[4] = {4096, 4096, 4096, 14336};
  std::vector<uint8_t*> hm(4 * L);
  int64_t slice[4];
  int64_t total = 0;
  for (int p = 0; p < 4; ++p) slice[p] = rows[p] * kk[p] * 2 / 1024 / ncu;
  for (int i = 0; i < 4 * L; ++i) {
    const size_t bytes = rows[i & 3] * kk[i & 3] * 2;
    if (hipMalloc(&hm[i], bytes) != hipSuccess) return 1;
    hipMemset(hm[i], 1, bytes);
    total += bytes;
  }
  uint8_t** dm;
  int64_t* ds;
  hipMalloc(&dm, sizeof(uint8_t*) * 4 * L);
  hipMalloc(&ds, sizeof(slice));
  hipMemcpy(dm, hm.data(), sizeof(uint8_t*) * 4 * L, hipMemcpyHostToDevice);
  hipMemcpy(ds, slice, sizeof(slice), hipMemcpyHostToDevice);
  hipFuncSetAttribute(reinterpret_cast<const void*>(probe_model<LOADERS>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      160 * 1024);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int it = 0; it < 3; ++it) {
    hipEventRecord(a);
    hipLaunchKernelGGL((probe_model<LOADERS>), dim3(ncu), dim3(256), LOADERS * 64 * 1024, 0, dm, ds, 4 * L, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    if (it == 2)
      printf("{\"pattern\": \"model\", \"loaders\": %d, \"GB\": %.2f, \"us\": %.1f, \"chip_TBps\": %.2f}\n", LOADERS,
             total / 1e9, ms * 1000, total / (ms * 1e9));
  }
  for (auto p : hm) hipFree(p);
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
  CHECK(hipFree(buf));
  run_model<1>(ncu, sink);
  run_model<2>(ncu, sink);
  CHECK(hipDeviceSynchronize());
  return 0;
}
