// One-shot all-reduce over xGMI peer memory (tensor-parallel decode messages).
//
// MI355X has 7 point-to-point xGMI links per GPU (fully connected 8-GPU mesh).
// A ring all-reduce (RCCL) moves data hop by hop, one link at a time; for the
// small, latency-bound messages of TP decode (T*H*2 bytes, 8 KiB..1 MiB) it is
// dominated by per-hop latency. Here every rank reads all peers' buffers
// directly through IPC-mapped pointers, so all links are used concurrently and
// the reduction takes one kernel:
//
//   block b (fixed 16 KiB chunk of the message):
//     1. copy my chunk of the input into my IPC buffer slot (gen & 1)
//     2. release (system scope) and raise flag[me][b] = gen in every peer's
//        signal array
//     3. wait until every peer raised flag[peer][b] >= gen in mine
//     4. sum chunk b over ranks 0..W-1 in fixed rank order (bit-identical
//        results on every rank) with fp32 accumulation; write the output
//   gen is a per-block counter kept in device memory, so the kernel is HIP
//   graph capturable (no host-side sequence number). gens[CAR_MAX_BLOCKS]
//   counts peer-wait timeouts (a missing peer never hangs the GPU).
//
// Double buffering (slot = gen & 1) makes reuse safe: before a block writes slot
// s at generation g, every peer has passed generation g-1 of the same block,
// hence finished reading generation g-2 (the previous user of slot s).
// Buffers and signals are allocated uncached (hipDeviceMallocUncached) so peer
// reads never see stale cache lines; flags use system-scope atomics.
// Two-shot variant (car2_kernel) for larger messages (prefill, 512 KiB..32 MiB at
// TP >= 4): the message is split into W rank shards; block b of every rank
//   1. stages chunk b of every shard into its IPC slot, signals phase 0
//   2. reduces chunk b of its OWN shard over all ranks (rank order), writes the
//      result to its output and back into its own slot, signals phase 1
//   3. copies chunk b of every other shard (already reduced by its owner)
// so each xGMI link carries ~2n/W bytes instead of n (one-shot), and every rank
// ends with the same bits (each shard is reduced exactly once). It has its own
// slots, signal arrays and generation counters, so the one-shot and two-shot
// paths never share a buffer region (the double-buffering argument above holds
// per block index within each path).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../kernels/common.h"

namespace xgk {

constexpr int CAR_MAX_RANKS = 8;
constexpr int CAR_MAX_BLOCKS = 512;
constexpr int CAR_CHUNK = 16384;    // bytes per block
constexpr int CAR_THREADS = 256;    // 256 x 64 B = 16 KiB

struct CarPtrs {
  uint8_t* data[CAR_MAX_RANKS];     // each rank's buffer: 2 slots x max_bytes
  uint32_t* sig[CAR_MAX_RANKS];     // each rank's signal array [CAR_MAX_RANKS][CAR_MAX_BLOCKS]
};

template <typename T>
__device__ __forceinline__ void acc8(float* a, uint4 v);

template <>
__device__ __forceinline__ void acc8<uint16_t>(float* a, uint4 v) {  // bf16
  float f[8];
  unpack8(v, f);
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] += f[i];
}

template <typename T>
__global__ void __launch_bounds__(CAR_THREADS) car_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                          int64_t nbytes, int64_t slot_bytes, CarPtrs p, int rank,
                                                          int world, uint32_t* __restrict__ gens) {
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const uint32_t gen = gens[b] + 1;
  const int64_t base = static_cast<int64_t>(b) * CAR_CHUNK;
  const int64_t slot_off = (gen & 1) * slot_bytes;
  // 1. stage my chunk (4 x 16 B per thread)
  uint4 mine[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t off = base + (static_cast<int64_t>(i) * CAR_THREADS + t) * 16;
    if (off < nbytes) {
      mine[i] = ld16(in + off);
      st16(p.data[rank] + slot_off + off, mine[i]);
    }
  }
  // 2. publish: every thread makes its stores visible system-wide, then one
  //    thread per peer raises my flag in that peer's signal array
  __threadfence_system();
  __syncthreads();
  if (t < world && t != rank) {
    __hip_atomic_store(p.sig[t] + rank * CAR_MAX_BLOCKS + b, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for every peer's flag for this block
  if (t < world && t != rank) {
    const uint32_t* f = p.sig[rank] + t * CAR_MAX_BLOCKS + b;
    uint32_t spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < gen) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 24)) {  // ~1 s: a peer never arrived -- record it and bail out rather than hang
        atomicAdd(gens + CAR_MAX_BLOCKS, 1u);
        break;
      }
    }
  }
  __syncthreads();
  __threadfence_system();  // acquire side for every thread before reading peer data
  // 4. reduce in rank order
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t off = base + (static_cast<int64_t>(i) * CAR_THREADS + t) * 16;
    if (off >= nbytes) continue;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < world; ++r) {
      const uint4 v = (r == rank) ? mine[i] : ld16_nt(p.data[r] + slot_off + off);
      acc8<T>(a, v);
    }
    st16(out + off, pack8(a));
  }
  if (t == 0) gens[b] = gen;
}

template <typename T>
__device__ __forceinline__ void car_signal_wait(const CarPtrs& p, int phase, int rank, int world, int b,
                                                uint32_t gen, uint32_t* timeouts) {
  const int t = threadIdx.x;
  __threadfence_system();
  __syncthreads();
  const int64_t ph = static_cast<int64_t>(phase) * CAR_MAX_RANKS * CAR_MAX_BLOCKS;
  if (t < world && t != rank)
    __hip_atomic_store(p.sig[t] + ph + rank * CAR_MAX_BLOCKS + b, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (t < world && t != rank) {
    const uint32_t* f = p.sig[rank] + ph + t * CAR_MAX_BLOCKS + b;
    uint32_t spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < gen) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 24)) {
        atomicAdd(timeouts, 1u);
        break;
      }
    }
  }
  __syncthreads();
  __threadfence_system();
}

template <typename T>
__global__ void __launch_bounds__(CAR_THREADS) car2_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                           int64_t nbytes, int64_t shard, int64_t slot_bytes,
                                                           CarPtrs p, int rank, int world,
                                                           uint32_t* __restrict__ gens) {
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const uint32_t gen = gens[b] + 1;
  const int64_t slot_off = (gen & 1) * slot_bytes;
  const int64_t cbase = static_cast<int64_t>(b) * CAR_CHUNK;
  uint8_t* mine = p.data[rank] + slot_off;
  // 1. stage chunk b of every shard (loads first, then stores: W*4 x 16 B in flight)
  for (int s = 0; s < world; ++s) {
    uint4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t o = cbase + (static_cast<int64_t>(i) * CAR_THREADS + t) * 16;
      const int64_t g = s * shard + o;
      if (o < shard && g < nbytes) v[i] = ld16(in + g);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t o = cbase + (static_cast<int64_t>(i) * CAR_THREADS + t) * 16;
      const int64_t g = s * shard + o;
      if (o < shard && g < nbytes) st16(mine + g, v[i]);
    }
  }
  car_signal_wait<T>(p, 0, rank, world, b, gen, gens + CAR_MAX_BLOCKS);
  // 2. reduce my shard's chunk b in rank order
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t o = cbase + (static_cast<int64_t>(i) * CAR_THREADS + t) * 16;
    const int64_t g = rank * shard + o;
    if (o >= shard || g >= nbytes) continue;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < world; ++r) acc8<T>(a, ld16_nt(p.data[r] + slot_off + g));
    const uint4 y = pack8(a);
    st16(out + g, y);
    st16(mine + g, y);
  }
  car_signal_wait<T>(p, 1, rank, world, b, gen, gens + CAR_MAX_BLOCKS);
  // 3. gather every other shard's chunk b from its owner
  for (int s = 0; s < world; ++s) {
    if (s == rank) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t o = cbase + (static_cast<int64_t>(i) * CAR_THREADS + t) * 16;
      const int64_t g = s * shard + o;
      if (o < shard && g < nbytes) st16(out + g, ld16_nt(p.data[s] + slot_off + g));
    }
  }
  if (t == 0) gens[b] = gen;
}

int car_max_blocks() { return CAR_MAX_BLOCKS; }
int car_chunk() { return CAR_CHUNK; }
int car_max_ranks() { return CAR_MAX_RANKS; }

// bf16 only (the activation dtype of every TP model here); nbytes % 16 == 0.
int custom_allreduce(const void* in, void* out, int64_t nbytes, int64_t slot_bytes, const uintptr_t* data_ptrs,
                     const uintptr_t* sig_ptrs, int rank, int world, uint32_t* gens, hipStream_t st) {
  if (world < 2 || world > CAR_MAX_RANKS || rank < 0 || rank >= world) return 1;
  if (nbytes <= 0 || nbytes % 16 || nbytes > slot_bytes) return 1;
  const int64_t blocks = (nbytes + CAR_CHUNK - 1) / CAR_CHUNK;
  if (blocks > CAR_MAX_BLOCKS) return 1;
  CarPtrs p{};
  for (int r = 0; r < world; ++r) {
    p.data[r] = reinterpret_cast<uint8_t*>(data_ptrs[r]);
    p.sig[r] = reinterpret_cast<uint32_t*>(sig_ptrs[r]);
  }
  hipLaunchKernelGGL(car_kernel<uint16_t>, dim3(static_cast<unsigned>(blocks)), dim3(CAR_THREADS), 0, st,
                     static_cast<const uint8_t*>(in), static_cast<uint8_t*>(out), nbytes, slot_bytes, p, rank, world,
                     gens);
  return 0;
}

// Two-shot: the signal arrays passed here hold 2 phases x [CAR_MAX_RANKS][CAR_MAX_BLOCKS].
int custom_allreduce_2shot(const void* in, void* out, int64_t nbytes, int64_t slot_bytes, const uintptr_t* data_ptrs,
                           const uintptr_t* sig_ptrs, int rank, int world, uint32_t* gens, hipStream_t st) {
  if (world < 2 || world > CAR_MAX_RANKS || rank < 0 || rank >= world) return 1;
  if (nbytes <= 0 || nbytes % 16 || nbytes > slot_bytes) return 1;
  const int64_t shard = ((nbytes + world - 1) / world + 15) / 16 * 16;
  const int64_t blocks = (shard + CAR_CHUNK - 1) / CAR_CHUNK;
  if (blocks > CAR_MAX_BLOCKS) return 1;
  CarPtrs p{};
  for (int r = 0; r < world; ++r) {
    p.data[r] = reinterpret_cast<uint8_t*>(data_ptrs[r]);
    p.sig[r] = reinterpret_cast<uint32_t*>(sig_ptrs[r]);
  }
  hipLaunchKernelGGL(car2_kernel<uint16_t>, dim3(static_cast<unsigned>(blocks)), dim3(CAR_THREADS), 0, st,
                     static_cast<const uint8_t*>(in), static_cast<uint8_t*>(out), nbytes, shard, slot_bytes, p, rank,
                     world, gens);
  return 0;
}

// ---- IPC buffer management (host) ------------------------------------------
int car_alloc_uncached(int64_t bytes, void** ptr) {
  if (hipExtMallocWithFlags(ptr, static_cast<size_t>(bytes), hipDeviceMallocUncached) != hipSuccess) return 1;
  if (hipMemset(*ptr, 0, static_cast<size_t>(bytes)) != hipSuccess) return 1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

int car_ipc_handle(void* ptr, hipIpcMemHandle_t* h) { return hipIpcGetMemHandle(h, ptr) == hipSuccess ? 0 : 1; }

int car_ipc_open(const hipIpcMemHandle_t* h, void** ptr) {
  return hipIpcOpenMemHandle(ptr, *h, hipIpcMemLazyEnablePeerAccess) == hipSuccess ? 0 : 1;
}

int car_ipc_close(void* ptr) { return hipIpcCloseMemHandle(ptr) == hipSuccess ? 0 : 1; }

int car_free(void* ptr) { return hipFree(ptr) == hipSuccess ? 0 : 1; }

}  // namespace xgk
