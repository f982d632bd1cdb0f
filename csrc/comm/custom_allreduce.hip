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
//   graph capturable (no host-side sequence number). A peer wait that times out
//   (the limit in ctl[1], see car_wait) bumps the device error counter ctl[0] and gives up instead of hanging
//   the GPU; the host reads the counter after every step (CustomAllReduce.check)
//   and fails the step, so a missing peer is an error, never a wrong sum.
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
#include "ll.h"

namespace xgk {

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

// Peer waits: ctl[0] counts timeouts (the host polls it after every step),
// ctl[1] is the wait limit in wall-clock ticks (wall_clock64, the device's constant
// real-time counter; the host writes it -- generous during warmup / graph capture,
// the configured collective timeout afterwards -- and captured graphs read the
// current value on every replay). A wait gives up at once when ctl[0] is already
// non-zero: after the first timeout of a step every later collective of that step
// returns immediately instead of spinning its own full limit, so a dead peer is
// reported within one limit, not one limit per collective.
__device__ __forceinline__ bool car_wait(const uint32_t* f, uint32_t gen, uint32_t* ctl) {
  if (__hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
  const uint64_t limit = __hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t t0 = wall_clock64();
  uint32_t spins = 0;
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < gen) {
    __builtin_amdgcn_s_sleep(2);
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

template <typename T>
__global__ void __launch_bounds__(CAR_THREADS) car_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                          int64_t nbytes, int64_t slot_bytes, CarPtrs p, int rank,
                                                          int world, uint32_t* __restrict__ gens,
                                                          uint32_t* __restrict__ err) {
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
    car_wait(f, gen, err);
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
    car_wait(f, gen, timeouts);
  }
  __syncthreads();
  __threadfence_system();
}

template <typename T>
__global__ void __launch_bounds__(CAR_THREADS) car2_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                           int64_t nbytes, int64_t shard, int64_t slot_bytes,
                                                           CarPtrs p, int rank, int world,
                                                           uint32_t* __restrict__ gens,
                                                           uint32_t* __restrict__ err) {
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const uint32_t gen = gens[b] + 1;
  const int64_t slot_off = (gen & 1) * slot_bytes;
  const int64_t cbase = static_cast<int64_t>(b) * CAR_CHUNK;
  // slot layout [block][shard][16 KiB]: block b's region is the same in every
  // launch whatever the message size (the per-block double-buffering argument)
  uint8_t* mine = p.data[rank] + slot_off;
  const int64_t bbase = static_cast<int64_t>(b) * world * CAR_CHUNK;
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
      const int64_t lo = (static_cast<int64_t>(i) * CAR_THREADS + t) * 16;
      const int64_t o = cbase + lo;
      const int64_t g = s * shard + o;
      if (o < shard && g < nbytes) st16(mine + bbase + s * CAR_CHUNK + lo, v[i]);
    }
  }
  car_signal_wait<T>(p, 0, rank, world, b, gen, err);
  // 2. reduce my shard's chunk b in rank order
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t lo = (static_cast<int64_t>(i) * CAR_THREADS + t) * 16;
    const int64_t o = cbase + lo;
    const int64_t g = rank * shard + o;
    if (o >= shard || g >= nbytes) continue;
    const int64_t so = bbase + rank * CAR_CHUNK + lo;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < world; ++r) acc8<T>(a, ld16_nt(p.data[r] + slot_off + so));
    const uint4 y = pack8(a);
    st16(out + g, y);
    st16(mine + so, y);
  }
  car_signal_wait<T>(p, 1, rank, world, b, gen, err);
  // 3. gather every other shard's chunk b from its owner
  for (int s = 0; s < world; ++s) {
    if (s == rank) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t lo = (static_cast<int64_t>(i) * CAR_THREADS + t) * 16;
      const int64_t o = cbase + lo;
      const int64_t g = s * shard + o;
      if (o < shard && g < nbytes) st16(out + g, ld16_nt(p.data[s] + slot_off + bbase + s * CAR_CHUNK + lo));
    }
  }
  if (t == 0) gens[b] = gen;
}

// Fused decode layer under TP (row-parallel O / down projections): one launch
// replaces reduce_partials -> all-reduce -> add + RMSNorm statistics.
//   block (t, chunk) owns row t, columns [chunk*1024, chunk*1024 + 1024) (128 lanes x 8):
//     1. sum this rank's S split-K fp32 partial slices, round to bf16 (the value
//        every rank contributes -- the message is bf16, as in the unfused path),
//        store into my IPC slot
//     2. signal / wait exactly as car_kernel (block index = t * nchunk + chunk)
//     3. resid = bf16(resid + sum over ranks in rank order) -- bit-identical on
//        every rank, so the replicated residual stream never diverges
//     4. the new residual's sum of squares -> ss_part[chunk * T + t] (the
//        RowStats layout of add_partials_resid: the next GEMM adds the H/1024
//        chunk sums in order and applies the RMSNorm as a row scale)
// T * H/1024 <= CAR_MAX_BLOCKS (decode: T <= 64, H <= 8192).
template <int SP>
__global__ void __launch_bounds__(128) car_resid_kernel(const float* __restrict__ part, int S, int T,
                                                        uint16_t* __restrict__ resid, float* __restrict__ ss_part,
                                                        int H, int64_t slot_bytes, CarPtrs p, int rank, int world,
                                                        uint32_t* __restrict__ gens, uint32_t* __restrict__ err) {
  __shared__ float red[2];
  const int t = blockIdx.x, chunk = blockIdx.y;
  const int b = t * gridDim.y + chunk;
  const int lane = threadIdx.x;
  const uint32_t gen = gens[b] + 1;
  const int64_t slot_off = (gen & 1) * slot_bytes;
  const int64_t e = static_cast<int64_t>(t) * H + (chunk * 128 + lane) * 8;  // element offset
  // 1. local split-K reduction -> bf16 contribution
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int ns = SP > 0 ? SP : S;
#pragma unroll
  for (int s = 0; s < ns; ++s) {
    const float* pp = part + static_cast<int64_t>(s) * T * H + e;
    const float4 a = *reinterpret_cast<const float4*>(pp);
    const float4 c = *reinterpret_cast<const float4*>(pp + 4);
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
    v[4] += c.x; v[5] += c.y; v[6] += c.z; v[7] += c.w;
  }
  const uint4 mine = pack8(v);
  const uint4 r_old = ld16(resid + e);
  st16(p.data[rank] + slot_off + e * 2, mine);
  // 2. publish + wait
  __threadfence_system();
  __syncthreads();
  if (lane < world && lane != rank)
    __hip_atomic_store(p.sig[lane] + rank * CAR_MAX_BLOCKS + b, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (lane < world && lane != rank) {
    const uint32_t* f = p.sig[rank] + lane * CAR_MAX_BLOCKS + b;
    car_wait(f, gen, err);
  }
  __syncthreads();
  __threadfence_system();
  // 3. cross-rank sum in rank order (all peer loads issued before the adds)
  uint4 pv[CAR_MAX_RANKS];
#pragma unroll
  for (int r = 0; r < CAR_MAX_RANKS; ++r)
    if (r < world) pv[r] = (r == rank) ? mine : ld16_nt(p.data[r] + slot_off + e * 2);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < CAR_MAX_RANKS; ++r)
    if (r < world) acc8<uint16_t>(acc, pv[r]);
  float ro[8];
  unpack8(r_old, ro);
#pragma unroll
  for (int i = 0; i < 8; ++i) ro[i] += acc[i];
  const uint4 pk = pack8(ro);
  st16(resid + e, pk);
  // 4. statistics of the stored (rounded) residual
  unpack8(pk, ro);
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) ss += ro[i] * ro[i];
  ss = block_sum(ss, red);
  if (lane == 0) {
    ss_part[static_cast<int64_t>(chunk) * T + t] = ss;
    gens[b] = gen;
  }
}

// ---------------------------------------------------------------------------------
// Push ("LL") protocol for latency-bound TP decode messages.
//
// The pull kernels above put a full synchronisation in front of the data: stage the
// message locally, fence system-wide, raise a flag in each peer, spin, fence again,
// then READ every peer's copy over xGMI -- a remote read round trip after the last
// flag arrives. Here each rank WRITES its contribution straight into every peer's
// receive region as 16-byte lines {d0, gen, d1, gen} (two 4-byte payload words, each
// carrying the generation): the receiver polls its OWN memory until both flags of a
// line equal the current generation. The flag travels in the same store as the data,
// so there is no fence, no separate flag word and no remote read; the cost is 2x the
// bytes on the wire, which is nothing at decode sizes (T * H * 2 bytes per rank).
//
// Receive region per rank: [2 parities][CAR_MAX_RANKS sources][lines]; a block's
// lines are at a fixed offset in every launch and parity = gen & 1, so the
// double-buffering argument of the pull kernels holds unchanged: before rank X writes
// parity p of block b at generation g into Y, X has received Y's generation g-1 of
// block b, which Y sent only after it finished reading generation g-2 (the previous
// user of parity p). The generation (not a toggling bit) in every line means a stale
// line of generation g-2 never matches.
// Fused residual all-reduce on the push protocol (same contract as car_resid_kernel:
// rank-ordered sum, bit-identical on every rank). Block (t, chunk), 128 lanes x 8
// elements; lane's 8 bf16 = 4 payload words = 2 lines per peer.
template <int SP>
__global__ void __launch_bounds__(128) car_ll_resid_kernel(const float* __restrict__ part, int S, int T,
                                                           uint16_t* __restrict__ resid, float* __restrict__ ss_part,
                                                           int H, int64_t region_bytes, CarPtrs p, int rank, int world,
                                                           uint32_t* __restrict__ gens, uint32_t* __restrict__ err,
                                                           int loop) {
  // loop (one-process --tp-shard simulation, comm.tp_allreduce_resid): every "peer"
  // region is this rank's own, lines go to source slot r and are polled but not added;
  // loop - 1 = a simulated link latency in wall-clock ticks
  __shared__ float red[2];
  const int t = blockIdx.x, chunk = blockIdx.y;
  const int b = t * gridDim.y + chunk;
  const int lane = threadIdx.x;
  const uint32_t gen = gens[b] + 1;
  const int64_t e = static_cast<int64_t>(t) * H + (chunk * 128 + lane) * 8;  // element offset
  // 1. local split-K reduction -> bf16 contribution (4 payload words)
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int ns = SP > 0 ? SP : S;
#pragma unroll
  for (int s = 0; s < ns; ++s) {
    const float* pp = part + static_cast<int64_t>(s) * T * H + e;
    const float4 a = *reinterpret_cast<const float4*>(pp);
    const float4 c = *reinterpret_cast<const float4*>(pp + 4);
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
    v[4] += c.x; v[5] += c.y; v[6] += c.z; v[7] += c.w;
  }
  const uint4 mine = pack8(v);
  const uint4 r_old = ld16(resid + e);
  // 2. push to every peer: lines at [parity][my rank][e / 4 .. + 2) of the peer's region
  const int64_t src_bytes = region_bytes / (2 * CAR_MAX_RANKS);  // per (parity, source)
  const int64_t line_off = (gen & 1) * (region_bytes / 2) + (e / 4) * 16;
  for (int r = 0; r < world; ++r) {
    if (r == rank) continue;
    uint8_t* dst = p.data[r] + line_off + static_cast<int64_t>(loop ? r : rank) * src_bytes;
    ll_store(dst, mine.x, mine.y, gen);
    ll_store(dst + 16, mine.z, mine.w, gen);
  }
  asm volatile("" ::: "memory");  // the pushes are issued before any poll
  if (loop > 1) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < static_cast<uint64_t>(loop - 1)) __builtin_amdgcn_s_sleep(1);
  }
  // 3. receive every peer's lines from my own region, sum in rank order
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  bool ok = true;
  for (int r = 0; r < world; ++r) {
    uint4 pv = mine;
    if (r != rank && ok) {
      uint32_t d[4];
      ok = ll_recv<2>(p.data[rank] + line_off + static_cast<int64_t>(r) * src_bytes, gen, err, d);
      if (loop) continue;
      pv = make_uint4(d[0], d[1], d[2], d[3]);
    }
    acc8<uint16_t>(acc, pv);
  }
  float ro[8];
  unpack8(r_old, ro);
#pragma unroll
  for (int i = 0; i < 8; ++i) ro[i] += acc[i];
  const uint4 pk = pack8(ro);
  st16(resid + e, pk);
  unpack8(pk, ro);
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) ss += ro[i] * ro[i];
  ss = block_sum(ss, red);
  if (lane == 0) {
    ss_part[static_cast<int64_t>(chunk) * T + t] = ss;
    gens[b] = gen;
  }
}

// Plain all-reduce (bf16, nbytes % 16 == 0) on the push protocol: block b owns the
// 16-byte groups [b * 256, b * 256 + 256) -- 4 KiB of message per block, 2 lines per
// group per peer.
constexpr int CAR_LL_GROUPS = 256;

__global__ void __launch_bounds__(CAR_LL_GROUPS) car_ll_kernel(const uint8_t* __restrict__ in,
                                                                uint8_t* __restrict__ out, int64_t nbytes,
                                                                int64_t region_bytes, CarPtrs p, int rank, int world,
                                                                uint32_t* __restrict__ gens,
                                                                uint32_t* __restrict__ err) {
  const int b = blockIdx.x;
  const uint32_t gen = gens[b] + 1;
  const int64_t grp = static_cast<int64_t>(b) * CAR_LL_GROUPS + threadIdx.x;
  const bool live = grp * 16 < nbytes;
  const int64_t src_bytes = region_bytes / (2 * CAR_MAX_RANKS);
  const int64_t line_off = (gen & 1) * (region_bytes / 2) + grp * 32;
  uint4 mine = make_uint4(0, 0, 0, 0);
  if (live) {
    mine = ld16(in + grp * 16);
    for (int r = 0; r < world; ++r) {
      if (r == rank) continue;
      uint8_t* dst = p.data[r] + line_off + static_cast<int64_t>(rank) * src_bytes;
      ll_store(dst, mine.x, mine.y, gen);
      ll_store(dst + 16, mine.z, mine.w, gen);
    }
    asm volatile("" ::: "memory");  // the pushes are issued before any poll
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    bool ok = true;
    for (int r = 0; r < world; ++r) {
      uint4 pv = mine;
      if (r != rank && ok) {
        uint32_t d[4];
        ok = ll_recv<2>(p.data[rank] + line_off + static_cast<int64_t>(r) * src_bytes, gen, err, d);
        pv = make_uint4(d[0], d[1], d[2], d[3]);
      }
      acc8<uint16_t>(acc, pv);
    }
    st16(out + grp * 16, pack8(acc));
  }
  __syncthreads();
  if (threadIdx.x == 0) gens[b] = gen;
}

int car_ll_max_bytes(int64_t region_bytes) {
  return static_cast<int>(region_bytes / (2 * CAR_MAX_RANKS) / 2);  // payload bytes per source line region
}

int custom_allreduce_resid_ll(const float* part, int S, int T, uint16_t* resid, float* ss_part, int H,
                              int64_t region_bytes, const uintptr_t* data_ptrs, int rank, int world, uint32_t* gens,
                              uint32_t* err, hipStream_t st, int loop) {
  if (world < 2 || world > CAR_MAX_RANKS || rank < 0 || rank >= world) return 1;
  if (T <= 0 || S <= 0 || H <= 0 || H % 1024) return 1;
  if (static_cast<int64_t>(T) * (H / 1024) > CAR_MAX_BLOCKS) return 1;
  if (static_cast<int64_t>(T) * H * 2 > car_ll_max_bytes(region_bytes)) return 1;
  CarPtrs p{};
  for (int r = 0; r < world; ++r) p.data[r] = reinterpret_cast<uint8_t*>(data_ptrs[r]);
  const dim3 g(T, H / 1024);
#define XGK_CARLL(SPV)                                                                                           \
  hipLaunchKernelGGL((car_ll_resid_kernel<SPV>), g, dim3(128), 0, st, part, S, T, resid, ss_part, H, region_bytes, \
                     p, rank, world, gens, err, loop)
  if (S == 1) XGK_CARLL(1);
  else if (S == 2) XGK_CARLL(2);
  else if (S == 4) XGK_CARLL(4);
  else if (S == 8) XGK_CARLL(8);
  else XGK_CARLL(0);
#undef XGK_CARLL
  return 0;
}

int custom_allreduce_ll(const void* in, void* out, int64_t nbytes, int64_t region_bytes, const uintptr_t* data_ptrs,
                        int rank, int world, uint32_t* gens, uint32_t* err, hipStream_t st) {
  if (world < 2 || world > CAR_MAX_RANKS || rank < 0 || rank >= world) return 1;
  if (nbytes <= 0 || nbytes % 16 || nbytes > car_ll_max_bytes(region_bytes)) return 1;
  const int64_t blocks = (nbytes / 16 + CAR_LL_GROUPS - 1) / CAR_LL_GROUPS;
  if (blocks > CAR_MAX_BLOCKS) return 1;
  CarPtrs p{};
  for (int r = 0; r < world; ++r) p.data[r] = reinterpret_cast<uint8_t*>(data_ptrs[r]);
  hipLaunchKernelGGL(car_ll_kernel, dim3(static_cast<unsigned>(blocks)), dim3(CAR_LL_GROUPS), 0, st,
                     static_cast<const uint8_t*>(in), static_cast<uint8_t*>(out), nbytes, region_bytes, p, rank, world,
                     gens, err);
  return 0;
}

int custom_allreduce_resid(const float* part, int S, int T, uint16_t* resid, float* ss_part, int H,
                           int64_t slot_bytes, const uintptr_t* data_ptrs, const uintptr_t* sig_ptrs, int rank,
                           int world, uint32_t* gens, uint32_t* err, hipStream_t st) {
  if (world < 2 || world > CAR_MAX_RANKS || rank < 0 || rank >= world) return 1;
  if (T <= 0 || S <= 0 || H <= 0 || H % 1024) return 1;
  if (static_cast<int64_t>(T) * (H / 1024) > CAR_MAX_BLOCKS) return 1;
  if (static_cast<int64_t>(T) * H * 2 > slot_bytes) return 1;
  CarPtrs p{};
  for (int r = 0; r < world; ++r) {
    p.data[r] = reinterpret_cast<uint8_t*>(data_ptrs[r]);
    p.sig[r] = reinterpret_cast<uint32_t*>(sig_ptrs[r]);
  }
  const dim3 g(T, H / 1024);
#define XGK_CARR(SPV)                                                                                          \
  hipLaunchKernelGGL((car_resid_kernel<SPV>), g, dim3(128), 0, st, part, S, T, resid, ss_part, H, slot_bytes, p, \
                     rank, world, gens, err)
  if (S == 1) XGK_CARR(1);
  else if (S == 2) XGK_CARR(2);
  else if (S == 4) XGK_CARR(4);
  else if (S == 8) XGK_CARR(8);
  else XGK_CARR(0);
#undef XGK_CARR
  return 0;
}

// All-gather along the last dimension through peer memory (the vocab-parallel LM
// head of a decode step: [T, V/W] bf16 logits per rank -> [T, V] everywhere).
// Graph capturable like car_kernel; every rank reads each peer's shard over its
// own xGMI link concurrently. Block b handles the 16 KiB chunks b, b + 512, ...
// of the flat shard (a fixed stride, NOT the grid size: a block's slot region must
// be the same in every launch for the per-block double-buffering argument) (rows x cb bytes, cb % 16 == 0): it stages them into its IPC
// slot and straight into its own output columns, signals once, waits for every
// peer's block b, then copies the peers' chunks into their output columns.
__global__ void __launch_bounds__(CAR_THREADS) car_gather_kernel(const uint8_t* __restrict__ in,
                                                                 uint8_t* __restrict__ out, uint32_t nbytes,
                                                                 uint32_t cb, int64_t slot_bytes, CarPtrs p, int rank,
                                                                 int world, uint32_t* __restrict__ gens,
                                                                 uint32_t* __restrict__ err) {
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const uint32_t gen = gens[b] + 1;
  const int64_t slot_off = (gen & 1) * slot_bytes;
  const int64_t row_bytes = static_cast<int64_t>(world) * cb;
  for (uint32_t base = static_cast<uint32_t>(b) * CAR_CHUNK; base < nbytes; base += CAR_MAX_BLOCKS * CAR_CHUNK) {
    uint4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t off = base + (i * CAR_THREADS + t) * 16;
      if (off < nbytes) v[i] = ld16(in + off);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t off = base + (i * CAR_THREADS + t) * 16;
      if (off < nbytes) {
        st16(p.data[rank] + slot_off + off, v[i]);
        st16(out + (off / cb) * row_bytes + static_cast<int64_t>(rank) * cb + off % cb, v[i]);
      }
    }
  }
  __threadfence_system();
  __syncthreads();
  if (t < world && t != rank)
    __hip_atomic_store(p.sig[t] + rank * CAR_MAX_BLOCKS + b, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (t < world && t != rank) {
    const uint32_t* f = p.sig[rank] + t * CAR_MAX_BLOCKS + b;
    car_wait(f, gen, err);
  }
  __syncthreads();
  __threadfence_system();
  for (int r = 0; r < world; ++r) {
    if (r == rank) continue;
    for (uint32_t base = static_cast<uint32_t>(b) * CAR_CHUNK; base < nbytes; base += CAR_MAX_BLOCKS * CAR_CHUNK) {
      uint4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t off = base + (i * CAR_THREADS + t) * 16;
        if (off < nbytes) v[i] = ld16_nt(p.data[r] + slot_off + off);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t off = base + (i * CAR_THREADS + t) * 16;
        if (off < nbytes) st16(out + (off / cb) * row_bytes + static_cast<int64_t>(r) * cb + off % cb, v[i]);
      }
    }
  }
  if (t == 0) gens[b] = gen;
}

int custom_allgather_lastdim(const void* in, void* out, int64_t rows, int64_t cb, int64_t slot_bytes,
                             const uintptr_t* data_ptrs, const uintptr_t* sig_ptrs, int rank, int world,
                             uint32_t* gens, uint32_t* err, hipStream_t st) {
  if (world < 2 || world > CAR_MAX_RANKS || rank < 0 || rank >= world) return 1;
  const int64_t nbytes = rows * cb;
  if (rows <= 0 || cb <= 0 || cb % 16 || nbytes > slot_bytes || nbytes >= (int64_t{1} << 31)) return 1;
  CarPtrs p{};
  for (int r = 0; r < world; ++r) {
    p.data[r] = reinterpret_cast<uint8_t*>(data_ptrs[r]);
    p.sig[r] = reinterpret_cast<uint32_t*>(sig_ptrs[r]);
  }
  const int64_t chunks = (nbytes + CAR_CHUNK - 1) / CAR_CHUNK;
  const int blocks = static_cast<int>(chunks < CAR_MAX_BLOCKS ? chunks : CAR_MAX_BLOCKS);
  hipLaunchKernelGGL(car_gather_kernel, dim3(blocks), dim3(CAR_THREADS), 0, st, static_cast<const uint8_t*>(in),
                     static_cast<uint8_t*>(out), static_cast<uint32_t>(nbytes), static_cast<uint32_t>(cb), slot_bytes,
                     p, rank, world, gens, err);
  return 0;
}

int car_max_blocks() { return CAR_MAX_BLOCKS; }
// wall_clock64() ticks per millisecond on the current device (the peer-wait limit unit)
int car_wallclock_khz() {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return 0;
  return khz;
}
int car_chunk() { return CAR_CHUNK; }
int car_max_ranks() { return CAR_MAX_RANKS; }

// bf16 only (the activation dtype of every TP model here); nbytes % 16 == 0.
int custom_allreduce(const void* in, void* out, int64_t nbytes, int64_t slot_bytes, const uintptr_t* data_ptrs,
                     const uintptr_t* sig_ptrs, int rank, int world, uint32_t* gens, uint32_t* err,
                     hipStream_t st) {
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
                     gens, err);
  return 0;
}

// Two-shot: the signal arrays passed here hold 2 phases x [CAR_MAX_RANKS][CAR_MAX_BLOCKS].
int custom_allreduce_2shot(const void* in, void* out, int64_t nbytes, int64_t slot_bytes, const uintptr_t* data_ptrs,
                           const uintptr_t* sig_ptrs, int rank, int world, uint32_t* gens, uint32_t* err,
                     hipStream_t st) {
  if (world < 2 || world > CAR_MAX_RANKS || rank < 0 || rank >= world) return 1;
  if (nbytes <= 0 || nbytes % 16 || nbytes > slot_bytes) return 1;
  const int64_t shard = ((nbytes + world - 1) / world + 15) / 16 * 16;
  const int64_t blocks = (shard + CAR_CHUNK - 1) / CAR_CHUNK;
  if (blocks > CAR_MAX_BLOCKS || blocks * world * CAR_CHUNK > slot_bytes) return 1;
  CarPtrs p{};
  for (int r = 0; r < world; ++r) {
    p.data[r] = reinterpret_cast<uint8_t*>(data_ptrs[r]);
    p.sig[r] = reinterpret_cast<uint32_t*>(sig_ptrs[r]);
  }
  hipLaunchKernelGGL(car2_kernel<uint16_t>, dim3(static_cast<unsigned>(blocks)), dim3(CAR_THREADS), 0, st,
                     static_cast<const uint8_t*>(in), static_cast<uint8_t*>(out), nbytes, shard, slot_bytes, p, rank,
                     world, gens, err);
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
