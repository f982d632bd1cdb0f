// gemm_m64 with LDS-DMA (global_load_lds_dwordx4) staging for BOTH operands.
//
// Same contract as gemm_m64 (16 < M <= 64, out = x . W^T, split-K partials /
// bf16 / fused SiLU-gate), different load path: the register-ring kernel feeds
// W to the MFMAs as fragment-shaped loads (16 rows x 64 B per wave instruction),
// which keeps the texture-address path busy at ~4 TB/s chip-wide; here every
// wave instruction moves 4 rows x 256 B (full lines) straight into LDS:
//   * K chunk = 128 (256 B per row); 3 LDS slots, 2 chunks in flight;
//   * W: each wave DMAs its own 16*NW rows into a wave-private region of the
//     slot; x: the 4 waves DMA 64 rows x 256 B (4 instructions each);
//   * LDS images are lane-linear (DMA writes base + lane*16) with the 16-B
//     granule XOR-swizzle (granule ^ (row & 15)) applied on the GLOBAL source
//     address, and undone on the ds_read_b128 fragment reads (conflict-free);
//   * one raw s_barrier per chunk after a COUNTED vmcnt (the next chunk stays in
//     flight across it), never __syncthreads (its fence would drain the DMA
//     queue); WAR: a slot is re-filled only after the barrier that follows its
//     last reads (cdna_hip_programming.md §5 "Pipelining across barriers").
//
// Fused decode layer (M64Epi; dense Llama decode path, xgserve/models/llama.py):
//   * the input RMSNorm as an epilogue row scale: x is the raw bf16 residual
//     stream, the norm weight is folded into W at load time, and output row m is
//     scaled by rsqrt(sum_sq[m] / K + eps) -- no normalised-activation kernel;
//   * GG_RESID: the residual add + the next norm's statistics inside the same
//     launch: write-through split-K slabs and an agent-scope arrival ticket per
//     column tile whose last workgroup reduces the tile into the bf16 residual
//     stream and the tile's per-row sum of squares; the consuming GEMM adds the
//     per-tile sums in a fixed order (deterministic).
//   * the statistics are loaded at kernel START (spread over the 16 lane groups x
//     waves of a row, so each lane holds <= 8 values) and combined in the epilogue
//     by xor-shuffles (+ one LDS step): their latency hides under the weight
//     stream instead of extending the tail.
#include <cstdlib>

#include <cstddef>

#include <algorithm>

#include "glds.h"
#include "../comm/ll.h"

namespace xgk {

enum : int { GG_BF16 = 0, GG_PARTIAL = 1, GG_SILU = 2, GG_RESID = 3, GG_MOE_RESID = 4, GG_AR = 5 };

// Fused-decode epilogue operands (all null / 0 for a plain GEMM).
//   ss_in / ss_n / ss_stride: RMSNorm statistics of the input rows as ss_n
//           partial sums of squares per row, ss_in[j * ss_stride + m], added in a
//           fixed order; output row m is scaled by rsqrt(sum / K + eps).
//           ss_n <= 8: any M (lane group g of row m sums j = g, g + 4);
//           8 < ss_n <= 128, M <= 16: wave w, group g sums j = 4w + g + 4 WV q,
//           q < 32 / WV (a 128-tile producer -- the 70B TP8 O / down at 64-column
//           tiles -- needs no pair combine);
//           8 < ss_n <= 64, M > 16 (MT = 4): lane m of wave w sums j = w + WV q (64 / WV
//           loads), the waves' sums added through LDS in wave order (deterministic).
//   GG_RESID: resid[m, n] += sum_s part[s, m, n] (bf16 residual stream, in place);
//           ss_out[tile * M + m] = sum over the tile's columns of resid[m, n]^2
//           (the next GEMM's ss_in with ss_n = gridDim.x). counters: gridDim.x tile
//           tickets, zero before the first launch; every ticket winner re-zeroes
//           its word, so each launch leaves them zero.
struct M64Epi {
  const float* ss_in;
  int ss_n;
  int ss_stride;
  float eps;
  uint16_t* resid;
  float* ss_out;
  int* counters;
  int krot = 0;  // set by m64g_launch (k_rotation): walk K chunks from a per-tile start
  // GG_AR (TP decode, row-parallel O / down): the tensor-parallel all-reduce in the
  // launch, operands in device memory (ArDesc below: kernel arguments stay in SGPRs)
  const struct ArDesc* ar = nullptr;
};

// GG_AR: GG_RESID with the tensor-parallel all-reduce inside the launch. The tile's
// last arriver sums its S slabs, rounds to bf16 (this rank's contribution, as in the
// unfused path) and pushes it to every peer as LL lines (comm/ll.h) at [parity]
// [source rank][element / 4] of the peer's receive region, then polls its OWN region
// for the peers' lines of the same tile and adds all contributions in rank order to
// the residual (bit-identical on every rank), with the tile's statistics. One
// generation per launch, kept per AR_GRAN-column granule (gens): every GG_AR launch
// covers all N columns, so each granule advances once per launch whatever the tile
// width (the O and down launches of a layer may differ) and the pull-free
// double-buffering argument of the LL all-reduce holds per line. loop: one-process
// TP-shard simulation -- the "peers" are this rank's own region (lines pushed to source
// slot r, polled, not added): the traffic and the waits of a `world`-rank group, the
// numerics of one rank; loop - 1 = a simulated link latency in wall-clock ticks, waited
// once per tile between the pushes and the polls. More column tiles than the consumer
// combines (64 per row, 128 at M <= 16; group 2): statistics per PAIR of tiles -- each
// tile stores its row sums to ss_tmp, the second of the pair to finish (ticket
// pair[tile / 2]) adds the two in order.
constexpr int AR_GRAN = 32;  // the narrowest GG_AR tile (16 x NW x WV columns)
struct ArDesc {
  uint8_t* data[CAR_MAX_RANKS];  // each rank's LL receive region (loop: all this rank's own)
  int64_t region;
  int rank, world, loop, group;
  uint32_t* gens;                // one generation per AR_GRAN columns (all equal after a launch)
  uint32_t* err;                 // [timeouts, wait limit] (the custom all-reduce's ctl)
  float* ss_tmp;
  int* pair;
};

// GG_MOE_RESID (grouped w2 of the fused decode layer, TP = 1): the MoE combine inside
// the w2 launch. Every workgroup stores its fp32 partial rows write-through and takes a
// ticket on its column tile; the tile's last arriver (all real row tiles x S splits
// have stored) adds, per token t, sum_j w[t, j] * sum_s part[s, dest[t, j]] over the
// tile's columns into the bf16 residual stream and writes the new residual's sum of
// squares ss_out[tile * T + t] (the next RMSNorm reads N / cols partial sums per row).
// Replaces the separate combine_resid launch (6 us per layer at Mixtral batch 1).
struct MoeResidEpi {
  const int32_t* dest;   // [T * k] padded row of each (token, choice), -1 = not local
  const float* w;        // [T * k] routing weights
  uint16_t* resid;       // [T, N] bf16 residual stream, updated in place
  float* ss_out;         // [N / cols, T]
  int* counters;         // one ticket per column tile, zero between launches
  int T;
  int k;
};

// K-chunk rotation. Workgroups that all start at K chunk 0 and walk in lockstep read the
// same column offset of weight rows 2*K bytes apart at the same moment, so the HBM
// requests of the whole grid pile onto a few channels: 8B gate_up at 64 rows streams at
// 4.9 TB/s in order and 6.2 TB/s rotated (profiles/r4_mw_probe.md). Each workgroup walks
// its chunk range from a tile-dependent start instead (the fp32 sum order changes, the
// result does not). Split-K grids (S > 2) are already spread over K and stay in order.
// Policy (set_k_rotation): 0 never, 1 when S <= 2 (default), 2 always.
static int g_krot_mode = 1;
void set_k_rotation(int mode) { g_krot_mode = mode; }
int k_rotation(int S) { return g_krot_mode == 2 || (g_krot_mode == 1 && S <= 2) ? 1 : 0; }

// Every wave drains its stores (write-through), then one relaxed agent-scope
// ticket; returns in every thread whether this workgroup drew `last_value`. The
// winner acquires (agent scope: drops this CU's stale L1 lines) before any of its
// waves reads what the others published, and re-arms the word. `flag` is an LDS
// word no wave touches concurrently (inside the staging array: ONE __shared__
// object per kernel, guide §5 "Three .s-level traps" (a)).
__device__ __forceinline__ bool agent_ticket(int* cnt, int last_value, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == last_value;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  const bool r = *flag != 0;
  __syncthreads();
  return r;
}

// Reduction of one column tile [tile*COLS, +COLS) x [0, M): the S fp32 slabs + the
// bf16 residual -> new residual and the tile's per-row sum of squares. The threads
// of one row are C4 = COLS/4 consecutive lanes of one wave (row sum = xor butterfly
// over them); every lane runs every butterfly. IB row-chunk passes share one batch
// of loads (IB x 4 slab reads + IB residual reads in flight before the first add):
// the slabs were written by other XCDs, so every read is a MALL round trip and a
// pass-by-pass loop paid one per NTHR x 16 B (~1 us per 16 KB at M = 64).
// ys (S == 1): the tile staged in LDS [M][COLS] by this workgroup instead of its slab
// (no store -> drain -> reload round trip). 4 < S <= 8: all S slab reads of an item in
// one batch (a 4-wide batch loop paid two MALL round trips per pass).
template <int COLS, int NTHR>
__device__ __forceinline__ void m64g_resid_reduce(const float* __restrict__ part, int S, int M, int N, int tile,
                                                  const M64Epi& epi, int r0 = 0, int r1 = -1,
                                                  const float* ys = nullptr) {
  constexpr int C4 = COLS / 4;
  constexpr int IB = 4;
  static_assert(64 % C4 == 0 && NTHR % C4 == 0, "row groups must not straddle waves");
  const int tid = threadIdx.x;
  const int n0 = tile * COLS;
  const int64_t slab = static_cast<int64_t>(M) * N;
  if (r1 < 0) r1 = M;
  const int nr = r1 - r0;
  for (int base = 0; base < nr * C4; base += IB * NTHR) {
    bool ok[IB];
    int m[IB], c[IB];
    int64_t off[IB];
    float y[IB][4];
    uint2 rv[IB];
#pragma unroll
    for (int i = 0; i < IB; ++i) {  // clamped unconditional addresses, masked after
      const int idx = base + i * NTHR + tid;
      ok[i] = idx < nr * C4;
      m[i] = r0 + (ok[i] ? idx / C4 : 0);
      c[i] = idx % C4;
      off[i] = static_cast<int64_t>(m[i]) * N + n0 + 4 * c[i];
      rv[i] = *reinterpret_cast<const uint2*>(epi.resid + off[i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) y[i][j] = 0.f;
    }
    if (ys != nullptr) {
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const float4 v = *reinterpret_cast<const float4*>(ys + (m[i] - r0) * COLS + 4 * c[i]);
        y[i][0] = v.x;
        y[i][1] = v.y;
        y[i][2] = v.z;
        y[i][3] = v.w;
      }
    } else if (S > 4 && S <= 8) {
      float4 v[IB][8];
#pragma unroll
      for (int i = 0; i < IB; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = *reinterpret_cast<const float4*>(part + min(j, S - 1) * slab + off[i]);
#pragma unroll
      for (int i = 0; i < IB; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float k = j < S ? 1.f : 0.f;
          y[i][0] += k * v[i][j].x;
          y[i][1] += k * v[i][j].y;
          y[i][2] += k * v[i][j].z;
          y[i][3] += k * v[i][j].w;
        }
    } else {
      for (int s0 = 0; s0 < S; s0 += 4) {
        float4 v[IB][4];
#pragma unroll
        for (int i = 0; i < IB; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) v[i][j] = *reinterpret_cast<const float4*>(part + min(s0 + j, S - 1) * slab + off[i]);
#pragma unroll
        for (int i = 0; i < IB; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float k = s0 + j < S ? 1.f : 0.f;
            y[i][0] += k * v[i][j].x;
            y[i][1] += k * v[i][j].y;
            y[i][2] += k * v[i][j].z;
            y[i][3] += k * v[i][j].w;
          }
      }
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      float sq = 0.f;
      if (ok[i]) {
        y[i][0] += __uint_as_float(rv[i].x << 16);
        y[i][1] += __uint_as_float(rv[i].x & 0xFFFF0000u);
        y[i][2] += __uint_as_float(rv[i].y << 16);
        y[i][3] += __uint_as_float(rv[i].y & 0xFFFF0000u);
        uint2 o;
        o.x = pack2(y[i][0], y[i][1]);
        o.y = pack2(y[i][2], y[i][3]);
        *reinterpret_cast<uint2*>(epi.resid + off[i]) = o;
        // the residual stream is bf16: the norm statistics use the rounded values
        const float a0 = __uint_as_float(o.x << 16), a1 = __uint_as_float(o.x & 0xFFFF0000u);
        const float a2 = __uint_as_float(o.y << 16), a3 = __uint_as_float(o.y & 0xFFFF0000u);
        sq = a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
      }
#pragma unroll
      for (int o = C4 / 2; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
      if (ok[i] && c[i] == 0) epi.ss_out[tile * M + m[i]] = sq;
    }
  }
}

// GG_RESID tail: tile ticket -> the last arriver reduces the tile.
template <int COLS, int NTHR>
__device__ __forceinline__ void m64g_resid_tail(const float* __restrict__ part, int S, int M, int N,
                                                const M64Epi& epi, int* flag, int bx, const float* ys = nullptr) {
  if (S > 1) {
    if (!agent_ticket(epi.counters + bx, S - 1, flag)) return;
  } else if (ys != nullptr) {
    __syncthreads();  // every wave's LDS stage
  } else {  // one split: the tile's own slab, written by every wave, read back in another layout
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  m64g_resid_reduce<COLS, NTHR>(part, S, M, N, bx, epi, 0, -1, ys);
}

// GG_AR tail (M64Epi::ar_*): tile ticket -> the last arriver reduces the S slabs,
// exchanges the bf16 tile with the TP peers over LL lines and folds the sum into the
// residual. One LL line = 4 columns of one row; the C4 = COLS / 4 lines of a row are
// consecutive lanes of one wave (row statistics by xor butterfly; every lane runs
// every butterfly).
template <int COLS, int NTHR>
__device__ __forceinline__ void m64g_ar_tail(const float* __restrict__ part, int S, int M, int N, const M64Epi& epi,
                                             int* flag, int bx, uint32_t dv, const float* ys = nullptr) {
  // ys (S == 1, a few rows): this workgroup's tile staged in LDS [M][COLS] instead of
  // the slab round trip through global memory
  // the descriptor, loaded into lanes 0..29 of every wave at kernel start (dv): read
  // back lane by lane (no global load in the tail, no SGPRs held across the loop)
  auto d32 = [&](int i) { return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(dv), i)); };
  auto d64 = [&](int i) { return static_cast<uint64_t>(d32(i)) | (static_cast<uint64_t>(d32(i + 1)) << 32); };
  // (fields read where they are used: few SGPRs live at once)
  auto peer = [&](int r) { return reinterpret_cast<uint8_t*>(d64(2 * r)); };
  auto region = [&] { return static_cast<int64_t>(d64(16)); };
  auto gens = [&] { return reinterpret_cast<uint32_t*>(d64(22)); };
  auto err = [&] { return reinterpret_cast<uint32_t*>(d64(24)); };
  const int rank = static_cast<int>(d32(18)), world = static_cast<int>(d32(19)), loop = static_cast<int>(d32(20));
  if (S > 1) {
    if (!agent_ticket(epi.counters + bx, S - 1, flag)) return;
  } else if (ys != nullptr) {
    __syncthreads();  // every wave's LDS stage
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's own slab stores
    __syncthreads();
  }
  constexpr int C4 = COLS / 4;
  static_assert(64 % C4 == 0 && NTHR % C4 == 0, "row groups must not straddle waves");
  const int tid = threadIdx.x;
  const int n0 = bx * COLS;
  const int64_t slab = static_cast<int64_t>(M) * N;
  // One generation per LAUNCH, not per tile: the O and down launches share the LL
  // region at different tile widths, so the words are kept per AR_GRAN-column granule
  // and every launch advances each granule once -- all equal, whatever COLS is.
  static_assert(COLS % AR_GRAN == 0, "GG_AR tiles cover whole granules");
  const uint32_t gen = gens()[n0 / AR_GRAN] + 1;
  const int64_t src_bytes = region() / (2 * CAR_MAX_RANKS);  // per (parity, source)
  const int64_t par = static_cast<int64_t>(gen & 1) * (region() / 2);
  uint8_t* const own = peer(rank);
  bool ok = true;
  for (int base = 0; base < M * C4; base += NTHR) {
    const int idx = base + tid;
    const bool act = idx < M * C4;
    const int m = act ? idx / C4 : 0, c = idx % C4;
    const int64_t e = static_cast<int64_t>(m) * N + n0 + 4 * c;  // element offset
    float y[4] = {0.f, 0.f, 0.f, 0.f};
    float sq = 0.f;
    if (act) {
      // the residual row segment is needed last: its load flies under the pushes and polls
      uint2 rv = *reinterpret_cast<const uint2*>(epi.resid + e);
      if (ys != nullptr) {
        const float4 v = *reinterpret_cast<const float4*>(ys + m * COLS + 4 * c);
        y[0] = v.x; y[1] = v.y; y[2] = v.z; y[3] = v.w;
      } else {
        for (int s0 = 0; s0 < S; s0 += 4) {
          float4 v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const float4*>(part + min(s0 + j, S - 1) * slab + e);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float k = s0 + j < S ? 1.f : 0.f;
            y[0] += k * v[j].x; y[1] += k * v[j].y; y[2] += k * v[j].z; y[3] += k * v[j].w;
          }
        }
      }
      const uint32_t w0 = pack2(y[0], y[1]), w1 = pack2(y[2], y[3]);  // this rank's bf16 contribution
      const int64_t line = par + (e / 4) * 16;
      for (int r = 0; r < world; ++r) {
        if (r == rank) continue;
        ll_store(peer(r) + line + static_cast<int64_t>(loop ? r : rank) * src_bytes, w0, w1,
                 gen);
      }
      asm volatile("" ::: "memory");  // every push is issued before the first poll
      if (loop > 1) {  // loopback simulation of a link latency (ticks)
        const uint64_t t0 = wall_clock64();
        while (wall_clock64() - t0 < static_cast<uint64_t>(loop - 1)) __builtin_amdgcn_s_sleep(1);
      }
      uint32_t d[CAR_MAX_RANKS][2];
      const uint32_t need = ((1u << world) - 1) & ~(1u << rank);
      if (ok) ok = ll_recv_multi(own + line, src_bytes, need, gen, err(), d);
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < world; ++r) {  // rank order: bit-identical on every rank
        uint32_t d0 = w0, d1 = w1;
        if (r != rank) {
          if (loop || !ok) continue;  // loopback: polled, not added
          d0 = d[r][0];
          d1 = d[r][1];
        }
        acc[0] += __uint_as_float(d0 << 16);
        acc[1] += __uint_as_float(d0 & 0xFFFF0000u);
        acc[2] += __uint_as_float(d1 << 16);
        acc[3] += __uint_as_float(d1 & 0xFFFF0000u);
      }
      acc[0] += __uint_as_float(rv.x << 16);
      acc[1] += __uint_as_float(rv.x & 0xFFFF0000u);
      acc[2] += __uint_as_float(rv.y << 16);
      acc[3] += __uint_as_float(rv.y & 0xFFFF0000u);
      rv.x = pack2(acc[0], acc[1]);
      rv.y = pack2(acc[2], acc[3]);
      *reinterpret_cast<uint2*>(epi.resid + e) = rv;
      const float a0 = __uint_as_float(rv.x << 16), a1 = __uint_as_float(rv.x & 0xFFFF0000u);
      const float a2 = __uint_as_float(rv.y << 16), a3 = __uint_as_float(rv.y & 0xFFFF0000u);
      sq = a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
    }
#pragma unroll
    for (int o = C4 / 2; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
    if (act && c == 0) {
      if (static_cast<int>(d32(21)) == 1) epi.ss_out[bx * M + m] = sq;
      else st4_sc1(reinterpret_cast<float*>(d64(26)) + bx * M + m, sq);
    }
  }
  if (tid < COLS / AR_GRAN) gens()[n0 / AR_GRAN + tid] = gen;
  if (static_cast<int>(d32(21)) == 1) return;
  // pair statistics: the later tile of the pair adds both row sums, in tile order
  if (!agent_ticket(reinterpret_cast<int*>(d64(28)) + bx / 2, 1, flag)) return;
  const int p0 = bx & ~1;
  const float* ss_tmp = reinterpret_cast<const float*>(d64(26));
  for (int m = tid; m < M; m += NTHR) epi.ss_out[(bx / 2) * M + m] = ss_tmp[p0 * M + m] + ss_tmp[(p0 + 1) * M + m];
}

// Split-K GG_SILU tail: every workgroup has stored its fp32 partial of the tile
// (write-through); the tile's last arriver sums the S slabs and applies the SiLU
// gate (gate / up rows interleaved in blocks of 16) into out [M, N / 2]. Lets the
// wide (8-wave, 256-column) tile run at M = 64: half the x bytes per weight byte
// of the 128-column tile, which is what bounds the per-CU LDS-DMA ingest there.
template <int COLS, int NTHR>
__device__ __forceinline__ void m64g_silu_tail(const float* __restrict__ part, int S, int M, int N,
                                               uint16_t* __restrict__ out, int* counters, int* flag, int bx) {
  if (!agent_ticket(counters + bx, S - 1, flag)) return;
  constexpr int O4 = COLS / 8;  // 4-wide output groups per row (COLS / 2 outputs)
  const int F = N / 2, n0 = bx * COLS;
  const int64_t slab = static_cast<int64_t>(M) * N;
  for (int idx = threadIdx.x; idx < M * O4; idx += NTHR) {
    const int m = idx / O4, oc = 4 * (idx % O4);
    const int64_t go = static_cast<int64_t>(m) * N + n0 + (oc >> 4) * 32 + (oc & 15);
    float gs[4] = {0.f, 0.f, 0.f, 0.f}, us[4] = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < S; ++s) {
      const float4 gv = *reinterpret_cast<const float4*>(part + s * slab + go);
      const float4 uv = *reinterpret_cast<const float4*>(part + s * slab + go + 16);
      gs[0] += gv.x; gs[1] += gv.y; gs[2] += gv.z; gs[3] += gv.w;
      us[0] += uv.x; us[1] += uv.y; us[2] += uv.z; us[3] += uv.w;
    }
    float o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = gs[r] / (1.f + __expf(-gs[r])) * us[r];
    uint2 v;
    v.x = pack2(o[0], o[1]);
    v.y = pack2(o[2], o[3]);
    *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * F + n0 / 2 + oc) = v;
  }
}

// Dense kernel, parametrised for the decode shapes (bench/gemm_bench.py picks):
//   NW  16-column MFMA tiles per wave (2 = 32 columns; required by the SiLU epilogue)
//   WV  waves per workgroup (4 or 2): fewer waves = more, smaller workgroups, so a
//       short N still puts a workgroup on every CU
//   KC  k per chunk (128: 256-B rows, 1 workgroup/CU; 64: 128-B rows, 2-3 per CU)
//   NT  non-temporal weight DMA (streamed once; keeps x resident in L2)
//   MT  16-row x tiles (4: 16 < M <= 64; 1: M <= 16 -- a quarter of the x DMA and
//       LDS per chunk, so the weight stream owns the load path at batch 1)
//   NS  LDS ring slots (NS - 1 chunks in flight across each barrier): 3, or deeper
//       for the one-x-tile (M <= 16) configurations, whose slots are small -- a
//       single workgroup per CU then keeps ~80 KB of weights in flight instead of 40
template <int NW, int WV, int KC, bool NT, int MT, int NS = 3>
__global__ void __launch_bounds__(64 * WV, 1) gemm_m64g_kernel(const uint16_t* __restrict__ x, int M, int K,
                                                               const uint16_t* __restrict__ w, int N,
                                                               float* __restrict__ part, uint16_t* __restrict__ out,
                                                               int mode, M64Epi epi) {
  constexpr int RB = KC * 2;                     // bytes per LDS row
  constexpr int GPR = KC / 8;                    // 16-B granules per row
  constexpr int RPI = 1024 / RB;                 // rows per DMA instruction (64 lanes x 16 B)
  constexpr int XROWS = 16 * MT;
  constexpr int XBYTES = XROWS * RB;
  constexpr int XI = XROWS / RPI / WV;           // x DMA instructions per wave per chunk
  constexpr int WROWS = 16 * NW;                 // weight rows per wave
  constexpr int WI = WROWS / RPI;                // weight DMA instructions per wave per chunk
  constexpr int WBYTES = WROWS * RB;             // per wave per slot
  constexpr int SLOT = XBYTES + WV * WBYTES;
  constexpr int G = XI + WI;
  static_assert(XI >= 1 && WI >= 1 && XROWS % (RPI * WV) == 0, "bad m64g geometry");
  static_assert(NS >= 3 && NS * SLOT <= 160 * 1024, "ring");
  __shared__ __attribute__((aligned(1024))) uint8_t lds0[NS == 3 ? SLOT : NS * SLOT];
  __shared__ __attribute__((aligned(1024))) uint8_t lds1[NS == 3 ? SLOT : 16];
  __shared__ __attribute__((aligned(1024))) uint8_t lds2[NS == 3 ? SLOT : 16];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  // tile bx of split s
  const int bx = blockIdx.x, S = gridDim.y, s = blockIdx.y;
  // split s takes chunks [s * nch / S, (s + 1) * nch / S): any S <= K / KC (uneven
  // splits fill the chip where K / KC has no divisor near 256 / column tiles)
  const int nch_all = K / KC;
  const int c_lo = s * nch_all / S;
  const int k0 = c_lo * KC;
  const int nchunks = (s + 1) * nch_all / S - c_lo;
  const int nbase = bx * (16 * NW * WV) + wid * WROWS;

  const int dr = lane / GPR, dj = lane % GPR;    // row within a DMA instruction, granule
  const uint16_t* wsrc[WI];
#pragma unroll
  for (int i = 0; i < WI; ++i) {
    const int r = RPI * i + dr;
    wsrc[i] = w + static_cast<int64_t>(nbase + r) * K + k0 + 8 * (dj ^ (r & (GPR - 1)));
  }
  const uint16_t* xsrc[XI];
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int r = RPI * (wid * XI + i) + dr;     // x row 0..XROWS-1
    xsrc[i] = x + static_cast<int64_t>(min(r, M - 1)) * K + k0 + 8 * (dj ^ (r & (GPR - 1)));
  }
  const int rot = epi.krot ? static_cast<int>((static_cast<unsigned>(bx) * 37u) % static_cast<unsigned>(nchunks)) : 0;

  auto chunk_k = [&](int c) {
    const int cr = c + rot;
    return (cr >= nchunks ? cr - nchunks : cr) * KC;
  };
  auto issue_x = [&](uint8_t* slot, int c) {
    const int kk = chunk_k(c);
#pragma unroll
    for (int i = 0; i < XI; ++i) glds16(xsrc[i] + kk, slot + RPI * (wid * XI + i) * RB);
  };
  auto issue_w = [&](uint8_t* slot, int c) {
    const int kk = chunk_k(c);
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      if constexpr (NT) glds16_nt(wsrc[i] + kk, slot + XBYTES + wid * WBYTES + i * 1024);
      else glds16(wsrc[i] + kk, slot + XBYTES + wid * WBYTES + i * 1024);
    }
  };
  auto issue = [&](uint8_t* slot, int c) {
    issue_x(slot, c);
    issue_w(slot, c);
  };

  f32x4_t acc[NW][MT];
#pragma unroll
  for (int nt = 0; nt < NW; ++nt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const uint8_t* slot) {
    const uint8_t* xs = slot;
    const uint8_t* ws = slot + XBYTES + wid * WBYTES;
#pragma unroll
    for (int t = 0; t < KC / 32; ++t) {
      const int phys = (4 * t + g) ^ (li & (GPR - 1));
      uint4 b[MT], a[NW];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) b[mt] = *reinterpret_cast<const uint4*>(xs + (16 * mt + li) * RB + phys * 16);
#pragma unroll
      for (int nt = 0; nt < NW; ++nt) a[nt] = *reinterpret_cast<const uint4*>(ws + (16 * nt + li) * RB + phys * 16);
#pragma unroll
      for (int nt = 0; nt < NW; ++nt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = mfma16x16x32(as_frag(a[nt]), as_frag(b[mt]), acc[nt][mt]);
    }
  };

  // chunk c lives in slot c % 3; per chunk: counted wait (chunk c+1 stays in
  // flight), barrier, DMA chunk c+2 into the slot freed by that barrier, compute c
  auto step = [&](uint8_t* cur, uint8_t* nxt2, int c) {
    if (c + 1 < nchunks) wait_vmcnt<G>();
    else wait_vmcnt<0>();
    raw_barrier();
    if (c + 2 < nchunks) issue(nxt2, c + 2);
    compute(cur);
  };

  // RMSNorm statistics of the input rows, loaded before the weight stream starts
  // (clamped unconditional loads, masked when combined; held in 8 registers)
  const bool has_ss = epi.ss_in != nullptr;
  // per-tile sums (ss_n > 8): M <= 16 spreads them over the waves too (wide); M > 16
  // (MT = 4, "tall"): lane = row, wave w sums j = w + WV q, combined through LDS
  const bool tall_ss = MT > 1 && has_ss && epi.ss_n > 8 && M > 16;
  const bool wide_ss = has_ss && epi.ss_n > 8 && !tall_ss;
  constexpr int TQ = MT > 1 ? 64 / WV : 1;
  constexpr int WQ = 32 / WV;  // wide statistics loads per lane (4 WV groups x WQ = 128 sums)
  float ssv[WQ > 8 ? WQ : 8];
  float ssb[TQ];
  // ring prologue: chunks 0 .. NS - 2 into their slots
  auto slot_of = [&](int j) -> uint8_t* {
    if constexpr (NS == 3) return j == 0 ? lds0 : lds1;
    else return lds0 + j * SLOT;
  };
  auto ld_ss = [&](int idx) { return epi.ss_in[idx]; };
  if (tall_ss) {
#pragma unroll
    for (int q = 0; q < TQ; ++q) ssb[q] = ld_ss(min(wid + WV * q, epi.ss_n - 1) * epi.ss_stride + min(lane, M - 1));
  } else if (has_ss) {
#pragma unroll
    for (int i = 0; i < (WQ > 8 ? WQ : 8); ++i) {
      if (wide_ss ? i >= WQ : (i >> 1) >= MT || i >= 8) break;
      const int mt = wide_ss ? 0 : i >> 1, q = wide_ss ? i : i & 1;
      const int j = wide_ss ? 4 * wid + g + 4 * WV * q : g + 4 * q;
      ssv[i] = ld_ss(min(j, epi.ss_n - 1) * epi.ss_stride + min(16 * mt + li, M - 1));
    }
  }
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (j < nchunks) issue(slot_of(j), j);

  if constexpr (NS == 3) {
    int c = 0;
    for (; c + 3 <= nchunks; c += 3) {
      step(lds0, lds2, c);
      step(lds1, lds0, c + 1);
      step(lds2, lds1, c + 2);
    }
    if (c < nchunks) step(lds0, lds2, c);
    if (c + 1 < nchunks) step(lds1, lds0, c + 1);
  } else {
    // NS-slot ring: chunk c in slot c % NS; before chunk c the chunks after it that
    // are already issued (rem = min(nchunks - 1 - c, NS - 2)) stay in flight
    for (int c = 0; c < nchunks; ++c) {
      const int rem = min(nchunks - 1 - c, NS - 2);
      if constexpr (NS >= 6) {
        if (rem >= 4) wait_vmcnt<4 * G>();
      }
      if constexpr (NS >= 5) {
        if (rem == 3) wait_vmcnt<3 * G>();
      }
      if constexpr (NS >= 4) {
        if (rem == 2) wait_vmcnt<2 * G>();
      }
      if (rem == 1) wait_vmcnt<G>();
      if (rem == 0) wait_vmcnt<0>();
      raw_barrier();
      if (c + NS - 1 < nchunks) issue(lds0 + ((c + NS - 1) % NS) * SLOT, c + NS - 1);
      compute(lds0 + (c % NS) * SLOT);
    }
  }

  if (has_ss) {  // input RMSNorm as a row scale of the (linear) output
    float tot[MT];
    if (tall_ss) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < TQ; ++q) v += wid + WV * q < epi.ss_n ? ssb[q] : 0.f;
      float* red = reinterpret_cast<float*>(lds0);
      __syncthreads();  // all waves are past their last slot read (no DMA in flight)
      red[wid * 64 + lane] = v;
      __syncthreads();
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float t = 0.f;
#pragma unroll
        for (int w2 = 0; w2 < WV; ++w2) t += red[w2 * 64 + 16 * mt + li];
        tot[mt] = t;
      }
      __syncthreads();  // red is re-used as the GG_RESID ticket flag below
    } else if (!wide_ss) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float v = (g < epi.ss_n ? ssv[2 * mt] : 0.f) + (g + 4 < epi.ss_n ? ssv[2 * mt + 1] : 0.f);
        v += __shfl_xor(v, 16, 64);
        tot[mt] = v + __shfl_xor(v, 32, 64);
      }
    } else {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < WQ; ++q) v += 4 * wid + g + 4 * WV * q < epi.ss_n ? ssv[q] : 0.f;
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      float* red = reinterpret_cast<float*>(lds0);
      __syncthreads();  // all waves are past their last slot read (no DMA in flight)
      if (g == 0) red[wid * 16 + li] = v;
      __syncthreads();
      float t = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < WV; ++w2) t += red[w2 * 16 + li];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) tot[mt] = t;  // M <= 16: only rows of mt 0 are real
      __syncthreads();  // red is re-used as the GG_RESID ticket flag below
    }
    const float inv_k = 1.f / static_cast<float>(K);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const float sc = rsqrtf(tot[mt] * inv_k + epi.eps);
#pragma unroll
      for (int nt = 0; nt < NW; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[nt][mt][r] *= sc;
    }
  }

  // GG_AR: the all-reduce descriptor (30 dwords) into lanes 0..29 of every wave, its
  // latency under the slab stores and the tile ticket (m64g_ar_tail reads it back with
  // readlane: no SGPRs held, no dependent load in the tail)
  uint32_t ar_dv = 0;
  if (mode == GG_AR) ar_dv = reinterpret_cast<const uint32_t*>(epi.ar)[lane < 30 ? lane : 29];
  // acc[nt][mt][r] = out[m = 16 mt + li][n = nbase + 16 nt + 4 g + r]
  const bool silu_split = NW == 2 && mode == GG_SILU && S > 1;
  constexpr int TCOLS = 16 * NW * WV;
  if ((mode == GG_AR || mode == GG_RESID) && S == 1 && 256 + M * TCOLS * 4 <= static_cast<int>(sizeof(lds0))) {
    // one split: the tile goes through LDS to the residual / all-reduce tail (no slab
    // store + drain + reload)
    __syncthreads();  // every wave is past its last ring read
    float* ys = reinterpret_cast<float*>(lds0 + 256);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = 16 * mt + li;
      if (m >= M) continue;
#pragma unroll
      for (int nt = 0; nt < NW; ++nt)
        *reinterpret_cast<float4*>(ys + m * TCOLS + (nbase - bx * TCOLS) + 16 * nt + 4 * g) =
            make_float4(acc[nt][mt][0], acc[nt][mt][1], acc[nt][mt][2], acc[nt][mt][3]);
    }
    if (mode == GG_AR) m64g_ar_tail<TCOLS, 64 * WV>(part, S, M, N, epi, reinterpret_cast<int*>(lds0), bx, ar_dv, ys);
    else m64g_resid_tail<TCOLS, 64 * WV>(part, S, M, N, epi, reinterpret_cast<int*>(lds0), bx, ys);
  } else if (mode == GG_PARTIAL || mode == GG_RESID || mode == GG_AR || silu_split) {
    float* pp = part + static_cast<int64_t>(s) * M * N;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = 16 * mt + li;
      if (m >= M) continue;
#pragma unroll
      for (int nt = 0; nt < NW; ++nt) {
        float* dst = pp + static_cast<int64_t>(m) * N + nbase + 16 * nt + 4 * g;
        if (mode != GG_PARTIAL) st16_sc1(dst, acc[nt][mt]);
        else *reinterpret_cast<float4*>(dst) = make_float4(acc[nt][mt][0], acc[nt][mt][1], acc[nt][mt][2], acc[nt][mt][3]);
      }
    }
    if (mode == GG_RESID)
      m64g_resid_tail<16 * NW * WV, 64 * WV>(part, S, M, N, epi, reinterpret_cast<int*>(lds0), bx);
    else if (mode == GG_AR)
      m64g_ar_tail<16 * NW * WV, 64 * WV>(part, S, M, N, epi, reinterpret_cast<int*>(lds0), bx, ar_dv);
    else if (silu_split)
      m64g_silu_tail<16 * NW * WV, 64 * WV>(part, S, M, N, out, epi.counters, reinterpret_cast<int*>(lds0), bx);
  } else if (mode == GG_BF16) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = 16 * mt + li;
      if (m >= M) continue;
#pragma unroll
      for (int nt = 0; nt < NW; ++nt) {
        uint2 v;
        v.x = pack2(acc[nt][mt][0], acc[nt][mt][1]);
        v.y = pack2(acc[nt][mt][2], acc[nt][mt][3]);
        *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * N + nbase + 16 * nt + 4 * g) = v;
      }
    }
  } else if (NW == 2) {
    const int F = N / 2, f0 = nbase / 2 + 4 * g;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = 16 * mt + li;
      if (m >= M) continue;
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float gt = acc[0][mt][r];
        o[r] = gt / (1.f + __expf(-gt)) * acc[NW - 1][mt][r];
      }
      uint2 v;
      v.x = pack2(o[0], o[1]);
      v.y = pack2(o[2], o[3]);
      *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * F + f0) = v;
    }
  }
}

// GG_MOE_RESID tail (MoeResidEpi): the column tile's last arriver combines every
// (token, choice) row's S partials into the residual stream.
template <int COLS, int NTHR>
__device__ __forceinline__ void moe_resid_tail(const float* __restrict__ part, int S, int P, int N,
                                               const MoeResidEpi& mre, int contributors, int* flag, int bx) {
  if (!agent_ticket(mre.counters + bx, contributors - 1, flag)) return;
  constexpr int G4 = COLS / 4;  // 4-column groups of the tile
  const int n0 = bx * COLS;
  const int64_t slab = static_cast<int64_t>(P) * N;
  const int lane = threadIdx.x & 63;
  // one row per G4 consecutive threads (G4 = 32: two rows per wave); the sum of
  // squares of a row is a reduction over its G4 lanes
  static_assert(64 % G4 == 0 && NTHR % G4 == 0, "moe_resid_tail geometry");
  for (int base = 0; base < mre.T * G4; base += NTHR) {
    const int idx = base + static_cast<int>(threadIdx.x);
    const int t = idx / G4, c = 4 * (idx % G4);
    const bool ok = t < mre.T;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    float sq = 0.f;
    if (ok) {
      for (int j = 0; j < mre.k; ++j) {
        const int p = mre.dest[t * mre.k + j];
        if (p < 0) continue;
        const float wt = mre.w[t * mre.k + j];
        float f[4] = {0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < S; ++s) {
          const float4 v = *reinterpret_cast<const float4*>(part + s * slab + static_cast<int64_t>(p) * N + n0 + c);
          f[0] += v.x; f[1] += v.y; f[2] += v.z; f[3] += v.w;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] += wt * f[i];
      }
      uint16_t* rp = mre.resid + static_cast<int64_t>(t) * N + n0 + c;
      const uint2 rv = *reinterpret_cast<const uint2*>(rp);
      float r[4] = {__uint_as_float(rv.x << 16), __uint_as_float(rv.x & 0xFFFF0000u),
                    __uint_as_float(rv.y << 16), __uint_as_float(rv.y & 0xFFFF0000u)};
      uint2 o;
      o.x = pack2(r[0] + a[0], r[1] + a[1]);
      o.y = pack2(r[2] + a[2], r[3] + a[3]);
      *reinterpret_cast<uint2*>(rp) = o;
      const float q[4] = {__uint_as_float(o.x << 16), __uint_as_float(o.x & 0xFFFF0000u),
                          __uint_as_float(o.y << 16), __uint_as_float(o.y & 0xFFFF0000u)};
      sq = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];  // statistics of the rounded residual
    }
#pragma unroll
    for (int o = G4 / 2; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
    if (ok && (lane % G4) == 0) mre.ss_out[static_cast<int64_t>(bx) * mre.T + t] = sq;
  }
}

template <int NW, int WV, int KC, bool NT, int MT>
__device__ __forceinline__ void grouped_body(const uint16_t* __restrict__ x, const int32_t* __restrict__ rows, int e,
                                             int p0, int p1, int rt0, int K, const uint16_t* __restrict__ w, int N,
                                             int P, float* __restrict__ part, uint16_t* __restrict__ out, int mode,
                                             uint8_t* lds0, uint8_t* lds1, uint8_t* lds2, int krot,
                                             const MoeResidEpi& mre, int contributors) {
  constexpr int RB = KC * 2;
  constexpr int GPR = KC / 8;
  constexpr int RPI = 1024 / RB;
  constexpr int XROWS = 16 * MT;
  constexpr int XBYTES = XROWS * RB;
  constexpr int XI = XROWS / RPI / WV;
  constexpr int WROWS = 16 * NW;
  constexpr int WI = WROWS / RPI;
  constexpr int WBYTES = WROWS * RB;
  constexpr int G = XI + WI;
  static_assert(XI >= 1 && WI >= 1 && XROWS % (RPI * WV) == 0, "bad m64g geometry");
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int S = gridDim.y, s = blockIdx.y;
  const int kws = K / S;
  const int k0 = s * kws;
  const int nchunks = kws / KC;
  const int nbase = blockIdx.x * (16 * NW * WV) + wid * WROWS;
  const int dr = lane / GPR, dj = lane % GPR;
  const uint16_t* we = w + static_cast<int64_t>(e) * N * K;
  const uint16_t* wsrc[WI];
#pragma unroll
  for (int i = 0; i < WI; ++i) {
    const int r = RPI * i + dr;
    wsrc[i] = we + static_cast<int64_t>(nbase + r) * K + k0 + 8 * (dj ^ (r & (GPR - 1)));
  }
  // non-temporal weight loads only when each expert's column tile is read once
  // (one 64-row tile); with several row tiles the re-reads should hit L2/MALL
  const bool nt = NT && (p1 - p0) <= 64;

  {
    const int rt = rt0;
    const int first = rows ? rows[rt] : rt;
    const uint16_t* xsrc[XI];
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int r = RPI * (wid * XI + i) + dr;
      int src = rows ? rows[rt + r] : rt + r;
      if (src < 0) src = first;
      xsrc[i] = x + static_cast<int64_t>(src) * K + k0 + 8 * (dj ^ (r & (GPR - 1)));
    }
    // K-chunk rotation (k_rotation): expert e's column tiles spread over K
    const int rot = krot ? static_cast<int>((blockIdx.x * 37u + e * 11u) % static_cast<unsigned>(nchunks)) : 0;
    auto issue = [&](uint8_t* slot, int c) {
      const int cr = c + rot;
      const int kk = (cr >= nchunks ? cr - nchunks : cr) * KC;
#pragma unroll
      for (int i = 0; i < XI; ++i) glds16(xsrc[i] + kk, slot + RPI * (wid * XI + i) * RB);
      if (nt) {
#pragma unroll
        for (int i = 0; i < WI; ++i) glds16_nt(wsrc[i] + kk, slot + XBYTES + wid * WBYTES + i * 1024);
      } else {
#pragma unroll
        for (int i = 0; i < WI; ++i) glds16(wsrc[i] + kk, slot + XBYTES + wid * WBYTES + i * 1024);
      }
    };
    f32x4_t acc[NW][MT];
#pragma unroll
    for (int nt_ = 0; nt_ < NW; ++nt_)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[nt_][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](const uint8_t* slot) {
      const uint8_t* xs = slot;
      const uint8_t* ws = slot + XBYTES + wid * WBYTES;
#pragma unroll
      for (int t = 0; t < KC / 32; ++t) {
        const int phys = (4 * t + g) ^ (li & (GPR - 1));
        uint4 b[MT], a[NW];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          b[mt] = *reinterpret_cast<const uint4*>(xs + (16 * mt + li) * RB + phys * 16);
#pragma unroll
        for (int nt_ = 0; nt_ < NW; ++nt_)
          a[nt_] = *reinterpret_cast<const uint4*>(ws + (16 * nt_ + li) * RB + phys * 16);
#pragma unroll
        for (int nt_ = 0; nt_ < NW; ++nt_)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[nt_][mt] = mfma16x16x32(as_frag(a[nt_]), as_frag(b[mt]), acc[nt_][mt]);
      }
    };
    auto step = [&](uint8_t* cur, uint8_t* nxt2, int c) {
      if (c + 1 < nchunks) wait_vmcnt<G>();
      else wait_vmcnt<0>();
      raw_barrier();
      if (c + 2 < nchunks) issue(nxt2, c + 2);
      compute(cur);
    };
    issue(lds0, 0);
    if (nchunks > 1) issue(lds1, 1);
    int c = 0;
    for (; c + 3 <= nchunks; c += 3) {
      step(lds0, lds2, c);
      step(lds1, lds0, c + 1);
      step(lds2, lds1, c + 2);
    }
    if (c < nchunks) step(lds0, lds2, c);
    if (c + 1 < nchunks) step(lds1, lds0, c + 1);

    if (mode == GG_PARTIAL || mode == GG_MOE_RESID) {
      float* pp = part + static_cast<int64_t>(s) * P * N;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = rt + 16 * mt + li;
#pragma unroll
        for (int nt_ = 0; nt_ < NW; ++nt_) {
          float* dst = pp + static_cast<int64_t>(m) * N + nbase + 16 * nt_ + 4 * g;
          if (mode == GG_MOE_RESID) st16_sc1(dst, acc[nt_][mt]);
          else *reinterpret_cast<float4*>(dst) = make_float4(acc[nt_][mt][0], acc[nt_][mt][1], acc[nt_][mt][2],
                                                             acc[nt_][mt][3]);
        }
      }
      if (mode == GG_MOE_RESID) moe_resid_tail<16 * NW * WV, 64 * WV>(part, S, P, N, mre, contributors,
                                                                       reinterpret_cast<int*>(lds0), blockIdx.x);
    } else if (mode == GG_BF16) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = rt + 16 * mt + li;
#pragma unroll
        for (int nt_ = 0; nt_ < NW; ++nt_) {
          uint2 v;
          v.x = pack2(acc[nt_][mt][0], acc[nt_][mt][1]);
          v.y = pack2(acc[nt_][mt][2], acc[nt_][mt][3]);
          *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * N + nbase + 16 * nt_ + 4 * g) = v;
        }
      }
    } else if (NW == 2) {
      const int F = N / 2, f0 = nbase / 2 + 4 * g;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = rt + 16 * mt + li;
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gt = acc[0][mt][r];
          o[r] = gt / (1.f + __expf(-gt)) * acc[NW - 1][mt][r];
        }
        uint2 v;
        v.x = pack2(o[0], o[1]);
        v.y = pack2(o[2], o[3]);
        *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * F + f0) = v;
      }
    }
  }
}

// Grouped (MoE) form of the same pipeline: W [E, N, K]; x rows gathered through
// the block-64 padded expert-sorted layout (rows[p] = source row, -1 = pad;
// rows == nullptr: x already in padded layout); offs[E+1] padded segment starts.
// Grid (column tiles, k-splits, P / 64 row tiles): one workgroup per row tile, so
// an expert's row tiles run concurrently -- the column tiles of one row tile
// (N / cols <= a few hundred) are fewer than the resident workgroups, so the
// next row tiles of the same weight tile are in flight together and re-read it
// from L2/MALL (a per-expert loop over row tiles serialised them). The column
// tile stays the fastest dimension: consecutive workgroups spread over the 8 XCDs
// (row-tile-fastest put a batch-1 step's two active experts on 2 XCDs). Row tiles
// past the last expert's segment (capacity padding) exit at once.
// Row-occupancy dispatch: `valid` (the sorted rows, -1 = pad) tells each workgroup
// how many of its 64 rows are real; it runs the 16-, 32- or 64-row body (MT_MAX
// caps it), so a decode step's ~16-30 rows per expert stage and multiply 1-2 x
// sub-tiles instead of 4 -- the x tile is re-read from L2 by every one of an
// expert's column tiles (448 for Mixtral w13), as many bytes as the weights.
// Rows past the body's 16*MT are never written (pads only: w2 runs the same body
// on the same rows, so it never reads them either).
template <int NW, int WV, int KC, bool NT, int MT_MAX>
__global__ void __launch_bounds__(64 * WV, 1) gemm_m64g_grouped_kernel(const uint16_t* __restrict__ x,
                                                                       const int32_t* __restrict__ rows,
                                                                       const int32_t* __restrict__ offs,
                                                                       const int32_t* __restrict__ valid, int E,
                                                                       int K, const uint16_t* __restrict__ w, int N,
                                                                       int P, float* __restrict__ part,
                                                                       uint16_t* __restrict__ out, int mode,
                                                                       int krot, MoeResidEpi mre) {
  constexpr int SLOT = 16 * MT_MAX * KC * 2 + WV * 16 * NW * KC * 2;
  __shared__ __attribute__((aligned(1024))) uint8_t lds0[SLOT];
  __shared__ __attribute__((aligned(1024))) uint8_t lds1[SLOT];
  __shared__ __attribute__((aligned(1024))) uint8_t lds2[SLOT];
  const int rt0 = blockIdx.z * 64;
  int e = -1;
  for (int i = 0; i < E; ++i)
    if (rt0 >= offs[i] && rt0 < offs[i + 1]) e = i;
  if (e < 0) return;  // capacity padding past the last segment
  const int p0 = offs[e], p1 = offs[e + 1];
  // GG_MOE_RESID: every real row tile x split stores, then tickets (offs is 64-aligned)
  const int contributors = (offs[E] >> 6) * static_cast<int>(gridDim.y);
  // MT_MAX 8 (prefill-sized steps): the 64-row tiles of an aligned pair within the
  // expert's segment run as ONE 128-row workgroup when both of them hold real rows -- the expert's weight tile is streamed once per
  // group instead of once per 64 rows (at ~144 rows per expert the re-reads are
  // what bound the GEMM). Every workgroup of a group counts the group's real rows
  // the same way; all but the leader exit when it takes them. Real rows lead each
  // segment, so the tiles past them are pads (never read by the combine).
  if constexpr (MT_MAX >= 8) {
    constexpr int GT = MT_MAX / 4;                // tiles per group (pairs); groups of three
                                                  // measured slower (profiles/r2_moe_pairs_ab.md)
    const int lt = (rt0 - p0) >> 6, ntl = (p1 - p0) >> 6;
    const int gs = lt / GT * GT, gn = min(GT, ntl - gs);
    if (gn >= 2) {
      const int r0 = p0 + 64 * gs, nrow = 64 * gn;
      const int t = threadIdx.x;
      int real = nrow;
      if (valid != nullptr) {
        real = __syncthreads_count(t < nrow && valid[r0 + t] >= 0);
        if constexpr (64 * WV < 64 * GT)
          real += __syncthreads_count(t + 64 * WV < nrow && valid[r0 + t + 64 * WV] >= 0);
      }
      const int need = (real + 63) >> 6;           // tiles holding real rows (they lead the segment)
      if (need >= 2) {
        if (lt != gs) return;                      // the group leader takes the group's real tiles
        grouped_body<NW, WV, KC, NT, 8>(x, rows, e, p0, p1, r0, K, w, N, P, part, out, mode, lds0, lds1, lds2, krot, mre, contributors);
        return;
      }
    }
  }
  int amt = MT_MAX;
  if (valid != nullptr && MT_MAX > 1) {
    const int t = threadIdx.x;
    const int real = __syncthreads_count(t < 64 && rt0 + t < p1 && valid[rt0 + t] >= 0);
    amt = (real + 15) / 16;
  }
  constexpr int RPI = 1024 / (KC * 2);
  constexpr bool MT1_OK = (16 / RPI / WV) >= 1;  // one 16-row x sub-tile is >= one DMA per wave
  if constexpr (MT_MAX >= 4) {
    if (amt > 2) {
      grouped_body<NW, WV, KC, NT, 4>(x, rows, e, p0, p1, rt0, K, w, N, P, part, out, mode, lds0, lds1, lds2, krot, mre, contributors);
      return;
    }
  }
  if constexpr (MT_MAX >= 2) {
    if (amt == 2 || !MT1_OK) {
      grouped_body<NW, WV, KC, NT, 2>(x, rows, e, p0, p1, rt0, K, w, N, P, part, out, mode, lds0, lds1, lds2, krot, mre, contributors);
      return;
    }
  }
  if constexpr (MT1_OK)
    grouped_body<NW, WV, KC, NT, 1>(x, rows, e, p0, p1, rt0, K, w, N, P, part, out, mode, lds0, lds1, lds2, krot, mre, contributors);
}

int m64g_cfg_kc(int cfg);

template <int NW>
static void launch_m64g_grouped(int cfg, dim3 grid, hipStream_t st, const uint16_t* x, const int32_t* rows,
                                const int32_t* offs, const int32_t* valid, int E, int K, const uint16_t* w, int N,
                                int P, float* part, uint16_t* out, int mode, bool mt1, bool mt8,
                                const MoeResidEpi& mre) {
#define XGK_GRP_MT(WV, KC, NT, MT)                                                                              \
  hipLaunchKernelGGL((gemm_m64g_grouped_kernel<NW, WV, KC, NT, MT>), grid, dim3(64 * WV), 0, st, x, rows, offs, \
                     valid, E, K, w, N, P, part, out, mode, k_rotation(static_cast<int>(grid.y)), mre)
#define XGK_GRP(WV, KC, NT)              \
  do {                                   \
    if (mt1) XGK_GRP_MT(WV, KC, NT, 1);  \
    else XGK_GRP_MT(WV, KC, NT, 4);      \
  } while (0)
  // 128-row pairs (KC 64 configs only: the x slot doubles)
#define XGK_GRP8(WV, KC, NT)                 \
  do {                                       \
    if (mt8) XGK_GRP_MT(WV, KC, NT, 8);      \
    else if (mt1) XGK_GRP_MT(WV, KC, NT, 1); \
    else XGK_GRP_MT(WV, KC, NT, 4);          \
  } while (0)
  // the 4-wave KC-64 configs have < 1 x DMA instruction per wave at 16 rows: MT >= 2
  switch (cfg) {
    case 1: XGK_GRP(4, 128, true); break;
    case 2:
      if (mt8) XGK_GRP_MT(4, 64, false, 8);
      else XGK_GRP_MT(4, 64, false, 4);
      break;
    case 3:
      if (mt8) XGK_GRP_MT(4, 64, true, 8);
      else XGK_GRP_MT(4, 64, true, 4);
      break;
    case 4: XGK_GRP8(2, 64, false); break;
    case 5: XGK_GRP8(2, 64, true); break;
    case 6: XGK_GRP(2, 128, true); break;
    default: XGK_GRP(4, 128, false); break;
  }
#undef XGK_GRP
#undef XGK_GRP8
#undef XGK_GRP_MT
}

int m64g_cfg_waves(int cfg);
int m64g_cfg_kc(int cfg);

// max_rows: a bound on the real rows of any expert (<= 16 selects the one-x-tile
// kernel; rows 16..63 of each padded tile are then left unwritten -- pads only).
// valid: the sorted rows (-1 = pad) for the row-occupancy dispatch, or nullptr (all 64 rows).
// pairs > 0: a bound on the (token, choice) rows over ALL local experts. The real
// 64-row tiles lead the padded layout (segments are packed, 64-aligned), and there are
// at most ceil(pairs / 64) + min(E, pairs) of them, so the grid stops there instead of
// at the capacity P / 64 (batch 1, Mixtral: 3 row tiles instead of 8 -- the empty
// workgroups each paid an offsets read before exiting).
int moe_gemm_m64g(const uint16_t* x, const int32_t* rows, const int32_t* offs, int E, int K, const uint16_t* w, int N,
                  int P, float* part, uint16_t* out, int S, int mode, int nw, int cfg, int max_rows, hipStream_t st,
                  const int32_t* valid, const MoeResidEpi* mre_in, int pairs) {
  if (E < 1 || P < 0 || P % 64 || S < 1 || (nw != 1 && nw != 2) || cfg < 0 || cfg > 6) return 1;
  if (mode != GG_BF16 && mode != GG_PARTIAL && mode != GG_SILU && mode != GG_MOE_RESID) return 1;
  const MoeResidEpi mre = mre_in ? *mre_in : MoeResidEpi{nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0};
  if (mode == GG_MOE_RESID && (mre.dest == nullptr || mre.w == nullptr || mre.resid == nullptr ||
                               mre.ss_out == nullptr || mre.counters == nullptr || mre.T < 1 || mre.k < 1 ||
                               max_rows > 256 || (16 * nw * m64g_cfg_waves(cfg)) % 4 ||
                               N / (16 * nw * m64g_cfg_waves(cfg)) > 64))  // the next norm sums <= 64 per row
    return 1;
  const int cols = 16 * nw * m64g_cfg_waves(cfg), kc = m64g_cfg_kc(cfg);
  if (K % (S * kc) || N % cols) return 1;
  if (mode == GG_SILU && (nw != 2 || S != 1)) return 1;
  if ((mode == GG_PARTIAL || mode == GG_MOE_RESID) && part == nullptr) return 1;
  if (mode != GG_PARTIAL && mode != GG_MOE_RESID && out == nullptr) return 1;
  if (P == 0) return 0;
  const int ztiles = pairs > 0 ? std::min(P / 64, (pairs + 63) / 64 + std::min(E, pairs)) : P / 64;
  const dim3 grid(N / cols, S, ztiles);
  const bool mt1 = max_rows <= 16 && cfg != 2 && cfg != 3;  // 16 x rows >= one DMA per wave
  // 128-row pairs for prefill-sized steps (> 256 pairs; decode keeps the 48 KB-slot
  // kernel and its occupancy), KC 64 configs only
  const bool mt8 = max_rows > 256 && m64g_cfg_kc(cfg) == 64;
  if (nw == 1) launch_m64g_grouped<1>(cfg, grid, st, x, rows, offs, valid, E, K, w, N, P, part, out, mode, mt1, mt8, mre);
  else launch_m64g_grouped<2>(cfg, grid, st, x, rows, offs, valid, E, K, w, N, P, part, out, mode, mt1, mt8, mre);
  return 0;
}

// cfg: 0 = (4 waves, KC 128), 1 = (4, 128, nt), 2 = (4, 64), 3 = (4, 64, nt),
//      4 = (2, 64), 5 = (2, 64, nt), 6 = (2, 128, nt), 7 = (8, 64, nt; four x tiles only:
//      a 16-row x tile is less than one DMA instruction per wave at 8 waves)
template <int NW>
static void launch_m64g(int cfg, dim3 grid, hipStream_t st, const uint16_t* x, int M, int K, const uint16_t* w, int N,
                        float* part, uint16_t* out, int mode, const M64Epi& epi) {
  // M <= 16: the one-x-tile kernel, except the 4-wave KC-64 configs (16 x rows would
  // be less than one DMA instruction per wave)
  const bool mt1 = M <= 16 && cfg != 2 && cfg != 3;
#define XGK_M64G(WV, KC, NT)                                                                                         \
  do {                                                                                                               \
    if (mt1)                                                                                                         \
      hipLaunchKernelGGL((gemm_m64g_kernel<NW, WV, KC, NT, 1>), grid, dim3(64 * WV), 0, st, x, M, K, w, N, part, out, \
                         mode, epi);                                                                                 \
    else                                                                                                             \
      hipLaunchKernelGGL((gemm_m64g_kernel<NW, WV, KC, NT, 4>), grid, dim3(64 * WV), 0, st, x, M, K, w, N, part, out, \
                         mode, epi);                                                                                 \
  } while (0)
#define XGK_M64G4(WV, KC, NT)                                                                                      \
  hipLaunchKernelGGL((gemm_m64g_kernel<NW, WV, KC, NT, 4>), grid, dim3(64 * WV), 0, st, x, M, K, w, N, part, out, \
                     mode, epi)
// deep-ring one-x-tile configurations (M <= 16 only)
#define XGK_M64G_DEEP(WV, KC, NT, NSV)                                                                             \
  hipLaunchKernelGGL((gemm_m64g_kernel<NW, WV, KC, NT, 1, NSV>), grid, dim3(64 * WV), 0, st, x, M, K, w, N, part, \
                     out, mode, epi)
  switch (cfg) {
    case 1: XGK_M64G(4, 128, true); break;
    case 2: XGK_M64G4(4, 64, false); break;
    case 3: XGK_M64G4(4, 64, true); break;
    case 4: XGK_M64G(2, 64, false); break;
    case 5: XGK_M64G(2, 64, true); break;
    case 6: XGK_M64G(2, 128, true); break;
    case 7: XGK_M64G4(8, 64, true); break;
    case 8: XGK_M64G_DEEP(2, 128, true, 5); break;
    case 9: XGK_M64G_DEEP(4, 128, true, 4); break;
    case 10: XGK_M64G_DEEP(2, 64, true, 6); break;
    default: XGK_M64G(4, 128, false); break;
  }
#undef XGK_M64G
#undef XGK_M64G4
#undef XGK_M64G_DEEP
}

int m64g_cfg_waves(int cfg) { return cfg == 7 ? 8 : cfg == 9 ? 4 : (cfg >= 4 ? 2 : 4); }
int m64g_cfg_kc(int cfg) {
  return (cfg == 2 || cfg == 3 || cfg == 4 || cfg == 5 || cfg == 7 || cfg == 10) ? 64 : 128;
}

// Host-side shape / operand checks shared by both entry points (0 = valid).
static int m64g_check(int M, int K, int N, const float* part, const uint16_t* out, int S, int mode, int nw, int cfg,
                      const M64Epi& epi) {
  if (M < 1 || M > 64 || S < 1 || (nw != 1 && nw != 2) || cfg < 0 || cfg > 10) return 1;
  if (cfg >= 8 && M > 16) return 1;  // deep-ring configurations: one x tile only
  if (mode < GG_BF16 || mode > GG_AR || mode == GG_MOE_RESID) return 1;
  // the consumer's statistics paths sum at most 64 partial sums per row, 128 at M <= 16
  if (epi.ss_in != nullptr && (epi.ss_n < 1 || epi.ss_n > (M <= 16 ? 128 : 64) || epi.ss_stride < M)) return 1;
  const int cols = 16 * nw * m64g_cfg_waves(cfg), kc = m64g_cfg_kc(cfg);
  if (K % kc || S > K / kc || N % cols) return 1;
  // split-K SiLU: fp32 slabs + one zeroed arrival ticket per column tile (m64g_silu_tail)
  if (mode == GG_SILU && (nw != 2 || (S > 1 && (part == nullptr || epi.counters == nullptr)))) return 1;
  if (mode == GG_BF16 && S != 1) return 1;
  if ((mode == GG_PARTIAL || mode == GG_RESID || mode == GG_AR) && part == nullptr) return 1;
  if ((mode == GG_BF16 || mode == GG_SILU) && out == nullptr) return 1;
  if ((mode == GG_RESID || mode == GG_AR) && (epi.resid == nullptr || epi.ss_out == nullptr || epi.counters == nullptr))
    return 1;
  if (mode == GG_AR && epi.ar == nullptr) return 1;  // (the descriptor is checked by the host wrapper)
  return 0;
}

static void m64g_launch(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, uint16_t* out, int S,
                        int mode, int nw, int cfg, const M64Epi& epi_in, hipStream_t st) {
  const int tiles = N / (16 * nw * m64g_cfg_waves(cfg));
  M64Epi epi = epi_in;
  epi.krot = k_rotation(S);
  const dim3 grid(tiles, S);
  if (nw == 1) launch_m64g<1>(cfg, grid, st, x, M, K, w, N, part, out, mode, epi);
  else launch_m64g<2>(cfg, grid, st, x, M, K, w, N, part, out, mode, epi);
}

int gemm_m64g(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, uint16_t* out, int S, int mode,
              int nw, int cfg, hipStream_t st) {
  const M64Epi epi{nullptr, 0, 0, 0.f, nullptr, nullptr, nullptr};
  if (mode == GG_RESID || mode == GG_AR || m64g_check(M, K, N, part, out, S, mode, nw, cfg, epi)) return 1;
  m64g_launch(x, M, K, w, N, part, out, S, mode, nw, cfg, epi, st);
  return 0;
}

// Fused-decode entry: the row-scaled input norm (ss_in) and/or the GG_RESID
// epilogue; ss_out holds (N / cols) * M floats, counters N / cols ints.
int gemm_m64g_ex(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, uint16_t* out, int S,
                 int mode, int nw, int cfg, const float* ss_in, int ss_n, int ss_stride, float eps, uint16_t* resid,
                 float* ss_out, int* counters, hipStream_t st) {
  const M64Epi epi{ss_in, ss_n, ss_stride, eps, resid, ss_out, counters};
  if (m64g_check(M, K, N, part, out, S, mode, nw, cfg, epi)) return 1;
  m64g_launch(x, M, K, w, N, part, out, S, mode, nw, cfg, epi, st);
  return 0;
}

// Row-parallel GEMM with the TP all-reduce + residual + statistics in the launch
// (GG_AR); desc: a device copy of ArDesc, validated by the host (linear.py
// m64_ar_resid_linear / comm.GemmArArgs).
int gemm_m64g_ar(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, int S, int nw, int cfg,
                 uint16_t* resid, float* ss_out, int* counters, const void* desc, hipStream_t st) {
  M64Epi epi{nullptr, 0, 0, 0.f, resid, ss_out, counters};
  epi.ar = static_cast<const ArDesc*>(desc);
  if (m64g_check(M, K, N, part, nullptr, S, GG_AR, nw, cfg, epi)) return 1;
  m64g_launch(x, M, K, w, N, part, nullptr, S, GG_AR, nw, cfg, epi, st);
  return 0;
}
int m64g_ar_desc_bytes() { return static_cast<int>(sizeof(ArDesc)); }
static_assert(sizeof(ArDesc) == 30 * 4 && offsetof(ArDesc, region) == 16 * 4 && offsetof(ArDesc, rank) == 18 * 4 &&
                  offsetof(ArDesc, gens) == 22 * 4 && offsetof(ArDesc, pair) == 28 * 4,
              "ArDesc: the tail reads it back by dword (m64g_ar_tail)");

}  // namespace xgk
