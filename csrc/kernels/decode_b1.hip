// Persistent batch-1 decode: every layer of a dense Llama-family model (and the final
// RMSNorm) in ONE launch of 256 workgroups, one per CU.
//
// Why: at batch 1 a decode step is a 14 GB once-read weight stream (Llama-3-8B); as
// five launches per layer every kernel boundary drains and refills the chip's memory
// pipeline (~1.2-1.9 us each, MI355X_MICROARCH.md price list "boundary") and the
// attention / combine kernels are pure latency with the weight stream stopped. Here
// the weight stream never stops: each CU's loader wave walks a STATIC sequence of
// weight lines (all layers, all projections) into an LDS ring, running ahead across
// the data dependencies ("prefetch-credit"), while three consumer waves compute.
//
// Roles per workgroup (4 waves):
//   wave 0      loader: 1-KiB lines (one global_load_lds_dwordx4 nt each) into a ring
//               of NSLOT 16-KiB slots; counted vmcnt waits, "landed" published in LDS;
//               a slot is refilled once every consumer has moved past it (cur[]).
//   waves 1..3  consumers: GEMV rows (v_dot2c_f32_bf16 on 16-B lane chunks, one wave
//               reduction per row), the hand-offs, attention, residual and norms.
// Row ownership (W = 256 workgroups, w = blockIdx.x):
//   QKV   : kv-head group h = w / (W / Hkv) owns its q rows (G heads), k and v rows;
//           its W / Hkv workgroups take equal contiguous slices (norm as a row scale).
//   attn  : workgroup i < S_att of group h = key split i (RoPE, KV append by the split
//           that owns the new key, online softmax) -> partials; then the same
//           workgroups combine one OPW-wide slice of the group's outputs each.
//   O     : rows [w * H/W, +H/W) (+ residual) ; GU: features [w * F/W, +F/W) (SiLU
//           gate, gate|up rows interleaved in blocks of 16) ; down: rows as O.
// Hand-offs between workgroups: 8-byte granules {tag, 32-bit value} written by ONE
// relaxed agent-scope atomic store each and swept with relaxed agent-scope loads
// until every tag matches (cdna_hip_programming.md §6 Guideline 16, R2: the data is
// the flag; no fence). tag = layer * 8 + edge + 1, never 0; the granule area is
// zeroed by a memset node before every launch. Every wait is bounded (ctl[1] ticks
// of the 100 MHz wall clock); a timeout bumps ctl[0], raises the workgroup's abort
// flag and every later wait returns at once, so the grid always drains.
//
// Numerics follow the fused multi-launch path (gemm_m64g + decode attention): norm
// statistics from the bf16 residual, projections in fp32, q/k/v rounded to bf16
// after RoPE, attention output and residual stream in bf16, SiLU-gate in fp32.
#include <algorithm>

#include "common.h"
#include "glds.h"

namespace xgk {
namespace b1 {

constexpr int NWG = 256;
constexpr int NLW = 2;          // loader waves (one wave's LDS-DMA issue tops out at ~19 GB/s per CU,
                                // two reach ~27: bench/dma_probe.hip)
constexpr int NCW = 2;          // consumer waves (4 waves per CU: 512 VGPRs each)
constexpr int NTHR = (NLW + NCW) * 64;
constexpr int CT = NCW * 64;    // consumer threads
constexpr int LINE = 1024;      // ring line: 64 lanes x 16 B
constexpr int SLOT = 16;        // lines per slot
constexpr int HD = 128;         // head dim

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));

enum { E_RESID = 0, E_QKV = 1, E_PART = 2, E_ATTN = 3, E_POST = 4, E_ACT = 5 };
enum { P_QKV = 0, P_O = 1, P_GU = 2, P_DN = 3 };

struct Args {
  const uint64_t* wptr;       // [L][4] qkv, o, gate_up (16-row interleaved), down
  const uint64_t* kvptr;      // [L][2] k_cache, v_cache  [blocks, Hkv, bs, 128] bf16
  const uint16_t* resid_in;   // [H] embedding row
  const uint16_t* final_norm; // [H]
  uint16_t* out;              // [H] normalised final hidden state
  const int32_t* positions;   // [1]
  const int32_t* slot_mapping;
  const int32_t* block_table; // [max_blocks] (row of the one sequence)
  const int32_t* seq_lens;    // [1] (includes the new token)
  const float* cos_sin;       // [max_pos, 128] = [cos | sin]
  uint64_t* gran;             // granule area (zeroed before each launch)
  int* ctl;                   // [0] timeouts, [1] wait limit in wall-clock ticks, [2] test: drop WG 0's QKV,
                              // [3] diagnostics: 1 = consumers ignore the ring, 2 = no weight loads
  int L, H, F, Hq, Hkv, bs, apply_rope;
  float eps, scale;
  // derived on the host (decode_b1_plan)
  int S_att, ring_lines;
  int off_xres, off_xbig, off_ctl;  // LDS byte offsets
  int g_resid, g_post, g_qkv, g_part, g_attn, g_act;  // granule offsets
  uint64_t* stamps;  // diagnostics (null in production): per-(workgroup, layer) phase clocks
  const uint64_t* runs;  // [NWG][runs_stride] {address, lines}: each workgroup's weight stream as
  int runs_stride;       // contiguous runs in line order (decode_b1_build_runs), {0, 0}-terminated
};
constexpr int NSTAMP = 18;

// LDS control block
struct Ctl {
  int landed[NLW];  // loader L: every line of ITS 8-line groups (g % NLW == L) below this landed
  int cur[NCW];     // first line each consumer may still read (consumers -> loaders)
  int cbar;         // consumer barrier arrivals
  int abort_;       // set on any timeout in this workgroup
  int pages[512];   // KV pages of this workgroup's key split (block_table[kb / bs ...])
  float red[16];    // cross-wave reduction scratch
  float res[256];   // per-item partial dot products of the current phase
};
constexpr int SEG = 8;  // ring lines per work item (one wave reduction each)

__device__ __forceinline__ uint32_t tag_of(int layer, int edge) { return static_cast<uint32_t>(layer * 8 + edge + 1); }

__device__ __forceinline__ int lds_ld(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_st(int* p, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Bounded wait bookkeeping (one per wave).
struct Spin {
  uint64_t t0 = 0;
  uint32_t n = 0;
  // true when the wait must give up (timeout here, or an abort raised elsewhere).
  // LDS polls sleep ~30 ns per pass; global (granule) polls ~0.25 us: every pass of a
  // sweep is L2 / fabric traffic that delays the weight stream of the whole chip.
  __device__ __forceinline__ bool tick(Ctl* c, int* ctl, uint64_t limit, bool global_check) {
    if (global_check)
      __builtin_amdgcn_s_sleep(2);
    else
      __builtin_amdgcn_s_sleep(1);
    if ((++n & (global_check ? 7 : 31)) != 0) return false;
    if (lds_ld(&c->abort_)) return true;
    if (global_check && __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
      __hip_atomic_store(&c->abort_, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return true;
    }
    const uint64_t t = wall_clock64();
    if (t0 == 0) t0 = t;
    if (t - t0 > limit) {
      if ((threadIdx.x & 63) == 0) atomicAdd(ctl, 1);
      __hip_atomic_store(&c->abort_, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return true;
    }
    return false;
  }
};

__device__ __forceinline__ void gstore(uint64_t* gran, int idx, uint32_t tag, uint32_t val) {
  __hip_atomic_store((gu64*)(gran + idx), (static_cast<unsigned long long>(tag) << 32) | val,
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t gload(const uint64_t* gran, int idx) {
  return __hip_atomic_load((gu64*)(const_cast<uint64_t*>(gran) + idx), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }

// Sum over the 64 lanes with DPP moves only (no LDS crossbar): xor 1, xor 2, half-row
// mirror, row mirror, then row_bcast15 / row_bcast31 fold the four rows into lane 63;
// the result is read back as a wave-uniform value.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xF, false));
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp_keep(float v) {  // masked-off rows keep v
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, ROW_MASK, 0xF, false));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_keep<0xB1>(v));
  v = fmaxf(v, dpp_keep<0x4E>(v));
  v = fmaxf(v, dpp_keep<0x141>(v));
  v = fmaxf(v, dpp_keep<0x140>(v));
  v = fmaxf(v, dpp_keep<0x142, 0xA>(v));
  v = fmaxf(v, dpp_keep<0x143, 0xC>(v));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp<0xB1>(v);         // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);         // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);        // row_half_mirror
  v += dpp<0x140>(v);        // row_mirror
  v += dpp<0x142, 0xA>(v);   // row_bcast15 -> rows 1, 3
  v += dpp<0x143, 0xC>(v);   // row_bcast31 -> rows 2, 3
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float bitsf(uint32_t u) { return __uint_as_float(u); }

// ---------------------------------------------------------------- work geometry
struct Geo {
  int H, F, Hq, Hkv, G, WPG, RPW, RO, FW, LH, LA, LF;
  int off_o, off_gu, off_dn, LL;
  __device__ __forceinline__ Geo(const Args& a) {
    H = a.H; F = a.F; Hq = a.Hq; Hkv = a.Hkv; G = Hq / Hkv;
    WPG = NWG / Hkv;
    RPW = (G + 2) * HD / WPG;
    RO = H / NWG;
    FW = F / NWG;
    LH = H / 512; LA = Hq * HD / 512; LF = F / 512;
    off_o = RPW * LH;
    off_gu = off_o + RO * LA;
    off_dn = off_gu + 2 * FW * LH;
    LL = off_dn + RO * LF;
  }
  // row (of the projection's weight) of row r of this workgroup in phase p
  __device__ __forceinline__ int row(int p, int w, int r) const {
    if (p == P_QKV) {
      const int h = w / WPG, idx = (w % WPG) * RPW + r;
      if (idx < G * HD) return h * G * HD + idx;
      if (idx < (G + 1) * HD) return Hq * HD + h * HD + (idx - G * HD);
      return (Hq + Hkv) * HD + h * HD + (idx - (G + 1) * HD);
    }
    if (p == P_GU) {  // the workgroup's gate / up rows in memory order (long contiguous runs)
      const int f0 = w * FW, f1 = f0 + FW;
      int base = 0;
      for (int b = f0 >> 4;; ++b) {
        const int lo = max(f0, 16 * b), cnt = min(f1, 16 * b + 16) - lo;
        if (r < base + 2 * cnt) {
          const int rr = r - base, up = rr >= cnt;
          return 32 * b + (lo & 15) + (up ? rr - cnt + 16 : rr);
        }
        base += 2 * cnt;
      }
    }
    return w * RO + r;  // O, down
  }
  // arithmetic selects (a switch here became a lookup table in scratch memory, whose
  // loads the loader's counted vmcnt waits then had to drain)
  // position of feature f's gate (up = 0) or up row in the workgroup's gate_up row order
  __device__ __forceinline__ int gu_pos(int w, int f, int up) const {
    const int f0 = w * FW, f1 = f0 + FW;
    int base = 0;
    for (int b = f0 >> 4; b < (f >> 4); ++b) base += 2 * (min(f1, 16 * b + 16) - max(f0, 16 * b));
    const int b = f >> 4, lo = max(f0, 16 * b), cnt = min(f1, 16 * b + 16) - lo;
    return base + up * cnt + (f - lo);
  }
  __device__ __forceinline__ int nrows(int p) const {
    return RO + (p == P_QKV) * (RPW - RO) + (p == P_GU) * (2 * FW - RO);
  }
  __device__ __forceinline__ int lpr(int p) const {
    return LH + (p == P_O) * (LA - LH) + (p == P_DN) * (LF - LH);
  }
  __device__ __forceinline__ int K(int p) const { return lpr(p) * 512; }
  __device__ __forceinline__ int poff(int p) const {
    return p == P_QKV ? 0 : p == P_O ? off_o : p == P_GU ? off_gu : off_dn;
  }
};

// ---------------------------------------------------------------- loader (wave 0)
__device__ __forceinline__ int min_cur(Ctl* c) {
  int m = lds_ld(&c->cur[0]);
#pragma unroll
  for (int i = 1; i < NCW; ++i) m = min(m, lds_ld(&c->cur[i]));
  return __builtin_amdgcn_readfirstlane(m);
}
__device__ __forceinline__ void publish(Ctl* c, int L, int& pub, int lines) {
  if (lines > pub) {
    pub = lines;
    lds_st(&c->landed[L], pub);
  }
}

// Loader wave L issues the 8-line groups g with g % NLW == L of the one static line
// sequence; its own DMAs are counted by its own vmcnt, so its published count covers
// its groups only (consumers check the loader of each line's group).
__device__ __forceinline__ void loader(const Args& a, Ctl* c, uint8_t* ring, int L) {
  const Geo g(a);  // a private copy: kept in registers (a shared reference put it in scratch)
  const int RL = a.ring_lines;
  const uint64_t limit = static_cast<uint64_t>(__hip_atomic_load(a.ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const int total = a.L * g.LL;
  int j = 0, pub = 0;
  bool dead = false;
  uint64_t free_wait = 0;
  if (a.ctl[3] & 2) {  // diagnostics: consumers alone
    lds_st(&c->landed[L], 0x7fffffff);
    return;
  }
  // the weight stream as contiguous runs (read through the scalar cache, a batch of 4
  // runs = one 64-B line at a time); rptr / rleft: the current run
  const int lane16 = (threadIdx.x & 63) * 16;
  // constant address space: uniform reads become scalar loads (lgkmcnt), never vector
  // loads, whose vmcnt would mix with the counted DMA waits
  typedef __attribute__((address_space(4))) const uint64_t cu64;
  cu64* rt = (cu64*)(a.runs) + static_cast<int64_t>(blockIdx.x) * a.runs_stride * 2;
  int k = 0;
  uint64_t rptr = rt[0];
  int rleft = static_cast<int>(rt[1]);
#define B1_NEXT_RUN()                                    \
  {                                                      \
    ++k;                                                 \
    rptr = rt[2 * k];                                    \
    rleft = static_cast<int>(rt[2 * k + 1]);             \
  }
#define B1_SKIP(N)                                       \
  {                                                      \
    int n_ = (N);                                        \
    while (n_ > 0 && rleft > 0) {                        \
      const int st_ = min(n_, rleft);                    \
      rptr += static_cast<uint64_t>(st_) * LINE;         \
      rleft -= st_;                                      \
      n_ -= st_;                                         \
      if (rleft == 0) B1_NEXT_RUN();                     \
    }                                                    \
  }
  B1_SKIP(8 * L);  // this loader's first group
  j = 8 * L;
  int rp = j % RL;
  for (; j < total; j += 8 * NLW) {
    // group of 8 lines [j, j + 8): it overwrites lines [j - RL, j - RL + 8), free once
    // every consumer holds nothing below j - RL + 8
    const int need = j + 8 - RL;
    if (need > 0 && min_cur(c) < need) {
      // ring full: publish what has landed in steps, keeping the rest of this loader's
      // DMA pipeline in flight (its groups j/8 - 2, - 4, - 6 may be outstanding here)
      const uint64_t tw = a.stamps ? wall_clock64() : 0;
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      publish(c, L, pub, j - 40);
      if (min_cur(c) < need) {
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        publish(c, L, pub, j - 24);
        if (min_cur(c) < need) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          publish(c, L, pub, j - 8);
          Spin sp;
          while (min_cur(c) < need)
            if (sp.tick(c, a.ctl, limit, false)) { dead = true; break; }
        }
      }
      if (a.stamps) free_wait += wall_clock64() - tw;
      if (dead) break;
    }
    const int n = min(8, total - j);
    for (int i = 0; i < n; ++i) {
      if (rleft <= 0) break;  // defensive: the table ended early (never issue past it)
      glds16_nt(reinterpret_cast<const uint8_t*>(rptr) + lane16, ring + (rp + i) * LINE);
      rptr += LINE;
      if (--rleft == 0) B1_NEXT_RUN();
    }
    B1_SKIP(8 * (NLW - 1));  // the other loaders' groups
    rp += 8 * NLW;
    if (rp >= RL) rp -= RL;
    // this loader's last 3 groups (24 DMAs) may still be in flight: its group j/8 - 6
    // (and every earlier one) has landed
    asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    publish(c, L, pub, j + 8 - 48);
  }
#undef B1_NEXT_RUN
#undef B1_SKIP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_st(&c->landed[L], dead ? 0x7fffffff : j);
  if (a.stamps && (threadIdx.x & 63) == 0 && L == 0) {
    uint64_t* st = a.stamps + static_cast<int64_t>(NWG) * a.L * NSTAMP + blockIdx.x * 4;
    st[0] = free_wait;
    st[1] = wall_clock64();
  }
}

// ---------------------------------------------------------------- consumer helpers
struct Cons {
  const Args& a;
  const Geo& g;
  Ctl* c;
  const uint8_t* ring;
  int cw, lane, ctid;
  int landed_c0, landed_c1;  // per-loader landed counts last seen
  int cbar_seq;
  int mode;
  uint64_t limit;
  uint64_t line_wait = 0;  // diagnostics: wall-clock ticks spent waiting for ring lines
  uint64_t* stp = nullptr;  // diagnostics: this workgroup's phase clocks (consumer thread 0)
  __device__ __forceinline__ void stamp(int layer, int i) {
    if (stp) stp[layer * NSTAMP + i] = wall_clock64();
  }
  __device__ __forceinline__ Cons(const Args& a_, const Geo& g_, Ctl* c_, const uint8_t* r_)
      : a(a_), g(g_), c(c_), ring(r_) {
    ctid = threadIdx.x - 64 * NLW;
    cw = __builtin_amdgcn_readfirstlane(ctid >> 6);  // wave-uniform: item loops and branches stay scalar
    lane = threadIdx.x & 63;
    landed_c0 = landed_c1 = 0;
    cbar_seq = 0;
    mode = a.ctl[3];
    limit = static_cast<uint64_t>(__hip_atomic_load(a.ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  __device__ __forceinline__ bool aborted() const { return lds_ld(&c->abort_) != 0; }

  // barrier of the three consumer waves (the loader never joins)
  __device__ __forceinline__ void cbar() {
    cbar_seq += NCW;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // LDS only: global traffic needs no barrier here
    if (lane == 0) __hip_atomic_fetch_add(&c->cbar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    Spin sp;
    while (lds_ld(&c->cbar) < cbar_seq)
      if (sp.tick(c, a.ctl, limit, false)) break;
    asm volatile("" ::: "memory");  // no LDS access moves above the poll (LDS is in order per wave)
  }
  __device__ __forceinline__ void set_cur(int line) {
    if (mode & 1) line = 0x7fffffff;  // diagnostics: the loader alone
    if (lane == 0) lds_st(&c->cur[cw], line);
  }
  __device__ __forceinline__ void wait_line(int j) {
    const int L = (j >> 3) & (NLW - 1);
    if (j < (L ? landed_c1 : landed_c0) || (mode & 1)) return;
    Spin sp;
    int l = lds_ld(&c->landed[L]);
    const uint64_t tw = (a.stamps && l <= j) ? wall_clock64() : 0;
    while (l <= j) {
      if (sp.tick(c, a.ctl, limit, false)) { l = 0x7fffffff; break; }
      l = lds_ld(&c->landed[L]);
    }
    asm volatile("" ::: "memory");
    if (tw) line_wait += wall_clock64() - tw;
    const int lu = __builtin_amdgcn_readfirstlane(l);
    if (L == 0) landed_c0 = lu; else landed_c1 = lu;
  }
  // one full row segment with x already in registers (phases whose rows are exactly one
  // segment: the same x for every item, read from LDS once per phase)
  __device__ __forceinline__ float dot_row_x(int j0, int rp0, const uint4* xr, int jrelease) {
    wait_line(j0);
    wait_line(j0 + SEG - 1);
    const int RL = a.ring_lines;
    uint4 wv[SEG];
#pragma unroll
    for (int i = 0; i < SEG; ++i) {
      const int rp = rp0 + i >= RL ? rp0 + i - RL : rp0 + i;
      wv[i] = *reinterpret_cast<const uint4*>(ring + rp * LINE + lane * 16);
    }
    set_cur(jrelease);
    float acc0 = 0.f, acc1 = 0.f;
#pragma unroll
    for (int i = 0; i < SEG; ++i) {
      acc0 = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, wv[i].x), __builtin_bit_cast(bf2_t, xr[i].x), acc0, false);
      acc1 = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, wv[i].y), __builtin_bit_cast(bf2_t, xr[i].y), acc1, false);
      acc0 = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, wv[i].z), __builtin_bit_cast(bf2_t, xr[i].z), acc0, false);
      acc1 = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, wv[i].w), __builtin_bit_cast(bf2_t, xr[i].w), acc1, false);
    }
    return wave_sum_dpp(acc0 + acc1);
  }

  __device__ __forceinline__ float dot_row(int j0, int nl, const uint16_t* x, int jrelease) {
    wait_line(j0);
    wait_line(j0 + nl - 1);
    const int RL = a.ring_lines;
    const int rp0 = j0 % RL;
    float acc0 = 0.f, acc1 = 0.f;
    if (nl == SEG) {  // full segment: branch-free, all 16 LDS reads in flight
      uint4 wv[SEG], xv[SEG];
#pragma unroll
      for (int i = 0; i < SEG; ++i) {
        const int rp = rp0 + i >= RL ? rp0 + i - RL : rp0 + i;
        wv[i] = *reinterpret_cast<const uint4*>(ring + rp * LINE + lane * 16);
        xv[i] = *reinterpret_cast<const uint4*>(x + i * 512 + lane * 8);
      }
      set_cur(jrelease);  // the item's lines are in registers once these reads return
#pragma unroll
      for (int i = 0; i < SEG; ++i) {
        acc0 = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, wv[i].x), __builtin_bit_cast(bf2_t, xv[i].x), acc0, false);
        acc1 = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, wv[i].y), __builtin_bit_cast(bf2_t, xv[i].y), acc1, false);
        acc0 = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, wv[i].z), __builtin_bit_cast(bf2_t, xv[i].z), acc0, false);
        acc1 = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, wv[i].w), __builtin_bit_cast(bf2_t, xv[i].w), acc1, false);
      }
    } else {  // a row's tail segment (K not a multiple of 4096)
      int rp = rp0;
      for (int i = 0; i < nl; ++i) {
        const uint4 wv = *reinterpret_cast<const uint4*>(ring + rp * LINE + lane * 16);
        const uint4 xv = *reinterpret_cast<const uint4*>(x + i * 512 + lane * 8);
        acc0 = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, wv.x), __builtin_bit_cast(bf2_t, xv.x), acc0, false);
        acc1 = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, wv.y), __builtin_bit_cast(bf2_t, xv.y), acc1, false);
        acc0 = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, wv.z), __builtin_bit_cast(bf2_t, xv.z), acc0, false);
        acc1 = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, wv.w), __builtin_bit_cast(bf2_t, xv.w), acc1, false);
        rp = rp + 1 == RL ? 0 : rp + 1;
      }
      set_cur(jrelease);
    }
    return wave_sum_dpp(acc0 + acc1);
  }

  // Sweep n granules (src index = map(i)) until every tag matches; data -> dst[i].
  // The three consumer waves split the work; callers cbar() after.
  template <int B = 16, typename Map>  // B <= 64 granules per lane per pass
  __device__ __forceinline__ void gather(int n, uint32_t tag, uint32_t* dst, Map map) {
    for (int base = cw * 64 * B; base < n; base += CT * B) {
      uint64_t v[B];
      uint64_t pend = 0;  // granules of this lane not matched yet: only those are re-read
#pragma unroll
      for (int k = 0; k < B; ++k)
        if (base + k * 64 + lane < n) pend |= 1ull << k;
      Spin sp;
      for (;;) {
        // every pending load issued before the first tag check (a check right after each
        // load made the sweep one round trip per granule)
#pragma unroll
        for (int k = 0; k < B; ++k)
          if (pend & (1ull << k)) v[k] = gload(a.gran, map(base + k * 64 + lane));
#pragma unroll
        for (int k = 0; k < B; ++k)
          if ((pend & (1ull << k)) && static_cast<uint32_t>(v[k] >> 32) == tag) pend &= ~(1ull << k);
        if (__all(pend == 0)) break;
        if (sp.tick(c, a.ctl, limit, true)) break;
      }
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const int i = base + k * 64 + lane;
        if (i < n) dst[i] = static_cast<uint32_t>(v[k]);
      }
    }
  }

  // sum of squares of the bf16 vector x[0:n] over the consumer threads -> rsqrt(ms + eps)
  __device__ __forceinline__ float norm_scale(const uint16_t* x, int n) {
    float s = 0.f;
    for (int i = ctid * 8; i < n; i += CT * 8) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + i), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) s += f[k] * f[k];
    }
    s = wave_sum(s);
    if (lane == 0) c->red[cw] = s;
    cbar();
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < NCW; ++i) tot += c->red[i];
    const float rs = rsqrtf(tot / static_cast<float>(n) + a.eps);
    cbar();  // red[] is reused by the next reduction
    return rs;
  }
};

__device__ __forceinline__ float bf16r(float f) { return bf2f(f2bf(f)); }

// ---------------------------------------------------------------- attention (split i of group h)
template <int GQ>  // query heads per kv head (compile time: loops over heads unroll without guards)
__device__ __forceinline__ void attention(Cons& k, int layer, int h, int i, uint8_t* scratch) {
  const Args& a = k.a;
  const Geo& g = k.g;
  constexpr int G = GQ;
  const int S = a.S_att;
  const int ctx = a.seq_lens[0], pos = a.positions[0], slot = a.slot_mapping[0];
  const int cs = (ctx + S - 1) / S;
  const int kb = min(i * cs, ctx), ke = min(kb + cs, ctx);
  // scratch layout (floats): gq[(G+2)*128] | qb (bf16 G*128) | knew, vnew (bf16 128 each)
  //                          | pw[NCW][64][8] | wm[NCW][G] wl[NCW][G] | wo[NCW][G][128]
  float* gq = reinterpret_cast<float*>(scratch);
  uint16_t* qb = reinterpret_cast<uint16_t*>(gq + (G + 2) * HD);
  uint16_t* knew = qb + G * HD;
  uint16_t* vnew = knew + HD;
  float* pw = reinterpret_cast<float*>(vnew + HD);
  float* wm = pw + NCW * 64 * 8;
  float* wl = wm + NCW * G;
  float* wo = wl + NCW * G;

  uint16_t* kc = reinterpret_cast<uint16_t*>(a.kvptr[layer * 2 + 0]);
  uint16_t* vc = reinterpret_cast<uint16_t*>(a.kvptr[layer * 2 + 1]);
  const int bs = a.bs;
  const int lane = k.lane;
  const int* pg = k.c->pages - kb / 16;  // pg[t / 16] = page of key t (t in [kb, ke))
  // each consumer wave takes a contiguous third of the split's keys, in chunks of 64
  const int nk = ke - kb, per = (nk + NCW - 1) / NCW;
  const int wb = min(kb + k.cw * per, ke), we = min(wb + per, ke);
  // K rows (lane = key) and V (lane = dim pair, one register per key) of a chunk. The
  // cached keys do not depend on this step, so the first chunk is requested BEFORE the
  // QKV hand-off: its HBM latency hides under the wait (a dependent load per key was
  // ~1.5 us each).
  uint4 kreg[HD / 8];
  uint32_t vreg[32];  // V of the chunk's first 32 keys (VGPR budget: 2 waves per SIMD)
// A chunk's (<= 64 keys) pages are at most five 16-key blocks: read them once (LDS),
// then every K / V address is arithmetic (a page lookup per key serialised ~64 LDS
// round trips in front of the loads).
#define B1_LOAD_CHUNK(T0)                                                                               \
  {                                                                                                     \
    const int b0_ = (T0) >> 4, o_ = (T0) & 15;                                                          \
    int pp_[5];                                                                                         \
    _Pragma("unroll") for (int q_ = 0; q_ < 5; ++q_) pp_[q_] = pg[min(b0_ + q_, (we - 1) >> 4)];       \
    auto page_ = [&](int q) { return q == 0 ? pp_[0] : q == 1 ? pp_[1] : q == 2 ? pp_[2] : q == 3 ? pp_[3] : pp_[4]; }; \
    const int t_ = (T0) + lane;                                                                         \
    if (t_ < we && t_ != ctx - 1) {                                                                     \
      const uint16_t* kr_ =                                                                             \
          kc + ((static_cast<int64_t>(page_((o_ + lane) >> 4)) * g.Hkv + h) * 16 + (t_ & 15)) * HD;     \
      _Pragma("unroll") for (int d_ = 0; d_ < HD / 8; ++d_) kreg[d_] =                                  \
          *reinterpret_cast<const uint4*>(kr_ + d_ * 8);                                                \
    }                                                                                                   \
    _Pragma("unroll") for (int tt_ = 0; tt_ < 32; ++tt_) {                                              \
      const int tk_ = (T0) + tt_;                                                                       \
      if (tk_ < we && tk_ != ctx - 1)                                                                   \
        vreg[tt_] = reinterpret_cast<const uint32_t*>(                                                  \
            vc + ((static_cast<int64_t>(page_((o_ + tt_) >> 4)) * g.Hkv + h) * 16 + (tk_ & 15)) * HD)[lane]; \
    }                                                                                                   \
  }
  if (wb < we) B1_LOAD_CHUNK(wb);
  k.stamp(layer, 10);

  // A: this group's q/k/v rows (fp32, normed projections)
  const int q0 = h * G * HD, k0 = g.Hq * HD + h * HD, v0 = (g.Hq + g.Hkv) * HD + h * HD;
  const int nq = (G + 2) * HD;
  k.gather(nq, tag_of(layer, E_QKV), reinterpret_cast<uint32_t*>(gq), [&](int x) {
    return a.g_qkv + (x < G * HD ? q0 + x : x < (G + 1) * HD ? k0 + (x - G * HD) : v0 + (x - (G + 1) * HD));
  });
  k.cbar();
  k.stamp(layer, 11);
  // B: RoPE (rotate-half pairs d, d + 64) and bf16 rounding
  const float* csr = a.cos_sin + static_cast<int64_t>(pos) * HD;
  for (int it = k.ctid; it < (G + 1) * 64 + 64; it += CT) {
    if (it < (G + 1) * 64) {
      const int hh = it >> 6, d = it & 63;
      float x1 = gq[hh * HD + d], x2 = gq[hh * HD + d + 64];
      if (a.apply_rope) {
        const float cv = csr[d], sv = csr[64 + d];
        const float y1 = x1 * cv - x2 * sv, y2 = x2 * cv + x1 * sv;
        x1 = y1;
        x2 = y2;
      }
      uint16_t* o = hh < G ? qb + hh * HD : knew;
      o[d] = f2bf(x1);
      o[d + 64] = f2bf(x2);
    } else {
      const int d = 2 * (it - (G + 1) * 64);
      vnew[d] = f2bf(gq[(G + 1) * HD + d]);
      vnew[d + 1] = f2bf(gq[(G + 1) * HD + d + 1]);
    }
  }
  k.cbar();
  k.stamp(layer, 12);
  // the split owning the new key appends it to the paged cache (read from LDS here;
  // the next step's launch reads it from the cache)
  if (slot >= 0 && kb <= ctx - 1 && ctx - 1 < ke && k.cw == 0) {
    const int64_t dst = ((static_cast<int64_t>(slot / bs) * g.Hkv + h) * bs + slot % bs) * HD;
    reinterpret_cast<uint32_t*>(kc + dst)[lane] = reinterpret_cast<const uint32_t*>(knew)[lane];
    reinterpret_cast<uint32_t*>(vc + dst)[lane] = reinterpret_cast<const uint32_t*>(vnew)[lane];
  }
  // C: online softmax over the wave's keys
  float m[G], l[G], o0[G], o1[G];
#pragma unroll
  for (int gg = 0; gg < G; ++gg) { m[gg] = -INFINITY; l[gg] = 0.f; o0[gg] = 0.f; o1[gg] = 0.f; }
  float* mypw = pw + k.cw * 64 * 8;  // [key][8 heads]: one b128 read gives 4 heads' p
  const uint32_t vnew_l = reinterpret_cast<const uint32_t*>(vnew)[lane];
  for (int t0 = wb; t0 < we; t0 += 64) {
    if (t0 != wb) B1_LOAD_CHUNK(t0);
    const int t = t0 + lane;
    const bool valid = t < we;
    if (t == ctx - 1) {
#pragma unroll
      for (int d = 0; d < HD / 8; ++d) kreg[d] = *reinterpret_cast<const uint4*>(knew + d * 8);
    }
    float s[G];
#pragma unroll
    for (int gg = 0; gg < G; ++gg) s[gg] = 0.f;
#pragma unroll
    for (int d = 0; d < HD / 8; ++d) {
      float kf[8];
      unpack8(kreg[d], kf);
#pragma unroll
      for (int gg = 0; gg < G; ++gg) {
        {
          float qf[8];
          unpack8(*reinterpret_cast<const uint4*>(qb + gg * HD + d * 8), qf);
#pragma unroll
          for (int e = 0; e < 8; ++e) s[gg] += qf[e] * kf[e];
        }
      }
    }
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      {
        const float sv = valid ? s[gg] * a.scale : -INFINITY;
        const float cm = wave_max_dpp(sv);
        const float nm = fmaxf(m[gg], cm);
        const float alpha = m[gg] == -INFINITY ? 0.f : __expf(m[gg] - nm);
        const float p = valid ? __expf(sv - nm) : 0.f;
        l[gg] = l[gg] * alpha + wave_sum_dpp(p);
        o0[gg] *= alpha;
        o1[gg] *= alpha;
        m[gg] = nm;
        mypw[lane * 8 + gg] = p;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int nt = min(64, we - t0);
    for (int half = 0; half < 2; ++half) {
      const int tb = half * 32;
      if (tb >= nt) break;
      if (half == 1) {  // keys 32..63 of the chunk: V loaded now
#pragma unroll
        for (int tt = 0; tt < 32; ++tt) {
          const int tk = t0 + 32 + tt;
          if (tk < we && tk != ctx - 1)
            vreg[tt] = reinterpret_cast<const uint32_t*>(
                vc + ((static_cast<int64_t>(pg[tk >> 4]) * g.Hkv + h) * 16 + (tk & 15)) * HD)[lane];
        }
      }
#pragma unroll
      for (int tt = 0; tt < 32; ++tt) {
        if (tb + tt < nt) {
          const uint32_t vv = (t0 + tb + tt == ctx - 1) ? vnew_l : vreg[tt];
          const float va = __uint_as_float(vv << 16), vb = __uint_as_float(vv & 0xFFFF0000u);
          const float4 pa = *reinterpret_cast<const float4*>(mypw + (tb + tt) * 8);
          const float4 pb = G > 4 ? *reinterpret_cast<const float4*>(mypw + (tb + tt) * 8 + 4) : pa;
          const float pv[8] = {pa.x, pa.y, pa.z, pa.w, pb.x, pb.y, pb.z, pb.w};  // heads >= G unused
#pragma unroll
          for (int gg = 0; gg < G; ++gg) {
            {
              o0[gg] += pv[gg] * va;
              o1[gg] += pv[gg] * vb;
            }
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
#undef B1_LOAD_CHUNK
#pragma unroll
  for (int gg = 0; gg < G; ++gg) {
    {
      if (lane == 0) {
        wm[k.cw * G + gg] = m[gg];
        wl[k.cw * G + gg] = l[gg];
      }
      wo[(k.cw * G + gg) * HD + 2 * lane] = o0[gg];
      wo[(k.cw * G + gg) * HD + 2 * lane + 1] = o1[gg];
    }
  }
  k.cbar();
  k.stamp(layer, 13);
  // D: merge the three waves and publish the split's partials: per head {m, l, o[128]}
  const uint32_t tp = tag_of(layer, E_PART);
  for (int e = k.ctid; e < G * (HD + 2); e += CT) {
    const int gg = e / (HD + 2), kk = e % (HD + 2);
    float M = -INFINITY;
    for (int w = 0; w < NCW; ++w) M = fmaxf(M, wm[w * G + gg]);
    float val;
    if (kk == 0) {
      val = M;
    } else {
      val = 0.f;
      for (int w = 0; w < NCW; ++w) {
        const float mw = wm[w * G + gg];
        const float f = (mw == -INFINITY) ? 0.f : __expf(mw - M);
        val += f * (kk == 1 ? wl[w * G + gg] : wo[(w * G + gg) * HD + kk - 2]);
      }
    }
    gstore(a.gran, a.g_part + ((h * S + i) * G + gg) * (HD + 2) + kk, tp, fbits(val));
  }
  k.cbar();
  k.stamp(layer, 14);
  // E: combine one OPW-wide slice of the group's G*128 outputs over the S splits
  const int OPW = G * HD / S;
  const int gs = (i * OPW) / HD, d0 = (i * OPW) % HD;
  const int per_s = OPW + 2;
  uint32_t* cb = reinterpret_cast<uint32_t*>(scratch);
  k.gather(S * per_s, tp, cb, [&](int x) {
    const int s_ = x / per_s, e_ = x % per_s;
    return a.g_part + ((h * S + s_) * G + gs) * (HD + 2) + (e_ < 2 ? e_ : 2 + d0 + e_ - 2);
  });
  k.cbar();
  k.stamp(layer, 15);
  // lane = split (S <= 32): max, weights and the denominator are wave reductions; each
  // wave reduces every third output pair (a serial loop over the splits per output was
  // ~5 us of dependent LDS reads)
  const uint32_t ta = tag_of(layer, E_ATTN);
  {
    const int sl = lane < S ? lane : 0;
    const float ms = lane < S ? bitsf(cb[sl * per_s]) : -INFINITY;
    const float M = wave_max(ms);
    const float f = ms == -INFINITY ? 0.f : __expf(ms - M);
    const float den = wave_sum_dpp(f * (lane < S ? bitsf(cb[sl * per_s + 1]) : 0.f));
    const float inv = den > 0.f ? 1.f / den : 0.f;
    for (int t = k.cw; t < OPW / 2; t += NCW) {
      const float n0 = wave_sum_dpp(f * bitsf(cb[sl * per_s + 2 + 2 * t]));
      const float n1 = wave_sum_dpp(f * bitsf(cb[sl * per_s + 3 + 2 * t]));
      if (lane == 0) gstore(a.gran, a.g_attn + ((h * G + gs) * HD + d0) / 2 + t, ta, pack2(n0 * inv, n1 * inv));
    }
  }
}

// ---------------------------------------------------------------- consumer main
// One projection phase: its rows split into work items of <= SEG lines, dealt round-
// robin to the consumer waves, so the three waves read adjacent lines and the ring
// space they hold back from the loader stays ~3 items (a whole-row unit per wave held
// the loader to a few lines of run-ahead on the 32-line gate_up units). Item partials
// go to c->res; the caller reduces them per row after a cbar.
__device__ __forceinline__ void phase_items(Cons& k, int jphase, int nrows, int lp, const uint16_t* x, int jnext,
                                            int stamp_layer = -1) {
  const int ipr = (lp + SEG - 1) / SEG;
  const int nit = (k.mode & 4) ? 0 : nrows * ipr;  // diagnostics: 4 = no projection work
  if (lp == SEG) {  // one item per row: x in registers, ring position stepped (no divisions)
    const int RL = k.a.ring_lines, step = NCW * SEG;
    uint4 xr[SEG];
#pragma unroll
    for (int i = 0; i < SEG; ++i) xr[i] = *reinterpret_cast<const uint4*>(x + i * 512 + k.lane * 8);
    int rp = (jphase + k.cw * SEG) % RL;
    if (k.cw < nit) k.set_cur(jphase + k.cw * SEG);
    if (stamp_layer >= 0) k.stamp(stamp_layer, 16);
    for (int it = k.cw; it < nit; it += NCW) {
      const int j0 = jphase + it * SEG;
      const float v = k.dot_row_x(j0, rp, xr, it + NCW < nit ? j0 + step : jnext);
      if (k.lane == 0) k.c->res[it] = v;
      rp += step;
      if (rp >= RL) rp -= RL;
    }
    if (stamp_layer >= 0) k.stamp(stamp_layer, 17);
    k.set_cur(jnext);
    k.cbar();
    return;
  }
  for (int it = k.cw; it < nit; it += NCW) {
    const int r = it / ipr, l0 = (it % ipr) * SEG;
    const int j0 = jphase + r * lp + l0;
    const int in = it + NCW;  // this wave's next item: its start is the new hold point
    const int jn = in < nit ? jphase + (in / ipr) * lp + (in % ipr) * SEG : jnext;
    k.set_cur(j0);
    const float v = k.dot_row(j0, min(SEG, lp - l0), x + l0 * 512, jn);
    if (k.lane == 0) k.c->res[it] = v;
  }
  k.set_cur(jnext);
  k.cbar();
}
__device__ __forceinline__ float row_sum(const Ctl* c, int r, int ipr) {
  float v = 0.f;
  for (int i = 0; i < ipr; ++i) v += c->res[r * ipr + i];
  return v;
}

template <int GQ>
__device__ __forceinline__ void consumer(const Args& a, Ctl* c, const uint8_t* ring, uint8_t* smem) {
  const Geo g(a);
  Cons k(a, g, c, ring);
  if (k.mode & 8) {  // diagnostics: the loader streams alone, the consumers leave
    k.set_cur(0x7fffffff);
    if (a.stamps && k.ctid == 0) a.stamps[static_cast<int64_t>(blockIdx.x) * a.L * NSTAMP] = wall_clock64();
    return;
  }
  uint16_t* xres = reinterpret_cast<uint16_t*>(smem + a.off_xres);
  uint16_t* xbig = reinterpret_cast<uint16_t*>(smem + a.off_xbig);
  const int w = blockIdx.x;
  const int h = w / g.WPG, gi = w % g.WPG;
  const int ct = k.ctid;
  const int iH = (g.LH + SEG - 1) / SEG, iA = (g.LA + SEG - 1) / SEG, iF = (g.LF + SEG - 1) / SEG;
  uint64_t* stp = (a.stamps && ct == 0) ? a.stamps + static_cast<int64_t>(w) * a.L * NSTAMP : nullptr;
  k.stp = stp;
  if (gi < a.S_att) {  // the key split's pages, read once for all layers
    const int ctx = a.seq_lens[0], cs = (ctx + a.S_att - 1) / a.S_att;
    const int kb = min(gi * cs, ctx), ke = min(kb + cs, ctx);
    if (ke > kb)
      for (int p = kb / a.bs + ct; p <= (ke - 1) / a.bs; p += CT) c->pages[p - kb / a.bs] = a.block_table[p];
  }
#define B1_STAMP(i) \
  if (stp) stp[layer * NSTAMP + (i)] = wall_clock64()
  for (int layer = 0; layer < a.L; ++layer) {
    const int lbase = layer * g.LL;
    B1_STAMP(0);
    // ---- residual stream in: the embedding row, or the previous layer's down outputs
    if (layer == 0) {
      for (int x = ct * 8; x < g.H; x += CT * 8)
        *reinterpret_cast<uint4*>(xres + x) = *reinterpret_cast<const uint4*>(a.resid_in + x);
    } else {
      k.gather(g.H / 2, tag_of(layer, E_RESID), reinterpret_cast<uint32_t*>(xres),
               [&](int x) { return a.g_resid + x; });
    }
    k.cbar();
    float rs = k.norm_scale(xres, g.H);
    B1_STAMP(1);
    // ---- QKV rows (norm as a row scale) -> fp32 granules
    phase_items(k, lbase, g.RPW, g.LH, xres, lbase + g.off_o);
    {
      const uint32_t tq = tag_of(layer, E_QKV);
      const bool drop = w == 0 && a.ctl[2] != 0;  // fault injection (tests: a dead producer)
      for (int r = ct; r < g.RPW; r += CT)
        if (!drop) gstore(a.gran, a.g_qkv + g.row(P_QKV, w, r), tq, fbits(row_sum(c, r, iH) * rs));
    }
    B1_STAMP(2);
    // ---- attention + combine (the first S_att workgroups of every kv-head group)
    if (gi < a.S_att) attention<GQ>(k, layer, h, gi, reinterpret_cast<uint8_t*>(xbig));
    k.cbar();
    B1_STAMP(3);
    k.gather(g.Hq * HD / 2, tag_of(layer, E_ATTN), reinterpret_cast<uint32_t*>(xbig),
             [&](int x) { return a.g_attn + x; });
    k.cbar();
    B1_STAMP(4);
    // ---- O rows + residual -> bf16x2 granules
    phase_items(k, lbase + g.off_o, g.RO, g.LA, xbig, lbase + g.off_gu);
    {
      const uint32_t tpo = tag_of(layer, E_POST);
      for (int u = ct; u < g.RO / 2; u += CT) {
        const int r0 = w * g.RO + 2 * u;
        gstore(a.gran, a.g_post + r0 / 2, tpo,
               pack2(bf2f(xres[r0]) + row_sum(c, 2 * u, iA), bf2f(xres[r0 + 1]) + row_sum(c, 2 * u + 1, iA)));
      }
    }
    B1_STAMP(5);
    k.cbar();  // every wave is done with the old residual in xres
    k.gather(g.H / 2, tag_of(layer, E_POST), reinterpret_cast<uint32_t*>(xres), [&](int x) { return a.g_post + x; });
    k.cbar();
    rs = k.norm_scale(xres, g.H);
    B1_STAMP(6);
    // ---- gate_up (rows in memory order, Geo::row) -> SiLU gate per feature pair
    phase_items(k, lbase + g.off_gu, 2 * g.FW, g.LH, xres, lbase + g.off_dn, layer);
    {
      const uint32_t tg = tag_of(layer, E_ACT);
      for (int u = ct; u < g.FW / 2; u += CT) {
        const int f = w * g.FW + 2 * u;
        const float g0 = row_sum(c, g.gu_pos(w, f, 0), iH) * rs, u0 = row_sum(c, g.gu_pos(w, f, 1), iH) * rs;
        const float g1 = row_sum(c, g.gu_pos(w, f + 1, 0), iH) * rs, u1 = row_sum(c, g.gu_pos(w, f + 1, 1), iH) * rs;
        gstore(a.gran, a.g_act + (w * g.FW) / 2 + u, tg,
               pack2(g0 / (1.f + __expf(-g0)) * u0, g1 / (1.f + __expf(-g1)) * u1));
      }
    }
    B1_STAMP(7);
    k.gather<40>(g.F / 2, tag_of(layer, E_ACT), reinterpret_cast<uint32_t*>(xbig), [&](int x) { return a.g_act + x; });
    k.cbar();
    B1_STAMP(8);
    // ---- down rows + residual -> the next layer's residual granules
    phase_items(k, lbase + g.off_dn, g.RO, g.LF, xbig, layer + 1 < a.L ? lbase + g.LL : 0x7fffffff);
    {
      const uint32_t tr = tag_of(layer + 1, E_RESID);
      for (int u = ct; u < g.RO / 2; u += CT) {
        const int r0 = w * g.RO + 2 * u;
        gstore(a.gran, a.g_resid + r0 / 2, tr,
               pack2(bf2f(xres[r0]) + row_sum(c, 2 * u, iF), bf2f(xres[r0 + 1]) + row_sum(c, 2 * u + 1, iF)));
      }
    }
    B1_STAMP(9);
    k.cbar();  // xres is overwritten by the next gather
  }
#undef B1_STAMP
  if (stp) a.stamps[static_cast<int64_t>(NWG) * a.L * NSTAMP + w * 4 + 2] = k.line_wait;
  // ---- final RMSNorm (workgroup 0)
  if (w == 0) {
    k.gather(g.H / 2, tag_of(a.L, E_RESID), reinterpret_cast<uint32_t*>(xres), [&](int x) { return a.g_resid + x; });
    k.cbar();
    const float rs = k.norm_scale(xres, g.H);
    for (int x = ct * 8; x < g.H; x += CT * 8) {
      float v[8], wf[8], o[8];
      unpack8(*reinterpret_cast<const uint4*>(xres + x), v);
      unpack8(*reinterpret_cast<const uint4*>(a.final_norm + x), wf);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = v[e] * rs * wf[e];
      *reinterpret_cast<uint4*>(a.out + x) = pack8(o);
    }
  }
}

template <int GQ>
__global__ void __launch_bounds__(NTHR, 1) decode_b1_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  Ctl* c = reinterpret_cast<Ctl*>(smem + a.off_ctl);
  if (threadIdx.x == 0) {
    for (int i = 0; i < NLW; ++i) c->landed[i] = 0;
    c->cbar = 0;
    c->abort_ = 0;
    for (int i = 0; i < NCW; ++i) c->cur[i] = 0;
  }
  __syncthreads();
  if (threadIdx.x < 64 * NLW)
    loader(a, c, smem, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
  else
    consumer<GQ>(a, c, smem, smem);
}

}  // namespace b1

// The loader's schedule: every (layer, phase, row) of workgroup w in line order,
// consecutive rows that are adjacent in memory merged into one run. Built once per
// model (the weights never move); the same Geo::row as the consumers, so the two
// sides cannot disagree on the order.
namespace b1 {
__global__ void decode_b1_runs_kernel(Args a, uint64_t* runs, int stride, int* overflow) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= NWG) return;
  const Geo g(a);
  uint64_t* rt = runs + static_cast<int64_t>(w) * stride * 2;
  int k = -1;
  uint64_t end = 0;
  for (int layer = 0; layer < a.L; ++layer)
    for (int p = 0; p < 4; ++p) {
      const int lp = g.lpr(p);
      const uint64_t W = a.wptr[layer * 4 + p];
      for (int r = 0; r < g.nrows(p); ++r) {
        const uint64_t ptr = W + static_cast<uint64_t>(g.row(p, w, r)) * lp * LINE;
        if (k >= 0 && ptr == end) {
          rt[2 * k + 1] += lp;
        } else {
          if (++k >= stride - 1) { atomicAdd(overflow, 1); return; }
          rt[2 * k] = ptr;
          rt[2 * k + 1] = lp;
        }
        end = ptr + static_cast<uint64_t>(lp) * LINE;
      }
    }
  rt[2 * (k + 1)] = 0;
  rt[2 * (k + 1) + 1] = 0;
}
}  // namespace b1

// ---------------------------------------------------------------- host side
// Plan: LDS carve-up, granule offsets, ring size. Returns the granule count, or -1
// when the shape is not supported (the caller keeps the multi-launch path).
int decode_b1_plan(int L, int H, int F, int Hq, int Hkv, int* out /*[13]*/) {
  using namespace b1;
  if (Hkv < 1 || Hq % Hkv || NWG % Hkv || H % (512 * 1) || F % 512 || (Hq * HD) % 512) return -1;
  const int G = Hq / Hkv, WPG = NWG / Hkv;
  if ((G != 1 && G != 2 && G != 4 && G != 8) || ((G + 2) * HD) % WPG) return -1;
  const int RPW = (G + 2) * HD / WPG, RO = H / NWG, FW = F / NWG;
  if (H % (2 * NWG) || F % (2 * NWG) || RPW < 1 || (FW % 2)) return -1;
  auto items = [](int rows, int K) { return rows * ((K / 512 + SEG - 1) / SEG); };
  if (items(RPW, H) > 256 || items(RO, Hq * HD) > 256 || items(2 * FW, H) > 256 || items(RO, F) > 256) return -1;
  const int S_att = WPG < 32 ? WPG : 32;
  if ((G * HD) % S_att || ((G * HD / S_att) % 2)) return -1;
  // LDS: ring | xres (H bf16) | xbig (max(Hq*128, F) bf16, also the attention scratch) | ctl
  const int xres = H * 2;
  const int scratch_attn = ((G + 2) * HD * 4 + G * HD * 2 + 2 * HD * 2 + NCW * 64 * 8 * 4 + 2 * NCW * G * 4 +
                            NCW * G * HD * 4);
  const int scratch_comb = S_att * (G * HD / S_att + 2) * 4;
  int xbig = std::max(std::max(Hq * HD, F) * 2, std::max(scratch_attn, scratch_comb));
  xbig = (xbig + 15) & ~15;
  const int ctl = static_cast<int>(sizeof(Ctl));
  const int lds_max = 160 * 1024;
  const int nslot = (lds_max - xres - xbig - ((ctl + 15) & ~15)) / (SLOT * LINE);
  if (nslot < 4) return -1;
  const int ring = nslot * SLOT * LINE;
  int o = 0;
  out[0] = S_att;
  out[1] = nslot * SLOT;
  out[2] = ring;                 // off_xres
  out[3] = ring + xres;          // off_xbig
  out[4] = ring + xres + xbig;   // off_ctl
  out[5] = ring + xres + xbig + ((ctl + 15) & ~15);  // LDS bytes
  out[6] = o; o += H / 2;                            // g_resid
  out[7] = o; o += H / 2;                            // g_post
  out[8] = o; o += (Hq + 2 * Hkv) * HD;              // g_qkv
  out[9] = o; o += Hkv * S_att * G * (HD + 2);       // g_part
  out[10] = o; o += Hq * HD / 2;                     // g_attn
  out[11] = o; o += F / 2;                           // g_act
  out[12] = L * (RPW + 2 * RO + 2 * FW) + 2;          // run-table entries per workgroup (bound)
  (void)L;
  return o;
}

static void b1_geometry(b1::Args& a, const int* pl, int L, int H, int F, int Hq, int Hkv) {
  a.L = L; a.H = H; a.F = F; a.Hq = Hq; a.Hkv = Hkv;
  a.S_att = pl[0]; a.ring_lines = pl[1];
  a.off_xres = pl[2]; a.off_xbig = pl[3]; a.off_ctl = pl[4];
  a.g_resid = pl[6]; a.g_post = pl[7]; a.g_qkv = pl[8]; a.g_part = pl[9]; a.g_attn = pl[10]; a.g_act = pl[11];
  a.runs_stride = pl[12];
}

// Once per model: the loaders' run tables (runs: NWG * plan[12] * 2 uint64).
int decode_b1_build_runs(const uint64_t* wptr, int L, int H, int F, int Hq, int Hkv, uint64_t* runs, int* overflow,
                         hipStream_t st) {
  using namespace b1;
  int pl[13];
  if (decode_b1_plan(L, H, F, Hq, Hkv, pl) < 0) return -1;
  Args a{};
  a.wptr = wptr;
  b1_geometry(a, pl, L, H, F, Hq, Hkv);
  hipLaunchKernelGGL(decode_b1_runs_kernel, dim3(NWG / 64), dim3(64), 0, st, a, runs, pl[12], overflow);
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

int decode_b1(const uint64_t* wptr, const uint64_t* kvptr, const uint16_t* resid_in, const uint16_t* final_norm,
              uint16_t* out, const int32_t* positions, const int32_t* slot_mapping, const int32_t* block_table,
              const int32_t* seq_lens, const float* cos_sin, uint64_t* gran, int* ctl, const uint64_t* runs, int L,
              int H, int F, int Hq, int Hkv, int bs, int apply_rope, float eps, float scale, uint64_t* stamps,
              hipStream_t st) {
  using namespace b1;
  int pl[13];
  const int ng = decode_b1_plan(L, H, F, Hq, Hkv, pl);
  if (ng < 0 || bs != 16) return -1;  // 16-key pages (attention address arithmetic)
  const int G = Hq / Hkv;
  const void* kern = G == 1   ? reinterpret_cast<const void*>(decode_b1_kernel<1>)
                     : G == 2 ? reinterpret_cast<const void*>(decode_b1_kernel<2>)
                     : G == 4 ? reinterpret_cast<const void*>(decode_b1_kernel<4>)
                     : G == 8 ? reinterpret_cast<const void*>(decode_b1_kernel<8>)
                              : nullptr;
  if (kern == nullptr) return -1;
  static bool attr_set[9] = {};
  if (!attr_set[G]) {
    if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess) return -2;
    attr_set[G] = true;
  }
  Args a{};
  a.wptr = wptr; a.kvptr = kvptr; a.resid_in = resid_in; a.final_norm = final_norm; a.out = out;
  a.positions = positions; a.slot_mapping = slot_mapping; a.block_table = block_table; a.seq_lens = seq_lens;
  a.cos_sin = cos_sin; a.gran = gran; a.ctl = ctl; a.runs = runs;
  b1_geometry(a, pl, L, H, F, Hq, Hkv);
  a.bs = bs; a.apply_rope = apply_rope;
  a.eps = eps; a.scale = scale;
  a.stamps = stamps;
  if (hipMemsetAsync(gran, 0, static_cast<size_t>(ng) * 8, st) != hipSuccess) return -3;
  void* args[] = {&a};
  if (hipLaunchKernel(kern, dim3(NWG), dim3(NTHR), args, pl[5], st) != hipSuccess) return -4;
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

}  // namespace xgk
