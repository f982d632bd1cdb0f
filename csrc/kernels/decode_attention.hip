// K6: paged decode attention (one query token per sequence), GQA, split-K (v2: MFMA for both products).
//
// Grid (Hkv, B, S): one workgroup per (kv head, sequence, key split); 4 waves.
// All G = Hq/Hkv query heads of a kv head are processed together so every K/V
// byte is read from HBM exactly once per step (decode is KV-bandwidth bound).
//
// Per 16-key tile (bs is a multiple of 16; a tile never straddles a page):
//   S^T[16 keys][16 heads] = K_tile . Q^T  on one MFMA chain
//     v_mfma_f32_16x16x32_bf16, A = K rows (16 B contiguous per lane, loaded
//     straight from the paged cache into the A-fragment layout: no LDS),
//     B = Q^T (resident in registers, heads >= G zero-padded);
//   online softmax per head: lane&15 is the head, its 16 keys sit in 4 regs x
//     4 lane groups -> 2 xor-shuffles;
//   O^T += V^T P^T on v_mfma_f32_16x16x16_bf16, V^T fragments read transposed
//     (ds_read_b64_tr_b16) from a wave-private LDS tile.
// Waves stride over tiles; the 4 wave states (m, l, O) merge through LDS at the
// end. With S > 1 each split writes (O/l, lse) and decode_combine reduces.
//
// Fused-QKV form (FQ; the dense decode layer, see gemm_m64g.hip): the QKV
// projection arrives as fp32 split-K partials. Each workgroup's prologue reduces
// the partials of ITS (sequence, kv head) -- the G query heads plus the k and v
// head --, rotates q and k with the RoPE table and, in the split that owns the
// sequence's last key, appends the new k/v row to the paged cache before its key
// loop reads it (same workgroup: ordered by vmcnt(0) + barrier; no other
// workgroup touches that row). This replaces rope_cache_partials and the q round
// trip through HBM: one launch less per layer.
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace xgk {

template <int D, int G, int NWAVES = 4>
struct DecodeCfg {
  static constexpr int KK = D / 32;        // 16x16x32 k-steps over the head dim (S^T)
  static constexpr int MT = D / 16;        // 16-dim output tiles (O^T)
  static constexpr int NCH = D / 8;        // 16-B chunks per key row
  static constexpr int VLD = 16 * NCH / 64;  // 16-B V chunks per lane per tile
  static constexpr int WAVES = NWAVES;
};

__device__ __forceinline__ f32x4_t mfma16x16x16(bf16x4_t a, bf16x4_t b, f32x4_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
#else
  return c;
#endif
}

template <int D>
__device__ __forceinline__ int dswz(int row, int ch) {
  return ch ^ (((row & 7) << 1) & (D / 8 - 1));
}

// Fused-QKV operands (FQ instantiations only).
struct QkvFuse {
  const float* part;            // [S, B, (Hq + 2 Hkv) * D] fp32 QKV split-K partials; row b = sequence b
  int S;
  const int32_t* positions;     // [B]
  const float* cos_sin;         // [max_pos, D] = [cos | sin], fp32
  const int32_t* slot_mapping;  // [B]; < 0: padding row (no cache write)
  uint16_t* k_cache;            // the kernel's kc / vc, writable
  uint16_t* v_cache;
  int apply_rope;
};

// f[0..4) = sum_s part[s * slab + off + 0..4): batches of 4 clamped loads issued
// before the adds (a runtime trip count with one load per iteration would chain S
// dependent L2 round trips); masked partials add exactly 0.
// S <= 8 (the decode QKV plans use 2-8 splits) takes ONE batch of loads, so the
// prologue pays one L2 round trip whatever the split.
__device__ __forceinline__ void sum_partials4(const float* __restrict__ part, int S, int64_t slab, int64_t off,
                                              float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) f[i] = 0.f;
  if (S > 4 && S <= 8) {
    // per-lane pointers stepped by one slab while i < S (clamped to the last split):
    // no per-split 64-bit scalar offsets (SGPR pressure)
    const float* p = part + off;
    float4 a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i] = *reinterpret_cast<const float4*>(p);
      if (i + 1 < S) p += slab;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float k = i < S ? 1.f : 0.f;
      f[0] += k * a[i].x; f[1] += k * a[i].y; f[2] += k * a[i].z; f[3] += k * a[i].w;
    }
    return;
  }
  for (int s0 = 0; s0 < S; s0 += 4) {
    float4 a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const float4*>(part + min(s0 + i, S - 1) * slab + off);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float k = s0 + i < S ? 1.f : 0.f;
      f[0] += k * a[i].x; f[1] += k * a[i].y; f[2] += k * a[i].z; f[3] += k * a[i].w;
    }
  }
}

__device__ __forceinline__ uint2 pack4(const float* f) { return make_uint2(pack2(f[0], f[1]), pack2(f[2], f[3])); }

// Prologue of the fused form: q (G heads, rotated) -> q_lds [G][D] bf16; when this
// split owns the last key and the row is real, the rotated k and the v row are
// written to the paged cache at slot_mapping[b]. One work item = 4 rotation pairs
// (or 4 v values): (G + 1) * D/8 + D/4 items spread over the 256 threads.
template <int D, int G>
__device__ __forceinline__ void decode_qkv_prologue(const QkvFuse& fq, int b, int kvh, int Hq, int Hkv, int bs,
                                                     bool owns_last, uint16_t* q_lds) {
  constexpr int HALF = D / 2, CPH = HALF / 4;  // rope work items (4 pairs each) per head
  const int64_t width = static_cast<int64_t>(Hq + 2 * Hkv) * D;
  const int64_t slab = static_cast<int64_t>(gridDim.y) * width;
  const int64_t row = static_cast<int64_t>(b) * width;
  const int slot = fq.slot_mapping[b];
  const bool wkv = owns_last && slot >= 0;
  const int64_t dst = wkv ? ((static_cast<int64_t>(slot / bs) * Hkv + kvh) * bs + slot % bs) * D : 0;
  const float* cs = fq.cos_sin + static_cast<int64_t>(fq.positions[b]) * D;
  const int n_rope = (G + 1) * CPH;
  for (int it = threadIdx.x; it < n_rope + D / 4; it += blockDim.x) {
    if (it < n_rope) {
      const int hh = it / CPH, c = it % CPH;  // hh < G: query head kvh*G + hh; hh == G: the k head
      if (hh == G && !wkv) continue;
      const int64_t col = static_cast<int64_t>(hh < G ? kvh * G + hh : Hq + kvh) * D + c * 4;
      float a[4], e[4];
      sum_partials4(fq.part, fq.S, slab, row + col, a);
      sum_partials4(fq.part, fq.S, slab, row + col + HALF, e);
      if (fq.apply_rope) {
        const float4 cv = *reinterpret_cast<const float4*>(cs + c * 4);
        const float4 sv = *reinterpret_cast<const float4*>(cs + HALF + c * 4);
        const float cc[4] = {cv.x, cv.y, cv.z, cv.w}, ss[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float x1 = a[i], x2 = e[i];
          a[i] = x1 * cc[i] - x2 * ss[i];
          e[i] = x2 * cc[i] + x1 * ss[i];
        }
      }
      uint16_t* o = hh < G ? q_lds + hh * D : fq.k_cache + dst;
      *reinterpret_cast<uint2*>(o + c * 4) = pack4(a);
      *reinterpret_cast<uint2*>(o + HALF + c * 4) = pack4(e);
    } else if (wkv) {
      const int c = it - n_rope;
      float f[4];
      sum_partials4(fq.part, fq.S, slab, row + static_cast<int64_t>(Hq + Hkv + kvh) * D + c * 4, f);
      *reinterpret_cast<uint2*>(fq.v_cache + dst + c * 4) = pack4(f);
    }
  }
  if (wkv) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the cache row lands before any wave reads it
}

// The same prologue in two halves for S <= 8 (every decode QKV plan): qkv_issue puts
// this thread's work item's partial loads (all 8 clamped splits) and RoPE factors in
// flight, the kernel then issues its K/V preloads, and qkv_finish waits only for the
// older prologue loads (in-order vmcnt) -- the prologue's L2 round trip, RoPE and
// cache append overlap the K/V HBM latency instead of queueing behind it.
template <int D>
struct QkvItem {
  float4 a[8], e[8];   // split partials: rotation-pair first / second halves (v item: e = a's address)
  float4 cv, sv;       // RoPE cos / sin of the 4 pairs
  int kind;            // 0 none, 1 q head (index hh), 2 k head, 3 v values
  int hh, c;
  int64_t dst;
};

template <int D, int G>
__device__ __forceinline__ void qkv_issue(const QkvFuse& fq, int b, int kvh, int Hq, int Hkv, int bs, bool owns_last,
                                          QkvItem<D>& w) {
  constexpr int HALF = D / 2, CPH = HALF / 4, NR = (G + 1) * CPH;
  static_assert(NR + D / 4 <= 256, "one prologue work item per thread");
  const int64_t width = static_cast<int64_t>(Hq + 2 * Hkv) * D;
  const int64_t slab = static_cast<int64_t>(gridDim.y) * width;
  const int64_t row = static_cast<int64_t>(b) * width;
  const int slot = fq.slot_mapping[b];
  const bool wkv = owns_last && slot >= 0;
  w.dst = wkv ? ((static_cast<int64_t>(slot / bs) * Hkv + kvh) * bs + slot % bs) * D : 0;
  const int it = threadIdx.x;
  int64_t col = 0;
  w.kind = 0;
  if (it < NR) {
    w.hh = it / CPH;
    w.c = it % CPH;
    if (w.hh < G || wkv) {
      w.kind = w.hh < G ? 1 : 2;
      col = static_cast<int64_t>(w.hh < G ? kvh * G + w.hh : Hq + kvh) * D + w.c * 4;
    }
  } else if (it < NR + D / 4 && wkv) {
    w.kind = 3;
    w.c = it - NR;
    col = static_cast<int64_t>(Hq + Hkv + kvh) * D + w.c * 4;
  }
  // unconditional loads (threads without an item re-read the slab's first line, a
  // v item its own line for the second half): loads under a branch make the
  // compiler's wait at the join conservative (a small vmcnt that drains the K/V
  // preloads issued after them)
  const float* p = fq.part + (w.kind == 0 ? 0 : row + col);
  const int eo = w.kind == 1 || w.kind == 2 ? HALF : 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    w.a[i] = *reinterpret_cast<const float4*>(p);
    w.e[i] = *reinterpret_cast<const float4*>(p + eo);
    if (i + 1 < fq.S) p += slab;
  }
  const int pos = fq.apply_rope ? fq.positions[b] : 0;
  const float* cs = (fq.apply_rope ? fq.cos_sin : fq.part) + static_cast<int64_t>(pos) * D;
  const int cc = w.kind == 1 || w.kind == 2 ? w.c * 4 : 0;
  w.cv = *reinterpret_cast<const float4*>(cs + cc);
  w.sv = *reinterpret_cast<const float4*>(cs + HALF + cc);
  asm volatile("" ::: "memory");  // keep these loads ahead of the K/V preloads
}

template <int D, int G>
__device__ __forceinline__ void qkv_finish(const QkvFuse& fq, QkvItem<D>& w, uint16_t* q_lds) {
  constexpr int HALF = D / 2;
  if (w.kind != 0) {
    float a[4] = {0.f, 0.f, 0.f, 0.f}, e[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float k = i < fq.S ? 1.f : 0.f;
      a[0] += k * w.a[i].x; a[1] += k * w.a[i].y; a[2] += k * w.a[i].z; a[3] += k * w.a[i].w;
      e[0] += k * w.e[i].x; e[1] += k * w.e[i].y; e[2] += k * w.e[i].z; e[3] += k * w.e[i].w;
    }
    if (w.kind == 3) {
      *reinterpret_cast<uint2*>(fq.v_cache + w.dst + w.c * 4) = pack4(a);
    } else {
      if (fq.apply_rope) {
        const float cc[4] = {w.cv.x, w.cv.y, w.cv.z, w.cv.w}, ss[4] = {w.sv.x, w.sv.y, w.sv.z, w.sv.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float x1 = a[i], x2 = e[i];
          a[i] = x1 * cc[i] - x2 * ss[i];
          e[i] = x2 * cc[i] + x1 * ss[i];
        }
      }
      // q rows through an LDS-qualified pointer: the compiler cannot merge them with the
      // k-cache stores into one flat store, which would make the barrier wait on vmcnt(0)
      if (w.kind == 1) {
        typedef __attribute__((address_space(3))) uint64_t lds_u64;
        lds_u64* o = (lds_u64*)(q_lds + w.hh * D);
        const uint2 pa = pack4(a), pe = pack4(e);
        o[w.c] = (static_cast<uint64_t>(pa.y) << 32) | pa.x;
        o[HALF / 4 + w.c] = (static_cast<uint64_t>(pe.y) << 32) | pe.x;
      } else {
        uint16_t* o = fq.k_cache + w.dst;
        *reinterpret_cast<uint2*>(o + w.c * 4) = pack4(a);
        *reinterpret_cast<uint2*>(o + HALF + w.c * 4) = pack4(e);
      }
    }
  }
  // the cache row lands before any wave reads it (waits for the K/V preloads too,
  // which by now have had the prologue's latency to arrive)
  if (w.kind >= 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Per 16-key tile and wave:
//   S^T[16 keys][16 heads] = K . Q^T     4 x v_mfma_f32_16x16x32_bf16 (K frags straight from HBM)
//   online softmax per head (lane&15 = head): 2 xor-shuffles per reduction,
//     alpha is lane-local so the O rescale needs no broadcast
//   O^T[d][h] += V^T . P^T               D/16 x v_mfma_f32_16x16x16_bf16; the S^T
//     accumulators ARE the P^T B-fragment (k = 4(lane>>4)+r), V^T fragments come
//     from a 4 KiB wave-private LDS tile via ds_read_b64_tr_b16
//   the next tile's K and V loads are issued before the current tile's math.
// kc / vc are not __restrict__: the fused form writes the new row through fq.
// softmax(lse)-weighted sum over splits of one output element: po[s * D], lse[s].
// All lse / partial loads of a 16-split batch are issued before any arithmetic
// (unconditional clamped loads, masked after): a batch-1 decode has few heads, so
// the reduce is pure latency and a dependent per-split loop costs ~7 us.
template <int D>
__device__ __forceinline__ float combine_splits(const float* __restrict__ lse, const float* __restrict__ po,
                                                int num_splits) {
  constexpr int SB = 16;
  float M = -INFINITY, den = 0.f, acc = 0.f;
  for (int s0 = 0; s0 < num_splits; s0 += SB) {
    float l[SB], v[SB];
#pragma unroll
    for (int i = 0; i < SB; ++i) {
      const int sc = min(s0 + i, num_splits - 1);
      l[i] = lse[sc];
      v[i] = po[static_cast<int64_t>(sc) * D];
    }
#pragma unroll
    for (int i = 0; i < SB; ++i)
      if (s0 + i >= num_splits) l[i] = -INFINITY;
    float m2 = M;
#pragma unroll
    for (int i = 0; i < SB; ++i) m2 = fmaxf(m2, l[i]);
    if (m2 == -INFINITY) continue;
    const float r = __expf(M - m2);  // rescale the running sums (M == -inf -> 0)
    den *= r;
    acc *= r;
#pragma unroll
    for (int i = 0; i < SB; ++i) {
      const float wgt = __expf(l[i] - m2);
      den += wgt;
      acc += wgt * v[i];
    }
    M = m2;
  }
  return den > 0.f ? acc / den : 0.f;
}

// KL (K through LDS): the K tile is fetched like V -- each wave instruction moves 4
// full 256-B key rows (coalesced) instead of 16 rows x 64 B in the MFMA A-fragment
// shape -- and staged into a wave-private, XOR-swizzled LDS tile whose ds_read_b128
// fragment reads are conflict-free; the fragment-shaped global loads occupy the
// texture-address path per byte moved, which caps the KV stream at 64 concurrent.
// (Measured and removed, A/B records in profiles/: an in-launch split combine by the
// last-arriving split, r1_inlaunch_combine_ab.md; O-weight prefetch workgroups inside
// this launch, r1_attn_prefetch_ab.md; 8 waves per workgroup, r1_decode_waves_c1.md.)
// PR (anatomy probes, bench/decode_cold.py --probe; output garbage): 0 = the kernel;
// 1 = no fused prologue (no QKV-partial reads / RoPE / KV append); 2 = no key loop;
// 3 = neither (launch + merge + store only); 4 = the kernel with cached (temporal) K/V loads.
// SPRO (FQ): the split prologue (qkv_issue before the K/V preloads, qkv_finish
// after; QKV plans with S <= 8 -- all of them today); false: the classic prologue.
template <int D, int G, bool FQ, bool KL = false, int NB = 2, int PR = 0, bool SPRO = true>
__global__ void __launch_bounds__(256) decode_attn_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const uint16_t* kc, const uint16_t* vc,
    const int32_t* __restrict__ block_tables, int bt_stride, const int32_t* __restrict__ seq_lens,
    float* __restrict__ part_out, float* __restrict__ part_lse, uint16_t* __restrict__ out, int64_t out_stride,
    int Hq, int Hkv, int bs, float scale, int num_splits, QkvFuse fq) {
  using C = DecodeCfg<D, G>;
  const int kvh = blockIdx.x, b = blockIdx.y, split = blockIdx.z;
  // wid through readfirstlane: wave-uniform to the compiler, so the page-table reads of
  // load_tile are scalar loads (lgkmcnt) and do not wait behind the prologue's vector loads
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int L = seq_lens[b];
  const int ntiles = (L + 15) >> 4;
  // tiles per split: an even share (a split past the sequence publishes lse = -inf)
  const int tps = (ntiles + num_splits - 1) / num_splits;
  const int t_begin = split * tps;
  const int t_end = min(ntiles, t_begin + tps);

  __shared__ __attribute__((aligned(16))) uint16_t v_lds[C::WAVES][16 * D];
  __shared__ __attribute__((aligned(16))) uint16_t k_lds[KL ? C::WAVES : 1][KL ? 16 * D : 8];
  __shared__ float m_lds[C::WAVES][16], l_lds[C::WAVES][16];
  __shared__ float o_lds[C::WAVES][G][D];
  __shared__ __attribute__((aligned(16))) uint16_t q_lds[FQ ? G * D : 8];

  const int32_t* bt = block_tables + static_cast<int64_t>(b) * bt_stride;
  const int64_t head_stride = static_cast<int64_t>(bs) * D;
  // NB register tiles per wave (K fragments + V rows): tiles t+W .. t+NB*W are in
  // flight while tile t is processed (one tile of lookahead left HBM idle between
  // a wave's tiles at 64 concurrent sequences)
  uint4 kf[NB][C::KK], vr[NB][C::VLD];
  // t < 0: a discarded load of the cache's first tile (keeps the preload count static)
  auto load_tile = [&](int t, uint4 (&kf)[C::KK], uint4 (&vr)[C::VLD]) {
    const int key0 = t * 16;
    const int64_t base = t < 0 ? 0
                               : (static_cast<int64_t>(bt[key0 / bs]) * Hkv + kvh) * head_stride +
                                     static_cast<int64_t>(key0 % bs) * D;
    // K/V are read once per step and a step's cache (GBs at 64 sequences) never fits the
    // L2 / Infinity Cache: non-temporal loads, 5.3 -> 6.1 TB/s at 2K keys (r4_decode_nt.md)
    auto ldkv = [](const uint16_t* p) { return PR == 4 ? ld16(p) : ld16_nt(p); };
    if constexpr (KL) {
      static_assert(C::KK == C::VLD, "K and V tiles split into the same chunks per lane");
#pragma unroll
      for (int i = 0; i < C::KK; ++i) {
        const int c = lane + 64 * i;  // chunk id in the 16 x NCH tile (4 full rows per instruction)
        kf[i] = ldkv(kc + base + (c / C::NCH) * D + (c % C::NCH) * 8);
      }
    } else {
      const uint16_t* kp = kc + base + li * D + 8 * g;
#pragma unroll
      for (int kk = 0; kk < C::KK; ++kk) kf[kk] = ldkv(kp + kk * 32);
    }
#pragma unroll
    for (int i = 0; i < C::VLD; ++i) {
      const int c = lane + 64 * i;  // chunk id in the 16 x NCH tile
      vr[i] = ldkv(vc + base + (c / C::NCH) * D + (c % C::NCH) * 8);
    }
  };
  const int t0 = t_begin + wid;
  // FQ: the first NB tiles of each wave are requested BEFORE the prologue (their
  // bytes do not depend on q), so the K/V latency overlaps the QKV-partial reads --
  // except the tile holding the key the prologue appends (the last one), which is
  // loaded after the prologue's barrier as before
  constexpr bool LOOP = PR != 2 && PR != 3;
  constexpr bool PRO = FQ && PR != 1 && PR != 3;
  // S <= 8 (SPRO): the prologue's own loads go out first (qkv_issue / qkv_finish). A
  // template choice, not a runtime branch, and the issue runs for every workgroup
  // (its loads stay in bounds for any L): loads under a branch, or registers the
  // other arm reuses, make the compiler's wait at the join drain everything after them
  constexpr bool SPLIT = PRO && SPRO;
  QkvItem<D> qi;
  if constexpr (SPLIT) qkv_issue<D, G>(fq, b, kvh, Hq, Hkv, bs, split == (ntiles - 1) / tps, qi);
  // every wave issues all NB preloads (skipped tiles as discarded loads): a static
  // count lets the compiler wait for the older prologue loads with vmcnt(NB * 8)
  // instead of vmcnt(0) at a control-flow join
  bool pre[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int tj = t0 + j * C::WAVES;
    pre[j] = LOOP && FQ && tj < t_end && tj != ntiles - 1;
    if constexpr (LOOP && FQ) load_tile(pre[j] ? tj : -1, kf[j], vr[j]);
  }
  if constexpr (FQ) {
    if constexpr (SPLIT) {
      if (L > 0) qkv_finish<D, G>(fq, qi, q_lds);
    } else if constexpr (PRO) {
      if (L > 0) decode_qkv_prologue<D, G>(fq, b, kvh, Hq, Hkv, bs, split == (ntiles - 1) / tps, q_lds);
    }
    __syncthreads();
  }

  // Q^T fragment: lane holds Q[head = li][32kk + 8g + j] (heads >= G are zero)
  bf16x8_t qf[C::KK];
  if constexpr (FQ) {
    const uint16_t* qp = q_lds + (li < G ? li : 0) * D;
#pragma unroll
    for (int kk = 0; kk < C::KK; ++kk)
      qf[kk] = as_frag(li < G ? *reinterpret_cast<const uint4*>(qp + kk * 32 + 8 * g) : make_uint4(0, 0, 0, 0));
  } else {
    const uint16_t* qp = q + static_cast<int64_t>(b) * q_stride + static_cast<int64_t>(kvh * G + li) * D;
#pragma unroll
    for (int kk = 0; kk < C::KK; ++kk) qf[kk] = as_frag(li < G ? ld16(qp + kk * 32 + 8 * g) : make_uint4(0, 0, 0, 0));
  }

  float m = -INFINITY, l = 0.f;  // per head li
  f32x4_t o[C::MT];
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt) o[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  uint16_t* my_v = v_lds[wid];
  uint16_t* my_k = k_lds[KL ? wid : 0];

  auto process = [&](int t, uint4 (&kfb)[C::KK], uint4 (&vrb)[C::VLD]) {
    uint4 kcur[C::KK];
    if constexpr (KL) {  // stage K rows, chunk ch of row r at granule ch ^ r (r < 16)
#pragma unroll
      for (int i = 0; i < C::KK; ++i) {
        const int c = lane + 64 * i;
        const int row = c / C::NCH, ch = c % C::NCH;
        st16(my_k + row * D + (ch ^ row) * 8, kfb[i]);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < C::KK; ++kk) kcur[kk] = kfb[kk];
    }
    // stage this tile's V rows into the wave-private LDS image (swizzled)
#pragma unroll
    for (int i = 0; i < C::VLD; ++i) {
      const int c = lane + 64 * i;
      const int row = c / C::NCH, ch = c % C::NCH;
      st16(my_v + row * D + dswz<D>(row, ch) * 8, vrb[i]);
    }
    if (t + NB * C::WAVES < t_end) load_tile(t + NB * C::WAVES, kfb, vrb);  // refill this register tile
    if constexpr (KL) {  // A fragment: key li, dims 32 kk + 8 g .. +8 (same wave wrote it: LDS order)
#pragma unroll
      for (int kk = 0; kk < C::KK; ++kk)
        kcur[kk] = *reinterpret_cast<const uint4*>(my_k + li * D + ((4 * kk + g) ^ li) * 8);
    }

    f32x4_t s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < C::KK; ++kk) s = mfma16x16x32(as_frag(kcur[kk]), qf[kk], s);

    // s[r] = S[key = 16t + 4g + r][head = li]
    const int key0 = t * 16 + 4 * g;
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[r] = key0 + r < L ? s[r] * scale : -INFINITY;
      mx = fmaxf(mx, s[r]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m, mx);
    const float alpha = __expf(m - m_new);  // first tile: m = -inf -> 0
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[r] = __expf(s[r] - m_new);
      ps += s[r];
    }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * alpha + ps;
    m = m_new;
    bf16x4_t pf;
    {
      const uint32_t lo = pack2(s[0], s[1]), hi = pack2(s[2], s[3]);
      pf = __builtin_bit_cast(bf16x4_t, make_uint2(lo, hi));
    }
    // O^T += V^T P^T ; lane (g, li) tr-reads keys 4g..4g+3 of dims 16mt + li
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[mt][r] *= alpha;
      const int row = 4 * g + (li >> 2);
      const int col = mt * 16 + 4 * (li & 3);
      const bf16x4_t vfrag = lds_read_tr16(my_v + row * D + dswz<D>(row, col >> 3) * 8 + (col & 7));
      o[mt] = mfma16x16x16(vfrag, pf, o[mt]);
    }
  };

#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int tj = t0 + j * C::WAVES;
    if (LOOP && tj < t_end && !pre[j]) load_tile(tj, kf[j], vr[j]);
  }
  for (int t = t0; LOOP && t < t_end; t += NB * C::WAVES) {
    bool done = false;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (!done && t + j * C::WAVES < t_end) process(t + j * C::WAVES, kf[j], vr[j]);
      else done = true;
    }
  }

  // ---- merge the 4 wave states: O^T[d = 16mt + 4g + r][h = li]
  if (lane < 16) {
    m_lds[wid][lane] = m;
    l_lds[wid][lane] = l;
  }
  if (li < G) {
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o_lds[wid][li][mt * 16 + 4 * g + r] = o[mt][r];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < G * D; idx += blockDim.x) {
    const int h = idx / D, d = idx % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < C::WAVES; ++w) M = fmaxf(M, m_lds[w][h]);
    float Ls = 0.f, O = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < C::WAVES; ++w) {
        const float e = __expf(m_lds[w][h] - M);
        Ls += l_lds[w][h] * e;
        O += o_lds[w][h][d] * e;
      }
    }
    const int qhead = kvh * G + h;
    const float res = Ls > 0.f ? O / Ls : 0.f;
    if (num_splits == 1) {
      out[static_cast<int64_t>(b) * out_stride + static_cast<int64_t>(qhead) * D + d] = f2bf(res);
    } else {
      const int64_t pi = (static_cast<int64_t>(b) * Hq + qhead) * num_splits + split;
      const float lse_v = Ls > 0.f ? M + __logf(Ls) : -INFINITY;
      part_out[pi * D + d] = res;
      if (d == 0) part_lse[pi] = lse_v;
    }
  }
}
// Split-K reduction launch: out[b, h, :] = sum_s softmax(lse)_s * part_out[b, h, s, :]
template <int D>
__global__ void __launch_bounds__(D) decode_combine_kernel(const float* __restrict__ part_out,
                                                           const float* __restrict__ part_lse,
                                                           uint16_t* __restrict__ out, int64_t out_stride,
                                                           int Hq, int num_splits) {
  const int bh = blockIdx.x;
  const int b = bh / Hq, h = bh % Hq;
  out[static_cast<int64_t>(b) * out_stride + static_cast<int64_t>(h) * D + threadIdx.x] =
      f2bf(combine_splits<D>(part_lse + static_cast<int64_t>(bh) * num_splits,
                             part_out + static_cast<int64_t>(bh) * num_splits * D + threadIdx.x, num_splits));
}

template <int D, int G, bool FQ>
static void launch_decode(const uint16_t* q, int64_t qs, const uint16_t* kc, const uint16_t* vc,
                          const int32_t* bt, int bts, const int32_t* sl, float* po, float* pl, uint16_t* out,
                          int64_t os, int B, int Hq, int Hkv, int bs, float scale, int S, const QkvFuse& fq,
                          hipStream_t st, int depth = 2) {
  // K through LDS for G <= 4; at G = 8 (one kv head per TP-8 rank of the 70B) the
  // fragment-shaped K loads measured 0.5-6 % faster. depth 3: three register tiles
  // in flight per wave (fused form, G <= 4)
  if constexpr (D == 128 && G <= 4 && FQ) {
#ifdef XGK_PROBES
    if (depth >= 11 && depth <= 14) {  // anatomy probes (depth = 10 + PR): xgserve/_build.py --probes
#define XGK_DECP(P)                                                                                                 \
  hipLaunchKernelGGL((decode_attn_kernel<D, G, FQ, true, 2, P>), dim3(Hkv, B, S), dim3(256), 0, st, q, qs, kc, vc, bt, \
                     bts, sl, po, pl, out, os, Hq, Hkv, bs, scale, S, fq)
      if (depth == 11) XGK_DECP(1);
      else if (depth == 12) XGK_DECP(2);
      else if (depth == 13) XGK_DECP(3);
      else XGK_DECP(4);
#undef XGK_DECP
      if (S > 1) hipLaunchKernelGGL(decode_combine_kernel<D>, dim3(B * Hq), dim3(D), 0, st, po, pl, out, os, Hq, S);
      return;
    }
#endif
  }
  // the split prologue handles QKV plans of <= 8 splits; depth 4 = the classic
  // prologue at depth 2 (A/B)
  const bool classic = FQ && (fq.S > 8 || depth == 4);
#define XGK_DEC(KL, NB, SP)                                                                                          \
  hipLaunchKernelGGL((decode_attn_kernel<D, G, FQ, KL, NB, 0, SP>), dim3(Hkv, B, S), dim3(256), 0, st, q, qs, kc, vc, \
                     bt, bts, sl, po, pl, out, os, Hq, Hkv, bs, scale, S, fq)
  if constexpr (D == 128 && G <= 4 && FQ) {
    if (depth == 3) {
      if (classic) XGK_DEC(true, 3, false);
      else XGK_DEC(true, 3, true);
    } else {
      if (classic) XGK_DEC(true, 2, false);
      else XGK_DEC(true, 2, true);
    }
  } else if constexpr (D == 128 && G <= 4) {
    XGK_DEC(true, 2, true);
  } else if constexpr (FQ) {
    if (classic) XGK_DEC(false, 2, false);
    else XGK_DEC(false, 2, true);
  } else {
    XGK_DEC(false, 2, true);
  }
#undef XGK_DEC
  if (S > 1) hipLaunchKernelGGL(decode_combine_kernel<D>, dim3(B * Hq), dim3(D), 0, st, po, pl, out, os, Hq, S);
}

// returns 0 on success, -1 for an unsupported (D, G) combination
int decode_attention(const uint16_t* q, int64_t q_stride, const uint16_t* kc, const uint16_t* vc,
                     const int32_t* bt, int bt_stride, const int32_t* seq_lens, float* part_out, float* part_lse,
                     uint16_t* out, int64_t out_stride, int B, int Hq, int Hkv, int D, int bs, float scale,
                     int num_splits, hipStream_t st) {
  if (B <= 0) return 0;
  if (bs % 16 != 0 || Hq % Hkv != 0) return -1;
  const int G = Hq / Hkv;
  const QkvFuse nofuse{nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
#define XGK_DEC(DD, GG)                                                                                  \
  if (D == DD && G == GG) {                                                                              \
    launch_decode<DD, GG, false>(q, q_stride, kc, vc, bt, bt_stride, seq_lens, part_out, part_lse, out,  \
                                 out_stride, B, Hq, Hkv, bs, scale, num_splits, nofuse, st);             \
    return 0;                                                                                            \
  }
  XGK_DEC(128, 1) XGK_DEC(128, 2) XGK_DEC(128, 4) XGK_DEC(128, 8) XGK_DEC(128, 16)
  XGK_DEC(64, 1) XGK_DEC(64, 2) XGK_DEC(64, 4) XGK_DEC(64, 8)
#undef XGK_DEC
  return -1;
}

// Fused-QKV decode attention (D = 128): part = QKV split-K partials [S_qkv, B, (Hq+2Hkv)*128].
int decode_attention_fq(const float* part, int S_qkv, const int32_t* positions, const float* cos_sin,
                        const int32_t* slots, uint16_t* kc, uint16_t* vc, const int32_t* bt, int bt_stride,
                        const int32_t* seq_lens, float* part_out, float* part_lse, uint16_t* out,
                        int64_t out_stride, int B, int Hq, int Hkv, int D, int bs, float scale, int num_splits,
                        int apply_rope, hipStream_t st, int depth) {
  if (B <= 0) return 0;
  if (part == nullptr || S_qkv < 1 || bs % 16 != 0 || Hq % Hkv != 0 || D != 128 || num_splits < 1) return -1;
  if (num_splits > 1 && (part_out == nullptr || part_lse == nullptr)) return -1;
#ifdef XGK_PROBES
  if (out == nullptr || depth < 2 || (depth > 4 && (depth < 11 || depth > 14))) return -1;
#else
  if (out == nullptr || depth < 2 || depth > 4) return -1;
#endif
  const QkvFuse fq{part, S_qkv, positions, cos_sin, slots, kc, vc, apply_rope};
  const int G = Hq / Hkv;
#define XGK_DECF(GG)                                                                                         \
  if (G == GG) {                                                                                             \
    launch_decode<128, GG, true>(nullptr, 0, kc, vc, bt, bt_stride, seq_lens, part_out, part_lse, out,       \
                                 out_stride, B, Hq, Hkv, bs, scale, num_splits, fq, st, depth);              \
    return 0;                                                                                                \
  }
  XGK_DECF(1) XGK_DECF(2) XGK_DECF(4) XGK_DECF(8)
#undef XGK_DECF
  return -1;
}

}  // namespace xgk
