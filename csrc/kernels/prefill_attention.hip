// K5: varlen causal flash attention over the paged KV cache (prefill, chunked
// prefill, prefix-cache hits, speculative verify), GQA.
//
// Grid (num_seqs * q_tiles, Hkv * G / GH); workgroup = GH query heads of ONE kv
// head x 64 query rows = 4*GH waves (16 rows per wave): the GH heads of a GQA group
// share every K/V tile they stream (read from HBM once per group slice instead of
// once per query head). KV streamed in 64-key tiles through a double-buffered LDS
// ring: the next tile's registers land in the other buffer right after this tile's
// MFMAs, so each tile costs one barrier. Query chunk i of a sequence
// with ctx cached keys sits at absolute position ctx + i and sees keys
// [0, ctx + i] -- the new chunk's K/V were already appended to the paged
// cache by rope_cache, so prefix-cached and chunked prefill are one code path.
//
// CDNA4 structure (cdna_hip_programming.md "Fused attention prefill"):
//   * swapped QK^T: S^T = K . Q^T with v_mfma_f32_16x16x32_bf16, so each lane
//     owns one query row (lane&15) and the row max / row sum are 2 xor-shuffles;
//   * K tile XOR-swizzled by (row & 15) on 16-B chunks -> the ds_read_b128 of
//     the A fragment is bank-conflict free (T2);
//   * P never leaves registers: the S^T accumulators ARE the B operand of
//     O^T += V^T P^T under a permuted k order (guide §3 "accumulator tile as
//     the next MFMA's operand"); V^T fragments come from ds_read_b64_tr_b16
//     (T10) on a V tile whose 16-B chunks are XOR-swizzled by (row&7)<<1 so the
//     transposed reads are conflict-free;
//   * the next KV tile's global loads are issued before the current tile's
//     MFMAs and written to LDS after the barrier (T14).
#include "common.h"
#include "glds.h"

namespace xgk {

template <int D, int GH = 1>
struct PrefillCfg {
  static constexpr int BM = 64;          // query rows per workgroup (per head)
  static constexpr int BN = 64;          // keys per KV tile
  static constexpr int KK = D / 32;      // k-steps of S^T
  static constexpr int MT = D / 16;      // 16-dim tiles of O^T
  static constexpr int NCH = D / 8;      // 16-B chunks per row
  static constexpr int THREADS = 256 * GH;
  static constexpr int LOADS = BN * NCH / THREADS;  // 16-B chunks per thread per tile (K and V each)
  static_assert(LOADS >= 1 && BN * NCH % THREADS == 0, "tile chunks must split evenly over the workgroup");
};

template <int D>
__device__ __forceinline__ int k_swz(int row, int ch) {
  return ch ^ (row & (PrefillCfg<D>::NCH - 1) & 15);
}
template <int D>
__device__ __forceinline__ int v_swz(int row, int ch) {
  return ch ^ (((row & 7) << 1) & (PrefillCfg<D>::NCH - 1));
}

template <int D, int GH>
__global__ void __launch_bounds__(256 * GH) prefill_attn_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ qsl, const int32_t* __restrict__ seq_lens, uint16_t* __restrict__ out,
    int64_t out_stride, int Hq, int Hkv, int bs, float scale, int tiles_per_seq) {
  using C = PrefillCfg<D, GH>;
  const int s = blockIdx.x / tiles_per_seq;
  const int qt = tiles_per_seq - 1 - (blockIdx.x % tiles_per_seq);  // heavy (late) tiles first
  const int q0 = qsl[s];
  const int qlen = qsl[s + 1] - q0;
  const int i0 = qt * C::BM;
  if (i0 >= qlen) return;
  const int L = seq_lens[s];
  const int ctx = L - qlen;
  const int lane = threadIdx.x & 63, wid_all = threadIdx.x >> 6;
  const int wid = wid_all & 3;                       // 16-row slice of the 64-row tile
  const int h = blockIdx.y * GH + (wid_all >> 2);    // this wave's query head
  const int kvh = (blockIdx.y * GH) / (Hq / Hkv);   // shared by the workgroup's GH heads
  const int g = lane >> 4, li = lane & 15;

  // one LDS array (double-buffered K and V tiles): [buf][K | V][BN * D]
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * C::BN * D];

  // Q^T fragment for this wave's 16 rows: lane holds Q[row li][32kk + 8g + j]
  const int my_row = i0 + wid * 16 + li;  // query index within the chunk
  bf16x8_t qf[C::KK];
  {
    const bool ok = my_row < qlen;
    const uint16_t* qp = q + static_cast<int64_t>(q0 + (ok ? my_row : 0)) * q_stride + static_cast<int64_t>(h) * D;
#pragma unroll
    for (int kk = 0; kk < C::KK; ++kk) qf[kk] = as_frag(ok ? ld16(qp + kk * 32 + 8 * g) : make_uint4(0, 0, 0, 0));
  }
  const int q_abs = ctx + my_row;

  const int kend = min(L, ctx + min(qlen, i0 + C::BM));  // exclusive causal bound for the workgroup
  const int ntiles = (kend + C::BN - 1) / C::BN;
  const int32_t* bt = block_tables + static_cast<int64_t>(s) * bt_stride;
  const int64_t head_stride = static_cast<int64_t>(bs) * D;

  uint4 kr[C::LOADS], vr[C::LOADS];
  auto gload = [&](int tile) {
#pragma unroll
    for (int it = 0; it < C::LOADS; ++it) {
      const int ci = threadIdx.x + it * C::THREADS;
      const int key = ci / C::NCH, ch = ci % C::NCH;
      const int kabs = tile * C::BN + key;
      if (kabs < L) {
        const int page = bt[kabs / bs];
        const int64_t off = (static_cast<int64_t>(page) * Hkv + kvh) * head_stride +
                            static_cast<int64_t>(kabs % bs) * D + ch * 8;
        kr[it] = ld16(kc + off);
        vr[it] = ld16(vc + off);
      } else {
        kr[it] = make_uint4(0, 0, 0, 0);
        vr[it] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto lstore = [&](int buf) {
    uint16_t* k_lds = lds + buf * 2 * C::BN * D;
    uint16_t* v_lds = k_lds + C::BN * D;
#pragma unroll
    for (int it = 0; it < C::LOADS; ++it) {
      const int ci = threadIdx.x + it * C::THREADS;
      const int key = ci / C::NCH, ch = ci % C::NCH;
      st16(k_lds + key * D + k_swz<D>(key, ch) * 8, kr[it]);
      st16(v_lds + key * D + v_swz<D>(key, ch) * 8, vr[it]);
    }
  };

  f32x4_t o[C::MT];
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt) o[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  if (ntiles > 0) {
    gload(0);
    lstore(0);
  }
  __syncthreads();
  for (int j = 0; j < ntiles; ++j) {
    if (j + 1 < ntiles) gload(j + 1);
    const int kv0 = j * C::BN;
    const uint16_t* k_lds = lds + (j & 1) * 2 * C::BN * D;
    const uint16_t* v_lds = k_lds + C::BN * D;

    // ---- S^T = K . Q^T : 4 subtiles of 16 keys
    f32x4_t sacc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      sacc[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int row = n * 16 + li;
#pragma unroll
      for (int kk = 0; kk < C::KK; ++kk) {
        const uint4 kfrag = *reinterpret_cast<const uint4*>(k_lds + row * D + k_swz<D>(row, 4 * kk + g) * 8);
        sacc[n] = mfma16x16x32(as_frag(kfrag), qf[kk], sacc[n]);
      }
    }
    // ---- online softmax on this lane's query row
    float mx = -INFINITY;
    const bool diag = kv0 + C::BN > ctx + i0;  // tile may cross the causal diagonal
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kabs = kv0 + n * 16 + g * 4 + r;
        float v = sacc[n][r] * scale;
        if (kabs >= L || (diag && kabs > q_abs)) v = -INFINITY;
        sacc[n][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m, mx);
    const float alpha = m_new == -INFINITY ? 1.f : __expf(m - m_new);
    float rs = 0.f;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = m_new == -INFINITY ? 0.f : __expf(sacc[n][r] - m_new);
        sacc[n][r] = p;
        rs += p;
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    m = m_new;
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[mt][r] *= alpha;

    // ---- O^T += V^T . P^T over two 32-key chunks (permuted k order)
#pragma unroll
    for (int sc = 0; sc < 2; ++sc) {
      uint4 pb;
      pb.x = pack2(sacc[2 * sc][0], sacc[2 * sc][1]);
      pb.y = pack2(sacc[2 * sc][2], sacc[2 * sc][3]);
      pb.z = pack2(sacc[2 * sc + 1][0], sacc[2 * sc + 1][1]);
      pb.w = pack2(sacc[2 * sc + 1][2], sacc[2 * sc + 1][3]);
      const bf16x8_t pfrag = as_frag(pb);
      const int qq = li >> 2, pp = li & 3;
      const int r0 = sc * 32 + 4 * g + qq;  // key row for elements 0..3
      const int r1 = r0 + 16;               // key row for elements 4..7
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt) {
        const int col = mt * 16 + 4 * pp;  // first dim of this lane's 4-element address
        const int ch = col >> 3, sub = col & 7;
        const bf16x4_t a0 = lds_read_tr16(v_lds + r0 * D + v_swz<D>(r0, ch) * 8 + sub);
        const bf16x4_t a1 = lds_read_tr16(v_lds + r1 * D + v_swz<D>(r1, ch) * 8 + sub);
        const bf16x8_t vfrag = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        o[mt] = mfma16x16x32(vfrag, pfrag, o[mt]);
      }
    }
    // tile j+1 into the other buffer: its last readers (tile j-1) all passed the
    // previous iteration's barrier, so one barrier per tile orders both hazards
    if (j + 1 < ntiles) lstore((j + 1) & 1);
    __syncthreads();
  }

  // ---- epilogue: O[row li][16mt + 4g + r] = o[mt][r] / l
  if (my_row < qlen) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    uint16_t* op = out + static_cast<int64_t>(q0 + my_row) * out_stride + static_cast<int64_t>(h) * D;
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt) {
      uint2 w;
      w.x = pack2(o[mt][0] * inv, o[mt][1] * inv);
      w.y = pack2(o[mt][2] * inv, o[mt][3] * inv);
      *reinterpret_cast<uint2*>(op + mt * 16 + 4 * g) = w;
    }
  }
}

// ---------------------------------------------------------------------------
// prefill_attn2_kernel: the D = 128 path (Llama-3 / Mixtral heads).
//
// The kernel above gives each wave 16 query rows, so every 1 KiB K or V fragment
// read from LDS feeds one 16x16x32 MFMA: at 256 B/clk of LDS per CU that caps the
// MFMA pipe near half rate, and its one-tile register prefetch behind a dependent
// block-table load leaves the HBM latency exposed on short prompts (the 512-token
// prompt of a continuous-batching step ran 29 us per layer). This kernel:
//   * 32 query rows per wave on v_mfma_f32_32x32x16_bf16: swapped S^T = K . Q^T
//     (Q^T fragments in registers, K rows by ds_read_b128), so a lane owns one
//     query row (lane & 31) and its 32 scores of a 64-key tile; row max / sum are
//     one xor-32 shuffle each. The S^T accumulator IS the B operand of
//     O^T += V^T . P^T (guide §3, permuted k order); V^T fragments come from
//     ds_read_b64_tr_b16. Half the LDS bytes per MFMA of the 16-row form;
//   * K and V tiles by LDS-DMA (global_load_lds_dwordx4, no staging registers,
//     no LDS stores) into an NSLOT-deep ring, NSLOT - 1 tiles ahead; the source
//     chunk is XOR-permuted so the DMA's lane-linear destination lands in the
//     image (b) layout of cdna_hip_programming.md T10 (row & 3, row >> 2 XOR),
//     conflict-free for both the K row reads and the V transposed reads;
//   * each wave's DMA rows of a tile lie in one KV page (bs % 16 == 0), so the
//     page index is a wave-uniform scalar load -- no dependent vector load, and
//     counted vmcnt waits see only the DMAs; keys past the sequence end are
//     clamped to its last row (finite data, probability 0);
//   * one raw s_barrier per tile; a wave skips the MFMAs of tiles wholly above
//     its rows' causal diagonal;
//   * grid = (row tile, head group) flattened with the head group fastest: at
//     8 kv-head groups each XCD streams one kv head's K/V; heavy (late) row
//     tiles of every sequence are dispatched first;
//   * KS = 2 key phases for short prompts: the waves of phase p take the odd / even
//     64-key tiles of a 128-key ring slot and merge (m, l, O) through LDS at the end,
//     halving the serial tile chain of the heaviest (last) row tile;
//   * softmax in base 2 with the scale folded into one FMA, row max / sum across the
//     two lane halves by v_permlane32_swap, and the O rescale skipped exactly when no
//     row of the wave raised its max (ballot).
// NW waves = GH query heads (one GQA group slice) x NW/GH/KS 32-row blocks x KS.
// ---------------------------------------------------------------------------
template <int NW, int GH, int KS, int NSLOT>
struct Pf2Cfg {
  static constexpr int D = 128;
  static constexpr int RB = NW / GH / KS;       // 32-row blocks per head
  static constexpr int BM = 32 * RB;            // query rows per workgroup (per head)
  static constexpr int BN = 64;                 // keys per compute tile
  static constexpr int SK = BN * KS;            // keys per ring slot (one tile per key phase)
  static constexpr int WROWS = SK / NW;         // DMA rows per wave per slot
  static constexpr int NDMA = WROWS / 4;        // 1-KiB DMAs per wave per slot, each of K and V
  static constexpr int TILE = BN * D * 2;       // bytes of one K (or V) 64-key tile
  static constexpr int SLOT = 2 * KS * TILE;    // [K phase 0 .. KS-1][V phase 0 .. KS-1]
  static_assert(NW % (GH * KS) == 0 && WROWS % 4 == 0 && WROWS <= 16 && NSLOT >= 2 && NSLOT <= 4, "wave layout");
  static_assert(NSLOT * SLOT <= 160 * 1024, "LDS");
};

// image (b): 256-B rows, 16-B chunk ch of row r at chunk slot ch ^ xsw(r)
__device__ __forceinline__ int pf2_xsw(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int pf2_off(int r, int ch) { return r * 256 + ((ch ^ pf2_xsw(r)) << 4); }

__device__ __forceinline__ f32x16_t mfma32x32x16(bf16x8_t a, bf16x8_t b, f32x16_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
#else
  return c;
#endif
}

__device__ __forceinline__ void sched_fence() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_sched_barrier(0);
#endif
}

// value combined with lane ^ 32's: v_permlane32_swap of x with itself leaves the
// low half's values in element 0 and the high half's in element 1, in every lane
__device__ __forceinline__ float xor32_max(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
#else
  return x;
#endif
}
__device__ __forceinline__ float xor32_sum(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
#else
  return x;
#endif
}

__device__ __forceinline__ float fast_exp2(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_exp2f(x);
#else
  return x;
#endif
}

template <int NW, int GH, int KS, int NSLOT>
__global__ void __launch_bounds__(64 * NW, (NW == 4 && NSLOT <= 2 ? 2 : 1)) prefill_attn2_kernel(
    const uint16_t* __restrict__ q, int64_t q_stride, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ qsl, const int32_t* __restrict__ seq_lens, uint16_t* __restrict__ out,
    int64_t out_stride, int num_seqs, int Hq, int Hkv, int bs, float scale_log2, int tiles_per_seq, int n_hg) {
  using C = Pf2Cfg<NW, GH, KS, NSLOT>;
  constexpr int D = C::D;
  const int bid = blockIdx.x;
  const int hg = bid % n_hg;
  const int rest = bid / n_hg;
  const int s = rest % num_seqs;
  const int qt = tiles_per_seq - 1 - rest / num_seqs;  // heavy (late) row tiles first
  const int q0 = qsl[s];
  const int qlen = qsl[s + 1] - q0;
  const int i0 = qt * C::BM;
  if (i0 >= qlen) return;
  const int L = seq_lens[s];
  const int ctx = L - qlen;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hh = w % GH, rb = (w / GH) % C::RB, kp = w / (GH * C::RB);  // head, row block, key phase
  const int h = hg * GH + hh;
  const int kvh = (hg * GH) / (Hq / Hkv);
  const int r = lane & 31, hf = lane >> 5;

  __shared__ __attribute__((aligned(16))) char lds[NSLOT * C::SLOT];

  // Q^T (B operand of S^T): lane holds Q[row r][16 ks + 8 hf + 0..7]
  const int my_row = i0 + rb * 32 + r;
  bf16x8_t qf[D / 16];
  {
    const int row = my_row < qlen ? my_row : 0;
    const uint16_t* qp = q + static_cast<int64_t>(q0 + row) * q_stride + static_cast<int64_t>(h) * D + 8 * hf;
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) qf[ks] = as_frag(ld16(qp + 16 * ks));
    // pin the loads' completion here, before the loop: hipcc's waitcnt pass does not
    // see the asm DMAs, and a wait it placed at the first use inside the loop would
    // count them
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) asm volatile("" : "+v"(qf[ks]));
  }
  // causal limit of this lane's row (rows past qlen: any finite limit, never stored)
  const int lim = min(ctx + my_row, L - 1);
  const int wave_hi = min(ctx + i0 + rb * 32 + 31, L - 1);  // largest limit in the wave
  const int wave_lo = ctx + i0 + rb * 32;                   // smallest
  const int kend = min(L, ctx + min(qlen, i0 + C::BM));
  const int ntiles = (kend + C::BN - 1) / C::BN;
  const int nslots = (ntiles + KS - 1) / KS;               // ring fills (super-tiles)
  const int32_t* btr = block_tables + static_cast<int64_t>(s) * bt_stride;

  auto issue = [&](int t) {  // super-tile t: keys [t * SK, + SK)
    char* kb = lds + (t % NSLOT) * C::SLOT;
    const int key0 = min(t * C::SK + w * C::WROWS, L - 1);
    const int pidx = key0 / bs;
    const int pg = btr[pidx];  // wave-uniform: scalar load
    const int64_t pbase = (static_cast<int64_t>(pg) * Hkv + kvh) * bs - static_cast<int64_t>(pidx) * bs;
#pragma unroll
    for (int i = 0; i < C::NDMA; ++i) {
      const int srow = w * C::WROWS + 4 * i + (lane >> 4);  // row in the super-tile
      const int kabs = min(t * C::SK + srow, L - 1);
      const int ch = (lane & 15) ^ pf2_xsw(srow & 63);
      const int64_t off = (pbase + kabs) * D + ch * 8;  // kabs lies in page pidx
      // phase srow / 64, row srow % 64 of its tile
      char* dst = kb + (srow >> 6) * C::TILE + ((w * C::WROWS + 4 * i) & 63) * 256;
      glds16(kc + off, dst);
      glds16(vc + off, dst + KS * C::TILE);
    }
  };

  f32x16_t o[D / 32];
#pragma unroll
  for (int db = 0; db < D / 32; ++db)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[db][e] = 0.f;
  float m = -INFINITY, l = 0.f;  // m in raw score units (scale applied inside exp2)

  wait_vmcnt<0>();  // Q fragments landed; from here on only the DMAs are counted
#pragma unroll
  for (int p = 0; p < NSLOT - 1; ++p)
    if (p < nslots) issue(p);

  const int g = lane >> 4, gi = lane & 15;
  const int tq = gi >> 2, tp = gi & 3;
  for (int j = 0; j < nslots; ++j) {
    // own DMAs of super-tile j done (later ones may stay in flight), then everyone's
    {
      const int ahead = min(NSLOT - 2, nslots - 1 - j);  // later super-tiles issued so far
      if constexpr (NSLOT >= 4) {
        if (ahead >= 2) wait_vmcnt<4 * C::NDMA>();
        else if (ahead == 1) wait_vmcnt<2 * C::NDMA>();
        else wait_vmcnt<0>();
      } else if constexpr (NSLOT == 3) {
        if (ahead >= 1) wait_vmcnt<2 * C::NDMA>();
        else wait_vmcnt<0>();
      } else {
        wait_vmcnt<0>();
      }
    }
    raw_barrier();
    if (j + NSLOT - 1 < nslots) issue(j + NSLOT - 1);
    const int tile = j * KS + kp;
    const int kv0 = tile * C::BN;
    if (tile >= ntiles || kv0 > wave_hi) continue;  // wave-uniform: nothing of this tile is visible
    // lane byte offsets into the tile (image (b)); per-read parts are one XOR with a
    // constant: K chunk 2 ks + hf -> ^ (ks << 5); V chunk 4 db + .. -> ^ (db << 6)
    const uint32_t kt_off = (j % NSLOT) * C::SLOT + kp * C::TILE;
    const uint32_t k_lane = (kt_off + r * 256) ^ (static_cast<uint32_t>(hf ^ pf2_xsw(r)) << 4);
    const uint32_t v_row = kt_off + KS * C::TILE + (4 * hf + tq) * 256 + 8 * (tp & 1);
    const uint32_t v_lane0 = (v_row + ((((2 * (g & 1) + (tp >> 1)) ^ (hf & 3)) << 4))) | (tq << 6);
    const uint32_t v_lane1 = (v_row + 8 * 256 + ((((2 * (g & 1) + (tp >> 1)) ^ ((hf + 2) & 3)) << 4))) | (tq << 6);

    // ---- S^T = K . Q^T: two 32-key blocks
    f32x16_t sacc[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int e = 0; e < 16; ++e) sacc[kb][e] = 0.f;
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        const uint4 kf = *reinterpret_cast<const uint4*>(lds + ((k_lane ^ (ks << 5)) + kb * 8192));
        sacc[kb] = mfma32x32x16(as_frag(kf), qf[ks], sacc[kb]);
      }
      sched_fence();  // bound the hoisted fragment reads (registers)
    }
    // ---- online softmax (base 2, scale folded into one FMA) on this lane's query row
    const bool need_mask = kv0 + C::BN - 1 > wave_lo || kv0 + C::BN > L;
    float mx = -INFINITY;
    if (need_mask) {
      // key kv0 + 4 hf + c (c a per-register constant) is visible iff c <= lim - kv0 - 4 hf
      const int vis = lim - kv0 - 4 * hf;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          if (kb * 32 + (e & 3) + 8 * (e >> 2) > vis) sacc[kb][e] = -INFINITY;
          mx = fmaxf(mx, sacc[kb][e]);
        }
    } else {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int e = 0; e < 16; ++e) mx = fmaxf(mx, sacc[kb][e]);
    }
    mx = xor32_max(mx);
    const float m_new = fmaxf(m, mx);
    const float nms = m_new == -INFINITY ? 0.f : -m_new * scale_log2;
    // exact rescale skip: no row of the wave raised its max -> alpha = 1 everywhere
    if (__builtin_amdgcn_ballot_w64(m_new > m) != 0) {
      const float alpha = fast_exp2(fmaf(m, scale_log2, nms));  // m = -inf -> 0
      l *= alpha;
#pragma unroll
      for (int db = 0; db < D / 32; ++db)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[db][e] *= alpha;
      m = m_new;
    }
    // pairwise: the fma / add pairs issue as packed v_pk_fma_f32 / v_pk_add_f32
    f32x2v_t rs2 = {0.f, 0.f};
    const f32x2v_t sc2 = {scale_log2, scale_log2}, nm2 = {nms, nms};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        f32x2v_t x = {sacc[kb][e], sacc[kb][e + 1]};
        x = x * sc2 + nm2;
        x[0] = fast_exp2(x[0]);
        x[1] = fast_exp2(x[1]);
        sacc[kb][e] = x[0];
        sacc[kb][e + 1] = x[1];
        rs2 += x;
      }
    l += xor32_sum(rs2[0] + rs2[1]);

    // ---- O^T += V^T . P^T: k-step (kb, ss) takes accumulator registers 8 ss .. 8 ss + 7
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        uint4 pb;
        pb.x = pack2(sacc[kb][8 * ss + 0], sacc[kb][8 * ss + 1]);
        pb.y = pack2(sacc[kb][8 * ss + 2], sacc[kb][8 * ss + 3]);
        pb.z = pack2(sacc[kb][8 * ss + 4], sacc[kb][8 * ss + 5]);
        pb.w = pack2(sacc[kb][8 * ss + 6], sacc[kb][8 * ss + 7]);
        const bf16x8_t pf = as_frag(pb);
        // rows kb*32 + 16 ss + 4 hf + tq (elements 0..3) and + 8 (elements 4..7)
#pragma unroll
        for (int db = 0; db < D / 32; ++db) {
          const uint32_t ro = (kb * 32 + 16 * ss) * 256;
          const bf16x4_t a0 = lds_read_tr16(reinterpret_cast<const uint16_t*>(lds + ((v_lane0 ^ (db << 6)) + ro)));
          const bf16x4_t a1 = lds_read_tr16(reinterpret_cast<const uint16_t*>(lds + ((v_lane1 ^ (db << 6)) + ro)));
          const bf16x8_t vf = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
          o[db] = mfma32x32x16(vf, pf, o[db]);
        }
        sched_fence();
      }
  }

  if constexpr (KS > 1) {
    // merge the key phases of each (head, row block) through the (drained) ring:
    // float slot [((pw * (KS - 1) + kp - 1) * 66 + idx) * 64 + lane], idx 0..63 = O, 64 = m, 65 = l
    static_assert(GH * C::RB * (KS - 1) * 66 * 64 * 4 <= NSLOT * C::SLOT, "merge area");
    float* mg = reinterpret_cast<float*>(lds);
    const int pw = w % (GH * C::RB);
    raw_barrier();  // every wave is past its last ring read (all DMAs were waited)
    if (kp > 0) {
      float* d = mg + (pw * (KS - 1) + kp - 1) * 66 * 64 + lane;
#pragma unroll
      for (int db = 0; db < D / 32; ++db)
#pragma unroll
        for (int e = 0; e < 16; ++e) d[(db * 16 + e) * 64] = o[db][e];
      d[64 * 64] = m;
      d[65 * 64] = l;
    }
    __syncthreads();
    if (kp > 0) return;
#pragma unroll
    for (int k = 1; k < KS; ++k) {
      const float* d = mg + (pw * (KS - 1) + k - 1) * 66 * 64 + lane;
      const float m2 = d[64 * 64], l2 = d[65 * 64];
      const float M = fmaxf(m, m2);
      const float Ms = M == -INFINITY ? 0.f : M * scale_log2;
      const float a1 = fast_exp2(m * scale_log2 - Ms), a2 = fast_exp2(m2 * scale_log2 - Ms);
      l = l * a1 + l2 * a2;
      m = M;
#pragma unroll
      for (int db = 0; db < D / 32; ++db)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[db][e] = o[db][e] * a1 + d[(db * 16 + e) * 64] * a2;
    }
  }

  // ---- epilogue: lane holds O[row r][32 db + 8 t + 4 hf + 0..3] in registers 4t .. 4t+3
  if (my_row < qlen) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    uint16_t* op = out + static_cast<int64_t>(q0 + my_row) * out_stride + static_cast<int64_t>(h) * D + 4 * hf;
#pragma unroll
    for (int db = 0; db < D / 32; ++db)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        uint2 v;
        v.x = pack2(o[db][4 * t + 0] * inv, o[db][4 * t + 1] * inv);
        v.y = pack2(o[db][4 * t + 2] * inv, o[db][4 * t + 3] * inv);
        *reinterpret_cast<uint2*>(op + db * 32 + 8 * t) = v;
      }
  }
}

// GQA grouping: GH query heads of one kv head per workgroup (4*GH waves). gh <= 0
// picks the widest GH in {4, 2, 1} dividing the group size that still gives >= 256
// workgroups (one per CU); measured (bench/prefill_bench.py, profiles/
// r2_prefill_bench.jsonl): Llama-3-8B heads at L = 8192: GH 1 / 2 / 4 = 287 / 315 /
// 443 TFLOP/s, L = 2048: 161 / 199 / 300; at L = 512 GH = 4 leaves CUs idle (66 vs
// 88). D = 64 supports GH <= 2.
int prefill_attention(const uint16_t* q, int64_t q_stride, const uint16_t* kc, const uint16_t* vc,
                      const int32_t* bt, int bt_stride, const int32_t* qsl, const int32_t* seq_lens,
                      uint16_t* out, int64_t out_stride, int num_seqs, int max_q_len, int Hq, int Hkv, int D,
                      int bs, float scale, hipStream_t st, int gh) {
  if (num_seqs <= 0 || max_q_len <= 0) return 0;
  if (bs % 16 != 0 || Hq % Hkv != 0) return -1;
  const int G = Hq / Hkv;
  // D = 128: prefill_attn2_kernel. gh == 0 picks the configuration; gh < 0 forces
  // -gh = 10 * NW + GH (A/B and tests); gh > 0 selects the 16-row kernel above.
  if (D == 128 && gh <= 0) {
    int nw = 0, ghh = 0, ns = 0, ks = 1;
    if (gh < 0) {  // -gh = 1000 * (KS - 1) + 100 * NSLOT + 10 * NW + GH (NSLOT 0: default)
      ks = 1 + (-gh) / 1000;
      ns = ((-gh) / 100) % 10;
      nw = ((-gh) / 10) % 10;
      ghh = (-gh) % 10;
    } else {
      ghh = G % 2 == 0 ? 2 : 1;
      // 8 waves: 128 rows x 2 heads once that still gives two workgroups per CU; else
      // 64 rows x 2 heads x 2 key phases (short prompts: half the serial tile chain).
      // profiles/r3_prefill_attn2.md: 8K 882 / 2K 598 / 512 17 us (8B heads)
      const int64_t wg8 = static_cast<int64_t>(num_seqs) * ((max_q_len + 32 * (8 / ghh) - 1) / (32 * (8 / ghh))) *
                          (Hq / ghh);
      nw = 8;
      ks = wg8 >= 512 ? 1 : 2;
    }
    if (ns == 0) ns = ks == 2 ? 2 : (nw == 8 ? 3 : 2);
    if (G % ghh != 0 || nw % (ghh * ks) != 0) return -1;
    const int bm = 32 * (nw / ghh / ks);
    const int tps = (max_q_len + bm - 1) / bm;
    const int n_hg = Hq / ghh;
    const float sl2 = scale * 1.4426950408889634f;
    dim3 grid(static_cast<unsigned>(static_cast<int64_t>(num_seqs) * tps * n_hg)), block(64 * nw);
#define XGK_PF2(NW, GH, KS, NS)                                                                              \
  hipLaunchKernelGGL((prefill_attn2_kernel<NW, GH, KS, NS>), grid, block, 0, st, q, q_stride, kc, vc, bt, \
                     bt_stride, qsl, seq_lens, out, out_stride, num_seqs, Hq, Hkv, bs, sl2, tps, n_hg)
    const int code = ((ks * 10 + ns) * 10 + nw) * 10 + ghh;
    switch (code) {
      case 1384: XGK_PF2(8, 4, 1, 3); break;
      case 1382: XGK_PF2(8, 2, 1, 3); break;
      case 1381: XGK_PF2(8, 1, 1, 3); break;
      case 1388: XGK_PF2(8, 8, 1, 3); break;
      case 1244: XGK_PF2(4, 4, 1, 2); break;
      case 1242: XGK_PF2(4, 2, 1, 2); break;
      case 1241: XGK_PF2(4, 1, 1, 2); break;
      case 2284: XGK_PF2(8, 4, 2, 2); break;
      case 2282: XGK_PF2(8, 2, 2, 2); break;
      case 2281: XGK_PF2(8, 1, 2, 2); break;
      default: return -1;
    }
#undef XGK_PF2
    return 0;
  }
  const int tps = (max_q_len + 63) / 64;
  if (gh <= 0) {
    gh = 1;
    for (int c = (D == 64 ? 2 : 4); c > 1; c >>= 1)
      if (G % c == 0 && static_cast<int64_t>(num_seqs) * tps * (Hq / c) >= 256) {
        gh = c;
        break;
      }
  }
  if (G % gh != 0 || (gh != 1 && gh != 2 && gh != 4)) return -1;
  dim3 grid(num_seqs * tps, Hq / gh), block(256 * gh);
#define XGK_PF(DV, GV)                                                                                          \
  hipLaunchKernelGGL((prefill_attn_kernel<DV, GV>), grid, block, 0, st, q, q_stride, kc, vc, bt, bt_stride, qsl, \
                     seq_lens, out, out_stride, Hq, Hkv, bs, scale, tps)
  if (D == 128) {
    if (gh == 1) XGK_PF(128, 1);
    else if (gh == 2) XGK_PF(128, 2);
    else XGK_PF(128, 4);
    return 0;
  }
  if (D == 64) {
    if (gh == 1) XGK_PF(64, 1);
    else if (gh == 2) XGK_PF(64, 2);
    else return -1;
    return 0;
  }
#undef XGK_PF
  return -1;
}

}  // namespace xgk
