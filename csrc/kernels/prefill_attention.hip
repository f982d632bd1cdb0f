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
