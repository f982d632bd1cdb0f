// Decode GEMM for 16 < M <= 64: out[M, N] = x[M, K] . W[N, K]^T, W streamed once.
//
// At batch 17..64 a Llama projection is still a weight stream (x is <= 0.5 MB
// per 4096-wide K and lives in L2), but x is now re-read by every column tile,
// so HOW x reaches the MFMAs decides the speed (cdna_hip_programming.md §5,
// "x through LDS in full lines ... NOT fragment-shaped loads"):
//   * workgroup = 4 waves, tile = 64 rows x BN columns (BN = 64 or 128), each
//     wave owns BN/4 weight rows for the whole K range of the workgroup;
//   * W goes HBM -> VGPRs as v_mfma_f32_16x16x32_bf16 A fragments through an
//     8-k-step register ring (one LDS chunk of W per wave in flight, 16 KiB per
//     wave at BN = 128, non-temporal: streamed once);
//   * x goes L2 -> VGPRs as full 128-B lines (line-shaped, 8 lanes per line),
//     then ds_write_b128 into a double-buffered [64][256] LDS chunk with a
//     16-B-granule XOR swizzle (row & 15), read back as B fragments with
//     ds_read_b128 (conflict-free); one __syncthreads per 8 k-steps, and since
//     no LDS-DMA is in flight it is a bare s_barrier: the W ring survives it;
//   * the x loads of chunk c+1 are issued before chunk c's W reloads, so the
//     ds_write at the end of the chunk waits only for them (in-order vmcnt);
//   * the last chunk is peeled (no reload), so W bytes read == W bytes;
//   * split-K over gridDim.y writes fp32 partials [S, M, N] consumed by the next
//     kernel's prologue (add_partials_rmsnorm / rope_cache_partials); SiLU-gate
//     epilogue for the block-16 interleaved gate|up layout (BN = 128, S = 1).
#include "common.h"

namespace xgk {

constexpr int GM_KC = 256;            // k per LDS chunk
constexpr int GM_STEPS = GM_KC / 32;  // 8 MFMA k-steps per chunk

enum GemmM64Mode : int { GM_BF16 = 0, GM_PARTIAL = 1, GM_SILU = 2 };

// LDS slot (16-B units) of granule c (0..31) of x row r in a [rows][256] bf16 chunk
__device__ __forceinline__ int gm_slot(int r, int c) { return (r << 5) | (c ^ (r & 15)); }

template <int NW>
struct GmW {
  uint4 w[GM_STEPS][NW];
};

template <bool NT>
__device__ __forceinline__ uint4 gm_ldw(const uint16_t* p) {
  if constexpr (NT) return ld16_nt(p);
  else return ld16(p);
}

// One LDS chunk (8 k-steps): MFMAs on ring stage W, reload W with the chunk at
// k offset kw (LOADW), stage x of the next chunk into nbuf (LOADX).
template <int MT, int NW, bool LOADW, bool LOADX, bool NT>
__device__ __forceinline__ void gm_chunk(GmW<NW>& W, uint4 (&X)[MT * 2], f32x4_t (&acc)[NW][MT],
                                         const uint4* __restrict__ buf, uint4* __restrict__ nbuf,
                                         const uint16_t* const (&wp)[NW], const uint16_t* const (&xp)[MT * 2],
                                         const int (&xi)[MT * 2], int kx, int kw, int li, int g) {
  if (LOADX) {
#pragma unroll
    for (int i = 0; i < MT * 2; ++i) X[i] = ld16(xp[i] + kx);
  }
#pragma unroll
  for (int t = 0; t < GM_STEPS; ++t) {
    uint4 b[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) b[mt] = buf[gm_slot(16 * mt + li, 4 * t + g)];
#pragma unroll
    for (int nt = 0; nt < NW; ++nt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = mfma16x16x32(as_frag(W.w[t][nt]), as_frag(b[mt]), acc[nt][mt]);
    if (LOADW) {
#pragma unroll
      for (int nt = 0; nt < NW; ++nt) W.w[t][nt] = gm_ldw<NT>(wp[nt] + kw + 32 * t);
    }
    // keep each reload next to the MFMAs that freed its registers (left alone,
    // the scheduler sinks all reloads to the chunk end and the ring drains)
    __builtin_amdgcn_sched_barrier(0);
  }
  if (LOADX) {
#pragma unroll
    for (int i = 0; i < MT * 2; ++i) nbuf[xi[i]] = X[i];
    __syncthreads();
  }
}

// RING = W chunks in flight (1: reload chunk c+1 while computing c; 2: c+2).
template <int MT, int NW, int RING, bool NT>
__global__ void __launch_bounds__(256, 2) gemm_m64_kernel(const uint16_t* __restrict__ x, int M, int K,
                                                          const uint16_t* __restrict__ w, int N,
                                                          float* __restrict__ part, uint16_t* __restrict__ out,
                                                          int mode) {
  constexpr int ROWS = 16 * MT;
  constexpr int XP = MT * 2;  // x granules per thread per chunk: ROWS*32 / 256
  __shared__ uint4 xs[2][ROWS * 32];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int S = gridDim.y, s = blockIdx.y;
  const int kws = K / S;
  const int k0 = s * kws;
  const int nchunks = kws / GM_KC;
  const int nbase = blockIdx.x * (64 * NW) + wid * (16 * NW);

  const uint16_t* wp[NW];
#pragma unroll
  for (int nt = 0; nt < NW; ++nt) wp[nt] = w + static_cast<int64_t>(nbase + 16 * nt + li) * K + k0 + 8 * g;
  const uint16_t* xp[XP];
  int xi[XP];
#pragma unroll
  for (int i = 0; i < XP; ++i) {
    const int p = tid + 256 * i, r = p >> 5, c = p & 31;
    xp[i] = x + static_cast<int64_t>(min(r, M - 1)) * K + k0 + 8 * c;
    xi[i] = gm_slot(r, c);
  }

  uint4 X[XP];
  GmW<NW> A, B;
#pragma unroll
  for (int i = 0; i < XP; ++i) X[i] = ld16(xp[i]);
#pragma unroll
  for (int t = 0; t < GM_STEPS; ++t)
#pragma unroll
    for (int nt = 0; nt < NW; ++nt) A.w[t][nt] = gm_ldw<NT>(wp[nt] + 32 * t);
  if (RING == 2 && nchunks > 1) {
#pragma unroll
    for (int t = 0; t < GM_STEPS; ++t)
#pragma unroll
      for (int nt = 0; nt < NW; ++nt) B.w[t][nt] = gm_ldw<NT>(wp[nt] + GM_KC + 32 * t);
  }
#pragma unroll
  for (int i = 0; i < XP; ++i) xs[0][xi[i]] = X[i];
  __syncthreads();

  f32x4_t acc[NW][MT];
#pragma unroll
  for (int nt = 0; nt < NW; ++nt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#define GM_CH(REG, LW, LX, kwc) \
  gm_chunk<MT, NW, LW, LX, NT>(REG, X, acc, xs[c & 1], xs[(c + 1) & 1], wp, xp, xi, (c + 1) * GM_KC, (kwc) * GM_KC, li, g)
  int c = 0;
  if (RING == 1) {
    for (; c + 1 < nchunks; ++c) GM_CH(A, true, true, c + 1);
    GM_CH(A, false, false, 0);
  } else {
    // stages alternate A (even chunks) / B (odd chunks); each reloads chunk c + 2
    for (; c + 3 < nchunks; c += 2) {
      GM_CH(A, true, true, c + 2);
      ++c;
      GM_CH(B, true, true, c + 2);
      --c;
    }
    const int r = nchunks - c;  // 1, 2 or 3 chunks left
    if (r == 3) {
      GM_CH(A, true, true, c + 2);
      ++c;
      GM_CH(B, false, true, 0);
      ++c;
      GM_CH(A, false, false, 0);
    } else if (r == 2) {
      GM_CH(A, false, true, 0);
      ++c;
      GM_CH(B, false, false, 0);
    } else {
      GM_CH(A, false, false, 0);
    }
  }
#undef GM_CH

  // acc[nt][mt][r] = out[m = 16 mt + li][n = nbase + 16 nt + 4 g + r]
  if (mode == GM_PARTIAL) {
    float* pp = part + static_cast<int64_t>(s) * M * N;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = 16 * mt + li;
      if (m >= M) continue;
#pragma unroll
      for (int nt = 0; nt < NW; ++nt)
        *reinterpret_cast<float4*>(pp + static_cast<int64_t>(m) * N + nbase + 16 * nt + 4 * g) =
            make_float4(acc[nt][mt][0], acc[nt][mt][1], acc[nt][mt][2], acc[nt][mt][3]);
    }
  } else if (mode == GM_BF16) {
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
  } else if (NW == 2) {  // GM_SILU: this wave's rows = gate then up of features nbase/2 .. +15
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

// ---------------------------------------------------------------------------
// Grouped (MoE) form. W is [E, N, K]; x rows come through the block-64 padded
// expert-sorted layout of moe_align (rows[p] = source row of padded row p, -1 =
// pad; offs[E + 1] = padded segment offsets; rows == nullptr: x is already in
// that layout). One workgroup per (column tile, k-split, expert) loops over the
// expert's 64-row tiles, so each column tile of an expert's weights leaves HBM
// once per step and later row tiles (prefill) re-read it from L2 / MALL.
// Output rows are padded positions: out / part have P = offs[E] rows.
template <int NW>
__global__ void __launch_bounds__(256, 2) gemm_m64_grouped_kernel(const uint16_t* __restrict__ x,
                                                                  const int32_t* __restrict__ rows,
                                                                  const int32_t* __restrict__ offs, int K,
                                                                  const uint16_t* __restrict__ w, int N, int P,
                                                                  float* __restrict__ part,
                                                                  uint16_t* __restrict__ out, int mode) {
  constexpr int MT = 4, XP = 8;
  __shared__ uint4 xs[2][64 * 32];
  const int e = blockIdx.z;
  const int p0 = offs[e], p1 = offs[e + 1];
  if (p1 <= p0) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int S = gridDim.y, s = blockIdx.y;
  const int kws = K / S;
  const int k0 = s * kws;
  const int nchunks = kws / GM_KC;
  const int nbase = blockIdx.x * (64 * NW) + wid * (16 * NW);
  const uint16_t* we = w + static_cast<int64_t>(e) * N * K;
  const uint16_t* wp[NW];
#pragma unroll
  for (int nt = 0; nt < NW; ++nt) wp[nt] = we + static_cast<int64_t>(nbase + 16 * nt + li) * K + k0 + 8 * g;

  for (int rt = p0; rt < p1; rt += 64) {
    if (rt != p0) __syncthreads();  // the previous tile's last chunk may still be read from xs
    const int first = rows ? rows[rt] : rt;  // a tile is never all padding
    const uint16_t* xp[XP];
    int xi[XP];
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int q = tid + 256 * i, r = q >> 5, c = q & 31;
      int src = rows ? rows[rt + r] : rt + r;
      if (src < 0) src = first;
      xp[i] = x + static_cast<int64_t>(src) * K + k0 + 8 * c;
      xi[i] = gm_slot(r, c);
    }
    uint4 X[XP];
    GmW<NW> A;
#pragma unroll
    for (int i = 0; i < XP; ++i) X[i] = ld16(xp[i]);
#pragma unroll
    for (int t = 0; t < GM_STEPS; ++t)
#pragma unroll
      for (int nt = 0; nt < NW; ++nt) A.w[t][nt] = ld16(wp[nt] + 32 * t);
#pragma unroll
    for (int i = 0; i < XP; ++i) xs[0][xi[i]] = X[i];
    __syncthreads();
    f32x4_t acc[NW][MT];
#pragma unroll
    for (int nt = 0; nt < NW; ++nt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    int c = 0;
    for (; c + 1 < nchunks; ++c)
      gm_chunk<MT, NW, true, true, false>(A, X, acc, xs[c & 1], xs[(c + 1) & 1], wp, xp, xi, (c + 1) * GM_KC,
                                          (c + 1) * GM_KC, li, g);
    gm_chunk<MT, NW, false, false, false>(A, X, acc, xs[c & 1], xs[(c + 1) & 1], wp, xp, xi, 0, 0, li, g);

    if (mode == GM_PARTIAL) {
      float* pp = part + static_cast<int64_t>(s) * P * N;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = rt + 16 * mt + li;
#pragma unroll
        for (int nt = 0; nt < NW; ++nt)
          *reinterpret_cast<float4*>(pp + static_cast<int64_t>(m) * N + nbase + 16 * nt + 4 * g) =
              make_float4(acc[nt][mt][0], acc[nt][mt][1], acc[nt][mt][2], acc[nt][mt][3]);
      }
    } else if (mode == GM_BF16) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = rt + 16 * mt + li;
#pragma unroll
        for (int nt = 0; nt < NW; ++nt) {
          uint2 v;
          v.x = pack2(acc[nt][mt][0], acc[nt][mt][1]);
          v.y = pack2(acc[nt][mt][2], acc[nt][mt][3]);
          *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * N + nbase + 16 * nt + 4 * g) = v;
        }
      }
    } else if (NW == 2) {  // GM_SILU on the block-16 interleaved gate|up rows of the expert
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

int moe_gemm_m64(const uint16_t* x, const int32_t* rows, const int32_t* offs, int E, int K, const uint16_t* w, int N,
                 int P, float* part, uint16_t* out, int S, int mode, int nw, hipStream_t st) {
  if (E < 1 || P < 0 || P % 64 || S < 1 || (nw != 1 && nw != 2)) return 1;
  if (K % (S * GM_KC) || N % (64 * nw)) return 1;
  if (mode == GM_SILU && (nw != 2 || S != 1)) return 1;
  if (mode == GM_PARTIAL && part == nullptr) return 1;
  if (mode != GM_PARTIAL && out == nullptr) return 1;
  if (P == 0) return 0;
  const dim3 grid(N / (64 * nw), S, E);
  if (nw == 1)
    hipLaunchKernelGGL(gemm_m64_grouped_kernel<1>, grid, dim3(256), 0, st, x, rows, offs, K, w, N, P, part, out, mode);
  else
    hipLaunchKernelGGL(gemm_m64_grouped_kernel<2>, grid, dim3(256), 0, st, x, rows, offs, K, w, N, P, part, out, mode);
  return 0;
}

template <int MT, int NW>
static void launch_gm(int tiles, int S, const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part,
                      uint16_t* out, int mode, int variant, hipStream_t st) {
  // variant bit0: ring depth 2 (else 1); bit1: default cache policy for W (else non-temporal)
  const dim3 grid(tiles, S);
  switch (variant & 3) {
    case 0: hipLaunchKernelGGL((gemm_m64_kernel<MT, NW, 1, true>), grid, dim3(256), 0, st, x, M, K, w, N, part, out, mode); break;
    case 1: hipLaunchKernelGGL((gemm_m64_kernel<MT, NW, 2, true>), grid, dim3(256), 0, st, x, M, K, w, N, part, out, mode); break;
    case 2: hipLaunchKernelGGL((gemm_m64_kernel<MT, NW, 1, false>), grid, dim3(256), 0, st, x, M, K, w, N, part, out, mode); break;
    default: hipLaunchKernelGGL((gemm_m64_kernel<MT, NW, 2, false>), grid, dim3(256), 0, st, x, M, K, w, N, part, out, mode); break;
  }
}

// nw: weight n-frags per wave (1 -> 64-column tiles, 2 -> 128). Returns nonzero on
// an unsupported shape (checked before any launch).
int gemm_m64(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, uint16_t* out, int S, int mode,
             int nw, int variant, hipStream_t st) {
  if (M < 1 || M > 64 || S < 1 || (nw != 1 && nw != 2)) return 1;
  if (K % (S * GM_KC) || N % (64 * nw)) return 1;
  if (mode == GM_SILU && (nw != 2 || S != 1)) return 1;
  if (mode == GM_PARTIAL && part == nullptr) return 1;
  if (mode != GM_PARTIAL && out == nullptr) return 1;
  const int tiles = N / (64 * nw);
  if (M <= 32) {
    if (nw == 1) launch_gm<2, 1>(tiles, S, x, M, K, w, N, part, out, mode, variant, st);
    else launch_gm<2, 2>(tiles, S, x, M, K, w, N, part, out, mode, variant, st);
  } else {
    if (nw == 1) launch_gm<4, 1>(tiles, S, x, M, K, w, N, part, out, mode, variant, st);
    else launch_gm<4, 2>(tiles, S, x, M, K, w, N, part, out, mode, variant, st);
  }
  return 0;
}

}  // namespace xgk
