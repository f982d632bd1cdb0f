// Decode-regime projection GEMM: out[M, N] = x[M, K] . W[N, K]^T for M <= 128.
//
// At decode batch sizes the Llama projections are pure weight streams (W is
// read once per step; x is <= 3.7 MB and L2-resident), so the kernel is built
// for HBM bandwidth, not MFMA rate (cdna_hip_programming.md §5: "GEMV / M <= 16
// decode weights: load straight to VGPRs, deep unroll, late vmcnt"):
//   * workgroup = 4 waves = 32 output columns (two 16-wide MFMA n-tiles); the
//     4 waves split the workgroup's K range, so every wave is an independent
//     weight stream with no barrier in its main loop;
//   * W rows go straight from HBM into v_mfma_f32_16x16x32_bf16 A fragments
//     (16 B per lane), x rows are read as B fragments from L2 (rows >= M are
//     clamped, their results discarded);
//   * named A/B register stages (loop unrolled by two, no runtime-indexed
//     register arrays) keep the next stage's loads in flight during the
//     current stage's MFMAs;
//   * one LDS reduction over the 4 waves at the end; split-K over gridDim.y
//     writes fp32 partials [S, M, N] that the CONSUMING kernel reduces in its
//     prologue (add_partials_rmsnorm / rope_cache_partials), so split-K costs no
//     extra launch;
//   * epilogue modes: bf16, fp32 partials, or SiLU-gate: with the block-16
//     interleaved gate|up layout a workgroup's two n-tiles are the gate and up
//     rows of the same 16 features -> silu(g)*u is written as [M, N/2].
#include "common.h"

namespace xgk {

constexpr int SK_BN = 32;     // columns per workgroup
constexpr int SK_WAVES = 4;

enum SkinnyMode : int { SK_BF16 = 0, SK_PARTIAL = 1, SK_SILU = 2 };

template <int MT, int KS>
struct Stage {
  uint4 w[KS][2];
  uint4 x[KS][MT];
};

template <int MT, int KS>
__device__ __forceinline__ void stage_load(Stage<MT, KS>& st, const uint16_t* w0, const uint16_t* w1,
                                           const uint16_t* const* xr, int k) {
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    st.w[ks][0] = ld16(w0 + k + ks * 32);
    st.w[ks][1] = ld16(w1 + k + ks * 32);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) st.x[ks][mt] = ld16(xr[mt] + k + ks * 32);
  }
}

template <int MT, int KS>
__device__ __forceinline__ void stage_mma(const Stage<MT, KS>& st, f32x4_t (&acc)[2][MT]) {
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = mfma16x16x32(as_frag(st.w[ks][nt]), as_frag(st.x[ks][mt]), acc[nt][mt]);
}

template <int MT, int KS>
__global__ void __launch_bounds__(256) skinny_gemm_kernel(const uint16_t* __restrict__ x, int M, int K,
                                                          const uint16_t* __restrict__ w, int N,
                                                          float* __restrict__ part, uint16_t* __restrict__ out,
                                                          int mode) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int n0 = blockIdx.x * SK_BN;
  const int S = gridDim.y, s = blockIdx.y;
  const int kwg = K / S;                 // K range of this workgroup
  const int kw = kwg / SK_WAVES;         // K range of this wave
  const int kb = s * kwg + wid * kw + 8 * g;

  const uint16_t* w0 = w + static_cast<int64_t>(n0 + li) * K + kb;
  const uint16_t* w1 = w + static_cast<int64_t>(n0 + 16 + li) * K + kb;
  const uint16_t* xr[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int row = min(mt * 16 + li, M - 1);
    xr[mt] = x + static_cast<int64_t>(row) * K + kb;
  }

  f32x4_t acc[2][MT];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  constexpr int STEP = KS * 32;
  const int nst = kw / STEP;             // stages per wave (host guarantees >= 1)
  // Loads of stage i+1 are in flight while stage i is multiplied. The steady
  // loop has no conditional loads (a conditional load makes hipcc merge
  // waitcnt states conservatively and drain vmcnt(0) every iteration).
  Stage<MT, KS> A, B;
  stage_load(A, w0, w1, xr, 0);
  int i = 0;
  for (; i + 2 < nst; i += 2) {
    stage_load(B, w0, w1, xr, (i + 1) * STEP);
    stage_mma(A, acc);
    stage_load(A, w0, w1, xr, (i + 2) * STEP);
    stage_mma(B, acc);
  }
  if (i + 1 < nst) {
    stage_load(B, w0, w1, xr, (i + 1) * STEP);
    stage_mma(A, acc);
    stage_mma(B, acc);
  } else {
    stage_mma(A, acc);
  }

  // ---- reduce the 4 waves' K slices through LDS
  // acc[nt][mt][r] = out[m = 16mt + li][n = n0 + 16nt + 4g + r]
  __shared__ float red[SK_WAVES - 1][2][MT][4][64];
  if (wid > 0) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wid - 1][nt][mt][r][lane] = acc[nt][mt][r];
  }
  __syncthreads();
  if (wid != 0) return;
#pragma unroll
  for (int ww = 0; ww < SK_WAVES - 1; ++ww)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[nt][mt][r] += red[ww][nt][mt][r][lane];

  if (mode == SK_PARTIAL) {
    float* pp = part + static_cast<int64_t>(s) * M * N;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + li;
      if (m >= M) continue;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        *reinterpret_cast<float4*>(pp + static_cast<int64_t>(m) * N + n0 + nt * 16 + 4 * g) =
            make_float4(acc[nt][mt][0], acc[nt][mt][1], acc[nt][mt][2], acc[nt][mt][3]);
    }
  } else if (mode == SK_BF16) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + li;
      if (m >= M) continue;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        uint2 v;
        v.x = pack2(acc[nt][mt][0], acc[nt][mt][1]);
        v.y = pack2(acc[nt][mt][2], acc[nt][mt][3]);
        *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * N + n0 + nt * 16 + 4 * g) = v;
      }
    }
  } else {  // SK_SILU: n-tile 0 = gate rows, n-tile 1 = up rows of features f0..f0+15
    const int F = N / 2;
    const int f0 = n0 / 2 + 4 * g;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + li;
      if (m >= M) continue;
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float gt = acc[0][mt][r];
        o[r] = gt / (1.f + __expf(-gt)) * acc[1][mt][r];
      }
      uint2 v;
      v.x = pack2(o[0], o[1]);
      v.y = pack2(o[2], o[3]);
      *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * F + f0) = v;
    }
  }
}

template <int MT, int KS>
static void launch_skinny(dim3 grid, const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part,
                          uint16_t* out, int mode, hipStream_t st) {
  hipLaunchKernelGGL((skinny_gemm_kernel<MT, KS>), grid, dim3(256), 0, st, x, M, K, w, N, part, out, mode);
}

// ---------------------------------------------------------------------------
// "Slab" variant for 16 < M <= 64: the workgroup's whole x slab
// [16*MT rows][Ks = K/S] (<= 128 KiB) is loaded into LDS once (one barrier),
// then each of the 4 waves streams its own 16 weight rows through an 8-deep
// register ring (8 k-steps = 8 KiB per wave in flight) with x B-fragments
// read from LDS: no barrier in the main loop, x read from L2 once per
// workgroup instead of once per wave. Tile 64 columns; split-K partials.
// ---------------------------------------------------------------------------
constexpr int SL_NKS = 32;            // k-steps per workgroup slice
constexpr int SL_KS = SL_NKS * 32;    // K slice per workgroup (fixed: K / split_k must equal it)

template <int MT>
__global__ void __launch_bounds__(256) skinny_slab_kernel(const uint16_t* __restrict__ x, int M, int K,
                                                          const uint16_t* __restrict__ w, int N,
                                                          float* __restrict__ part, uint16_t* __restrict__ out,
                                                          int mode) {
  extern __shared__ __attribute__((aligned(16))) uint16_t xs[];  // [16*MT][Ks], 16-B chunks swizzled
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int n0 = blockIdx.x * 64;
  const int S = gridDim.y, s = blockIdx.y;
  const int Ks = K / S;
  const int kb = s * Ks;
  const int nch = Ks / 8;  // 16-B chunks per slab row
  const uint16_t* wrow = w + static_cast<int64_t>(n0 + wid * 16 + li) * K + kb + 8 * g;

  // The wave's ENTIRE weight slice (SL_NKS k-steps = 32 KiB per wave, 128 VGPRs)
  // is requested before anything else: at one workgroup per CU the register
  // file is there to hold it, and all of the HBM latency overlaps the slab fill.
  uint4 wr[SL_NKS];
#pragma unroll
  for (int ks = 0; ks < SL_NKS; ++ks) wr[ks] = ld16_nt(wrow + ks * 32);

  // slab fill (rows >= M are zero): 16 independent loads in flight per thread
  // before their LDS stores -- a load->store loop would serialise L2 latencies.
  const int total = 16 * MT * nch;
  for (int p0 = 0; p0 < total; p0 += 256 * 16) {
    uint4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int p = p0 + u * 256 + threadIdx.x;
      const int row = p / nch, ch = p % nch;
      const int rr = min(row, M - 1);
      v[u] = p < total ? ld16(x + static_cast<int64_t>(rr) * K + kb + ch * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int p = p0 + u * 256 + threadIdx.x;
      if (p >= total) continue;
      const int row = p / nch, ch = p % nch;
      st16(xs + static_cast<int64_t>(row) * Ks + ((ch ^ (row & 15)) * 8), row < M ? v[u] : make_uint4(0, 0, 0, 0));
    }
  }
  __syncthreads();

  f32x4_t acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int ks = 0; ks < SL_NKS; ++ks) {
    const bf16x8_t a = as_frag(wr[ks]);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int row = mt * 16 + li;
      const int ch = ks * 4 + g;
      const uint4 b = *reinterpret_cast<const uint4*>(xs + static_cast<int64_t>(row) * Ks + ((ch ^ (row & 15)) * 8));
      acc[mt] = mfma16x16x32(a, as_frag(b), acc[mt]);
    }
  }

  // acc[mt][r] = out[m = 16mt + li][n = n0 + 16wid + 4g + r]
  if (mode == SK_PARTIAL) {
    float* pp = part + static_cast<int64_t>(s) * M * N;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + li;
      if (m < M)
        *reinterpret_cast<float4*>(pp + static_cast<int64_t>(m) * N + n0 + wid * 16 + 4 * g) =
            make_float4(acc[mt][0], acc[mt][1], acc[mt][2], acc[mt][3]);
    }
  } else {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + li;
      if (m >= M) continue;
      uint2 v;
      v.x = pack2(acc[mt][0], acc[mt][1]);
      v.y = pack2(acc[mt][2], acc[mt][3]);
      *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * N + n0 + wid * 16 + 4 * g) = v;
    }
  }
}

constexpr int SL_MAX_LDS = 128 * 1024;

// 0 = launched, -1 = shape not supported by the slab kernel
static int launch_slab(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, uint16_t* out,
                       int split_k, int mode, hipStream_t st) {
  if (M <= 16 || M > 64 || N % 64 || mode == SK_SILU) return -1;
  const int MT = M <= 32 ? 2 : 4;
  const int Ks = K / split_k;
  if (K % split_k || Ks != SL_KS) return -1;
  const size_t lds = static_cast<size_t>(16 * MT) * Ks * 2;
  if (lds > SL_MAX_LDS) return -1;
  dim3 grid(N / 64, split_k);
  static bool attr_set = false;  // opt in to > 64 KiB dynamic LDS once (not a stream op: graph-safe)
  if (!attr_set) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&skinny_slab_kernel<2>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, SL_MAX_LDS) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(&skinny_slab_kernel<4>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, SL_MAX_LDS) != hipSuccess)
      return -1;  // the LDS opt-in failed: the caller reports the unsupported launch
    attr_set = true;
  }
  if (MT == 2)
    hipLaunchKernelGGL(skinny_slab_kernel<2>, grid, dim3(256), lds, st, x, M, K, w, N, part, out, mode);
  else
    hipLaunchKernelGGL(skinny_slab_kernel<4>, grid, dim3(256), lds, st, x, M, K, w, N, part, out, mode);
  return 0;
}

// Largest per-workgroup K slice the slab kernel can hold for M rows (0 = not applicable).
int skinny_slab_kmax(int M) {
  if (M <= 16 || M > 64) return 0;
  return SL_KS;  // the slab kernel takes exactly this K slice per workgroup
}

// K must be a multiple of split_k * 4 waves * stage depth (KS*32); returns -1 otherwise.
int skinny_gemm(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, uint16_t* out, int split_k,
                int mode, hipStream_t st) {
  if (M <= 0) return 0;
  if (M > 128 || N % SK_BN || split_k <= 0) return -1;
  if (mode != SK_PARTIAL && split_k != 1) return -1;
  if (M > 16 && M <= 64 && launch_slab(x, M, K, w, N, part, out, split_k, mode, st) == 0) return 0;
  const int MT = M <= 16 ? 1 : M <= 32 ? 2 : M <= 64 ? 4 : 8;
  const int KS = MT >= 8 ? 1 : 2;
  if (K % (split_k * SK_WAVES * KS * 32)) return -1;
  dim3 grid(N / SK_BN, split_k);
  switch (MT) {
    case 1: launch_skinny<1, 2>(grid, x, M, K, w, N, part, out, mode, st); break;
    case 2: launch_skinny<2, 2>(grid, x, M, K, w, N, part, out, mode, st); break;
    case 4: launch_skinny<4, 2>(grid, x, M, K, w, N, part, out, mode, st); break;
    default: launch_skinny<8, 1>(grid, x, M, K, w, N, part, out, mode, st); break;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// Split-K consumers
// ---------------------------------------------------------------------------
// residual[t] += sum_s part[s, t]; out[t] = rmsnorm(residual[t]) * w
// SP > 0: compile-time partial count (every load of a chunk issued before the
// adds); SP == 0: runtime S.
template <int VPT, int SP>
__global__ void __launch_bounds__(256) add_partials_rmsnorm_kernel(const float* __restrict__ part, int S, int T,
                                                                   uint16_t* __restrict__ residual,
                                                                   const uint16_t* __restrict__ w,
                                                                   uint16_t* __restrict__ out, int H, float eps) {
  __shared__ float red[8];
  const int row = blockIdx.x;
  const int nchunk = H >> 3;
  uint16_t* rr = residual + static_cast<int64_t>(row) * H;
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = threadIdx.x + k * blockDim.x;
    if (c < nchunk) {
      unpack8(ld16(rr + c * 8), v[k]);
      if constexpr (SP > 0) {
        float4 a[SP], b[SP];
#pragma unroll
        for (int s = 0; s < SP; ++s) {
          const float* pp = part + (static_cast<int64_t>(s) * T + row) * H + c * 8;
          a[s] = *reinterpret_cast<const float4*>(pp);
          b[s] = *reinterpret_cast<const float4*>(pp + 4);
        }
#pragma unroll
        for (int s = 0; s < SP; ++s) {
          v[k][0] += a[s].x; v[k][1] += a[s].y; v[k][2] += a[s].z; v[k][3] += a[s].w;
          v[k][4] += b[s].x; v[k][5] += b[s].y; v[k][6] += b[s].z; v[k][7] += b[s].w;
        }
      } else {
        for (int s = 0; s < S; ++s) {
          const float* pp = part + (static_cast<int64_t>(s) * T + row) * H + c * 8;
          const float4 a = *reinterpret_cast<const float4*>(pp);
          const float4 b = *reinterpret_cast<const float4*>(pp + 4);
          v[k][0] += a.x; v[k][1] += a.y; v[k][2] += a.z; v[k][3] += a.w;
          v[k][4] += b.x; v[k][5] += b.y; v[k][6] += b.z; v[k][7] += b.w;
        }
      }
      const uint4 pk = pack8(v[k]);
      st16(rr + c * 8, pk);
      unpack8(pk, v[k]);
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[k][i] * v[k][i];
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / static_cast<float>(H) + eps);
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int c = threadIdx.x + k * blockDim.x;
    if (c < nchunk) {
      float wf[8], o[8];
      unpack8(ld16(w + c * 8), wf);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = v[k][i] * inv * wf[i];
      st16(out + static_cast<int64_t>(row) * H + c * 8, pack8(o));
    }
  }
}

void add_partials_rmsnorm(const float* part, int S, int T, uint16_t* residual, const uint16_t* w, uint16_t* out,
                          int H, float eps, hipStream_t st) {
  if (T <= 0) return;
  const int nchunk = H / 8;
  const int thr = nchunk >= 256 ? 256 : ((nchunk + 63) / 64) * 64;
  int vpt = (nchunk + thr - 1) / thr;
  vpt = vpt <= 1 ? 1 : vpt <= 2 ? 2 : vpt <= 4 ? 4 : 8;
  dim3 g(T), b(thr);
#define XGK_APR(V, SPV) hipLaunchKernelGGL((add_partials_rmsnorm_kernel<V, SPV>), g, b, 0, st, part, S, T, residual, \
                                           w, out, H, eps)
#define XGK_APR_S(V)            \
  if (S == 1) XGK_APR(V, 1);    \
  else if (S == 2) XGK_APR(V, 2); \
  else if (S == 4) XGK_APR(V, 4); \
  else if (S == 8) XGK_APR(V, 8); \
  else XGK_APR(V, 0);
  switch (vpt) {
    case 1: XGK_APR_S(1); break;
    case 2: XGK_APR_S(2); break;
    case 4: XGK_APR_S(4); break;
    default: XGK_APR_S(8); break;
  }
#undef XGK_APR_S
#undef XGK_APR
}

// Fused decode layer, large split-K slabs (M ~ 64 decode): residual[t] +=
// sum_s part[s, t] (bf16, in place) and the new residual's sums of squares per
// 1024-column chunk, ss_part[chunk * T + t]; the next GEMM adds the H/1024 chunk
// sums in order (deterministic) and applies the RMSNorm as a row scale. One
// 128-thread workgroup per (row, chunk): 8 columns per lane, every partial load
// issued before the adds; 4-8x the workgroups of add_partials_rmsnorm.
//
// Simulated TP all-reduce (a --tp-shard run stands in for one rank of a TP group):
// sim_ticks > 0 makes every workgroup wait that many ticks of the 100 MHz wall clock
// first -- the peer round trip of the one-shot xGMI all-reduce -- so the simulation
// exposes collective latency (profiles/r3_tp_ar_overlap.md).
template <int SP>
__global__ void __launch_bounds__(128) add_partials_resid_kernel(const float* __restrict__ part, int S, int T,
                                                                  uint16_t* __restrict__ residual,
                                                                  float* __restrict__ ss_part, int H, uint64_t sim_ticks) {
  __shared__ float red[8];
  const int nchunk = H / 1024;
  if (sim_ticks) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < sim_ticks) __builtin_amdgcn_s_sleep(1);
  }
  const int t = blockIdx.x / nchunk, chunk = blockIdx.x % nchunk;
  const int col = (chunk * 128 + threadIdx.x) * 8;
  uint16_t* rr = residual + static_cast<int64_t>(t) * H + col;
  float v[8];
  unpack8(ld16(rr), v);
  if constexpr (SP > 0) {
    float4 a[SP], b[SP];
#pragma unroll
    for (int s = 0; s < SP; ++s) {
      const float* pp = part + (static_cast<int64_t>(s) * T + t) * H + col;
      a[s] = *reinterpret_cast<const float4*>(pp);
      b[s] = *reinterpret_cast<const float4*>(pp + 4);
    }
#pragma unroll
    for (int s = 0; s < SP; ++s) {
      v[0] += a[s].x; v[1] += a[s].y; v[2] += a[s].z; v[3] += a[s].w;
      v[4] += b[s].x; v[5] += b[s].y; v[6] += b[s].z; v[7] += b[s].w;
    }
  } else {
    for (int s = 0; s < S; ++s) {
      const float* pp = part + (static_cast<int64_t>(s) * T + t) * H + col;
      const float4 a = *reinterpret_cast<const float4*>(pp);
      const float4 b = *reinterpret_cast<const float4*>(pp + 4);
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
      v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    }
  }
  const uint4 pk = pack8(v);
  st16(rr, pk);
  unpack8(pk, v);  // statistics of the rounded (stored) residual
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) ss += v[i] * v[i];
  ss = block_sum(ss, red);
  if (threadIdx.x == 0) ss_part[static_cast<int64_t>(chunk) * T + t] = ss;
}

void add_partials_resid(const float* part, int S, int T, uint16_t* residual, float* ss_part, int H,
                        hipStream_t st, uint64_t sim_ticks) {
  if (T <= 0) return;
  const dim3 g(T * (H / 1024));
#define XGK_APRS(SPV) \
  hipLaunchKernelGGL((add_partials_resid_kernel<SPV>), g, dim3(128), 0, st, part, S, T, residual, ss_part, H, sim_ticks)
  if (S == 1) XGK_APRS(1);
  else if (S == 2) XGK_APRS(2);
  else if (S == 4) XGK_APRS(4);
  else if (S == 8) XGK_APRS(8);
  else XGK_APRS(0);
#undef XGK_APRS
}

// out[t, :] = bf16(sum_s part[s, t, :])  (used when a collective needs the sum)
__global__ void __launch_bounds__(256) reduce_partials_kernel(const float* __restrict__ part, int S, int64_t n,
                                                              uint16_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n / 4;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    float4 a = reinterpret_cast<const float4*>(part)[i];
    for (int s = 1; s < S; ++s) {
      const float4 b = reinterpret_cast<const float4*>(part + s * n)[i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    uint2 v;
    v.x = pack2(a.x, a.y);
    v.y = pack2(a.z, a.w);
    reinterpret_cast<uint2*>(out)[i] = v;
  }
}

void reduce_partials(const float* part, int S, int64_t n, uint16_t* out, hipStream_t st) {
  if (n <= 0) return;
  int64_t g = (n / 4 + 255) / 256;
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(g < 2048 ? g : 2048), dim3(256), 0, st, part, S, n, out);
}

}  // namespace xgk
