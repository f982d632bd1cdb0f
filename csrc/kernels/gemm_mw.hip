// gemm_mw: weight-streaming MFMA GEMM for mid-sized M (64 < M <= 320): the
// mixed continuous-batching step (decode rows + a bounded prefill chunk) and
// prompt-sized steps that are still weight-stream-bound on MI355X.
//
//   out[M, N] = x[M, K] . W[N, K]^T        (bf16 in, fp32 accumulate)
//
// At M ~ 192 a step needs ~190 FLOP per weight byte, i.e. ~1.1 PFLOP/s of bf16
// MFMA beside a ~6 TB/s weight stream -- the kernel has to keep BOTH busy. The
// decode kernel (gemm_m64g) gives each wave its own weight rows and all M rows of
// x; at M = 192 its x tile would be re-read from L2 by every 128-column tile at 3x
// the weight bytes and its LDS reads would outrun the MFMAs. Here:
//
//   * one 512-thread workgroup per CU (8 waves as WN x WM, 2 waves per SIMD);
//     the workgroup owns a WCOLS = WN*16*NWT column tile and every one of the
//     XROWS = WM*16*MTW x rows, so x bytes per weight byte = M / WCOLS;
//   * wave (wn, wm) computes 16*NWT columns x 16*MTW rows with
//     v_mfma_f32_16x16x32_bf16 (W fragment = A, x fragment = B):
//     per 32-deep k step NWT + MTW ds_read_b128 feed NWT*MTW MFMAs;
//   * both operands arrive by LDS-DMA (global_load_lds_dwordx4, 8 rows x 128 B per
//     wave instruction) into lane-linear images with the 16-B granule XOR-swizzle
//     (granule ^ row & 7) applied on the global source address and undone on the
//     fragment reads (conflict-free ds_read_b128, cdna_hip_programming.md T2);
//   * K chunks of 64; the weight ring is D chunks deep (D+1 slots), the x ring D-1
//     deep (D slots): vmcnt retires in issue order, so x(c) must be issued before
//     W(c+1) -- the per-chunk issue order is x(c+D-1), W(c+D) and the counted wait
//     before chunk c leaves W(c+1..c+D-1) and x(c+1..c+D-2) in flight across the
//     raw s_barrier (cdna_hip_programming.md §5 "Pipelining across barriers");
//   * split-K for grids that would not fill 256 CUs: fp32 partial slabs
//     [S, M, N] reduced by the consumer kernel (rope_cache_partials /
//     add_partials_rmsnorm), uneven chunk ranges allowed;
//   * XCD-grouped block order: the workgroups of one split sit on the same XCDs, so
//     each XCD's L2 holds only its K range of x (the down projection's x is 7 MB at
//     M = 256, more than one 4 MB L2).
// Epilogues: fp32 partials, bf16, or the SiLU gate of a block-16 interleaved
// gate|up weight (split 1).
#include "glds.h"

namespace xgk {

int k_rotation(int S);  // gemm_m64g.hip

enum : int { MW_BF16 = 0, MW_PARTIAL = 1, MW_SILU = 2 };

// PR: anatomy-probe code paths of round 4 (profiles/r4_mw_probe.md), now always 0:
// PR & 7 selects compiled-out pipeline parts, PR & 8 forces K rotation.
template <int WN, int NWT, int MTW, int D, bool NT, int PR = 0>
__global__ void __launch_bounds__(512, 1) gemm_mw_kernel(const uint16_t* __restrict__ x, int M, int K,
                                                          const uint16_t* __restrict__ w, int N, int S,
                                                          float* __restrict__ part, uint16_t* __restrict__ out,
                                                          int mode, int krot) {
  constexpr int WM = 8 / WN;
  constexpr int KC = 64, RB = 128, RPI = 8;     // k per chunk, bytes per LDS row, rows per DMA instruction
  constexpr int WCOLS = WN * 16 * NWT;
  constexpr int XROWS = WM * 16 * MTW;
  constexpr int WSLOT = WCOLS * RB;
  constexpr int XSLOT = XROWS * RB;
  constexpr int WI = WCOLS / RPI / 8;           // weight DMA instructions per wave per chunk
  constexpr int XI = XROWS / RPI / 8;           // x DMA instructions per wave per chunk
  static_assert(WN * WM == 8 && WI >= 1 && XI >= 1 && WCOLS % 64 == 0 && XROWS % 64 == 0, "bad gemm_mw geometry");
  static_assert(D >= 2 && D <= 4, "ring depth");
  static_assert((D + 1) * WSLOT + D * XSLOT <= 160 * 1024, "LDS");
  // ONE __shared__ object (cdna_hip_programming.md §5 "Three .s-level traps" (a))
  __shared__ __attribute__((aligned(1024))) uint8_t smem[(D + 1) * WSLOT + D * XSLOT];
  uint8_t* const wring = smem;
  uint8_t* const xring = smem + (D + 1) * WSLOT;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int wn = wid % WN, wm = wid / WN;

  // XCD-grouped virtual block id (bijective for any grid size): blocks that share
  // an XCD (same blockIdx % 8) get consecutive ids -> mostly one split per XCD
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7;
  const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int ntiles = N / WCOLS;
  const int s = v / ntiles, tile = v - s * ntiles;
  const int nch_all = K / KC;
  const int c_lo = s * nch_all / S, c_hi = (s + 1) * nch_all / S;
  const int nch = c_hi - c_lo;
  const int k0 = c_lo * KC;
  const int n0 = tile * WCOLS;

  // DMA sources: wave instruction i covers rows 8 gi .. 8 gi + 7 (gi = wid * I + i);
  // lane -> (row dr = lane / 8, physical granule dj = lane % 8) holding logical
  // granule dj ^ dr
  const int dr = lane >> 3, dj = lane & 7;
  const uint16_t* wsrc[WI];
#pragma unroll
  for (int i = 0; i < WI; ++i)
    wsrc[i] = w + static_cast<int64_t>(n0 + 8 * (wid * WI + i) + dr) * K + k0 + 8 * (dj ^ dr);
  const uint16_t* xsrc[XI];
#pragma unroll
  for (int i = 0; i < XI; ++i)
    xsrc[i] = x + static_cast<int64_t>(min(8 * (wid * XI + i) + dr, M - 1)) * K + k0 + 8 * (dj ^ dr);

  constexpr int PK = PR & 7;
  const int rot = ((PR & 8) || krot) ? (tile * 37) % nch : 0;  // K-chunk rotation (gemm_m64g.hip k_rotation)
  auto kof = [&](int c) {
    const int cc = c + rot;
    return (cc >= nch ? cc - nch : cc) * KC;
  };
  auto issue_w = [&](int c) {
    if constexpr (PK == 2 || PK == 4 || PK == 5) return;
    uint8_t* slot = wring + (c % (D + 1)) * WSLOT;
    const int kk = kof(c);
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      if constexpr (NT) glds16_nt(wsrc[i] + kk, slot + (wid * WI + i) * 1024);
      else glds16(wsrc[i] + kk, slot + (wid * WI + i) * 1024);
    }
  };
  auto issue_x = [&](int c) {
    if constexpr (PK == 2 || PK == 3 || PK == 6) return;
    uint8_t* slot = xring + (c % D) * XSLOT;
    const int kk = kof(c);
#pragma unroll
    for (int i = 0; i < XI; ++i) glds16(xsrc[i] + kk, slot + (wid * XI + i) * 1024);
  };

  f32x4_t acc[NWT][MTW];
#pragma unroll
  for (int nt = 0; nt < NWT; ++nt)
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) acc[nt][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int wrow0 = wn * 16 * NWT, xrow0 = wm * 16 * MTW;
  auto compute = [&](int c) {
    const uint8_t* ws = wring + (c % (D + 1)) * WSLOT;
    const uint8_t* xs = xring + (c % D) * XSLOT;
#pragma unroll
    for (int t = 0; t < KC / 32; ++t) {
      const int phys = (4 * t + g) ^ (li & 7);
      uint4 a[NWT], b[MTW];
#pragma unroll
      for (int nt = 0; nt < NWT; ++nt)
        a[nt] = *reinterpret_cast<const uint4*>(ws + (wrow0 + 16 * nt + li) * RB + phys * 16);
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt)
        b[mt] = *reinterpret_cast<const uint4*>(xs + (xrow0 + 16 * mt + li) * RB + phys * 16);
#pragma unroll
      for (int nt = 0; nt < NWT; ++nt)
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt) acc[nt][mt] = mfma16x16x32(as_frag(a[nt]), as_frag(b[mt]), acc[nt][mt]);
    }
  };

  // Issue order: chunk j (j = -D .. nch-1, the negative ones are the prologue)
  // issues x(j + D - 1) then W(j + D), each only if it exists. Before chunk c,
  // x(c) must have landed; issued after it are W(c+1) and, per later chunk,
  // x(c+1..c+D-2) / W(c+2..c+D-1). With rem = min(nch - 1 - c, D - 1) chunks still
  // ahead, the exact count left in flight is rem W groups + min(rem, D - 2) x groups.
  auto wait_for = [&](int c) {
    const int rem = min(nch - 1 - c, D - 1);
    if constexpr (D >= 4) {
      if (rem >= 3) { wait_vmcnt<3 * WI + 2 * XI>(); return; }
    }
    if constexpr (D >= 3) {
      if (rem >= 2) { wait_vmcnt<2 * WI + (D - 2 < 2 ? D - 2 : 2) * XI>(); return; }
    }
    if (rem >= 1) wait_vmcnt<WI + (D >= 3 ? XI : 0)>();
    else wait_vmcnt<0>();
  };

  // prologue: W0, x0, W1, x1, W2, ..., x(D-2), W(D-1)
  issue_w(0);
#pragma unroll
  for (int j = 1; j < D; ++j) {
    if (j - 1 < nch) issue_x(j - 1);
    if (j < nch) issue_w(j);
  }
  for (int c = 0; c < nch; ++c) {
    wait_for(c);
    raw_barrier();
    // refills the slots read by chunk c - 1 (every wave is past the barrier)
    if (c + D - 1 < nch) issue_x(c + D - 1);
    if (c + D < nch) issue_w(c + D);
    if constexpr (PK != 1 && PK != 5 && PK != 6) compute(c);
  }

  // acc[nt][mt][r] = out[m = xrow0 + 16 mt + li][n = n0 + wrow0 + 16 nt + 4 g + r]
  if (mode == MW_PARTIAL) {
    float* pp = part + static_cast<int64_t>(s) * M * N;
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
      const int m = xrow0 + 16 * mt + li;
      if (m >= M) continue;
#pragma unroll
      for (int nt = 0; nt < NWT; ++nt)
        *reinterpret_cast<float4*>(pp + static_cast<int64_t>(m) * N + n0 + wrow0 + 16 * nt + 4 * g) =
            make_float4(acc[nt][mt][0], acc[nt][mt][1], acc[nt][mt][2], acc[nt][mt][3]);
    }
  } else if (mode == MW_BF16) {
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
      const int m = xrow0 + 16 * mt + li;
      if (m >= M) continue;
#pragma unroll
      for (int nt = 0; nt < NWT; ++nt) {
        uint2 o;
        o.x = pack2(acc[nt][mt][0], acc[nt][mt][1]);
        o.y = pack2(acc[nt][mt][2], acc[nt][mt][3]);
        *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * N + n0 + wrow0 + 16 * nt + 4 * g) = o;
      }
    }
  } else if constexpr (NWT % 2 == 0) {
    // SiLU gate: n-tiles 2j (gate) / 2j + 1 (up) are one interleaved 16-row block pair
    const int F = N / 2, f0 = (n0 + wrow0) / 2 + 4 * g;
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
      const int m = xrow0 + 16 * mt + li;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < NWT / 2; ++j) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gt = acc[2 * j][mt][r];
          o[r] = gt / (1.f + __expf(-gt)) * acc[2 * j + 1][mt][r];
        }
        uint2 v2;
        v2.x = pack2(o[0], o[1]);
        v2.y = pack2(o[2], o[3]);
        *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * F + f0 + 16 * j) = v2;
      }
    }
  }
}

// (Measured and removed in round 5 -- records kept in profiles/: the split-role rings
// "gemm_mw2" (waves 0-3 weights, 4-7 x; r4_mw_sweep.md, r4_mw2_sweep.jsonl) and the
// software-pipelined "gemm_mw3" (one ring of whole chunks, reads of chunk c + 1 under
// chunk c's MFMAs; r4_mw_sweep_v1.jsonl) never beat the kernel above on a default plan,
// and the anatomy probes (PR != 0, r4_mw_probe.md) were measurement builds.)

// cfg -> (WN, NWT, D, NT): 0 = 4 x 2 waves, 256 columns, ring 2, nt weights;
// 1 = 4 x 2, 128 columns, ring 3, nt; 2 = 4 x 2, 128 columns, ring 2, nt; 3 / 4 = 0 / 1
// with default-policy weight loads; 5 = 2 x 4 waves, 128 columns, ring 3, nt;
// 6 = 2 x 4 waves, 256 columns, ring 2, nt. The x tile follows M: 32-row steps on the
// 4 x 2 layouts (64 .. 320 rows), 64-row steps on the 2 x 4 ones (64 .. 256).
int mw_cfg_cols(int cfg) { return (cfg == 0 || cfg == 3 || cfg == 6) ? 256 : 128; }
static int mw_cfg_wn(int cfg) { return cfg >= 5 ? 2 : 4; }

template <int WN, int NWT, int MTW, int D>
constexpr bool mw_fits() {
  constexpr int WM = 8 / WN;
  return (WM * 16 * MTW) % 64 == 0 && (D + 1) * (WN * 16 * NWT * 128) + D * (WM * 16 * MTW * 128) <= 160 * 1024;
}

template <int WN, int NWT, int D, bool NT>
static int launch_mw(int mtw, dim3 grid, hipStream_t st, const uint16_t* x, int M, int K, const uint16_t* w, int N,
                     int S, float* part, uint16_t* out, int mode) {
#define XGK_MW(MTW)                                                                                             \
  case MTW:                                                                                                     \
    if constexpr (mw_fits<WN, NWT, MTW, D>()) {                                                                 \
      hipLaunchKernelGGL((gemm_mw_kernel<WN, NWT, MTW, D, NT>), grid, dim3(512), 0, st, x, M, K, w, N, S, part, \
                         out, mode, k_rotation(S));                                                             \
      return 0;                                                                                                 \
    }                                                                                                           \
    return 1;
  if constexpr (WN == 4) {
    switch (mtw) {
      XGK_MW(2)
      XGK_MW(4)
      XGK_MW(6)
      XGK_MW(8)
      XGK_MW(10)
      default: return 1;
    }
  } else {
    switch (mtw) {
      XGK_MW(1)
      XGK_MW(2)
      XGK_MW(3)
      XGK_MW(4)
      default: return 1;
    }
  }
#undef XGK_MW
}

// x [M, K] bf16 row-major, w [N, K] bf16 row-major. mode MW_PARTIAL: part [S, M, N]
// fp32; MW_BF16: out [M, N]; MW_SILU: out [M, N / 2] (S = 1). 0 = launched, 1 = a
// shape / configuration this kernel does not take (M beyond the cfg's LDS budget).
int gemm_mw(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, uint16_t* out, int S, int mode,
            int cfg, hipStream_t st) {
  if (M < 1 || M > 320 || cfg < 0 || cfg >= 7 || S < 1 || K % 64 || S > K / 64) return 1;
  const int cols = mw_cfg_cols(cfg);
  if (N % cols) return 1;
  if (mode == MW_PARTIAL) {
    if (part == nullptr) return 1;
  } else if (mode == MW_BF16 || mode == MW_SILU) {
    if (out == nullptr || S != 1) return 1;
  } else {
    return 1;
  }
  const dim3 grid((N / cols) * S);
  int mtw;
  if (mw_cfg_wn(cfg) == 4) mtw = M <= 64 ? 2 : M <= 128 ? 4 : M <= 192 ? 6 : M <= 256 ? 8 : 10;
  else mtw = (M + 63) / 64;
  switch (cfg) {
    case 0: return launch_mw<4, 4, 2, true>(mtw, grid, st, x, M, K, w, N, S, part, out, mode);
    case 1: return launch_mw<4, 2, 3, true>(mtw, grid, st, x, M, K, w, N, S, part, out, mode);
    case 2: return launch_mw<4, 2, 2, true>(mtw, grid, st, x, M, K, w, N, S, part, out, mode);
    case 3: return launch_mw<4, 4, 2, false>(mtw, grid, st, x, M, K, w, N, S, part, out, mode);
    case 4: return launch_mw<4, 2, 3, false>(mtw, grid, st, x, M, K, w, N, S, part, out, mode);
    case 5: return launch_mw<2, 4, 3, true>(mtw, grid, st, x, M, K, w, N, S, part, out, mode);
    default: return launch_mw<2, 8, 2, true>(mtw, grid, st, x, M, K, w, N, S, part, out, mode);
  }
}

}  // namespace xgk
