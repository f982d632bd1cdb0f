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

// PR (anatomy probes, bench/gemm_bench.py --mw-probe; results are garbage unless the
// low bits are 0): PR & 7: 0 = the kernel; 1 = DMA + waits + barriers only (no
// fragment reads / MFMA); 2 = fragment reads + MFMA + barriers only (no DMA); 3 = no x
// DMA (weights only); 4 = no weight DMA; 5 = x DMA only; 6 = weight DMA only.
// PR & 8: every workgroup walks its K chunks from a tile-dependent start (rotated), so
// the workgroups of an XCD read different x lines at any moment (results exact).
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

// Split-role rings (cfg >= 7). The single-ring kernel above issues x and W from every
// wave, so vmcnt's in-order retirement ties x's lead to the weights' and the x
// slots eat the LDS that deeper weight rings need -- at M = 192 it keeps ~56 KB in
// flight per CU, and measured per-CU ingest (~42 GB/s) is exactly that over a
// ~1.3 us loaded latency (profiles/r4_mw_sweep.md). vmcnt is PER WAVE: here waves
// 0-3 issue only weight DMAs (DW-slot ring, DW-1 chunks ahead) and waves 4-7 only x
// DMAs (DX slots, DX-1 ahead, L2-resident), so each role's counted wait sees its own
// stream only, and the weight ring gets the LDS: e.g. 128 columns x DW = 6 keeps 80
// KB of weights in flight. Every wave still computes its (wn, wm) tile.
// Input RMSNorm as an epilogue row scale (the fused decode layer's contract, see
// gemm_m64g.hip M64Epi): x is the raw bf16 residual stream, the norm weight is folded
// into W, and output row m is scaled by rsqrt(sum_j ss_in[j * ss_stride + m] / K + eps)
// (ss_n partial sums of squares, added in order). ss_in == nullptr: no scale.
struct MwEpi {
  const float* ss_in;
  int ss_n;
  int ss_stride;
  float eps;
};

template <int WN, int NWT, int MTW, int DW, int DX, bool NT>
__global__ void __launch_bounds__(512, 1) gemm_mw2_kernel(const uint16_t* __restrict__ x, int M, int K,
                                                           const uint16_t* __restrict__ w, int N, int S,
                                                           float* __restrict__ part, uint16_t* __restrict__ out,
                                                           int mode, MwEpi epi, int krot) {
  constexpr int WM = 8 / WN;
  constexpr int KC = 64, RB = 128, RPI = 8;
  constexpr int WCOLS = WN * 16 * NWT;
  constexpr int XROWS = WM * 16 * MTW;
  constexpr int WSLOT = WCOLS * RB;
  constexpr int XSLOT = XROWS * RB;
  constexpr int WI = WCOLS / RPI / 4;           // weight DMA instructions per W-wave per chunk
  constexpr int XI = XROWS / RPI / 4;           // x DMA instructions per x-wave per chunk
  static_assert(WN * WM == 8 && WI >= 1 && XI >= 1 && WCOLS % 32 == 0 && XROWS % 32 == 0, "bad gemm_mw2 geometry");
  static_assert(DW >= 2 && DW <= 9 && DX >= 2 && DX <= 4, "ring depths");
  static_assert(DW * WSLOT + DX * XSLOT <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) uint8_t smem[DW * WSLOT + DX * XSLOT];
  uint8_t* const wring = smem;
  uint8_t* const xring = smem + DW * WSLOT;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int wn = wid % WN, wm = wid / WN;
  const bool wload = wid < 4;                   // DMA role: weights (waves 0-3) or x (4-7)
  const int rw = wid & 3;                       // index within the role

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

  const int dr = lane >> 3, dj = lane & 7;
  constexpr int NI = WI > XI ? WI : XI;
  const uint16_t* src[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    if (wload) {
      const int row = 8 * (rw * WI + (i < WI ? i : 0)) + dr;
      src[i] = w + static_cast<int64_t>(n0 + row) * K + k0 + 8 * (dj ^ dr);
    } else {
      const int row = 8 * (rw * XI + (i < XI ? i : 0)) + dr;
      src[i] = x + static_cast<int64_t>(min(row, M - 1)) * K + k0 + 8 * (dj ^ dr);
    }
  }
  const int rot = krot ? (tile * 37) % nch : 0;  // K-chunk rotation (gemm_m64g.hip k_rotation)
  auto kof = [&](int c) {
    const int cc = c + rot;
    return (cc >= nch ? cc - nch : cc) * KC;
  };
  auto issue_w = [&](int c) {
    uint8_t* slot = wring + (c % DW) * WSLOT;
    const int kk = kof(c);
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      if constexpr (NT) glds16_nt(src[i] + kk, slot + (rw * WI + i) * 1024);
      else glds16(src[i] + kk, slot + (rw * WI + i) * 1024);
    }
  };
  auto issue_x = [&](int c) {
    uint8_t* slot = xring + (c % DX) * XSLOT;
    const int kk = kof(c);
#pragma unroll
    for (int i = 0; i < XI; ++i) glds16(src[i] + kk, slot + (rw * XI + i) * 1024);
  };

  f32x4_t acc[NWT][MTW];
#pragma unroll
  for (int nt = 0; nt < NWT; ++nt)
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) acc[nt][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int wrow0 = wn * 16 * NWT, xrow0 = wm * 16 * MTW;
  auto compute = [&](int c) {
    const uint8_t* ws = wring + (c % DW) * WSLOT;
    const uint8_t* xs = xring + (c % DX) * XSLOT;
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

  // each role leaves the chunks after c that it already issued in flight:
  // rem = min(nch - 1 - c, ring depth - 2) groups of its own instructions
  auto wait_role = [&](int c) {
    if (wload) {
      const int rem = min(nch - 1 - c, DW - 2);
      if constexpr (DW >= 9) { if (rem == 7) { wait_vmcnt<7 * WI>(); return; } }
      if constexpr (DW >= 8) { if (rem == 6) { wait_vmcnt<6 * WI>(); return; } }
      if constexpr (DW >= 7) { if (rem == 5) { wait_vmcnt<5 * WI>(); return; } }
      if constexpr (DW >= 6) { if (rem == 4) { wait_vmcnt<4 * WI>(); return; } }
      if constexpr (DW >= 5) { if (rem == 3) { wait_vmcnt<3 * WI>(); return; } }
      if constexpr (DW >= 4) { if (rem == 2) { wait_vmcnt<2 * WI>(); return; } }
      if constexpr (DW >= 3) { if (rem == 1) { wait_vmcnt<WI>(); return; } }
      wait_vmcnt<0>();
    } else {
      const int rem = min(nch - 1 - c, DX - 2);
      if constexpr (DX >= 4) { if (rem == 2) { wait_vmcnt<2 * XI>(); return; } }
      if constexpr (DX >= 3) { if (rem == 1) { wait_vmcnt<XI>(); return; } }
      wait_vmcnt<0>();
    }
  };

  // norm statistics of this lane's rows: lane group g sums j = g, g + 4, ... (loaded
  // before the weight stream starts; older than every DMA, so the counted waits hold)
  constexpr int SQ = 4;  // up to 4 * SQ = 16 partial sums per row
  const bool has_ss = epi.ss_in != nullptr;
  float ssv[MTW][SQ];
  if (has_ss) {
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
      for (int q = 0; q < SQ; ++q)
        ssv[mt][q] = epi.ss_in[min(g + 4 * q, epi.ss_n - 1) * epi.ss_stride + min(xrow0 + 16 * mt + li, M - 1)];
  }
  if (wload) {
#pragma unroll
    for (int j = 0; j < DW - 1; ++j)
      if (j < nch) issue_w(j);
  } else {
#pragma unroll
    for (int j = 0; j < DX - 1; ++j)
      if (j < nch) issue_x(j);
  }
  for (int c = 0; c < nch; ++c) {
    wait_role(c);
    raw_barrier();
    // refill the slots chunk c - 1 used (every wave is past the barrier)
    if (wload) {
      if (c + DW - 1 < nch) issue_w(c + DW - 1);
    } else {
      if (c + DX - 1 < nch) issue_x(c + DX - 1);
    }
    compute(c);
  }

  if (has_ss) {  // input RMSNorm as a row scale of the (linear) output
    const float inv_k = 1.f / static_cast<float>(K);
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < SQ; ++q) v += g + 4 * q < epi.ss_n ? ssv[mt][q] : 0.f;
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const float sc = rsqrtf(v * inv_k + epi.eps);
#pragma unroll
      for (int nt = 0; nt < NWT; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[nt][mt][r] *= sc;
    }
  }

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

// Software-pipelined variant (cfg >= 15). The anatomy probes (profiles/r4_mw_probe.md)
// show the compute side alone at ~2x the MFMA issue time at M >= 192: each chunk ran
// barrier -> fragment reads -> MFMAs, so every chunk exposed the LDS latency and the
// 8-wave read burst. Here one ring of R slots holds a whole chunk (W tile + x tile),
// every wave DMAs its share of both, and the fragments of chunk c + 1 are read into a
// second register set while chunk c's MFMAs run:
//   per chunk c:  lgkmcnt(0) (this wave's reads of chunk c are in registers)
//                 counted vmcnt (this wave's DMAs of chunk c + 1 landed)
//                 s_barrier     (all waves: chunk c + 1 in LDS, slot c % R no longer read)
//                 DMA chunk c + R into slot c % R
//                 ds_read chunk c + 1 -> the other register set
//                 MFMAs of chunk c
// so R - 1 chunks stay in flight and the reads hide under the MFMAs. Epilogues as
// gemm_mw2 (partials / bf16 / SiLU-gate, optional input-RMSNorm row scale).
template <int WN, int NWT, int MTW, int R, bool NT>
__global__ void __launch_bounds__(512, 1) gemm_mw3_kernel(const uint16_t* __restrict__ x, int M, int K,
                                                           const uint16_t* __restrict__ w, int N, int S,
                                                           float* __restrict__ part, uint16_t* __restrict__ out,
                                                           int mode, MwEpi epi, int krot) {
  constexpr int WM = 8 / WN;
  constexpr int KC = 64, RB = 128, RPI = 8, KT = KC / 32;
  constexpr int WCOLS = WN * 16 * NWT;
  constexpr int XROWS = WM * 16 * MTW;
  constexpr int WSLOT = WCOLS * RB;
  constexpr int SLOT = WSLOT + XROWS * RB;
  constexpr int WI = WCOLS / RPI / 8;           // weight DMA instructions per wave per chunk
  constexpr int XI = XROWS / RPI / 8;           // x DMA instructions per wave per chunk
  constexpr int G = WI + XI;
  static_assert(WN * WM == 8 && WI >= 1 && XI >= 1 && WCOLS % 64 == 0 && XROWS % 64 == 0, "bad gemm_mw3 geometry");
  static_assert(R >= 2 && R <= 5 && R * SLOT <= 160 * 1024, "ring");
  __shared__ __attribute__((aligned(1024))) uint8_t smem[R * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int wn = wid % WN, wm = wid / WN;

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

  const int dr = lane >> 3, dj = lane & 7;
  const uint16_t* wsrc[WI];
#pragma unroll
  for (int i = 0; i < WI; ++i)
    wsrc[i] = w + static_cast<int64_t>(n0 + 8 * (wid * WI + i) + dr) * K + k0 + 8 * (dj ^ dr);
  const uint16_t* xsrc[XI];
#pragma unroll
  for (int i = 0; i < XI; ++i)
    xsrc[i] = x + static_cast<int64_t>(min(8 * (wid * XI + i) + dr, M - 1)) * K + k0 + 8 * (dj ^ dr);
  const int rot = krot ? (tile * 37) % nch : 0;  // K-chunk rotation (gemm_m64g.hip k_rotation)

  auto issue = [&](int c) {
    uint8_t* base = smem + (c % R) * SLOT;
    const int cc = c + rot;
    const int kk = (cc >= nch ? cc - nch : cc) * KC;
#pragma unroll
    for (int i = 0; i < XI; ++i) glds16(xsrc[i] + kk, base + WSLOT + (wid * XI + i) * 1024);
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      if constexpr (NT) glds16_nt(wsrc[i] + kk, base + (wid * WI + i) * 1024);
      else glds16(wsrc[i] + kk, base + (wid * WI + i) * 1024);
    }
  };

  f32x4_t acc[NWT][MTW];
#pragma unroll
  for (int nt = 0; nt < NWT; ++nt)
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) acc[nt][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int wrow0 = wn * 16 * NWT, xrow0 = wm * 16 * MTW;
  auto read = [&](int c, uint4 (&a)[KT][NWT], uint4 (&b)[KT][MTW]) {
    const uint8_t* ws = smem + (c % R) * SLOT;
    const uint8_t* xs = ws + WSLOT;
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const int phys = (4 * t + g) ^ (li & 7);
#pragma unroll
      for (int nt = 0; nt < NWT; ++nt)
        a[t][nt] = *reinterpret_cast<const uint4*>(ws + (wrow0 + 16 * nt + li) * RB + phys * 16);
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt)
        b[t][mt] = *reinterpret_cast<const uint4*>(xs + (xrow0 + 16 * mt + li) * RB + phys * 16);
    }
  };
  auto mma = [&](const uint4 (&a)[KT][NWT], const uint4 (&b)[KT][MTW]) {
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int nt = 0; nt < NWT; ++nt)
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt) acc[nt][mt] = mfma16x16x32(as_frag(a[t][nt]), as_frag(b[t][mt]), acc[nt][mt]);
  };
  // this wave's DMAs of chunk c landed, `after` = groups issued after chunk c (<= R - 1)
  auto wait_after = [&](int after) {
    if constexpr (R >= 5) { if (after >= 4) { wait_vmcnt<4 * G>(); return; } }
    if constexpr (R >= 4) { if (after == 3) { wait_vmcnt<3 * G>(); return; } }
    if constexpr (R >= 3) { if (after == 2) { wait_vmcnt<2 * G>(); return; } }
    if (after == 1) { wait_vmcnt<G>(); return; }
    wait_vmcnt<0>();
  };

  constexpr int SQ = 4;
  const bool has_ss = epi.ss_in != nullptr;
  float ssv[MTW][SQ];
  if (has_ss) {
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
      for (int q = 0; q < SQ; ++q)
        ssv[mt][q] = epi.ss_in[min(g + 4 * q, epi.ss_n - 1) * epi.ss_stride + min(xrow0 + 16 * mt + li, M - 1)];
  }

  // prologue: chunks 0 .. R-1; chunk 0 landed everywhere; its fragments -> set A
#pragma unroll
  for (int j = 0; j < R; ++j)
    if (j < nch) issue(j);
  wait_after(min(R - 1, nch - 1));
  raw_barrier();
  uint4 fa[KT][NWT], fb[KT][MTW], ga[KT][NWT], gb[KT][MTW];
  read(0, fa, fb);
  // one chunk: a / b hold chunk c (reads in flight), a2 / b2 receive chunk c + 1
  auto step = [&](int c, uint4 (&a)[KT][NWT], uint4 (&b)[KT][MTW], uint4 (&a2)[KT][NWT], uint4 (&b2)[KT][MTW]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (c + 1 < nch) wait_after(min(R - 2, nch - 2 - c));
    raw_barrier();
    if (c + R < nch) issue(c + R);
    if (c + 1 < nch) read(c + 1, a2, b2);
    mma(a, b);
  };
  int c = 0;
  for (; c + 1 < nch; c += 2) {
    step(c, fa, fb, ga, gb);
    step(c + 1, ga, gb, fa, fb);
  }
  if (c < nch) step(c, fa, fb, ga, gb);

  if (has_ss) {  // input RMSNorm as a row scale of the (linear) output
    const float inv_k = 1.f / static_cast<float>(K);
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
      float vs = 0.f;
#pragma unroll
      for (int q = 0; q < SQ; ++q) vs += g + 4 * q < epi.ss_n ? ssv[mt][q] : 0.f;
      vs += __shfl_xor(vs, 16, 64);
      vs += __shfl_xor(vs, 32, 64);
      const float sc = rsqrtf(vs * inv_k + epi.eps);
#pragma unroll
      for (int nt = 0; nt < NWT; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[nt][mt][r] *= sc;
    }
  }

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

template <int WN, int NWT, int MTW, int DW, int DX>
constexpr bool mw2_fits() {
  constexpr int WM = 8 / WN;
  return DW * (WN * 16 * NWT * 128) + DX * (WM * 16 * MTW * 128) <= 160 * 1024;
}

template <int WN, int NWT, int DW, int DX>
static int launch_mw2(int mtw, dim3 grid, hipStream_t st, const uint16_t* x, int M, int K, const uint16_t* w, int N,
                      int S, float* part, uint16_t* out, int mode, const MwEpi& epi) {
#define XGK_MW2(MTW)                                                                                              \
  case MTW:                                                                                                       \
    if constexpr (mw2_fits<WN, NWT, MTW, DW, DX>()) {                                                             \
      hipLaunchKernelGGL((gemm_mw2_kernel<WN, NWT, MTW, DW, DX, true>), grid, dim3(512), 0, st, x, M, K, w, N, S, \
                         part, out, mode, epi, k_rotation(S));                                                    \
      return 0;                                                                                                   \
    }                                                                                                             \
    return 1;
  switch (mtw) {
    XGK_MW2(1)
    XGK_MW2(2)
    XGK_MW2(3)
    XGK_MW2(4)
    XGK_MW2(5)
    XGK_MW2(6)
    XGK_MW2(7)
    XGK_MW2(8)
    XGK_MW2(9)
    XGK_MW2(10)
    default: return 1;
  }
#undef XGK_MW2
}

// split-role configurations: (WN, NWT, DW, DX)
struct Mw2Cfg { int wn, nwt, dw, dx; };
static constexpr Mw2Cfg kMw2[] = {
    {4, 2, 6, 2},   // 7: 128 columns, 5 weight chunks ahead
    {2, 4, 6, 2},   // 8: same, 2 x 4 waves
    {4, 2, 5, 3},   // 9: 128 columns, 4 ahead, x 2 ahead
    {4, 4, 3, 2},   // 10: 256 columns, 2 ahead
    {2, 8, 3, 2},   // 11: same, 2 x 4 waves
    {4, 2, 8, 2},   // 12: 128 columns, 7 ahead (M <= 128)
    {2, 4, 8, 2},   // 13: same, 2 x 4 waves
    {4, 4, 4, 2},   // 14: 256 columns, 3 ahead (M <= 128)
};
template <int WN, int NWT, int MTW, int R>
constexpr bool mw3_fits() {
  constexpr int WM = 8 / WN;
  // two fragment sets + the accumulators in 256 VGPRs: at most 8 (NWT + MTW) x 2 KT
  // fragment registers beside 4 NWT MTW accumulators (4 x 8 / 2 x 4 waves: MTW <= 6 / 4)
  return (WM * 16 * MTW) % 64 == 0 && R * (WN * 16 * NWT * 128 + WM * 16 * MTW * 128) <= 160 * 1024 &&
         16 * (NWT + MTW) + 4 * NWT * MTW <= 200;
}

template <int WN, int NWT, int R>
static int launch_mw3(int M, dim3 grid, hipStream_t st, const uint16_t* x, int K, const uint16_t* w, int N, int S,
                      float* part, uint16_t* out, int mode, const MwEpi& epi) {
  constexpr int RPW = (8 / WN) * 16;   // x rows per MTW step
  constexpr int STEP = 64 / RPW > 0 ? 64 / RPW : 1;  // MTW granularity so x rows stay a multiple of 64
  const int mtw = ((M + RPW - 1) / RPW + STEP - 1) / STEP * STEP;
#define XGK_MW3(MTW)                                                                                            \
  case MTW:                                                                                                     \
    if constexpr (mw3_fits<WN, NWT, MTW, R>()) {                                                                \
      hipLaunchKernelGGL((gemm_mw3_kernel<WN, NWT, MTW, R, true>), grid, dim3(512), 0, st, x, M, K, w, N, S,    \
                         part, out, mode, epi, k_rotation(S));                                                  \
      return 0;                                                                                                 \
    }                                                                                                           \
    return 1;
  switch (mtw) {
    XGK_MW3(1)
    XGK_MW3(2)
    XGK_MW3(3)
    XGK_MW3(4)
    XGK_MW3(5)
    XGK_MW3(6)
    XGK_MW3(8)
    XGK_MW3(10)
    default: return 1;
  }
#undef XGK_MW3
}

// software-pipelined configurations (cfg 15 + i): (WN, NWT, R)
static constexpr Mw2Cfg kMw3[] = {
    {4, 2, 4, 0},   // 15: 128 columns, 4-slot ring (M <= 192)
    {4, 2, 3, 0},   // 16: 128 columns, 3 slots (M <= 256)
    {2, 4, 4, 0},   // 17: 2 x 4 waves, 128 columns, 4 slots (M <= 192)
    {2, 4, 3, 0},   // 18: 2 x 4 waves, 3 slots (M <= 256)
    {4, 2, 5, 0},   // 19: 128 columns, 5 slots (M <= 128)
    {4, 4, 3, 0},   // 20: 256 columns, 3 slots (M <= 128)
    {2, 4, 5, 0},   // 21: 2 x 4 waves, 128 columns, 5 slots (M <= 128)
};
constexpr int kMw2Cfgs = 7 + static_cast<int>(sizeof(kMw2) / sizeof(kMw2[0]));
constexpr int kMwCfgs = kMw2Cfgs + static_cast<int>(sizeof(kMw3) / sizeof(kMw3[0]));

int mw_cfg_cols_any(int cfg) {
  if (cfg < 7) return mw_cfg_cols(cfg);
  if (cfg >= kMw2Cfgs) return kMw3[cfg - kMw2Cfgs].wn * 16 * kMw3[cfg - kMw2Cfgs].nwt;
  return kMw2[cfg - 7].wn * 16 * kMw2[cfg - 7].nwt;
}

// x [M, K] bf16 row-major, w [N, K] bf16 row-major. mode MW_PARTIAL: part [S, M, N]
// fp32; MW_BF16: out [M, N]; MW_SILU: out [M, N / 2] (S = 1). 0 = launched, 1 = a
// shape / configuration this kernel does not take (M beyond the cfg's LDS budget).
static int gemm_mw_impl(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, uint16_t* out, int S,
                        int mode, int cfg, const MwEpi& epi, hipStream_t st) {
  if (M < 1 || M > 320 || cfg < 0 || cfg >= kMwCfgs || S < 1 || K % 64 || S > K / 64) return 1;
  if (epi.ss_in != nullptr && (cfg < 7 || epi.ss_n < 1 || epi.ss_n > 16 || epi.ss_stride < M)) return 1;
  const int cols = mw_cfg_cols_any(cfg);
  if (N % cols) return 1;
  if (mode == MW_PARTIAL) {
    if (part == nullptr) return 1;
  } else if (mode == MW_BF16 || mode == MW_SILU) {
    if (out == nullptr || S != 1) return 1;
  } else {
    return 1;
  }
  const dim3 grid((N / cols) * S);
  if (cfg >= kMw2Cfgs) {
    switch (cfg - kMw2Cfgs) {
      case 0: return launch_mw3<4, 2, 4>(M, grid, st, x, K, w, N, S, part, out, mode, epi);
      case 1: return launch_mw3<4, 2, 3>(M, grid, st, x, K, w, N, S, part, out, mode, epi);
      case 2: return launch_mw3<2, 4, 4>(M, grid, st, x, K, w, N, S, part, out, mode, epi);
      case 3: return launch_mw3<2, 4, 3>(M, grid, st, x, K, w, N, S, part, out, mode, epi);
      case 4: return launch_mw3<4, 2, 5>(M, grid, st, x, K, w, N, S, part, out, mode, epi);
      case 5: return launch_mw3<4, 4, 3>(M, grid, st, x, K, w, N, S, part, out, mode, epi);
      default: return launch_mw3<2, 4, 5>(M, grid, st, x, K, w, N, S, part, out, mode, epi);
    }
  }
  if (cfg >= 7) {
    const Mw2Cfg c = kMw2[cfg - 7];
    const int rows_per = (8 / c.wn) * 16;
    const int mtw = (M + rows_per - 1) / rows_per;
    switch (cfg) {
      case 7: return launch_mw2<4, 2, 6, 2>(mtw, grid, st, x, M, K, w, N, S, part, out, mode, epi);
      case 8: return launch_mw2<2, 4, 6, 2>(mtw, grid, st, x, M, K, w, N, S, part, out, mode, epi);
      case 9: return launch_mw2<4, 2, 5, 3>(mtw, grid, st, x, M, K, w, N, S, part, out, mode, epi);
      case 10: return launch_mw2<4, 4, 3, 2>(mtw, grid, st, x, M, K, w, N, S, part, out, mode, epi);
      case 11: return launch_mw2<2, 8, 3, 2>(mtw, grid, st, x, M, K, w, N, S, part, out, mode, epi);
      case 12: return launch_mw2<4, 2, 8, 2>(mtw, grid, st, x, M, K, w, N, S, part, out, mode, epi);
      case 13: return launch_mw2<2, 4, 8, 2>(mtw, grid, st, x, M, K, w, N, S, part, out, mode, epi);
      default: return launch_mw2<4, 4, 4, 2>(mtw, grid, st, x, M, K, w, N, S, part, out, mode, epi);
    }
  }
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

// Anatomy probes of the two best mid-M configurations (cfg 1: 4 x 2 waves, cfg 5: 2 x 4
// waves; 128 columns, ring 3, nt weights) at 64-row steps of M (PR as above).
template <int PR>
static int launch_mw_probe(int cfg, int M, dim3 grid, hipStream_t st, const uint16_t* x, int K, const uint16_t* w,
                           int N, int S, float* part, uint16_t* out, int mode) {
#define XGK_MWP(WN, NWT, MTW)                                                                                   \
  hipLaunchKernelGGL((gemm_mw_kernel<WN, NWT, MTW, 3, true, PR>), grid, dim3(512), 0, st, x, M, K, w, N, S, \
                     part, out, mode, 0);                                                                       \
  return 0;
  const int q = (M + 63) / 64;
  if (cfg == 1) {
    if (q == 1) { XGK_MWP(4, 2, 2) }
    if (q == 2) { XGK_MWP(4, 2, 4) }
    if (q == 3) { XGK_MWP(4, 2, 6) }
    if (q == 4) { XGK_MWP(4, 2, 8) }
  } else if (cfg == 5) {
    if (q == 1) { XGK_MWP(2, 4, 1) }
    if (q == 2) { XGK_MWP(2, 4, 2) }
    if (q == 3) { XGK_MWP(2, 4, 3) }
    if (q == 4) { XGK_MWP(2, 4, 4) }
  }
#undef XGK_MWP
  return 1;
}

int gemm_mw_probe(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, uint16_t* out, int S,
                  int mode, int cfg, int probe, hipStream_t st) {
  if (M < 1 || M > 256 || S < 1 || K % 64 || S > K / 64 || N % 128 || (cfg != 1 && cfg != 5)) return 1;
  if (mode == MW_PARTIAL ? part == nullptr : (out == nullptr || S != 1)) return 1;
  const dim3 grid((N / 128) * S);
  switch (probe) {
#define XGK_MWPC(P) \
  case P: return launch_mw_probe<P>(cfg, M, grid, st, x, K, w, N, S, part, out, mode);
    XGK_MWPC(0) XGK_MWPC(1) XGK_MWPC(2) XGK_MWPC(3) XGK_MWPC(4) XGK_MWPC(5) XGK_MWPC(6)
    XGK_MWPC(8) XGK_MWPC(9) XGK_MWPC(13)
#undef XGK_MWPC
    default: return 1;
  }
}

int gemm_mw(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, uint16_t* out, int S, int mode,
            int cfg, hipStream_t st) {
  return gemm_mw_impl(x, M, K, w, N, part, out, S, mode, cfg, MwEpi{nullptr, 0, 0, 0.f}, st);
}

// with the input RMSNorm as a row scale (split-role configurations only; ss_n <= 16)
int gemm_mw_ss(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, uint16_t* out, int S, int mode,
               int cfg, const float* ss_in, int ss_n, int ss_stride, float eps, hipStream_t st) {
  return gemm_mw_impl(x, M, K, w, N, part, out, S, mode, cfg, MwEpi{ss_in, ss_n, ss_stride, eps}, st);
}

}  // namespace xgk
