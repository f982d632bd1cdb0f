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
#include "common.h"

namespace xgk {

constexpr int GG_KC = 128;              // k per chunk (one slot)
constexpr int GG_SLOTS = 3;
constexpr int GG_XBYTES = 64 * 256;     // x rows x bytes per chunk

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

// The DMA is issued from inline asm so that hipcc's waitcnt pass does not see it:
// with the builtin it serialises the DMAs of different slots (vmcnt(0) between
// them and before every fragment read). Completion is then tracked ONLY by the
// explicit counted waits below; "memory" keeps the compiler from moving LDS
// reads across them.
__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)(lds_base))));
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :
      : "v"(src), "s"(lds)
      : "memory", "m0");
#endif
}

__device__ __forceinline__ void glds16_nt(const void* src, void* lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)(lds_base))));
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off nt"
      :
      : "v"(src), "s"(lds)
      : "memory", "m0");
#endif
}

// s_waitcnt vmcnt(N) (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14; expcnt, lgkmcnt left at max)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#endif
}

__device__ __forceinline__ void raw_barrier() {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_barrier" ::: "memory");
#endif
}

enum : int { GG_BF16 = 0, GG_PARTIAL = 1, GG_SILU = 2 };

// Dense kernel, parametrised for the decode shapes (bench/gemm_bench.py picks):
//   NW  16-column MFMA tiles per wave (2 = 32 columns; required by the SiLU epilogue)
//   WV  waves per workgroup (4 or 2): fewer waves = more, smaller workgroups, so a
//       short N still puts a workgroup on every CU
//   KC  k per chunk (128: 256-B rows, 1 workgroup/CU; 64: 128-B rows, 2-3 per CU)
//   NT  non-temporal weight DMA (streamed once; keeps x resident in L2)
template <int NW, int WV, int KC, bool NT>
__global__ void __launch_bounds__(64 * WV, 1) gemm_m64g_kernel(const uint16_t* __restrict__ x, int M, int K,
                                                               const uint16_t* __restrict__ w, int N,
                                                               float* __restrict__ part, uint16_t* __restrict__ out,
                                                               int mode) {
  constexpr int MT = 4;
  constexpr int RB = KC * 2;                     // bytes per LDS row
  constexpr int GPR = KC / 8;                    // 16-B granules per row
  constexpr int RPI = 1024 / RB;                 // rows per DMA instruction (64 lanes x 16 B)
  constexpr int XBYTES = 64 * RB;
  constexpr int XI = 64 / RPI / WV;              // x DMA instructions per wave per chunk
  constexpr int WROWS = 16 * NW;                 // weight rows per wave
  constexpr int WI = WROWS / RPI;                // weight DMA instructions per wave per chunk
  constexpr int WBYTES = WROWS * RB;             // per wave per slot
  constexpr int SLOT = XBYTES + WV * WBYTES;
  constexpr int G = XI + WI;
  static_assert(XI >= 1 && WI >= 1 && 64 % (RPI * WV) == 0, "bad m64g geometry");
  __shared__ __attribute__((aligned(1024))) uint8_t lds0[SLOT];
  __shared__ __attribute__((aligned(1024))) uint8_t lds1[SLOT];
  __shared__ __attribute__((aligned(1024))) uint8_t lds2[SLOT];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int S = gridDim.y, s = blockIdx.y;
  const int kws = K / S;
  const int k0 = s * kws;
  const int nchunks = kws / KC;
  const int nbase = blockIdx.x * (16 * NW * WV) + wid * WROWS;

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
    const int r = RPI * (wid * XI + i) + dr;     // x row 0..63
    xsrc[i] = x + static_cast<int64_t>(min(r, M - 1)) * K + k0 + 8 * (dj ^ (r & (GPR - 1)));
  }

  auto issue = [&](uint8_t* slot, int c) {
    const int kk = c * KC;
#pragma unroll
    for (int i = 0; i < XI; ++i) glds16(xsrc[i] + kk, slot + RPI * (wid * XI + i) * RB);
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      if constexpr (NT) glds16_nt(wsrc[i] + kk, slot + XBYTES + wid * WBYTES + i * 1024);
      else glds16(wsrc[i] + kk, slot + XBYTES + wid * WBYTES + i * 1024);
    }
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

  // acc[nt][mt][r] = out[m = 16 mt + li][n = nbase + 16 nt + 4 g + r]
  if (mode == GG_PARTIAL) {
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

// Grouped (MoE) form of the same pipeline: W [E, N, K]; x rows gathered through
// the block-64 padded expert-sorted layout (rows[p] = source row, -1 = pad;
// rows == nullptr: x already in padded layout); offs[E+1] padded segment starts.
// One workgroup per (column tile, k-split, expert) loops over the expert's
// 64-row tiles (the same weight column tile is re-read from L2/MALL, not HBM).
template <int NW, int WV, int KC, bool NT>
__global__ void __launch_bounds__(64 * WV, 1) gemm_m64g_grouped_kernel(const uint16_t* __restrict__ x,
                                                                       const int32_t* __restrict__ rows,
                                                                       const int32_t* __restrict__ offs, int K,
                                                                       const uint16_t* __restrict__ w, int N, int P,
                                                                       float* __restrict__ part,
                                                                       uint16_t* __restrict__ out, int mode) {
  constexpr int MT = 4;
  constexpr int RB = KC * 2;
  constexpr int GPR = KC / 8;
  constexpr int RPI = 1024 / RB;
  constexpr int XBYTES = 64 * RB;
  constexpr int XI = 64 / RPI / WV;
  constexpr int WROWS = 16 * NW;
  constexpr int WI = WROWS / RPI;
  constexpr int WBYTES = WROWS * RB;
  constexpr int SLOT = XBYTES + WV * WBYTES;
  constexpr int G = XI + WI;
  static_assert(XI >= 1 && WI >= 1 && 64 % (RPI * WV) == 0, "bad m64g geometry");
  __shared__ __attribute__((aligned(1024))) uint8_t lds0[SLOT];
  __shared__ __attribute__((aligned(1024))) uint8_t lds1[SLOT];
  __shared__ __attribute__((aligned(1024))) uint8_t lds2[SLOT];

  const int e = blockIdx.z;
  const int p0 = offs[e], p1 = offs[e + 1];
  if (p1 <= p0) return;
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

  for (int rt = p0; rt < p1; rt += 64) {
    if (rt != p0) raw_barrier();  // the previous tile's last slot may still be read
    const int first = rows ? rows[rt] : rt;
    const uint16_t* xsrc[XI];
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int r = RPI * (wid * XI + i) + dr;
      int src = rows ? rows[rt + r] : rt + r;
      if (src < 0) src = first;
      xsrc[i] = x + static_cast<int64_t>(src) * K + k0 + 8 * (dj ^ (r & (GPR - 1)));
    }
    auto issue = [&](uint8_t* slot, int c) {
      const int kk = c * KC;
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

    if (mode == GG_PARTIAL) {
      float* pp = part + static_cast<int64_t>(s) * P * N;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = rt + 16 * mt + li;
#pragma unroll
        for (int nt_ = 0; nt_ < NW; ++nt_)
          *reinterpret_cast<float4*>(pp + static_cast<int64_t>(m) * N + nbase + 16 * nt_ + 4 * g) =
              make_float4(acc[nt_][mt][0], acc[nt_][mt][1], acc[nt_][mt][2], acc[nt_][mt][3]);
      }
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

template <int NW>
static void launch_m64g_grouped(int cfg, dim3 grid, hipStream_t st, const uint16_t* x, const int32_t* rows,
                                const int32_t* offs, int K, const uint16_t* w, int N, int P, float* part,
                                uint16_t* out, int mode) {
#define XGK_GRP(WV, KC, NT)                                                                                    \
  hipLaunchKernelGGL((gemm_m64g_grouped_kernel<NW, WV, KC, NT>), grid, dim3(64 * WV), 0, st, x, rows, offs, K, w, \
                     N, P, part, out, mode)
  switch (cfg) {
    case 1: XGK_GRP(4, 128, true); break;
    case 2: XGK_GRP(4, 64, false); break;
    case 3: XGK_GRP(4, 64, true); break;
    case 4: XGK_GRP(2, 64, false); break;
    case 5: XGK_GRP(2, 64, true); break;
    case 6: XGK_GRP(2, 128, true); break;
    default: XGK_GRP(4, 128, false); break;
  }
#undef XGK_GRP
}

int m64g_cfg_waves(int cfg);
int m64g_cfg_kc(int cfg);

int moe_gemm_m64g(const uint16_t* x, const int32_t* rows, const int32_t* offs, int E, int K, const uint16_t* w, int N,
                  int P, float* part, uint16_t* out, int S, int mode, int nw, int cfg, hipStream_t st) {
  if (E < 1 || P < 0 || P % 64 || S < 1 || (nw != 1 && nw != 2) || cfg < 0 || cfg > 6) return 1;
  const int cols = 16 * nw * m64g_cfg_waves(cfg), kc = m64g_cfg_kc(cfg);
  if (K % (S * kc) || N % cols) return 1;
  if (mode == GG_SILU && (nw != 2 || S != 1)) return 1;
  if (mode == GG_PARTIAL && part == nullptr) return 1;
  if (mode != GG_PARTIAL && out == nullptr) return 1;
  if (P == 0) return 0;
  const dim3 grid(N / cols, S, E);
  if (nw == 1) launch_m64g_grouped<1>(cfg, grid, st, x, rows, offs, K, w, N, P, part, out, mode);
  else launch_m64g_grouped<2>(cfg, grid, st, x, rows, offs, K, w, N, P, part, out, mode);
  return 0;
}

// cfg: 0 = (4 waves, KC 128), 1 = (4, 128, nt), 2 = (4, 64), 3 = (4, 64, nt),
//      4 = (2, 64), 5 = (2, 64, nt), 6 = (2, 128, nt)
template <int NW>
static void launch_m64g(int cfg, dim3 grid, hipStream_t st, const uint16_t* x, int M, int K, const uint16_t* w, int N,
                        float* part, uint16_t* out, int mode) {
  switch (cfg) {
    case 1: hipLaunchKernelGGL((gemm_m64g_kernel<NW, 4, 128, true>), grid, dim3(256), 0, st, x, M, K, w, N, part, out, mode); break;
    case 2: hipLaunchKernelGGL((gemm_m64g_kernel<NW, 4, 64, false>), grid, dim3(256), 0, st, x, M, K, w, N, part, out, mode); break;
    case 3: hipLaunchKernelGGL((gemm_m64g_kernel<NW, 4, 64, true>), grid, dim3(256), 0, st, x, M, K, w, N, part, out, mode); break;
    case 4: hipLaunchKernelGGL((gemm_m64g_kernel<NW, 2, 64, false>), grid, dim3(128), 0, st, x, M, K, w, N, part, out, mode); break;
    case 5: hipLaunchKernelGGL((gemm_m64g_kernel<NW, 2, 64, true>), grid, dim3(128), 0, st, x, M, K, w, N, part, out, mode); break;
    case 6: hipLaunchKernelGGL((gemm_m64g_kernel<NW, 2, 128, true>), grid, dim3(128), 0, st, x, M, K, w, N, part, out, mode); break;
    default: hipLaunchKernelGGL((gemm_m64g_kernel<NW, 4, 128, false>), grid, dim3(256), 0, st, x, M, K, w, N, part, out, mode); break;
  }
}

int m64g_cfg_waves(int cfg) { return cfg >= 4 ? 2 : 4; }
int m64g_cfg_kc(int cfg) { return (cfg == 2 || cfg == 3 || cfg == 4 || cfg == 5) ? 64 : 128; }

int gemm_m64g(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, uint16_t* out, int S, int mode,
              int nw, int cfg, hipStream_t st) {
  if (M < 1 || M > 64 || S < 1 || (nw != 1 && nw != 2) || cfg < 0 || cfg > 6) return 1;
  const int wv = m64g_cfg_waves(cfg), kc = m64g_cfg_kc(cfg);
  const int cols = 16 * nw * wv;
  if (K % (S * kc) || N % cols) return 1;
  if (mode == GG_SILU && (nw != 2 || S != 1)) return 1;
  if (mode == GG_PARTIAL && part == nullptr) return 1;
  if (mode != GG_PARTIAL && out == nullptr) return 1;
  const dim3 grid(N / cols, S);
  if (nw == 1) launch_m64g<1>(cfg, grid, st, x, M, K, w, N, part, out, mode);
  else launch_m64g<2>(cfg, grid, st, x, M, K, w, N, part, out, mode);
  return 0;
}

}  // namespace xgk
