// Decode GEMM with FP8 weights (OCP E4M3, one fp32 scale per output channel) and
// bf16 activations: out = x . (diag(s) W8)^T for M <= 64 (decode batches).
//
// Weight-only FP8 halves the bytes of a bandwidth-bound decode step. The weights
// stream through the same LDS-DMA pipeline as gemm_m64g (3 slots, 2 chunks in
// flight, counted vmcnt + raw barrier, non-temporal weight DMA); each A fragment is
// read as 8 fp8 bytes and widened to bf16 in registers with v_cvt_scalef32_pk_bf16_fp8
// (exact: every E4M3 value is representable in bf16), then the bf16 MFMA
// (16x16x32) runs as in the bf16 kernel. The per-channel scale is applied to the
// fp32 accumulators in the epilogue. Activations stay bf16 (no activation
// quantisation): the accuracy is that of the rounded weights alone.
//
//   weights [N, K] uint8 (E4M3), scale [N] fp32; x [M, K] bf16 (M <= 64; MT = 1
//   x tile of 16 rows for M <= 16, MT = 4 tiles for 16 < M <= 64, KC 128 only).
//   LDS: x rows 2*KC bytes, weight rows KC bytes, 16-B granules XOR-swizzled by
//   row on the GLOBAL source address (DMA writes are lane-linear).
//   modes: W8_PARTIAL -> fp32 split-K partials [S, M, N] (reduced by the consumer
//   kernel, like gemm_m64g's); W8_SILU -> bf16 silu(gate) * up from block-16
//   interleaved gate|up rows (split 1).
//
// Weight formats (FMT; Req 10.3 quantization levels, weight-only, bf16 activations):
//   WQ_FP8   E4M3 codes, fp32 scale per output channel (above);
//   WQ_INT8  symmetric int8 codes, fp32 scale per output channel: each byte widened
//            exactly (|q| <= 127 is a bf16 integer), scale in the epilogue as for FP8;
//   WQ_INT4  symmetric 4-bit codes in groups of WQ_GROUP = 128 k per output channel,
//            fp32 scale per (group, channel) [K / 128][N]. Stored offset-binary
//            (u = q + 8) and packed so that one 32-bit word holds 8 consecutive k
//            with element 2j at bits 4j and element 2j + 1 at bits 16 + 4j: one
//            v_and_or per bf16 PAIR builds 0x4300 | u = 128 + u = 136 + q (exact
//            bf16). The MFMA accumulates sum x (136 + q) per group; an all-ones
//            MFMA gives sum x over the same group, and at each group end
//            acc += s_group (acc_group - 136 sum x). Rows are KC / 2 bytes; the
//            workgroup's scales are staged in LDS before the DMA pipeline starts
//            (no VGPR-destination global load beside the in-flight LDS-DMA).
#include "glds.h"

namespace xgk {

enum : int { W8_PARTIAL = 1, W8_SILU = 2 };
enum : int { WQ_FP8 = 0, WQ_INT8 = 1, WQ_INT4 = 2 };
constexpr int WQ_GROUP = 128;
constexpr int WQ_SC_FLOATS = 4096;  // int4 scales staged per workgroup (groups x columns)

// 8 int8 codes (k order) -> bf16x8 A fragment (exact)
__device__ __forceinline__ bf16x8_t int8x8_to_bf16(uint2 v) {
  uint32_t o[4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint32_t wv = j ? v.y : v.x;
    const float a = static_cast<float>(static_cast<int8_t>(wv & 0xFF));
    const float b = static_cast<float>(static_cast<int8_t>((wv >> 8) & 0xFF));
    const float c = static_cast<float>(static_cast<int8_t>((wv >> 16) & 0xFF));
    const float d = static_cast<float>(static_cast<int8_t>(wv >> 24));
    // exact integers: the bf16 of each is its top 16 bits
    o[2 * j] = (__float_as_uint(a) >> 16) | (__float_as_uint(b) & 0xFFFF0000u);
    o[2 * j + 1] = (__float_as_uint(c) >> 16) | (__float_as_uint(d) & 0xFFFF0000u);
  }
  return as_frag(make_uint4(o[0], o[1], o[2], o[3]));
}

// 8 offset-binary nibbles (pair-interleaved, see WQ_INT4) -> bf16x8 of 136 + q
__device__ __forceinline__ bf16x8_t u4x8_to_bf16(uint32_t v) {
  return as_frag(make_uint4((v & 0x000F000Fu) | 0x43004300u, ((v >> 4) & 0x000F000Fu) | 0x43004300u,
                            ((v >> 8) & 0x000F000Fu) | 0x43004300u, ((v >> 12) & 0x000F000Fu) | 0x43004300u));
}

// 8 E4M3 bytes (k order) -> bf16x8 A fragment
__device__ __forceinline__ bf16x8_t fp8x8_to_bf16(uint2 v) {
#if defined(__HIP_DEVICE_COMPILE__)
  const auto a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.x, 1.0f, false);
  const auto b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.x, 1.0f, true);
  const auto c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.y, 1.0f, false);
  const auto d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.y, 1.0f, true);
  return as_frag(make_uint4(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b),
                            __builtin_bit_cast(uint32_t, c), __builtin_bit_cast(uint32_t, d)));
#else
  return bf16x8_t{};
#endif
}

//   NW  16-column MFMA tiles per wave (SiLU needs 2: one gate + one up tile)
//   WV  waves per workgroup
//   KC  k per chunk (fp8 row = KC bytes, bf16 x row = 2 KC bytes)
template <int NW, int WV, int KC, int MT, int FMT = WQ_FP8>
__global__ void __launch_bounds__(64 * WV, 1) gemm_w8_kernel(const uint16_t* __restrict__ x, int M, int K,
                                                             const uint8_t* __restrict__ w,
                                                             const float* __restrict__ wscale, int N,
                                                             float* __restrict__ part, uint16_t* __restrict__ out,
                                                             int mode) {
  constexpr bool I4 = FMT == WQ_INT4;
  constexpr int XRB = KC * 2, WRB = I4 ? KC / 2 : KC;  // bytes per LDS row
  constexpr int XG = XRB / 16, WG = WRB / 16;    // 16-B granules per row
  constexpr int XRPI = 1024 / XRB, WRPI = 1024 / WRB;  // rows per DMA instruction
  constexpr int XROWS = 16 * MT;
  constexpr int XBYTES = XROWS * XRB;
  constexpr int XI = XROWS / XRPI / WV;          // x DMA instructions per wave per chunk
  constexpr int WROWS = 16 * NW;
  constexpr int WI = WROWS / WRPI;               // weight DMA instructions per wave per chunk
  constexpr int WBYTES = WROWS * WRB;
  constexpr int SLOT = XBYTES + WV * WBYTES;
  constexpr int G = XI + WI;
  static_assert(XI >= 1 && WI >= 1 && XROWS % (XRPI * WV) == 0 && WROWS % WRPI == 0, "bad w8 geometry");
  __shared__ __attribute__((aligned(1024))) uint8_t lds0[SLOT];
  __shared__ __attribute__((aligned(1024))) uint8_t lds1[SLOT];
  __shared__ __attribute__((aligned(1024))) uint8_t lds2[SLOT];
  // int4: this workgroup's group scales [group][column] (unused otherwise)
  __shared__ __attribute__((aligned(16))) float sc_lds[I4 ? WQ_SC_FLOATS : 4];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int S = gridDim.y, s = blockIdx.y;
  const int kws = K / S;
  const int k0 = s * kws;
  const int nchunks = kws / KC;
  const int nbase = blockIdx.x * (16 * NW * WV) + wid * WROWS;

  const uint8_t* wsrc[WI];
  {
    const int dr = lane / WG, dj = lane % WG;
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const int r = WRPI * i + dr;
      wsrc[i] = w + static_cast<int64_t>(nbase + r) * (I4 ? K / 2 : K) + (I4 ? k0 / 2 : k0) +
                16 * (dj ^ (r & (WG - 1)));
    }
  }
  const uint16_t* xsrc[XI];
  {
    const int dr = lane / XG, dj = lane % XG;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int r = XRPI * (wid * XI + i) + dr;  // x row 0..XROWS-1
      xsrc[i] = x + static_cast<int64_t>(min(r, M - 1)) * K + k0 + 8 * (dj ^ (r & (XG - 1)));
    }
  }

  auto issue = [&](uint8_t* slot, int c) {
    const int kk = c * KC;
#pragma unroll
    for (int i = 0; i < XI; ++i) glds16(xsrc[i] + kk, slot + XRPI * (wid * XI + i) * XRB);
#pragma unroll
    for (int i = 0; i < WI; ++i) glds16_nt(wsrc[i] + (I4 ? kk / 2 : kk), slot + XBYTES + wid * WBYTES + i * 1024);
  };

  f32x4_t acc[NW][MT];
#pragma unroll
  for (int nt = 0; nt < NW; ++nt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // int4: the open group's sum x (136 + q) and sum x (every row of an all-ones MFMA)
  f32x4_t accg[I4 ? NW : 1][I4 ? MT : 1];
  f32x4_t xs[I4 ? MT : 1];
  constexpr int COLS = 16 * NW * WV;
  const int g0 = k0 / WQ_GROUP;  // first group of this split
  if constexpr (I4) {
#pragma unroll
    for (int nt = 0; nt < NW; ++nt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) accg[nt][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) xs[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // stage the scales before any LDS-DMA is in flight (host: groups x COLS <= WQ_SC_FLOATS)
    const int ng = kws / WQ_GROUP, col0 = blockIdx.x * COLS;
    for (int i = tid; i < ng * COLS; i += 64 * WV) sc_lds[i] = wscale[static_cast<int64_t>(g0 + i / COLS) * N + col0 +
                                                                      i % COLS];
    __syncthreads();
  }
  const bf16x8_t ones = as_frag(make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u));
  // fold the group that ends at chunk c, k step t (int4)
  auto fold = [&](int gi) {
#pragma unroll
    for (int nt = 0; nt < NW; ++nt) {
      const float4 sc = *reinterpret_cast<const float4*>(sc_lds + gi * COLS + wid * WROWS + 16 * nt + 4 * g);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        acc[nt][mt][0] += sc.x * (accg[nt][mt][0] - 136.f * xs[mt][0]);
        acc[nt][mt][1] += sc.y * (accg[nt][mt][1] - 136.f * xs[mt][1]);
        acc[nt][mt][2] += sc.z * (accg[nt][mt][2] - 136.f * xs[mt][2]);
        acc[nt][mt][3] += sc.w * (accg[nt][mt][3] - 136.f * xs[mt][3]);
        accg[nt][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) xs[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  };

  auto compute = [&](const uint8_t* slot, int c) {
    const uint8_t* xsl = slot;
    const uint8_t* ws = slot + XBYTES + wid * WBYTES;
#pragma unroll
    for (int t = 0; t < KC / 32; ++t) {
      // x (B operand): row 16 mt + li, k = 32t + 8g.. -> bf16 granule 4t + g
      uint4 b[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int xr = 16 * mt + li;
        b[mt] = *reinterpret_cast<const uint4*>(xsl + xr * XRB + (((4 * t + g) ^ (xr & (XG - 1))) * 16));
      }
#pragma unroll
      for (int nt = 0; nt < NW; ++nt) {
        const int row = 16 * nt + li;
        bf16x8_t a;
        if constexpr (I4) {
          // W row 16 nt + li, k = 32t + 8g.. -> 4-bit granule t, bytes 4g .. 4g + 3
          a = u4x8_to_bf16(*reinterpret_cast<const uint32_t*>(ws + row * WRB + ((t ^ (row & (WG - 1))) * 16) +
                                                              4 * g));
        } else {
          // W (A operand): row 16 nt + li, k = 32t + 8g.. -> byte granule 2t + g/2, byte (g & 1) * 8
          const uint2 a8 = *reinterpret_cast<const uint2*>(ws + row * WRB +
                                                           (((2 * t + (g >> 1)) ^ (row & (WG - 1))) * 16) +
                                                           (g & 1) * 8);
          a = FMT == WQ_INT8 ? int8x8_to_bf16(a8) : fp8x8_to_bf16(a8);
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          if constexpr (I4) accg[nt][mt] = mfma16x16x32(a, as_frag(b[mt]), accg[nt][mt]);
          else acc[nt][mt] = mfma16x16x32(a, as_frag(b[mt]), acc[nt][mt]);
        }
      }
      if constexpr (I4) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) xs[mt] = mfma16x16x32(ones, as_frag(b[mt]), xs[mt]);
        if ((t + 1) % (WQ_GROUP / 32) == 0) fold((c * KC + 32 * t) / WQ_GROUP);
      }
    }
  };

  auto step = [&](uint8_t* cur, uint8_t* nxt2, int c) {
    if (c + 1 < nchunks) wait_vmcnt<G>();
    else wait_vmcnt<0>();
    raw_barrier();
    if (c + 2 < nchunks) issue(nxt2, c + 2);
    compute(cur, c);
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

  // acc[nt][mt][r] = out[m = 16 mt + li][n = nbase + 16 nt + 4 g + r] / scale[n]
  // (int4: the group scales are already folded in)
#pragma unroll
  for (int nt = 0; nt < (I4 ? 0 : NW); ++nt) {
    const float4 sc = *reinterpret_cast<const float4*>(wscale + nbase + 16 * nt + 4 * g);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      acc[nt][mt][0] *= sc.x;
      acc[nt][mt][1] *= sc.y;
      acc[nt][mt][2] *= sc.z;
      acc[nt][mt][3] *= sc.w;
    }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = 16 * mt + li;
    if (m >= M) continue;
    if (mode == W8_PARTIAL) {
      float* pp = part + static_cast<int64_t>(s) * M * N + static_cast<int64_t>(m) * N;
#pragma unroll
      for (int nt = 0; nt < NW; ++nt)
        *reinterpret_cast<float4*>(pp + nbase + 16 * nt + 4 * g) =
            make_float4(acc[nt][mt][0], acc[nt][mt][1], acc[nt][mt][2], acc[nt][mt][3]);
    } else if (NW == 2) {
      const int F = N / 2, f0 = nbase / 2 + 4 * g;
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

// cfg: 0 = (NW 2, 4 waves, KC 128), 1 = (2, 2, 128), 2 = (1, 4, 128), 3 = (2, 2, 256), 4 = (2, 4, 256)
static int w8_cfg_cols(int cfg) {
  switch (cfg) {
    case 0: return 128;
    case 1: return 64;
    case 2: return 64;
    case 3: return 64;
    case 4: return 128;
    default: return 0;
  }
}
static int w8_cfg_kc(int cfg) { return cfg >= 3 ? 256 : 128; }
static int w8_cfg_nw(int cfg) { return cfg == 2 ? 1 : 2; }

template <int FMT>
static void launch_w8(int cfg, bool mt1, dim3 grid, hipStream_t st, const uint16_t* x, int M, int K, const uint8_t* w,
                      const float* scale, int N, float* part, uint16_t* out, int mode) {
#define XGK_W8(NW, WV, KC, MT)                                                                                 \
  hipLaunchKernelGGL((gemm_w8_kernel<NW, WV, KC, MT, FMT>), grid, dim3(64 * WV), 0, st, x, M, K, w, scale, N, part, \
                     out, mode)
  switch (cfg) {
    case 0: if (mt1) XGK_W8(2, 4, 128, 1); else XGK_W8(2, 4, 128, 4); break;
    case 1: if (mt1) XGK_W8(2, 2, 128, 1); else XGK_W8(2, 2, 128, 4); break;
    case 2: if (mt1) XGK_W8(1, 4, 128, 1); else XGK_W8(1, 4, 128, 4); break;
    case 3: XGK_W8(2, 2, 256, 1); break;
    default: XGK_W8(2, 4, 256, 1); break;
  }
#undef XGK_W8
}

// fmt: WQ_FP8 / WQ_INT8 (scale [N]) or WQ_INT4 (w [N, K / 2] packed, scale [K / 128, N])
int gemm_w8(const uint16_t* x, int M, int K, const uint8_t* w, const float* scale, int N, float* part,
            uint16_t* out, int S, int mode, int cfg, hipStream_t st, int fmt) {
  if (M < 1 || M > 64 || S < 1 || cfg < 0 || cfg > 4 || fmt < WQ_FP8 || fmt > WQ_INT4) return 1;
  if (M > 16 && cfg >= 3) return 1;  // KC 256 with four x tiles exceeds the LDS
  if (mode != W8_PARTIAL && mode != W8_SILU) return 1;
  const int cols = w8_cfg_cols(cfg), kc = w8_cfg_kc(cfg);
  if (N % cols || K % (S * kc)) return 1;
  if (mode == W8_SILU && (w8_cfg_nw(cfg) != 2 || S != 1 || out == nullptr)) return 1;
  if (mode == W8_PARTIAL && part == nullptr) return 1;
  // int4: whole groups per split, and the workgroup's scales fit its LDS stage
  if (fmt == WQ_INT4 && ((K / S) % WQ_GROUP || (K / S / WQ_GROUP) * cols > WQ_SC_FLOATS)) return 1;
  const dim3 grid(N / cols, S);
  const bool mt1 = M <= 16;
  if (fmt == WQ_FP8) launch_w8<WQ_FP8>(cfg, mt1, grid, st, x, M, K, w, scale, N, part, out, mode);
  else if (fmt == WQ_INT8) launch_w8<WQ_INT8>(cfg, mt1, grid, st, x, M, K, w, scale, N, part, out, mode);
  else launch_w8<WQ_INT4>(cfg, mt1, grid, st, x, M, K, w, scale, N, part, out, mode);
  return 0;
}

}  // namespace xgk
