// gemm_pf: prompt-sized MFMA GEMM (M ~ 256 .. 8192) for the projections of mixed
// continuous-batching steps and prefill:
//
//   out[M, N] = x[M, K] . W[N, K]^T        (bf16 in, fp32 accumulate)
//
// Replaces the library GEMM of the mixed step (VERDICT r4 "next round" #1): at
// M ~ 575 the four projections of a Llama-3-8B layer are ~250 GFLOP, compute-
// bound, so the kernel is built around keeping the matrix pipe busy
// (cdna_hip_programming.md §5 "The 256² 8-phase template", §5.5 T1-T5):
//
//   * one 512-thread workgroup per CU owns a BM x 256 output tile (BM = 128 / 192
//     / 256) over 64-deep K tiles; 8 waves as 2 (M) x 4 (N): wave (wr, wc) owns
//     BM/2 rows x 64 columns, v_mfma_f32_16x16x32_bf16 (the DVFS-favourable shape,
//     MI355X_MICROARCH.md "DVFS give-back" item 7) with the W fragment as the MFMA
//     A operand, so each lane ends with 4 consecutive output columns of one row;
//   * a K tile is consumed in P = BM/64 PHASES; phase q covers 32 rows of each
//     wave's half (64 A rows of the tile), so its A rows are free for restaging as
//     soon as phase q is over. The W tile (256 rows) is read into registers once,
//     in phase 0. Two LDS slots (K tiles t and t+1); the pieces of tile t+2 are
//     re-staged into tile t's slot phase by phase as they are released, so ~1.5 K
//     tiles of LDS-DMA stay in flight across the barriers under counted
//     s_waitcnt vmcnt(N) (never 0 in steady state; §5 "Pipelining across
//     barriers") -- the counts come from a constexpr simulation of the issue
//     order (pf_wait_count);
//   * both operands by global_load_lds_dwordx4 (8 rows x 128 B per wave
//     instruction) into lane-linear images, 16-B granule XOR-swizzle (granule ^
//     row & 7) on the global SOURCE address and on the ds_read_b128 fragment
//     reads (rule 21 / T2);
//   * ping-pong: waves 4-7 (wr = 1) run one barrier behind waves 0-3, so on every
//     SIMD (waves w and w + 4 share one) one wave's MFMA segment overlaps its
//     partner's fragment reads + DMA issue. Every piece is waited for one barrier
//     earlier than its first reader needs ("one barrier MORE when two wave groups
//     run staggered", §5 "Read a staged buffer one phase AFTER the wait"), and the
//     fragment reads retire (lgkmcnt(0)) before the barrier that ends their
//     segment, so a slot region can be re-staged in the very next phase (WAR);
//   * XCD-bijective block order with the M tiles of one W tile adjacent, so a W
//     tile's M tiles run on one XCD and read it through one L2 (T1); optional
//     K-tile rotation per W tile (the lock-step HBM stream of r4_mw_probe.md);
//   * split-K (uneven ranges) for grids that would not fill the chip: fp32
//     partials [S, M, N] reduced by the consumer (rope_cache_partials /
//     add_partials_rmsnorm), like every other projection kernel here.
// Epilogues: bf16, fp32 partials, or silu(gate) * up of a block-16 interleaved
// gate|up weight (the SiLU-gate fused: no [M, 2F] intermediate).
// Grouped form (gemm_pf_grouped, GRP): the prompt-sized expert GEMMs of an MoE layer
// over moe_align's expert-sorted rows -- one tile per expert segment, so each expert's
// weights stream once per step (profiles/r5_moe_pf.md).
#include <type_traits>

#include "glds.h"

namespace xgk {

int k_rotation(int S);  // gemm_m64g.hip

enum : int { PF_BF16 = 0, PF_PARTIAL = 1, PF_SILU = 2 };
constexpr int PF_GROUP_M = 8;  // M tiles per group of the tile order
// K-tile rotation per W tile (set_pf_krot(1); off by default): it spreads the
// lock-step HBM stream of the weight-streaming kernels, but here it would put the
// N tiles that share an A panel on different K tiles and lose that panel's L2 reuse
static int pf_krot = 0;
void set_pf_krot(int on) { pf_krot = on; }

namespace pf {
constexpr int BN = 256;  // output columns per workgroup (4 waves x 64)
constexpr int NBW = 4;   // W-tile DMA instructions per wave per K tile (256 rows x 128 B / 8 waves / 1 KB)

// Steady-state DMA issue order per wave (P phases per K tile, NA = A-piece DMA
// instructions per wave per phase, lag L). Global phase of (tile t, phase p) is
// tP + p. A piece q of tile u is read in global phase uP + q and its LDS region is
// re-staged (for tile u + 2) L phases later: issued in global phase uP + q + L.
// L = 1: the phase right after the last read -- the fragment reads retire before that
// phase's first barrier (lgkmcnt(0) ahead of the barrier); L = 2: the template form,
// the reads retire after the barrier, just ahead of the MFMAs (one phase less of DMA
// in flight). W piece i of tile u (the W image is read in phase 0 of tile u - 2) is
// issued in global phase (u - 2)P + L + i % P. Within a phase: A pieces, then W.
constexpr int b_rel(int P, int L, int i) { return L + i % P; }      // global phase offset from (u - 2)P
constexpr int b_phase(int P, int L, int i) { return b_rel(P, L, i) % P; }
constexpr int nb_in_phase(int P, int L, int ph) {
  int c = 0;
  for (int i = 0; i < NBW; ++i) c += b_phase(P, L, i) == ph ? 1 : 0;
  return c;
}
// the A piece issued in phase ph and how many tiles ahead its target is (1 or 2)
constexpr int a_piece(int P, int L, int ph) { return (ph - L % P + P) % P; }
constexpr int a_ahead(int P, int L, int ph) { return 2 - (a_piece(P, L, ph) + L) / P; }
constexpr int b_ahead(int P, int L, int i) { return 2 - b_rel(P, L, i) / P; }
constexpr int n_issue(int P, int L, int NA, int ph) { return NA + nb_in_phase(P, L, ph); }
constexpr int tile_issues(int P, int L, int NA) {
  int s = 0;
  for (int ph = 0; ph < P; ++ph) s += n_issue(P, L, NA, ph);
  return s;
}
constexpr int pos(int P, int L, int NA, int tau, int ph, int j) {
  int o = 0;
  for (int q = 0; q < ph; ++q) o += n_issue(P, L, NA, q);
  return tau * tile_issues(P, L, NA) + o + j;
}
// the last A DMA of A piece q of tile u
constexpr int pos_a(int P, int L, int NA, int u, int q) {
  return pos(P, L, NA, u - 2 + (q + L) / P, (q + L) % P, NA - 1);
}
constexpr int pos_b(int P, int L, int NA, int u, int i) {
  const int ph = b_phase(P, L, i);
  int j = NA;
  for (int i2 = 0; i2 < i; ++i2) j += b_phase(P, L, i2) == ph ? 1 : 0;
  return pos(P, L, NA, u - 2 + b_rel(P, L, i) / P, ph, j);
}
// vmcnt that retires everything phase p of a steady-state tile reads (A piece p,
// plus the whole W tile at p = 0), counted where the wait sits: after the issues
// of the previous phase, before those of phase p
constexpr int wait_count(int P, int L, int NA, int p) {
  const int t = 8;
  int latest = pos_a(P, L, NA, t, p);
  if (p == 0)
    for (int i = 0; i < NBW; ++i) latest = latest > pos_b(P, L, NA, t, i) ? latest : pos_b(P, L, NA, t, i);
  return pos(P, L, NA, t, p, 0) - 1 - latest;
}
// the largest tile an issue of phase ph targets, relative to the phase's tile
constexpr int max_ahead(int P, int L, int ph) {
  int m = a_ahead(P, L, ph);
  for (int i = 0; i < NBW; ++i)
    if (b_phase(P, L, i) == ph && b_ahead(P, L, i) > m) m = b_ahead(P, L, i);
  return m;
}
static_assert(wait_count(4, 1, 1, 0) == 6 && wait_count(4, 1, 1, 1) == 13 && wait_count(4, 1, 1, 2) == 13 &&
                  wait_count(4, 1, 1, 3) == 13, "pf wait counts (P = 4)");
static_assert(wait_count(2, 1, 2, 0) == 4 && wait_count(2, 1, 2, 1) == 10, "pf wait counts (P = 2, NA = 2)");
static_assert(a_piece(3, 1, 0) == 2 && a_ahead(3, 1, 0) == 1 && a_piece(3, 1, 1) == 0 && a_ahead(3, 1, 1) == 2,
              "pf lag-1 order");
static_assert(a_piece(3, 2, 0) == 1 && a_ahead(3, 2, 0) == 1 && a_piece(3, 2, 1) == 2 && a_ahead(3, 2, 1) == 1 &&
                  a_piece(3, 2, 2) == 0 && a_ahead(3, 2, 2) == 2,
              "pf lag-2 order");
}  // namespace pf

template <int P, int L, int NA, int PH>
__device__ __forceinline__ void pf_wait(bool steady) {
  if (steady) wait_vmcnt<pf::wait_count(P, L, NA, PH)>();
  else wait_vmcnt<0>();
}

// Grouped (MoE expert) form, GRP: the M dimension is moe_align's expert-sorted,
// 64-padded row space [P]; expert e owns rows [offs[e], offs[e + 1]) and its own
// weight w + e * w_stride. Tile slot mi of a column tile walks the experts' tiles in
// order (expert e has ceil(segment / BM) of them); slots past the last tile exit.
// A row p of a tile reads x row rows[p] (rows == nullptr: row p; -1 = a pad: row 0,
// finite data never combined), rows past the segment end are not stored.
struct PfGrp {
  const int32_t* rows;
  const int32_t* offs;
  int E;
  int mt;            // tile slots per column tile (host bound on the experts' tiles)
  int64_t w_stride;  // elements between two experts' [N, K] weights
};

template <int BM, int MTP, bool NT, int PR = 0, int LAG = 1, bool GRP = false>
__global__ void __launch_bounds__(512, 1) gemm_pf_kernel(const uint16_t* __restrict__ x, int M, int K,
                                                          const uint16_t* __restrict__ w, int N, int S,
                                                          float* __restrict__ part, uint16_t* __restrict__ out,
                                                          int mode, int krot, PfGrp grp) {
  // MTP: 16-row m tiles per wave per phase -> a phase is MTP x 4 x 2 MFMAs per wave
  // and releases 32 MTP A rows = 4 MTP DMA pieces of 8 rows; wave w issues pieces
  // w, w + 8, ... (MTP = 3: 12 pieces -> waves 0-3 two, waves 4-7 one; NA0 / NA1 are
  // the per-wave counts of the two groups, and each group's waits count its own)
  constexpr int P = BM / (32 * MTP);
  constexpr int NPC = 4 * MTP;                       // pieces per A phase block
  constexpr int NA0 = (NPC + 7) / 8;                 // pieces per wave, waves 0-3
  constexpr int NA1 = NPC / 8;                       // waves 4-7
  constexpr int NA = NA0;
  constexpr int PB = 32 * MTP * 128;       // bytes of one A phase block
  constexpr int BN = pf::BN;
  constexpr int ASZ = BM * 128;            // A image: P phase blocks
  constexpr int SLOT = ASZ + BN * 128;     // + the W image
  constexpr int NACC = P * MTP * 4;        // f32x4 accumulators per lane
  static_assert(P >= 2 && P * 32 * MTP == BM && MTP >= 2 && MTP <= 4 && NA1 >= 1, "gemm_pf geometry");
  static_assert(2 * SLOT <= 160 * 1024, "LDS");
  // ONE __shared__ object (cdna_hip_programming.md §5 "Three .s-level traps" (a))
  __shared__ __attribute__((aligned(1024))) uint8_t smem[2 * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;   // wave-uniform (scalar): guards barriers below
  const int g = lane >> 4, li = lane & 15;

  // XCD-bijective virtual block id (T1)
  const int TM = (M + BM - 1) / BM, TN = N / BN;
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7;
  const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int per_split = (GRP ? grp.mt : TM) * TN;
  const int nk_all = K / 64;
  // grouped order: GM M tiles x every N tile per group, M fastest inside a group, so
  // the ~32 workgroups an XCD runs at once share a few A and W panels (L2 hits)
  const int GM = TM < PF_GROUP_M ? TM : PF_GROUP_M;
  auto tile_mn = [&](int u, int& m0, int& n0) {
    const int gsz = GM * TN, gid = u / gsz, first_m = gid * GM;
    const int gm = TM - first_m < GM ? TM - first_m : GM;
    const int ug = u - gid * gsz;
    m0 = (first_m + ug % gm) * BM;
    n0 = (ug / gm) * BN;
  };

  // DMA lanes: row dr of an 8-row piece, physical granule dj holding logical dj ^ dr
  const int dr = lane >> 3, dj = lane & 7;
  const int sw = 8 * (dj ^ dr);
  const int wrow = wc * 64;          // W rows of this wave within the W image
  const int arl = wr * 16 * MTP;     // this wave's rows within an A phase block
  const int sl = li & 7;             // swizzle key of every fragment row this lane reads

  f32x4_t acc[P][MTP][4];
  // fragments read straight into the MFMA operand type (a uint4 -> bf16x8 bit_cast made
  // hipcc shuffle every fragment's middle dwords through VALU moves before each MFMA)
  bf16x8_t bfr[4][2];
  bf16x8_t afr[MTP][2];

  // ---- one K range [kt_lo, kt_lo + nk) of the tile at (m0, n0) into acc
  auto compute = [&](int m0, int n0, int kt_lo, int nk, int m_hi, const uint16_t* wb) {
    const int rot = krot ? ((n0 / BN) * 37) % nk : 0;
    // A phase block q: rows [wr 0: 16 MTP rows][wr 1: 16 MTP rows]; piece pc = wid + 8 a
    // of wave wid fills block rows 8 pc .. 8 pc + 7
    const uint16_t* asrc[P][NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const int pc = wid + 8 * a < NPC ? wid + 8 * a : wid;   // (an unused slot of waves 4-7)
      const int br = 8 * pc + dr;
      const int half = br / (16 * MTP);
      const int r = half * (BM / 2) + br - half * 16 * MTP;
#pragma unroll
      for (int q = 0; q < P; ++q) {
        int row = min(m0 + r + 16 * MTP * q, m_hi - 1);
        if constexpr (GRP) {
          if (grp.rows != nullptr) row = max(grp.rows[row], 0);
        }
        asrc[q][a] = x + static_cast<int64_t>(row) * K + sw;
      }
    }
    const uint16_t* bsrc = wb + static_cast<int64_t>(n0 + 32 * wid + dr) * K + sw;  // + 8 i rows per piece
    auto kof = [&](int t) {
      const int tt = t + rot;
      return (kt_lo + (tt >= nk ? tt - nk : tt)) * 64;
    };
    auto issue_a = [&](int t, int q) {
      if constexpr (PR == 1) return;
#pragma unroll
      for (int a = 0; a < NA; ++a)
        if (a < NA1 || wr == 0)
          glds16(asrc[q][a] + kof(t), smem + (t & 1) * SLOT + q * PB + (wid + 8 * a) * 1024);
    };
    auto issue_b = [&](int t, int i) {
      if constexpr (PR == 1) return;
      const uint16_t* src = bsrc + static_cast<int64_t>(8 * i) * K + kof(t);
      uint8_t* dst = smem + (t & 1) * SLOT + ASZ + (4 * wid + i) * 1024;
      if constexpr (NT) glds16_nt(src, dst);
      else glds16(src, dst);
    };
    // the DMA of phase PH of tile t (steady-state order, pf:: above); targets outside
    // [0, nk) are skipped (the prologue runs virtual tiles -2 and -1)
    auto issue_phase = [&](int t, auto ph_c) {
      constexpr int PH = decltype(ph_c)::value;
      constexpr int QA = pf::a_piece(P, LAG, PH), UA = pf::a_ahead(P, LAG, PH);
      if (t + UA >= 0 && t + UA < nk) issue_a(t + UA, QA);
#pragma unroll
      for (int i = 0; i < pf::NBW; ++i)
        if (pf::b_phase(P, LAG, i) == PH) {
          const int ub = t + pf::b_ahead(P, LAG, i);
          if (ub >= 0 && ub < nk) issue_b(ub, i);
        }
    };
    auto issue_tile = [&](int t) {
      issue_phase(t, std::integral_constant<int, 0>{});
      issue_phase(t, std::integral_constant<int, 1>{});
      if constexpr (P > 2) issue_phase(t, std::integral_constant<int, (P > 2 ? 2 : 0)>{});
      if constexpr (P > 3) issue_phase(t, std::integral_constant<int, (P > 3 ? 3 : 0)>{});
    };

#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
      for (int mt = 0; mt < MTP; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[q][mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // every wave is past the previous range's LDS reads before its slots are refilled
    __syncthreads();
    // prologue: the issues of (virtual) tiles -2 and -1, in steady-state order
    issue_tile(-2);
    issue_tile(-1);
    // wait for what (tile 0, phase 0) reads; the steady count holds iff every issue
    // between that piece and the wait exists (nk >= 2: every prologue target does)
    if (wr == 0) pf_wait<P, LAG, NA0, 0>(nk >= 2);
    else pf_wait<P, LAG, NA1, 0>(nk >= 2);
    if (wr == 1) raw_barrier();  // the stagger: waves 4-7 one barrier behind

    auto phase = [&](int t, auto ph_c) {
      constexpr int p = decltype(ph_c)::value;
      const uint8_t* slot = smem + (t & 1) * SLOT;
      // the wait at the end of this phase retires what the NEXT phase reads
      constexpr int PN = (p + 1 < P) ? p + 1 : 0;
      const int tt = (p + 1 < P) ? t : t + 1;
      const bool need = tt < nk;
      // the count holds iff the last phase before the wait (p of tile t) issued all
      // its DMA (its largest target is below nk; targets grow with the phase)
      const bool steady = t + pf::max_ahead(P, LAG, p) <= nk - 1;
      // ---- load segment: this phase's DMA, then the fragment reads
      raw_barrier();
      __builtin_amdgcn_sched_barrier(0);
      issue_phase(t, ph_c);
      if constexpr (p == 0) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            bfr[nt][ks] = *reinterpret_cast<const bf16x8_t*>(slot + ASZ + (wrow + 16 * nt + li) * 128 +
                                                              (((4 * ks + g) ^ sl) << 4));
      }
#pragma unroll
      for (int mt = 0; mt < MTP; ++mt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          afr[mt][ks] = *reinterpret_cast<const bf16x8_t*>(slot + p * PB + (arl + 16 * mt + li) * 128 +
                                                            (((4 * ks + g) ^ sl) << 4));
      // LAG 1: fragment reads retire before the barrier (the region is re-staged next
      // phase); LAG 2: they retire ahead of the MFMAs that use them (compiler waits)
      if constexpr (LAG == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (wr == 1 && need) pf_wait<P, LAG, NA1, PN>(steady);
      raw_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- MFMA segment
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < (PR == 2 ? 0 : 2); ++ks)
#pragma unroll
        for (int mt = 0; mt < MTP; ++mt)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
            acc[p][mt][nt] = mfma16x16x32(bfr[nt][ks], afr[mt][ks], acc[p][mt][nt]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (wr == 0 && need) pf_wait<P, LAG, NA0, PN>(steady);
    };
    for (int t = 0; t < nk; ++t) {
      phase(t, std::integral_constant<int, 0>{});
      phase(t, std::integral_constant<int, 1>{});
      if constexpr (P > 2) phase(t, std::integral_constant<int, (P > 2 ? 2 : 0)>{});
      if constexpr (P > 3) phase(t, std::integral_constant<int, (P > 3 ? 3 : 0)>{});
    }
    if (wr == 0) raw_barrier();  // equal barrier counts in both groups
  };

  // ---- epilogue of a finished tile (split s of S for PF_PARTIAL)
  // acc[q][mt][nt][r] = out[m = m0 + wr BM/2 + 16 MTP q + 16 mt + li][n = n0 + wrow + 16 nt + 4 g + r]
  auto epilogue = [&](int m0, int n0, int s, int m_hi) {
    const int mb = m0 + wr * (BM / 2) + li;
    const int nb0 = n0 + wrow + 4 * g;
    if (mode == PF_PARTIAL) {
      float* pp = part + static_cast<int64_t>(s) * M * N;
#pragma unroll
      for (int q = 0; q < P; ++q)
#pragma unroll
        for (int mt = 0; mt < MTP; ++mt) {
          const int m = mb + 16 * MTP * q + 16 * mt;
          if (m >= m_hi) continue;
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
            *reinterpret_cast<float4*>(pp + static_cast<int64_t>(m) * N + nb0 + 16 * nt) =
                make_float4(acc[q][mt][nt][0], acc[q][mt][nt][1], acc[q][mt][nt][2], acc[q][mt][nt][3]);
        }
    } else if (mode == PF_BF16) {
#pragma unroll
      for (int q = 0; q < P; ++q)
#pragma unroll
        for (int mt = 0; mt < MTP; ++mt) {
          const int m = mb + 16 * MTP * q + 16 * mt;
          if (m >= m_hi) continue;
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            uint2 o;
            o.x = pack2(acc[q][mt][nt][0], acc[q][mt][nt][1]);
            o.y = pack2(acc[q][mt][nt][2], acc[q][mt][nt][3]);
            *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * N + nb0 + 16 * nt) = o;
          }
        }
    } else {
      // SiLU gate: n tiles 2j (gate) / 2j + 1 (up) are one interleaved 16-row block pair
      const int F = N / 2, f0 = (n0 + wrow) / 2 + 4 * g;
#pragma unroll
      for (int q = 0; q < P; ++q)
#pragma unroll
        for (int mt = 0; mt < MTP; ++mt) {
          const int m = mb + 16 * MTP * q + 16 * mt;
          if (m >= m_hi) continue;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            float o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float gt = acc[q][mt][2 * j][r];
              o[r] = gt / (1.f + __expf(-gt)) * acc[q][mt][2 * j + 1][r];
            }
            uint2 v2;
            v2.x = pack2(o[0], o[1]);
            v2.y = pack2(o[2], o[3]);
            *reinterpret_cast<uint2*>(out + static_cast<int64_t>(m) * F + f0 + 16 * j) = v2;
          }
        }
    }
  };

  // data-parallel: one (tile, split) per workgroup
  {
    // GRP: the tile slots past the experts' last tile are empty and sit at the end of
    // the order, so the dispatch order itself (block b on XCD b % 8) spreads the real
    // tiles over every XCD; the XCD-contiguous order v would leave whole XCDs idle
    const int vg = GRP ? bid : v;
    const int s = vg / per_split;
    int m0, n0, m_hi = M;
    const uint16_t* wb = w;
    if constexpr (GRP) {
      // tile slot mi of column tile n: the mi-th (expert, row tile) in expert order
      const int u = vg - s * per_split, mi = u / TN;
      n0 = (u - mi * TN) * BN;
      int e = 0, base = 0, lo = 0, hi = 0;
      for (; e < grp.E; ++e) {
        lo = grp.offs[e];
        hi = grp.offs[e + 1];
        const int nt = (hi - lo + BM - 1) / BM;
        if (mi < base + nt) break;
        base += nt;
      }
      if (e == grp.E) return;  // past the last tile: the whole workgroup leaves (uniform)
      m0 = lo + (mi - base) * BM;
      m_hi = hi;
      wb = w + static_cast<int64_t>(e) * grp.w_stride;
    } else {
      tile_mn(v - s * per_split, m0, n0);
    }
    const int kt_lo = s * nk_all / S;
    compute(m0, n0, kt_lo, (s + 1) * nk_all / S - kt_lo, m_hi, wb);
    epilogue(m0, n0, s, m_hi);
  }
}

template <int BM, int MTP, bool NT, int PR = 0, int LAG = 1>
static int launch_pf(int tiles, hipStream_t st, const uint16_t* x, int M, int K, const uint16_t* w, int N, int S,
                     float* part, uint16_t* out, int mode) {
  const PfGrp ng{nullptr, nullptr, 0, 0, 0};
  hipLaunchKernelGGL((gemm_pf_kernel<BM, MTP, NT, PR, LAG>), dim3(tiles * S), dim3(512), 0, st, x, M, K, w, N, S, part,
                     out, mode, pf_krot, ng);
  return static_cast<int>(hipGetLastError());
}

// cfg % 16 -> (BM, MTP): 0 (256, 2)  1 (192, 2)  2 (128, 2)  3 (256, 4)  4 (192, 3)  5 (288, 3);
// with DMA lag 2 (fragment reads retire after the barrier; 3+ phases only): 6 (288, 3)
// 7 (256, 2)  8 (192, 2);
// cfg / 16: 0 the kernel, 1 no DMA, 2 no MFMA (anatomy probes, bench/pf_gemm_bench.py
// --probe: garbage results). W stays on cached DMA (non-temporal measured slower: the
// M tiles of a W tile re-read it through L2).
int pf_cfg_bm(int cfg) {
  switch (cfg & 15) {
    case 1: case 4: case 8: return 192;
    case 2: return 128;
    case 5: case 6: return 288;
    default: return 256;
  }
}

template <int PR>
static int launch_pf_cfg(int c, int tiles, hipStream_t st, const uint16_t* x, int M, int K, const uint16_t* w, int N,
                         int S, float* part, uint16_t* out, int mode) {
  switch (c) {
    case 0: return launch_pf<256, 2, false, PR>(tiles, st, x, M, K, w, N, S, part, out, mode);
    case 1: return launch_pf<192, 2, false, PR>(tiles, st, x, M, K, w, N, S, part, out, mode);
    case 2: return launch_pf<128, 2, false, PR>(tiles, st, x, M, K, w, N, S, part, out, mode);
    case 3: return launch_pf<256, 4, false, PR>(tiles, st, x, M, K, w, N, S, part, out, mode);
    case 4: return launch_pf<192, 3, false, PR>(tiles, st, x, M, K, w, N, S, part, out, mode);
    case 5: return launch_pf<288, 3, false, PR>(tiles, st, x, M, K, w, N, S, part, out, mode);
    case 6: return launch_pf<288, 3, false, PR, 2>(tiles, st, x, M, K, w, N, S, part, out, mode);
    case 7: return launch_pf<256, 2, false, PR, 2>(tiles, st, x, M, K, w, N, S, part, out, mode);
    case 8: return launch_pf<192, 2, false, PR, 2>(tiles, st, x, M, K, w, N, S, part, out, mode);
    default: return 1;
  }
}

// grouped (MoE): data-parallel only, no K rotation
template <int BM, int MTP, int LAG>
static int launch_pf_grp(int tiles, hipStream_t st, const uint16_t* x, int M, int K, const uint16_t* w, int N, int S,
                         float* part, uint16_t* out, int mode, const PfGrp& grp) {
  hipLaunchKernelGGL((gemm_pf_kernel<BM, MTP, false, 0, LAG, true>), dim3(tiles * S), dim3(512), 0, st, x, M, K, w, N,
                     S, part, out, mode, 0, grp);
  return static_cast<int>(hipGetLastError());
}

// Grouped (MoE experts, moe_align layout): out / part rows are the P sorted rows; w is
// [E, N, K]; rows gathers x (nullptr: x is already in sorted order); max_pairs bounds
// the real rows over all experts (sizes the grid: sum over experts of ceil(segment / BM)
// <= (max_pairs + 63 E) / BM + E). Lag-2 configs 6 / 7 / 8 only.
int gemm_pf_grouped(const uint16_t* x, const int32_t* rows, const int32_t* offs, int E, int P, int K,
                    const uint16_t* w, int N, int max_pairs, float* part, uint16_t* out, int S, int mode, int cfg,
                    hipStream_t st) {
  if (E < 1 || P < 1 || P % 64 || max_pairs < 1 || offs == nullptr || K < 64 || K % 64 || N < pf::BN ||
      N % pf::BN || S < 1 || S > K / 64 || cfg < 6 || cfg > 8)
    return 1;
  if (mode == PF_PARTIAL) {
    if (part == nullptr) return 1;
  } else if (mode == PF_BF16 || mode == PF_SILU) {
    if (out == nullptr || S != 1) return 1;
  } else {
    return 1;
  }
  const int bm = pf_cfg_bm(cfg);
  const int mt = (max_pairs + 63 * E) / bm + E;
  const PfGrp grp{rows, offs, E, mt, static_cast<int64_t>(N) * K};
  const int tiles = mt * (N / pf::BN);
  switch (cfg) {
    case 6: return launch_pf_grp<288, 3, 2>(tiles, st, x, P, K, w, N, S, part, out, mode, grp);
    case 7: return launch_pf_grp<256, 2, 2>(tiles, st, x, P, K, w, N, S, part, out, mode, grp);
    default: return launch_pf_grp<192, 2, 2>(tiles, st, x, P, K, w, N, S, part, out, mode, grp);
  }
}

int gemm_pf(const uint16_t* x, int M, int K, const uint16_t* w, int N, float* part, uint16_t* out, int S, int mode,
            int cfg, hipStream_t st) {
  if (M < 1 || K < 64 || K % 64 || N < pf::BN || N % pf::BN || S < 1 || S > K / 64 || cfg < 0 || cfg >= 48)
    return 1;
  if (mode == PF_PARTIAL) {
    if (part == nullptr) return 1;
  } else if (mode == PF_BF16 || mode == PF_SILU) {
    if (out == nullptr || S != 1) return 1;
  } else {
    return 1;
  }
  const int bm = pf_cfg_bm(cfg);
  const int tiles = ((M + bm - 1) / bm) * (N / pf::BN);
  switch (cfg / 16) {
    case 0: return launch_pf_cfg<0>(cfg % 16, tiles, st, x, M, K, w, N, S, part, out, mode);
#ifdef XGK_PROBES  // anatomy probes (no DMA / no MFMA): measurement builds only (xgserve/_build.py --probes)
    case 1: return launch_pf_cfg<1>(cfg % 16, tiles, st, x, M, K, w, N, S, part, out, mode);
    default: return launch_pf_cfg<2>(cfg % 16, tiles, st, x, M, K, w, N, S, part, out, mode);
#else
    default: return 1;
#endif
  }
}

}  // namespace xgk
