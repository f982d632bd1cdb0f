// K12: Mixture-of-Experts building blocks (Mixtral-style top-k routing).
//
//   moe_topk_softmax : router logits [T, E] -> top-k (weights, expert ids); the
//                      weights are the softmax over the selected k logits
//                      (== softmax-then-renormalise, Mixtral semantics) or the
//                      plain softmax probabilities when renorm == 0.
//   moe_align        : one workgroup builds the expert-sorted, block_m-padded
//                      row layout for this rank's experts: sorted_rows[p] =
//                      token of padded row p (-1 = pad), expert_offsets[E+1],
//                      dest[t*k+j] = padded row of (token t, choice j) or -1
//                      when the expert lives on another EP rank.
//   (the grouped expert GEMMs are gemm_m64_grouped in gemm_m64.hip: W [E, N, K]
//    streamed once per step per column tile, fused SiLU-gate on w13)
//   moe_combine      : out[t] = sum_j w[t, j] * y[dest[t*k + j]], y bf16 or
//                      fp32 split-K partials of the w2 GEMM (also the EP source-side
//                      unpermute: y = rows returned by the expert owners).
//   ep_plan / ep_scatter : expert-parallel dispatch -- deterministic per-destination
//                      slots (fixed-capacity or count-exact packed layout), local
//                      expert ids for the owners, the row copy into the send buffer.
#include "common.h"

namespace xgk {

// ---------------------------------------------------------------- routing
template <typename T>
__device__ __forceinline__ float ldv(const T* p, int64_t i);
template <> __device__ __forceinline__ float ldv<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
template <> __device__ __forceinline__ float ldv<float>(const float* p, int64_t i) { return p[i]; }

template <typename T>
__global__ void topk_softmax_kernel(const T* __restrict__ logits, int T_, int E, int k, int renorm,
                                    float* __restrict__ w, int32_t* __restrict__ ids) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T_) return;
  float v[64];
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) {
    v[e] = ldv<T>(logits, static_cast<int64_t>(t) * E + e);
    mx = fmaxf(mx, v[e]);
  }
  float den = 0.f;
  for (int e = 0; e < E; ++e) den += __expf(v[e] - mx);
  unsigned long long used = 0;
  float sel[16];
  int sid[16];
  float ssum = 0.f;
  for (int j = 0; j < k; ++j) {
    int best = -1;
    float bv = -INFINITY;
    for (int e = 0; e < E; ++e)
      if (!((used >> e) & 1ull) && (best < 0 || v[e] > bv)) { best = e; bv = v[e]; }
    used |= 1ull << best;
    sid[j] = best;
    sel[j] = __expf(bv - mx) / den;
    ssum += sel[j];
  }
  for (int j = 0; j < k; ++j) {
    w[static_cast<int64_t>(t) * k + j] = renorm ? sel[j] / ssum : sel[j];
    ids[static_cast<int64_t>(t) * k + j] = sid[j];
  }
}

void moe_topk_softmax(const void* logits, int is_f32, int T, int E, int k, int renorm, float* w, int32_t* ids,
                      hipStream_t st) {
  if (T <= 0) return;
  dim3 g((T + 127) / 128), b(128);
  if (is_f32)
    hipLaunchKernelGGL(topk_softmax_kernel<float>, g, b, 0, st, (const float*)logits, T, E, k, renorm, w, ids);
  else
    hipLaunchKernelGGL(topk_softmax_kernel<uint16_t>, g, b, 0, st, (const uint16_t*)logits, T, E, k, renorm, w,
                       ids);
}

// Router GEMV + softmax + top-k in one launch (replaces a tiny hipBLASLt GEMM and
// the topk kernel on the decode path): one workgroup per token, each thread dots
// 8-element chunks of the hidden row with all EM (>= E) router rows in fp32,
// block reduction, then lane 0 selects the top k (softmax over all E, optionally
// renormalised over the chosen k: Mixtral semantics).
// Fused-decode form (NORM): h is the raw residual stream; the workgroup first takes
// the row's RMSNorm (sum of squares, block reduction), writes the normalised row
// hn = bf16(x * rsqrt(mean(x^2) + eps) * norm_w) for the expert GEMMs and routes on
// those bf16 values -- the post-attention RMSNorm launch disappears.
template <int EM, bool NORM = false>
__global__ void __launch_bounds__(256) route_kernel(const uint16_t* __restrict__ h, const uint16_t* __restrict__ wr,
                                                    int H, int E, int k, int renorm, float* __restrict__ w,
                                                    int32_t* __restrict__ ids, const uint16_t* __restrict__ norm_w = nullptr,
                                                    float eps = 0.f, uint16_t* __restrict__ hn = nullptr) {
  __shared__ float red[4][EM];
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float acc[EM];
#pragma unroll
  for (int e = 0; e < EM; ++e) acc[e] = 0.f;
  const uint16_t* hr = h + static_cast<int64_t>(t) * H;
  float scale = 1.f;
  if constexpr (NORM) {
    float ss = 0.f;
    for (int c = threadIdx.x; c < H / 8; c += 256) {
      float x[8];
      unpack8(ld16(hr + c * 8), x);
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += x[i] * x[i];
    }
    ss = wave_sum(ss);
    if (lane == 0) red[wid][0] = ss;
    __syncthreads();
    ss = red[0][0] + red[1][0] + red[2][0] + red[3][0];
    __syncthreads();  // red is reused for the router sums below
    scale = rsqrtf(ss / static_cast<float>(H) + eps);
  }
  for (int c = threadIdx.x; c < H / 8; c += 256) {
    float x[8];
    unpack8(ld16(hr + c * 8), x);
    if constexpr (NORM) {
      float g[8];
      unpack8(ld16(norm_w + c * 8), g);
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = x[i] * scale * g[i];
      const uint4 q = pack8(x);
      st16(hn + static_cast<int64_t>(t) * H + c * 8, q);
      unpack8(q, x);  // route on the bf16 values the experts will see
    }
#pragma unroll
    for (int e = 0; e < EM; ++e) {
      if (e < E) {
        float r[8];
        unpack8(ld16(wr + static_cast<int64_t>(e) * H + c * 8), r);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[e] += x[i] * r[i];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EM; ++e) {
    const float v = wave_sum(acc[e]);
    if (lane == 0) red[wid][e] = v;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  float v[EM];
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) {
    v[e] = red[0][e] + red[1][e] + red[2][e] + red[3][e];
    mx = fmaxf(mx, v[e]);
  }
  float den = 0.f;
  for (int e = 0; e < E; ++e) den += __expf(v[e] - mx);
  unsigned long long used = 0;
  float sel[16];
  int sid[16];
  float ssum = 0.f;
  for (int j = 0; j < k; ++j) {
    int best = -1;
    float bv = -INFINITY;
    for (int e = 0; e < E; ++e)
      if (!((used >> e) & 1ull) && (best < 0 || v[e] > bv)) { best = e; bv = v[e]; }
    used |= 1ull << best;
    sid[j] = best;
    sel[j] = __expf(bv - mx) / den;
    ssum += sel[j];
  }
  for (int j = 0; j < k; ++j) {
    w[static_cast<int64_t>(t) * k + j] = renorm ? sel[j] / ssum : sel[j];
    ids[static_cast<int64_t>(t) * k + j] = sid[j];
  }
}

// One-round-trip router (route2): 512 threads, each owning CPT 8-element chunks of the
// hidden row; every load the workgroup needs (the row, the norm weight, all E router
// rows) is issued before any arithmetic, so the launch costs one memory latency instead
// of route_kernel's three dependent rounds (norm pass, then per-chunk router loads):
// Mixtral batch 1 spent 10.8 us per layer in route_kernel<8, true> (profiles/
// r4_mixtral_c1_kernels.md) on 8 KB of activations + 64 KB of router weights.
// Single-token steps (batch-1 decode) can take the expert layout of moe_align in the
// same launch (RA.sorted_rows != nullptr): the one workgroup that routed the token
// writes offsets / sorted_rows / dest exactly as align_kernel would for T = 1 (top-k
// experts are distinct, so each holds at most one row) -- one launch less per layer.
struct RouteAlign {
  int32_t* sorted_rows;  // [cap]
  int32_t* offsets;      // [E_local + 1]
  int32_t* dest;         // [k]
  int E_local, expert_offset, block_m, cap;
};

// Wave 0 of route2_kernel: the same selection with lane e holding expert e (E <= 64):
// the router sums (fixed order over the waves), the softmax max / denominator and each
// of the k argmax rounds are wave reductions instead of thread 0's serial loops (about
// 2 us of dependent LDS reads and branches per launch at Mixtral batch 1). Ties go to
// the lowest expert index (as the reference top-k); the softmax denominator is a tree sum.
template <int EM, int NWV>
__device__ __forceinline__ void route_select_wave(const float (*red)[EM + 1], int E, int k, int renorm, int t,
                                                  float* __restrict__ w, int32_t* __restrict__ ids,
                                                  const RouteAlign& ra, bool align, int* s_off, int* s_pos) {
  const int lane = threadIdx.x & 63;
  float v = -INFINITY;
  if (lane < E) {
    v = 0.f;
#pragma unroll
    for (int q = 0; q < NWV; ++q) v += red[q][lane];
  }
  const float mx = wave_max(v);
  const float den = wave_sum(lane < E ? __expf(v - mx) : 0.f);
  bool used = false;
  float ssum = 0.f, my_sel = 0.f;
  int my_id = 0;
  for (int j = 0; j < k; ++j) {
    // argmax over the unused experts, lowest index on ties
    float bv = (lane < E && !used) ? v : -INFINITY;
    int bi = (lane < E && !used) ? lane : 64;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    const float sel = __expf(bv - mx) / den;
    ssum += sel;
    if (lane == bi) used = true;
    if (lane == j) { my_sel = sel; my_id = bi; }
    if (align && lane == 0) s_pos[j] = bi;  // expert ids for now; rows below
  }
  if (lane < k) {
    w[static_cast<int64_t>(t) * k + lane] = renorm ? my_sel / ssum : my_sel;
    ids[static_cast<int64_t>(t) * k + lane] = my_id;
  }
  if (align && lane == 0) {  // align_kernel's layout for the k pairs of this one token
    int cnt[EM];
    for (int e = 0; e < ra.E_local; ++e) cnt[e] = 0;
    for (int j = 0; j < k; ++j) {
      const int e = s_pos[j] - ra.expert_offset;
      if (e >= 0 && e < ra.E_local) ++cnt[e];
    }
    s_off[0] = 0;
    for (int e = 0; e < ra.E_local; ++e) s_off[e + 1] = s_off[e] + (cnt[e] + ra.block_m - 1) / ra.block_m * ra.block_m;
    for (int j = 0; j < k; ++j) {
      const int e = s_pos[j] - ra.expert_offset;
      s_pos[j] = (e >= 0 && e < ra.E_local) ? s_off[e] : -1;  // distinct experts: one row each
    }
  }
}

template <int EM, bool NORM, int CPT>
__global__ void __launch_bounds__(512) route2_kernel(const uint16_t* __restrict__ h, const uint16_t* __restrict__ wr,
                                                     int H, int E, int k, int renorm, float* __restrict__ w,
                                                     int32_t* __restrict__ ids, const uint16_t* __restrict__ norm_w,
                                                     float eps, uint16_t* __restrict__ hn, RouteAlign ra) {
  constexpr int NWV = 8;
  __shared__ float red[NWV][EM + 1];
  __shared__ int s_off[EM + 1], s_pos[16];
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nch = H / 8;
  const uint16_t* hr = h + static_cast<int64_t>(t) * H;
  uint4 xv[CPT], gv[CPT], rv[CPT][EM];
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = min(threadIdx.x + 512 * i, nch - 1);
    xv[i] = ld16(hr + c * 8);
    if constexpr (NORM) gv[i] = ld16(norm_w + c * 8);
#pragma unroll
    for (int e = 0; e < EM; ++e) rv[i][e] = ld16(wr + static_cast<int64_t>(min(e, E - 1)) * H + c * 8);
  }
  float scale = 1.f;
  if constexpr (NORM) {
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      if (threadIdx.x + 512 * i >= nch) break;
      float x[8];
      unpack8(xv[i], x);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += x[j] * x[j];
    }
    ss = wave_sum(ss);
    if (lane == 0) red[wid][EM] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int v = 0; v < NWV; ++v) tot += red[v][EM];
    scale = rsqrtf(tot / static_cast<float>(H) + eps);
  }
  float acc[EM];
#pragma unroll
  for (int e = 0; e < EM; ++e) acc[e] = 0.f;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + 512 * i;
    if (c >= nch) break;
    float x[8];
    unpack8(xv[i], x);
    if constexpr (NORM) {
      float g[8];
      unpack8(gv[i], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = x[j] * scale * g[j];
      const uint4 q = pack8(x);
      st16(hn + static_cast<int64_t>(t) * H + c * 8, q);
      unpack8(q, x);  // route on the bf16 values the experts will see
    }
#pragma unroll
    for (int e = 0; e < EM; ++e) {
      float r[8];
      unpack8(rv[i][e], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[e] += x[j] * r[j];
    }
  }
#pragma unroll
  for (int e = 0; e < EM; ++e) {
    const float v = wave_sum(acc[e]);
    if (lane == 0) red[wid][e] = v;
  }
  __syncthreads();
  const bool align = ra.sorted_rows != nullptr;  // T == 1 (host-checked)
  if (wid == 0) route_select_wave<EM, NWV>(red, E, k, renorm, t, w, ids, ra, align, s_off, s_pos);
  if (!align) return;
  __syncthreads();
  for (int e = threadIdx.x; e <= ra.E_local; e += blockDim.x) ra.offsets[e] = s_off[e];
  for (int j = threadIdx.x; j < k; j += blockDim.x) ra.dest[j] = s_pos[j];
  for (int p = threadIdx.x; p < ra.cap; p += blockDim.x) {
    int r = -1;
    for (int j = 0; j < k; ++j)
      if (s_pos[j] == p) r = 0;
    ra.sorted_rows[p] = r;
  }
}

int moe_route(const uint16_t* h, const uint16_t* wr, int T, int H, int E, int k, int renorm, float* w, int32_t* ids,
              hipStream_t st, const uint16_t* norm_w, float eps, uint16_t* hn, int32_t* al_rows, int32_t* al_offs,
              int32_t* al_dest, int al_E, int al_eoff, int al_bm) {
  if (T <= 0) return 0;
  if (H % 8 || E < 1 || E > 64 || k < 1 || k > 16 || k > E) return 1;
  if ((norm_w == nullptr) != (hn == nullptr)) return 1;
  const dim3 g(T), b(256);
  RouteAlign ra{nullptr, nullptr, nullptr, 0, 0, 1, 0};
  if (al_rows != nullptr) {  // the layout in the same launch: one token, <= 8 local experts
    if (T != 1 || E > 8 || al_E < 1 || al_E > 8 || al_bm < 1 || al_offs == nullptr || al_dest == nullptr) return 1;
    const int cap = (k + al_E * (al_bm - 1) + al_bm - 1) / al_bm * al_bm;
    ra = RouteAlign{al_rows, al_offs, al_dest, al_E, al_eoff, al_bm, cap};
  }
  // up to 8 experts and 4 chunks per thread (H <= 16384): the one-round-trip router
  if (E <= 8 && H <= 8 * 512 * 4) {
    const int cpt = (H / 8 + 511) / 512;
#define XGK_R2(NORM, CPT)                                                                                         \
  hipLaunchKernelGGL((route2_kernel<8, NORM, CPT>), g, dim3(512), 0, st, h, wr, H, E, k, renorm, w, ids, norm_w, \
                     eps, hn, ra)
    if (norm_w != nullptr) {
      if (cpt == 1) XGK_R2(true, 1);
      else if (cpt == 2) XGK_R2(true, 2);
      else XGK_R2(true, 4);
    } else {
      if (cpt == 1) XGK_R2(false, 1);
      else if (cpt == 2) XGK_R2(false, 2);
      else XGK_R2(false, 4);
    }
#undef XGK_R2
    return 0;
  }
  if (ra.sorted_rows != nullptr) return 1;
  if (norm_w != nullptr) {
    if (E <= 8) hipLaunchKernelGGL((route_kernel<8, true>), g, b, 0, st, h, wr, H, E, k, renorm, w, ids, norm_w, eps, hn);
    else if (E <= 16) hipLaunchKernelGGL((route_kernel<16, true>), g, b, 0, st, h, wr, H, E, k, renorm, w, ids, norm_w, eps, hn);
    else hipLaunchKernelGGL((route_kernel<64, true>), g, b, 0, st, h, wr, H, E, k, renorm, w, ids, norm_w, eps, hn);
    return 0;
  }
  if (E <= 8)
    hipLaunchKernelGGL((route_kernel<8, false>), g, b, 0, st, h, wr, H, E, k, renorm, w, ids, nullptr, 0.f, nullptr);
  else if (E <= 16)
    hipLaunchKernelGGL((route_kernel<16, false>), g, b, 0, st, h, wr, H, E, k, renorm, w, ids, nullptr, 0.f, nullptr);
  else
    hipLaunchKernelGGL((route_kernel<64, false>), g, b, 0, st, h, wr, H, E, k, renorm, w, ids, nullptr, 0.f, nullptr);
  return 0;
}

// ---------------------------------------------------------------- layout
// Expert-parallel aware: a pair (t, j) whose global expert ids[t*k+j] is outside
// [expert_offset, expert_offset + E) belongs to another rank: dest = -1, not placed.
// sorted_rows holds cap = T*k + E*(block_m-1) rounded up to block_m entries (-1 = pad);
// offsets[E+1] are block_m-padded segment starts; dest[t*k+j] = padded row of the pair.
__global__ void __launch_bounds__(1024) align_kernel(const int32_t* __restrict__ ids, int n_pairs, int k, int E,
                                                     int expert_offset, int block_m, int32_t* __restrict__ sorted_rows,
                                                     int32_t* __restrict__ offsets, int32_t* __restrict__ dest,
                                                     int cap) {
  __shared__ int cnt[256];
  __shared__ int off[257];
  __shared__ int fill[256];
  for (int e = threadIdx.x; e < E; e += blockDim.x) { cnt[e] = 0; fill[e] = 0; }
  __syncthreads();
  for (int i = threadIdx.x; i < n_pairs; i += blockDim.x) {
    const int e = ids[i] - expert_offset;
    if (e >= 0 && e < E) atomicAdd(&cnt[e], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    off[0] = 0;
    for (int e = 0; e < E; ++e) off[e + 1] = off[e] + (cnt[e] + block_m - 1) / block_m * block_m;
  }
  __syncthreads();
  for (int e = threadIdx.x; e <= E; e += blockDim.x) offsets[e] = off[e];
  for (int p = threadIdx.x; p < cap; p += blockDim.x) sorted_rows[p] = -1;
  __syncthreads();
  for (int i = threadIdx.x; i < n_pairs; i += blockDim.x) {
    const int e = ids[i] - expert_offset;
    if (e < 0 || e >= E) {
      dest[i] = -1;
      continue;
    }
    const int pos = off[e] + atomicAdd(&fill[e], 1);
    sorted_rows[pos] = i / k;
    dest[i] = pos;
  }
}

void moe_align(const int32_t* ids, int T, int k, int E, int expert_offset, int block_m, int32_t* sorted_rows,
               int32_t* offsets, int32_t* dest, hipStream_t st) {
  int cap = T * k + E * (block_m - 1);
  cap = (cap + block_m - 1) / block_m * block_m;
  hipLaunchKernelGGL(align_kernel, dim3(1), dim3(1024), 0, st, ids, T * k, k, E, expert_offset, block_m, sorted_rows,
                     offsets, dest, cap);
}

// ---------------------------------------------------------------- combine
// out[t] = sum_j w[t, j] * sum_s part[s][dest[t*k + j]]   (dest < 0: another rank's expert)
// y is either bf16 [P, H] (S == 0) or fp32 split-K partials [S, P, H].
template <int SP>
__global__ void __launch_bounds__(256) combine_kernel(const void* __restrict__ y, int S, int P,
                                                      const int32_t* __restrict__ dest, const float* __restrict__ w,
                                                      void* __restrict__ out, int k, int H, int out_f32) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const int p = dest[t * k + j];
      if (p < 0) continue;
      const float wt = w[t * k + j];
      float f[8];
      if constexpr (SP == 0) {
        unpack8(ld16(static_cast<const uint16_t*>(y) + static_cast<int64_t>(p) * H + c * 8), f);
      } else {
        float4 a[SP], b[SP];
#pragma unroll
        for (int s = 0; s < SP; ++s) {
          const float* q = static_cast<const float*>(y) + (static_cast<int64_t>(s) * P + p) * H + c * 8;
          a[s] = *reinterpret_cast<const float4*>(q);
          b[s] = *reinterpret_cast<const float4*>(q + 4);
        }
        for (int i = 0; i < 8; ++i) f[i] = 0.f;
#pragma unroll
        for (int s = 0; s < SP; ++s) {
          f[0] += a[s].x; f[1] += a[s].y; f[2] += a[s].z; f[3] += a[s].w;
          f[4] += b[s].x; f[5] += b[s].y; f[6] += b[s].z; f[7] += b[s].w;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += wt * f[i];
    }
    if (out_f32) {  // fp32 rows for a TP all-reduce: no bf16 rounding, no cast launch
      float* o = static_cast<float*>(out) + static_cast<int64_t>(t) * H + c * 8;
      *reinterpret_cast<float4*>(o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      *reinterpret_cast<float4*>(o + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
    } else {
      st16(static_cast<uint16_t*>(out) + static_cast<int64_t>(t) * H + c * 8, pack8(acc));
    }
  }
}

// Fused-decode form: resid[t] += sum_j w[t, j] * sum_s part[s][dest[t*k + j]] in place
// (bf16 residual stream) and ss[c * T + t] = sum over 1024-column chunk c of the new
// residual row squared (the next layer's RMSNorm statistics, read by gemm_m64g).
// One workgroup per token; H <= 8192.
template <int SP>
__global__ void __launch_bounds__(256) combine_resid_kernel(const float* __restrict__ part, int P,
                                                            const int32_t* __restrict__ dest,
                                                            const float* __restrict__ w, uint16_t* __restrict__ resid,
                                                            float* __restrict__ ss, int T, int k, int H) {
  __shared__ float red[4][8];
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float sq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // per 1024-column chunk
  for (int c = threadIdx.x; c < H / 8; c += 256) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const int p = dest[t * k + j];
      if (p < 0) continue;
      const float wt = w[t * k + j];
      float f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int s = 0; s < SP; ++s) {
        const float* q = part + (static_cast<int64_t>(s) * P + p) * H + c * 8;
        const float4 a = *reinterpret_cast<const float4*>(q);
        const float4 b = *reinterpret_cast<const float4*>(q + 4);
        f[0] += a.x; f[1] += a.y; f[2] += a.z; f[3] += a.w;
        f[4] += b.x; f[5] += b.y; f[6] += b.z; f[7] += b.w;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += wt * f[i];
    }
    uint16_t* rp = resid + static_cast<int64_t>(t) * H + c * 8;
    float r[8];
    unpack8(ld16(rp), r);
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] += acc[i];
    const uint4 o = pack8(r);
    st16(rp, o);
    unpack8(o, r);  // statistics of the rounded bf16 residual
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) v += r[i] * r[i];
    const int chunk = (c * 8) >> 10;
#pragma unroll
    for (int q = 0; q < 8; ++q) sq[q] += chunk == q ? v : 0.f;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float v = wave_sum(sq[q]);
    if (lane == 0) red[wid][q] = v;
  }
  __syncthreads();
  if (threadIdx.x < H / 1024) {
    const int q = threadIdx.x;
    ss[static_cast<int64_t>(q) * T + t] = red[0][q] + red[1][q] + red[2][q] + red[3][q];
  }
}

int moe_combine_resid(const float* part, int S, int P, const int32_t* dest, const float* w, uint16_t* resid, float* ss,
                      int T, int k, int H, hipStream_t st) {
  if (T <= 0) return 0;
  if (H % 1024 || H > 8192) return 1;
  const dim3 g(T), b(256);
  switch (S) {
    case 1: hipLaunchKernelGGL(combine_resid_kernel<1>, g, b, 0, st, part, P, dest, w, resid, ss, T, k, H); return 0;
    case 2: hipLaunchKernelGGL(combine_resid_kernel<2>, g, b, 0, st, part, P, dest, w, resid, ss, T, k, H); return 0;
    case 4: hipLaunchKernelGGL(combine_resid_kernel<4>, g, b, 0, st, part, P, dest, w, resid, ss, T, k, H); return 0;
    default: return 1;
  }
}

int moe_combine(const void* y, int S, int P, const int32_t* dest, const float* w, void* out, int T, int k, int H,
                hipStream_t st, int out_f32) {
  if (T <= 0) return 0;
  if (H % 8) return 1;
  const dim3 g(T), b(256);
  switch (S) {
    case 0: hipLaunchKernelGGL(combine_kernel<0>, g, b, 0, st, y, S, P, dest, w, out, k, H, out_f32); return 0;
    case 1: hipLaunchKernelGGL(combine_kernel<1>, g, b, 0, st, y, S, P, dest, w, out, k, H, out_f32); return 0;
    case 2: hipLaunchKernelGGL(combine_kernel<2>, g, b, 0, st, y, S, P, dest, w, out, k, H, out_f32); return 0;
    case 4: hipLaunchKernelGGL(combine_kernel<4>, g, b, 0, st, y, S, P, dest, w, out, k, H, out_f32); return 0;
    default: return 1;
  }
}

// ---------------------------------------------------------------- expert-parallel dispatch
// (llama.py LlamaLayer._moe_alltoall: a rank routes its token slice and ships each
// (token, choice) row to the rank owning that expert, rank r owning global experts
// [r * E_local, (r + 1) * E_local).)
//
// ep_plan: ONE workgroup plans the whole dispatch. Pair i goes to d = ids[i] / E_local
// at a stable, deterministic slot: slot[i] = base[d] + #{i' < i : d(i') = d}, where
// base[d] = d * cap (fixed-capacity layout: a graph-capturable all_to_all with equal
// splits) or the exclusive prefix of the per-destination counts (packed layout: the
// count-exact all_to_all of eager steps). send_eid[slot] = the owner's LOCAL expert id;
// unused capacity slots get -1, which the owner's moe_align skips (no padding rows
// routed to any expert). counts[d] = pairs for rank d. Pairs with an out-of-range id
// get slot -1 (never sent, never combined).
// Each thread owns a contiguous chunk of pairs: per-destination counts in registers
// -> block exclusive scan (wave shuffles + per-wave totals in LDS) -> second pass
// assigns slots in pair order.
constexpr int EP_MAX_RANKS = 8;
constexpr int EP_PLAN_THREADS = 1024;

__global__ void __launch_bounds__(EP_PLAN_THREADS) ep_plan_kernel(const int32_t* __restrict__ ids, int n_pairs,
                                                                   int E_local, int tp, int cap, int packed,
                                                                   int32_t* __restrict__ slot,
                                                                   int32_t* __restrict__ send_eid,
                                                                   int32_t* __restrict__ counts) {
  constexpr int NWAVE = EP_PLAN_THREADS / 64;
  __shared__ int wave_tot[EP_MAX_RANKS][NWAVE];
  __shared__ int base_s[EP_MAX_RANKS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int chunk = (n_pairs + EP_PLAN_THREADS - 1) / EP_PLAN_THREADS;
  const int i0 = min(n_pairs, tid * chunk), i1 = min(n_pairs, i0 + chunk);
  const int n_eid = packed ? n_pairs : tp * cap;
  if (!packed)
    for (int s = tid; s < n_eid; s += EP_PLAN_THREADS) send_eid[s] = -1;
  int cnt[EP_MAX_RANKS];
#pragma unroll
  for (int d = 0; d < EP_MAX_RANKS; ++d) cnt[d] = 0;
  const int n_exp = E_local * tp;
  for (int i = i0; i < i1; ++i) {
    const int e = ids[i];
    const int d = (e >= 0 && e < n_exp) ? e / E_local : -1;
#pragma unroll
    for (int q = 0; q < EP_MAX_RANKS; ++q) cnt[q] += (d == q);
  }
  // exclusive prefix over threads, per destination
  int excl[EP_MAX_RANKS];
#pragma unroll
  for (int d = 0; d < EP_MAX_RANKS; ++d) {
    int v = cnt[d];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(v, o, 64);
      if (lane >= o) v += u;
    }
    excl[d] = v - cnt[d];
    if (lane == 63) wave_tot[d][wid] = v;
  }
  __syncthreads();  // also orders the -1 fill before the slot writes below
  if (tid == 0) {
    int acc = 0;
    for (int d = 0; d < EP_MAX_RANKS; ++d) {
      int tot = 0;
      for (int w = 0; w < NWAVE; ++w) tot += wave_tot[d][w];
      base_s[d] = packed ? acc : d * cap;
      if (d < tp) {
        counts[d] = tot;
        acc += tot;
      }
    }
  }
#pragma unroll
  for (int d = 0; d < EP_MAX_RANKS; ++d)
    for (int w = 0; w < wid; ++w) excl[d] += wave_tot[d][w];
  __syncthreads();
  for (int i = i0; i < i1; ++i) {
    const int e = ids[i];
    const int d = (e >= 0 && e < n_exp) ? e / E_local : -1;
    int s = -1;
#pragma unroll
    for (int q = 0; q < EP_MAX_RANKS; ++q)
      if (d == q) s = base_s[q] + excl[q]++;
    slot[i] = s;
    if (s >= 0) send_eid[s] = e - d * E_local;
  }
}

int ep_plan(const int32_t* ids, int n_pairs, int E_local, int tp, int cap, int packed, int32_t* slot, int32_t* send_eid,
            int32_t* counts, hipStream_t st) {
  if (tp < 1 || tp > EP_MAX_RANKS || E_local < 1 || n_pairs < 0 || (!packed && cap < 0)) return 1;
  hipLaunchKernelGGL(ep_plan_kernel, dim3(1), dim3(EP_PLAN_THREADS), 0, st, ids, n_pairs, E_local, tp, cap, packed,
                     slot, send_eid, counts);
  return 0;
}

// ep_scatter: send[slot[i]] = x[i / k] (one wave per pair, 16-B vector copies).
__global__ void __launch_bounds__(256) ep_scatter_kernel(const uint16_t* __restrict__ x, int64_t x_stride, int k,
                                                         const int32_t* __restrict__ slot, int n_pairs, int H,
                                                         uint16_t* __restrict__ send) {
  const int pair = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (pair >= n_pairs) return;
  const int s = slot[pair];
  if (s < 0) return;
  const uint16_t* src = x + static_cast<int64_t>(pair / k) * x_stride;
  uint16_t* dst = send + static_cast<int64_t>(s) * H;
  for (int c = lane; c < H / 8; c += 64) st16(dst + 8 * c, ld16(src + 8 * c));
}

int ep_scatter(const uint16_t* x, int64_t x_stride, int k, const int32_t* slot, int n_pairs, int H, uint16_t* send,
               hipStream_t st) {
  if (n_pairs <= 0) return 0;
  if (H % 8 || x_stride % 8 || k < 1) return 1;
  hipLaunchKernelGGL(ep_scatter_kernel, dim3((n_pairs + 3) / 4), dim3(256), 0, st, x, x_stride, k, slot, n_pairs, H,
                     send);
  return 0;
}


}  // namespace xgk
