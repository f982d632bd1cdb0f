// K12: Mixture-of-Experts building blocks (Mixtral-style top-k routing).
//
//   moe_topk_softmax : router logits [T, E] -> top-k (weights, expert ids); the
//                      weights are the softmax over the selected k logits
//                      (== softmax-then-renormalise, Mixtral semantics) or the
//                      plain softmax probabilities when renorm == 0.
//   moe_align        : one workgroup builds the expert-sorted, block_m-padded
//                      row layout: sorted_rows[p] = token of padded row p (-1 =
//                      pad), expert_offsets[E+1], tile_expert[tile], dest[t*k+j]
//                      = padded row of (token t, choice j).
//   moe_grouped_gemm : out[p, :] = x[rows[p], :] @ W[e(p)]^T for every expert
//                      at once (W stored [E, N, K], the nn.Linear layout). A
//                      64x64 tile per workgroup: the gathered 64-row x slab is
//                      staged in LDS (XOR-swizzled, shared by the 4 waves), each
//                      wave streams its own 16 weight rows straight into MFMA
//                      B fragments (weights are read once: GEMV-regime rule),
//                      v_mfma_f32_16x16x32_bf16, next-chunk loads issued before
//                      the current chunk's MFMAs.
//   moe_combine      : out[t] = sum_j w[t, j] * y[dest[t*k + j]].
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

// ---------------------------------------------------------------- layout
// sorted_rows must hold T*k + E*(block_m-1) entries; tile_expert the same / block_m.
__global__ void __launch_bounds__(1024) align_kernel(const int32_t* __restrict__ ids, int n_pairs, int k, int E,
                                                     int block_m, int32_t* __restrict__ sorted_rows,
                                                     int32_t* __restrict__ offsets, int32_t* __restrict__ tile_expert,
                                                     int32_t* __restrict__ dest, int cap) {
  __shared__ int cnt[256];
  __shared__ int off[257];
  __shared__ int fill[256];
  for (int e = threadIdx.x; e < E; e += blockDim.x) { cnt[e] = 0; fill[e] = 0; }
  __syncthreads();
  for (int i = threadIdx.x; i < n_pairs; i += blockDim.x) atomicAdd(&cnt[ids[i]], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    off[0] = 0;
    for (int e = 0; e < E; ++e) off[e + 1] = off[e] + (cnt[e] + block_m - 1) / block_m * block_m;
  }
  __syncthreads();
  for (int e = threadIdx.x; e <= E; e += blockDim.x) offsets[e] = off[e];
  const int total = off[E];
  for (int p = threadIdx.x; p < cap; p += blockDim.x) sorted_rows[p] = -1;
  const int ntile_cap = cap / block_m;
  for (int tl = threadIdx.x; tl < ntile_cap; tl += blockDim.x) {
    const int p = tl * block_m;
    int e = -1;
    if (p < total)
      for (int x = 0; x < E; ++x)
        if (p >= off[x] && p < off[x + 1]) { e = x; break; }
    tile_expert[tl] = e;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n_pairs; i += blockDim.x) {
    const int e = ids[i];
    const int pos = off[e] + atomicAdd(&fill[e], 1);
    sorted_rows[pos] = i / k;
    dest[i] = pos;
  }
}

void moe_align(const int32_t* ids, int T, int k, int E, int block_m, int32_t* sorted_rows, int32_t* offsets,
               int32_t* tile_expert, int32_t* dest, hipStream_t st) {
  const int cap = T * k + E * (block_m - 1);
  hipLaunchKernelGGL(align_kernel, dim3(1), dim3(1024), 0, st, ids, T * k, k, E, block_m, sorted_rows, offsets,
                     tile_expert, dest, cap);
}

// ---------------------------------------------------------------- grouped GEMM
// tile 64 rows x 64 cols, K chunk 64. x rows gathered through rows[] when gather.
constexpr int GG_BM = 64, GG_BN = 64, GG_BK = 64;

__global__ void __launch_bounds__(256) grouped_gemm_kernel(const uint16_t* __restrict__ x,
                                                           const int32_t* __restrict__ rows,
                                                           const uint16_t* __restrict__ w, uint16_t* __restrict__ out,
                                                           const int32_t* __restrict__ tile_expert, int N, int K,
                                                           int gather) {
  const int tile = blockIdx.x;
  const int e = tile_expert[tile];
  if (e < 0) return;
  const int n0 = blockIdx.y * GG_BN;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  __shared__ __attribute__((aligned(16))) uint16_t xs[GG_BM * GG_BK];  // 8 KiB, [row][8 chunks] swizzled

  // staging role: 256 threads x 2 chunks of 16 B = 64 rows x 64 k
  int src_row[2];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int ci = threadIdx.x + it * 256;
    const int r = ci >> 3;
    const int p = tile * GG_BM + r;
    src_row[it] = gather ? rows[p] : p;
  }
  const uint16_t* wrow = w + (static_cast<int64_t>(e) * N + n0 + wid * 16 + li) * K;

  uint4 xr[2], wr[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int ci = threadIdx.x + it * 256;
      const int ch = ci & 7;
      xr[it] = src_row[it] >= 0 ? ld16(x + static_cast<int64_t>(src_row[it]) * K + k0 + ch * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) wr[ks] = ld16(wrow + k0 + ks * 32 + 8 * g);
  };
  auto lstore = [&]() {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int ci = threadIdx.x + it * 256;
      const int r = ci >> 3, ch = ci & 7;
      st16(xs + r * GG_BK + ((ch ^ (r & 7)) * 8), xr[it]);
    }
  };

  f32x4_t acc[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  gload(0);
  for (int k0 = 0; k0 < K; k0 += GG_BK) {
    __syncthreads();
    lstore();
    const uint4 wcur0 = wr[0], wcur1 = wr[1];
    __syncthreads();
    if (k0 + GG_BK < K) gload(k0 + GG_BK);
    // out^T tile for this wave: C[n = 16wid + li][m] ... we compute C = X . W^T with
    // A = X rows (from LDS), B = W^T (lane holds W[n = li][k = 8g + j])
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8_t bfrag = as_frag(ks == 0 ? wcur0 : wcur1);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int r = mt * 16 + li;
        const int ch = ks * 4 + g;
        const uint4 a = *reinterpret_cast<const uint4*>(xs + r * GG_BK + ((ch ^ (r & 7)) * 8));
        acc[mt] = mfma16x16x32(as_frag(a), bfrag, acc[mt]);
      }
    }
  }
  // C layout: acc[mt][r] = out[row = 16mt + 4g + r][col = 16wid + li]
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = tile * GG_BM + mt * 16 + 4 * g + r;
      out[static_cast<int64_t>(p) * N + n0 + wid * 16 + li] = f2bf(acc[mt][r]);
    }
}

void moe_grouped_gemm(const uint16_t* x, const int32_t* rows, const uint16_t* w, uint16_t* out, const int32_t* offs,
                      const int32_t* tile_expert, int max_tiles, int N, int K, int gather, int x_rows,
                      int num_experts, hipStream_t st) {
  (void)offs;
  (void)x_rows;
  (void)num_experts;
  if (max_tiles <= 0) return;
  hipLaunchKernelGGL(grouped_gemm_kernel, dim3(max_tiles, N / GG_BN), dim3(256), 0, st, x, rows, w, out, tile_expert,
                     N, K, gather);
}

// ---------------------------------------------------------------- combine
__global__ void __launch_bounds__(256) combine_kernel(const uint16_t* __restrict__ y, const int32_t* __restrict__ dest,
                                                      const float* __restrict__ w, uint16_t* __restrict__ out, int k,
                                                      int H) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const int p = dest[t * k + j];
      const float wt = w[t * k + j];
      if (wt == 0.f) continue;  // dropped (non-local) choice: its row may be unwritten
      float f[8];
      unpack8(ld16(y + static_cast<int64_t>(p) * H + c * 8), f);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += wt * f[i];
    }
    st16(out + static_cast<int64_t>(t) * H + c * 8, pack8(acc));
  }
}

void moe_combine(const uint16_t* y, const int32_t* dest, const float* w, uint16_t* out, int T, int k, int H,
                 hipStream_t st) {
  if (T <= 0) return;
  hipLaunchKernelGGL(combine_kernel, dim3(T), dim3(256), 0, st, y, dest, w, out, k, H);
}

void silu_and_mul(const uint16_t* in, uint16_t* out, int T, int F, int interleave16, hipStream_t st);
void moe_silu_mul_gather(const uint16_t* in, uint16_t* out, int rows, int F, hipStream_t st) {
  silu_and_mul(in, out, rows, F, 0, st);
}

}  // namespace xgk
