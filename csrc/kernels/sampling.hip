// K9: token sampling on the logits rows of a decode/prefill step.
//
// argmax_logprob: greedy path. One 1024-thread workgroup per row streams the
//   row once (16-B loads of 8 bf16 / 4 f32), tracking the (max, argmax) pair and
//   an online log-sum-exp, so the chosen token's logprob comes for free.
// sample_gumbel: temperature (+ top-k / top-p) sampling in one kernel:
//   * top-p/top-k are applied through a threshold on the logit found by a
//     bisection over [row max - 30*T, row max] on the L2-resident row
//     (<= 24 passes), no sort;
//   * the draw is Gumbel-max: argmax(logit/T - log(-log u)), u from a
//     per-(seed, step, row, index) counter hash, so a fixed seed reproduces.
#include "common.h"

namespace xgk {

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

template <typename T>
__device__ __forceinline__ int load_vec(const T* row, int i, float* f);

template <>
__device__ __forceinline__ int load_vec<uint16_t>(const uint16_t* row, int i, float* f) {
  unpack8(ld16(row + i * 8), f);
  return 8;
}
template <>
__device__ __forceinline__ int load_vec<float>(const float* row, int i, float* f) {
  const float4 v = *reinterpret_cast<const float4*>(row + i * 4);
  f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
  return 4;
}
template <typename T> struct VecW { static constexpr int W = 8; };
template <> struct VecW<float> { static constexpr int W = 4; };

template <typename T>
__device__ __forceinline__ float scalar_at(const T* row, int i);
template <> __device__ __forceinline__ float scalar_at<uint16_t>(const uint16_t* r, int i) { return bf2f(r[i]); }
template <> __device__ __forceinline__ float scalar_at<float>(const float* r, int i) { return r[i]; }

// reduce (val, idx) max with lowest index on ties, plus (m, s) log-sum-exp
struct ArgLse {
  float v; int i; float m; float s;
};
__device__ __forceinline__ ArgLse merge(ArgLse a, ArgLse b) {
  ArgLse r;
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) { r.v = b.v; r.i = b.i; } else { r.v = a.v; r.i = a.i; }
  r.m = fmaxf(a.m, b.m);
  r.s = (a.m == -INFINITY ? 0.f : a.s * __expf(a.m - r.m)) + (b.m == -INFINITY ? 0.f : b.s * __expf(b.m - r.m));
  return r;
}

template <typename T>
__global__ void __launch_bounds__(1024) argmax_kernel(const T* __restrict__ logits, int64_t stride, int V,
                                                      int32_t* __restrict__ out_tok, float* __restrict__ out_lp) {
  constexpr int W = VecW<T>::W;
  const T* row = logits + blockIdx.x * stride;
  ArgLse a{-INFINITY, 0x7fffffff, -INFINITY, 0.f};
  const int nv = V / W;
  for (int c = threadIdx.x; c < nv; c += blockDim.x) {
    float f[8];
    load_vec<T>(row, c, f);
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const float x = f[k];
      if (x > a.v) { a.v = x; a.i = c * W + k; }
      if (x > a.m) { a.s = a.s * __expf(a.m - x) + 1.f; a.m = x; } else { a.s += __expf(x - a.m); }
    }
  }
  for (int i = nv * W + threadIdx.x; i < V; i += blockDim.x) {
    const float x = scalar_at<T>(row, i);
    if (x > a.v) { a.v = x; a.i = i; }
    if (x > a.m) { a.s = a.s * __expf(a.m - x) + 1.f; a.m = x; } else { a.s += __expf(x - a.m); }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgLse b{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64), __shfl_xor(a.m, o, 64), __shfl_xor(a.s, o, 64)};
    a = merge(a, b);
  }
  __shared__ ArgLse red[16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    ArgLse r = red[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = merge(r, red[w]);
    out_tok[blockIdx.x] = r.i;
    if (out_lp) out_lp[blockIdx.x] = r.v - (r.m + __logf(r.s));
  }
}

// --------------------------------------------------------------------------
// Gumbel-max sampling with optional top-k / top-p thresholds.
// temps[row] <= 0 means greedy for that row.
// --------------------------------------------------------------------------
template <typename T>
__device__ float block_reduce_max(float v, float* sh) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r = fmaxf(r, sh[w]);
  return r;
}
__device__ float block_reduce_sum(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r += sh[w];
  return r;
}

template <typename T>
__global__ void __launch_bounds__(1024) sample_kernel(const T* __restrict__ logits, int64_t stride, int V,
                                                      const float* __restrict__ temps,
                                                      const float* __restrict__ top_ps,
                                                      const int32_t* __restrict__ top_ks,
                                                      const uint64_t* __restrict__ seeds, uint64_t step,
                                                      int32_t* __restrict__ out_tok, float* __restrict__ out_lp) {
  __shared__ float sh[16];
  __shared__ ArgLse red[16];
  const T* row = logits + blockIdx.x * stride;
  const float temp = temps[blockIdx.x];
  const float top_p = top_ps ? top_ps[blockIdx.x] : 1.f;
  const int top_k = top_ks ? top_ks[blockIdx.x] : 0;
  const bool greedy = !(temp > 0.f);
  const float it = greedy ? 1.f : 1.f / temp;

  // pass 1: row max and log-sum-exp of logits/T
  float mx = -INFINITY, se = 0.f;
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float x = scalar_at<T>(row, i) * it;
    if (x > mx) { se = se * __expf(mx - x) + 1.f; mx = x; } else { se += __expf(x - mx); }
  }
  const float M = block_reduce_max<T>(mx, sh);
  const float S = block_reduce_sum(mx == -INFINITY ? 0.f : se * __expf(mx - M), sh);
  const float logZ = M + __logf(S);

  // threshold: keep x/T >= thr. Bisection on mass (top-p) and count (top-k).
  // thr_p: the largest threshold whose kept mass is still >= top_p;
  // thr_k: the smallest threshold that keeps <= top_k tokens; keep x >= max.
  float thr = -INFINITY;
  const bool use_p = !greedy && top_p < 1.f, use_k = !greedy && top_k > 0 && top_k < V;
  if (use_p || use_k) {
    float lo_p = M - 40.f, hi_p = M, lo_k = M - 40.f, hi_k = M;
    for (int iter = 0; iter < 24; ++iter) {
      const float mid_p = 0.5f * (lo_p + hi_p), mid_k = 0.5f * (lo_k + hi_k);
      float mass = 0.f, cnt = 0.f;
      for (int i = threadIdx.x; i < V; i += blockDim.x) {
        const float x = scalar_at<T>(row, i) * it;
        if (x >= mid_p) mass += __expf(x - logZ);
        if (x >= mid_k) cnt += 1.f;
      }
      mass = block_reduce_sum(mass, sh);
      cnt = block_reduce_sum(cnt, sh);
      if (mass >= top_p) lo_p = mid_p; else hi_p = mid_p;
      if (cnt <= static_cast<float>(top_k)) hi_k = mid_k; else lo_k = mid_k;
    }
    if (use_p) thr = lo_p;
    if (use_k) thr = fmaxf(thr, hi_k);
    thr = fminf(thr, M);  // the argmax token is always kept
  }

  // pass 2: Gumbel-max draw over kept tokens
  const uint64_t seed = seeds ? seeds[blockIdx.x] : 0x9E3779B97F4A7C15ull;
  // the stream depends only on (seed, step): rows that share a seed draw identically
  const uint32_t key = hash32(static_cast<uint32_t>(seed) ^ hash32(static_cast<uint32_t>(seed >> 32) + 0x85ebca6bU) ^
                              hash32(static_cast<uint32_t>(step) * 0x27d4eb2fU + 0x165667b1U));
  ArgLse a{-INFINITY, 0x7fffffff, -INFINITY, 0.f};
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float x = scalar_at<T>(row, i) * it;
    if (x < thr) continue;
    float score = x;
    if (!greedy) {
      const uint32_t hsh = hash32(key ^ hash32(static_cast<uint32_t>(i) * 0x9E3779B9U));
      const float u = (static_cast<float>(hsh >> 8) + 0.5f) * (1.f / 16777216.f);
      score = x - __logf(-__logf(u));
    }
    if (score > a.v) { a.v = score; a.i = i; a.m = x; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgLse b{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64), __shfl_xor(a.m, o, 64), 0.f};
    if (b.v > a.v || (b.v == a.v && b.i < a.i)) a = b;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    ArgLse r = red[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
      if (red[w].v > r.v || (red[w].v == r.v && red[w].i < r.i)) r = red[w];
    out_tok[blockIdx.x] = r.i;
    if (out_lp) out_lp[blockIdx.x] = r.m - logZ;  // logprob under the temperature-scaled distribution
  }
}

void argmax_logprob(const void* logits, int is_f32, int64_t stride, int B, int V, int32_t* tok, float* lp,
                    hipStream_t st) {
  if (B <= 0) return;
  if (is_f32)
    hipLaunchKernelGGL(argmax_kernel<float>, dim3(B), dim3(1024), 0, st, (const float*)logits, stride, V, tok, lp);
  else
    hipLaunchKernelGGL(argmax_kernel<uint16_t>, dim3(B), dim3(1024), 0, st, (const uint16_t*)logits, stride, V,
                       tok, lp);
}

void sample_tokens(const void* logits, int is_f32, int64_t stride, int B, int V, const float* temps,
                   const float* top_ps, const int32_t* top_ks, const uint64_t* seeds, uint64_t step, int32_t* tok,
                   float* lp, hipStream_t st) {
  if (B <= 0) return;
  if (is_f32)
    hipLaunchKernelGGL(sample_kernel<float>, dim3(B), dim3(1024), 0, st, (const float*)logits, stride, V, temps,
                       top_ps, top_ks, seeds, step, tok, lp);
  else
    hipLaunchKernelGGL(sample_kernel<uint16_t>, dim3(B), dim3(1024), 0, st, (const uint16_t*)logits, stride, V,
                       temps, top_ps, top_ks, seeds, step, tok, lp);
}

// --------------------------------------------------------------------------
// K11 (part): per-segment sums of hidden rows for mean pooling (embeddings).
// out[s, :] += sum_{t in [cu[s], cu[s+1])} hidden[t, :]   (fp32 accumulate)
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256) segment_sum_kernel(const uint16_t* __restrict__ hidden, int H,
                                                          const int32_t* __restrict__ cu,
                                                          const int32_t* __restrict__ out_rows,
                                                          float* __restrict__ out) {
  const int s = blockIdx.x;
  const int dst = out_rows ? out_rows[s] : s;
  if (dst < 0) return;
  const int t0 = cu[s], t1 = cu[s + 1];
  for (int c = blockIdx.y * blockDim.x + threadIdx.x; c < H / 8; c += gridDim.y * blockDim.x) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int t = t0; t < t1; ++t) {
      float f[8];
      unpack8(ld16(hidden + static_cast<int64_t>(t) * H + c * 8), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += f[k];
    }
    float* o = out + static_cast<int64_t>(dst) * H + c * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] += acc[k];
  }
}

void segment_sum(const uint16_t* hidden, int H, const int32_t* cu, const int32_t* out_rows, float* out, int S,
                 hipStream_t st) {
  if (S <= 0) return;
  const int chunks = H / 8;
  const int gy = (chunks + 255) / 256;
  hipLaunchKernelGGL(segment_sum_kernel, dim3(S, gy), dim3(256), 0, st, hidden, H, cu, out_rows, out);
}

// Asynchronous scheduling: a step planned before the previous one finished has
// placeholder ids for its decode rows; ids[i] <- prev[src[i]] (the previous step's
// sampled token of that sequence) where src[i] >= 0. Runs first inside the decode
// graph (src all -1 on ordinary steps: a no-op).
__global__ void __launch_bounds__(256) subst_tokens_kernel(int32_t* __restrict__ ids, const int32_t* __restrict__ src,
                                                           const int32_t* __restrict__ prev, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int s = src[i];
    if (s >= 0) ids[i] = prev[s];
  }
}

void subst_tokens(int32_t* ids, const int32_t* src, const int32_t* prev, int n, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(subst_tokens_kernel, dim3((n + 255) / 256), dim3(256), 0, st, ids, src, prev, n);
}

// K11: embeddings output -- mean-pool + L2 normalise on the device. For each
// finished request i: v = acc[rows[i]] / counts[i]; out[i] = v / max(||v||, 1e-12);
// the accumulator row is re-zeroed for the slot's next owner. One workgroup per row.
__global__ void __launch_bounds__(256) mean_l2norm_rows_kernel(float* __restrict__ acc, const int32_t* __restrict__ rows,
                                                               const int32_t* __restrict__ counts,
                                                               float* __restrict__ out, int H) {
  __shared__ float red[4];
  const int i = blockIdx.x;
  float* a = acc + static_cast<int64_t>(rows[i]) * H;
  const float inv_n = 1.f / static_cast<float>(counts[i] > 0 ? counts[i] : 1);
  float s = 0.f;
  for (int c = threadIdx.x; c < H; c += blockDim.x) {
    const float v = a[c] * inv_n;
    s += v * v;
  }
  s = block_sum(s, red);
  const float scale = inv_n / fmaxf(sqrtf(s), 1e-12f);
  float* o = out + static_cast<int64_t>(i) * H;
  for (int c = threadIdx.x; c < H; c += blockDim.x) {
    o[c] = a[c] * scale;
    a[c] = 0.f;
  }
}

void mean_l2norm_rows(float* acc, const int32_t* rows, const int32_t* counts, float* out, int n, int H,
                      hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(mean_l2norm_rows_kernel, dim3(n), dim3(256), 0, st, acc, rows, counts, out, H);
}

}  // namespace xgk
