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
#include "glds.h"

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
  constexpr int U = 8;  // 16-B vectors in flight per thread
  const T* row = logits + blockIdx.x * stride;
  ArgLse a{-INFINITY, 0x7fffffff, -INFINITY, 0.f};
  const int nv = V / W;
  // batches of U vectors: every load of a batch is issued before any is used
  // (clamped, masked after), so a 128K-entry row costs ~2 memory round trips per
  // thread instead of one per vector; the log-sum-exp is updated once per batch
  for (int c0 = threadIdx.x; c0 < nv; c0 += U * blockDim.x) {
    uint4 raw[U];
#pragma unroll
    for (int u = 0; u < U; ++u) raw[u] = ld16(row + static_cast<int64_t>(min(c0 + u * (int)blockDim.x, nv - 1)) * W);
    float f[U][W];
    float bm = -INFINITY;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (W == 8) {
        unpack8(raw[u], f[u]);
      } else {
        f[u][0] = __uint_as_float(raw[u].x); f[u][1] = __uint_as_float(raw[u].y);
        f[u][2] = __uint_as_float(raw[u].z); f[u][3] = __uint_as_float(raw[u].w);
      }
      const bool ok = c0 + u * (int)blockDim.x < nv;
#pragma unroll
      for (int k = 0; k < W; ++k) {
        if (!ok) f[u][k] = -INFINITY;
        const float x = f[u][k];
        if (x > a.v) { a.v = x; a.i = (c0 + u * (int)blockDim.x) * W + k; }
        bm = fmaxf(bm, x);
      }
    }
    if (bm == -INFINITY) continue;
    const float mn = fmaxf(a.m, bm);
    float bs = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < W; ++k) bs += __expf(f[u][k] - mn);  // masked: exp(-inf) = 0
    a.s = (a.m == -INFINITY ? 0.f : a.s * __expf(a.m - mn)) + bs;
    a.m = mn;
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

// --------------------------------------------------------------------------
// Split-row sampler (sample v2): P workgroups per row, four launches, no bisection.
//   K1 samp_stats: per-chunk (max, sum exp) of y = logit / T.
//   K2 samp_hist1 (rows with top-p / top-k): a 1024-bin histogram of u = M - y over
//      [0, 40) -- fixed-point probability mass (u64, order-independent, so a fixed seed
//      reproduces) and counts -- merged into the row's global histogram with atomics;
//      the row's last workgroup (ticket) finds the boundary bins bp (top-p) and bk
//      (top-k) from the cumulative sums and re-zeroes the histogram.
//   K3 samp_hist2: the same over 1024 sub-bins of the two boundary bins -> (sp, sk).
//   K4 samp_draw: Gumbel-max over the kept tokens (bin, sub-bin) <= the boundary,
//      per chunk; the row's last workgroup merges the chunks in order.
// Kept set: top-p -- the smallest prefix by descending y whose mass reaches top_p, at
// sub-bin resolution (40 / 2^20 in y); top-k -- every token of the bins / sub-bins
// whose cumulative count stays <= k; the row's argmax always. The draw is the v1
// kernel's (same counter hash per (seed, step, index)). Each pass re-reads its chunk
// (L2-resident after K1) with batched loads.
namespace samp {
constexpr int NT = 256;       // threads per workgroup
constexpr int NB = 1024;      // bins per histogram level
constexpr int PMAX = 64;      // workgroups per row
constexpr float RANGE = 40.f; // u beyond this is never kept by top-p / top-k
constexpr float FIX = 1099511627776.f;  // 2^40: fixed-point probability mass

// per-row workspace (bytes), zero before the first launch; every ticket winner
// re-zeroes what it consumed, so each call leaves it zero
struct Row {
  float stats[PMAX][2];                 // K1 partials (m, s)
  float draw[PMAX][4];                  // K4 partials (score, idx bits, y, -)
  unsigned long long h1m[NB];
  unsigned int h1c[NB];
  unsigned long long h2m[NB];
  unsigned int h2c[NB];
  unsigned long long mass_before_p;     // K2 -> K3
  int bp, bk, cnt_before_k, sp, sk;     // bp / bk == NB: no boundary (keep u < RANGE)
  int tickets[4];
};
}  // namespace samp

size_t sample_ws_row_bytes() { return (sizeof(samp::Row) + 255) & ~size_t(255); }

template <typename T>
struct SampRow {
  const T* row;
  int lo, hi;  // this workgroup's chunk [lo, hi)
  // f(i, x) over the chunk, each thread in increasing i. 16-B vectors (8 in flight per
  // thread) when the chunk start is 16-B aligned, else scalar loads (8 in flight).
  template <class F>
  __device__ __forceinline__ void visit(F f) const {
    constexpr int W = VecW<T>::W, U = 8;
    const T* base = row + lo;
    const bool vec = (reinterpret_cast<uintptr_t>(base) & 15) == 0;
    int done = lo;
    if (vec) {
      const int nvec = (hi - lo) / W;
      for (int v0 = static_cast<int>(threadIdx.x); v0 < nvec; v0 += U * samp::NT) {
        uint4 raw[U];
#pragma unroll
        for (int u = 0; u < U; ++u) raw[u] = ld16(base + static_cast<int64_t>(min(v0 + u * samp::NT, nvec - 1)) * W);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int vi = v0 + u * samp::NT;
          if (vi >= nvec) break;
          float fv[8];
          if constexpr (W == 8) {
            unpack8(raw[u], fv);
          } else {
            fv[0] = __uint_as_float(raw[u].x); fv[1] = __uint_as_float(raw[u].y);
            fv[2] = __uint_as_float(raw[u].z); fv[3] = __uint_as_float(raw[u].w);
          }
#pragma unroll
          for (int k = 0; k < W; ++k) f(lo + vi * W + k, fv[k]);
        }
      }
      done = lo + nvec * W;
    }
    for (int i0 = done + static_cast<int>(threadIdx.x); i0 < hi; i0 += U * samp::NT) {
      float v[U];
#pragma unroll
      for (int j = 0; j < U; ++j) v[j] = scalar_at<T>(row, min(i0 + j * samp::NT, hi - 1));
#pragma unroll
      for (int j = 0; j < U; ++j)
        if (i0 + j * samp::NT < hi) f(i0 + j * samp::NT, v[j]);
    }
  }
};

struct SampParams {
  float it;       // 1 / T (1 for greedy rows)
  bool greedy, use_p, use_k;
  float top_p;
  int top_k;
};

__device__ __forceinline__ SampParams samp_params(int b, int V, const float* temps, const float* top_ps,
                                                  const int32_t* top_ks) {
  SampParams q;
  const float temp = temps[b];
  q.greedy = !(temp > 0.f);
  q.it = q.greedy ? 1.f : 1.f / temp;
  q.top_p = top_ps ? top_ps[b] : 1.f;
  q.top_k = top_ks ? top_ks[b] : 0;
  q.use_p = !q.greedy && q.top_p < 1.f;
  q.use_k = !q.greedy && q.top_k > 0 && q.top_k < V;
  return q;
}

// (M, logZ) of the row from the K1 partials, combined in a fixed order by wave 0
// (deterministic); every thread gets the result.
__device__ __forceinline__ void samp_row_stats(const samp::Row& r, int P, float& M, float& logZ) {
  __shared__ float sh[2];
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    float m = l < P ? r.stats[l][0] : -INFINITY, sv = l < P ? r.stats[l][1] : 0.f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(sv, o, 64);
      const float mn = fmaxf(m, m2);
      sv = (m == -INFINITY ? 0.f : sv * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
      m = mn;
    }
    if (l == 0) { sh[0] = m; sh[1] = m + __logf(sv); }
  }
  __syncthreads();
  M = sh[0];
  logZ = sh[1];
}

__device__ __forceinline__ void samp_chunk(int V, int P, int p, int& lo, int& hi) {
  const int per = ((V + P - 1) / P + 7) & ~7;
  lo = min(V, p * per);
  hi = min(V, lo + per);
}

template <typename T>
__global__ void __launch_bounds__(samp::NT) samp_stats_kernel(const T* __restrict__ logits, int64_t stride, int V,
                                                             const float* __restrict__ temps, samp::Row* ws) {
  const int b = blockIdx.y, p = blockIdx.x, P = gridDim.x;
  const float temp = temps[b];
  const float it = temp > 0.f ? 1.f / temp : 1.f;
  SampRow<T> sr{logits + b * stride, 0, 0};
  samp_chunk(V, P, p, sr.lo, sr.hi);
  float m = -INFINITY, sv = 0.f;
  sr.visit([&](int, float x) {
    const float y = x * it;
    if (y > m) { sv = (m == -INFINITY ? 0.f : sv * __expf(m - y)) + 1.f; m = y; } else { sv += __expf(y - m); }
  });
  __shared__ float rm[samp::NT / 64], rs[samp::NT / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(sv, o, 64);
    const float mn = fmaxf(m, m2);
    sv = (m == -INFINITY ? 0.f : sv * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
    m = mn;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { rm[wid] = m; rs[wid] = sv; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = -INFINITY, S = 0.f;
    for (int w = 0; w < samp::NT / 64; ++w) {
      const float mn = fmaxf(M, rm[w]);
      S = (M == -INFINITY ? 0.f : S * __expf(M - mn)) + (rm[w] == -INFINITY ? 0.f : rs[w] * __expf(rm[w] - mn));
      M = mn;
    }
    ws[b].stats[p][0] = M;
    ws[b].stats[p][1] = S;
  }
}

// Row ticket (see gemm_m64g.hip agent_ticket): drain, one relaxed agent-scope add;
// the winner acquires before reading what the other workgroups published.
__device__ __forceinline__ bool samp_ticket(int* cnt, int last_value) {
  __shared__ int flag;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == last_value;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    flag = last;
  }
  __syncthreads();
  return flag != 0;
}

// First bin (in order) where base + cumulative mass reaches `target` (or NB) and first
// bin where base + cumulative count exceeds `kmax` (or NB), with the exclusive prefix
// at those bins. Run by a whole workgroup over global histograms h_m / h_c, which it
// re-zeroes.
__device__ void samp_scan(unsigned long long* h_m, unsigned int* h_c, bool do_p, unsigned long long target,
                          bool do_k, long long kmax, int& bin_p, unsigned long long& before_p, int& bin_k,
                          long long& before_k) {
  constexpr int PER = samp::NB / samp::NT;
  __shared__ unsigned long long sm[samp::NT];
  __shared__ long long sc[samp::NT];
  __shared__ int best_p, best_k;
  const int t = threadIdx.x;
  unsigned long long lm[PER];
  unsigned int lc[PER];
  unsigned long long tm = 0;
  long long tc = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    lm[j] = do_p ? __hip_atomic_load(h_m + t * PER + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    lc[j] = do_k ? __hip_atomic_load(h_c + t * PER + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    tm += lm[j];
    tc += lc[j];
  }
  if (t == 0) { best_p = samp::NB; best_k = samp::NB; }
  sm[t] = tm;
  sc[t] = tc;
  __syncthreads();
  for (int o = 1; o < samp::NT; o <<= 1) {  // inclusive Hillis-Steele scan
    const unsigned long long am = t >= o ? sm[t - o] : 0ull;
    const long long ac = t >= o ? sc[t - o] : 0ll;
    __syncthreads();
    sm[t] += am;
    sc[t] += ac;
    __syncthreads();
  }
  unsigned long long cm = sm[t] - tm;  // exclusive
  long long cc = sc[t] - tc;
  int fp = samp::NB, fk = samp::NB;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if (fp == samp::NB && cm + lm[j] >= target) fp = t * PER + j;
    if (fk == samp::NB && cc + lc[j] > kmax) fk = t * PER + j;
    if (fp == samp::NB) cm += lm[j];
    if (fk == samp::NB) cc += lc[j];
  }
  if (do_p && fp < samp::NB) atomicMin(&best_p, fp);
  if (do_k && fk < samp::NB) atomicMin(&best_k, fk);
  __syncthreads();
  bin_p = best_p;
  bin_k = best_k;
  // the owners of the boundary bins publish the exclusive prefixes
  __shared__ unsigned long long bp_before;
  __shared__ long long bk_before;
  if (do_p && fp == best_p && fp < samp::NB) bp_before = cm;
  if (do_k && fk == best_k && fk < samp::NB) bk_before = cc;
  __syncthreads();
  before_p = bin_p < samp::NB ? bp_before : 0ull;
  before_k = bin_k < samp::NB ? bk_before : 0ll;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if (do_p) h_m[t * PER + j] = 0ull;
    if (do_k) h_c[t * PER + j] = 0u;
  }
}

// level-1 bin of u = M - y (>= NB: outside the range) and the sub-bin within it
__device__ __forceinline__ int samp_bin(float u, int& sub) {
  const float tt = u * (samp::NB / samp::RANGE);
  const int b = tt < static_cast<float>(samp::NB) ? static_cast<int>(tt) : samp::NB;
  sub = min(samp::NB - 1, max(0, static_cast<int>((tt - static_cast<float>(b)) * samp::NB)));
  return b;
}

template <typename T, int LEVEL>
__global__ void __launch_bounds__(samp::NT) samp_hist_kernel(const T* __restrict__ logits, int64_t stride, int V,
                                                            const float* __restrict__ temps,
                                                            const float* __restrict__ top_ps,
                                                            const int32_t* __restrict__ top_ks, samp::Row* ws) {
  const int b = blockIdx.y, p = blockIdx.x, P = gridDim.x;
  const SampParams q = samp_params(b, V, temps, top_ps, top_ks);
  samp::Row& r = ws[b];
  if (!q.use_p && !q.use_k) return;  // uniform per row: no workgroup of it takes a ticket
  const bool do_p = q.use_p && (LEVEL == 1 || r.bp < samp::NB);
  const bool do_k = q.use_k && (LEVEL == 1 || r.bk < samp::NB);
  if (!do_p && !do_k) return;
  const int bp = LEVEL == 2 ? r.bp : 0, bk = LEVEL == 2 ? r.bk : 0;
  float M, logZ;
  samp_row_stats(r, P, M, logZ);
  __shared__ unsigned long long hm[samp::NB];
  __shared__ unsigned int hc[samp::NB];
  for (int i = threadIdx.x; i < samp::NB; i += samp::NT) { hm[i] = 0ull; hc[i] = 0u; }
  __syncthreads();
  SampRow<T> sr{logits + b * stride, 0, 0};
  samp_chunk(V, P, p, sr.lo, sr.hi);
  sr.visit([&](int, float x) {
    const float y = x * q.it;
    int sub;
    const int bin = samp_bin(M - y, sub);
    if (bin >= samp::NB) return;
    if (LEVEL == 1) {
      if (do_p) atomicAdd(&hm[bin], static_cast<unsigned long long>(__expf(y - logZ) * samp::FIX));
      if (do_k) atomicAdd(&hc[bin], 1u);
    } else {
      if (do_p && bin == bp) atomicAdd(&hm[sub], static_cast<unsigned long long>(__expf(y - logZ) * samp::FIX));
      if (do_k && bin == bk) atomicAdd(&hc[sub], 1u);
    }
  });
  __syncthreads();
  unsigned long long* gm = LEVEL == 1 ? r.h1m : r.h2m;
  unsigned int* gc = LEVEL == 1 ? r.h1c : r.h2c;
  for (int i = threadIdx.x; i < samp::NB; i += samp::NT) {
    if (do_p && hm[i]) atomicAdd(gm + i, hm[i]);
    if (do_k && hc[i]) atomicAdd(gc + i, hc[i]);
  }
  if (!samp_ticket(&r.tickets[LEVEL], P - 1)) return;
  const unsigned long long target = static_cast<unsigned long long>(static_cast<double>(q.top_p) * samp::FIX);
  const unsigned long long base_p = LEVEL == 1 ? 0ull : r.mass_before_p;
  const long long base_k = LEVEL == 1 ? 0ll : r.cnt_before_k;
  int fp, fk;
  unsigned long long bef_p;
  long long bef_k;
  samp_scan(gm, gc, do_p, target > base_p ? target - base_p : 0ull, do_k, q.top_k - base_k, fp, bef_p, fk, bef_k);
  if (threadIdx.x == 0) {
    if (LEVEL == 1) {
      r.bp = q.use_p ? fp : samp::NB;
      r.bk = q.use_k ? fk : samp::NB;
      r.mass_before_p = bef_p;
      r.cnt_before_k = static_cast<int>(bef_k);
    } else {
      r.sp = do_p ? (fp < samp::NB ? fp : samp::NB - 1) : 0;  // sub-bins <= sp kept
      r.sk = do_k ? fk : 0;                                   // sub-bins < sk kept
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(samp::NT) samp_draw_kernel(const T* __restrict__ logits, int64_t stride, int V,
                                                            const float* __restrict__ temps,
                                                            const float* __restrict__ top_ps,
                                                            const int32_t* __restrict__ top_ks,
                                                            const uint64_t* __restrict__ seeds, uint64_t step,
                                                            samp::Row* ws, int32_t* __restrict__ out_tok,
                                                            float* __restrict__ out_lp) {
  const int b = blockIdx.y, p = blockIdx.x, P = gridDim.x;
  const SampParams q = samp_params(b, V, temps, top_ps, top_ks);
  samp::Row& r = ws[b];
  float M, logZ;
  samp_row_stats(r, P, M, logZ);
  const int bp = q.use_p ? r.bp : samp::NB, bk = q.use_k ? r.bk : samp::NB;
  const int sp = bp < samp::NB ? r.sp : 0, sk = bk < samp::NB ? r.sk : 0;
  const uint64_t seed = seeds ? seeds[b] : 0x9E3779B97F4A7C15ull;
  const uint32_t key = hash32(static_cast<uint32_t>(seed) ^ hash32(static_cast<uint32_t>(seed >> 32) + 0x85ebca6bU) ^
                              hash32(static_cast<uint32_t>(step) * 0x27d4eb2fU + 0x165667b1U));
  float bv = -INFINITY, by = -INFINITY;
  int bi = 0x7fffffff;
  SampRow<T> sr{logits + b * stride, 0, 0};
  samp_chunk(V, P, p, sr.lo, sr.hi);
  const bool filt = q.use_p || q.use_k;
  // Gumbel noise is bounded: u <= 1 - 2^-25 gives -log(-log u) < 17.33, so a token with
  // y + GMAX below this thread's best score cannot win -- skipped without its hash
  // (exact: the draw is unchanged)
  constexpr float GMAX = 17.5f;
  sr.visit([&](int i, float x) {
    const float y = x * q.it;
    if (!q.greedy && y + GMAX < bv) return;
    if (filt && y < M) {  // the row max is always kept
      int sub;
      const int bin = samp_bin(M - y, sub);
      if (bin >= samp::NB) return;
      if (q.use_p && bp < samp::NB && (bin > bp || (bin == bp && sub > sp))) return;
      if (q.use_k && bk < samp::NB && (bin > bk || (bin == bk && sub >= sk))) return;
    }
    float score = y;
    if (!q.greedy) {
      const uint32_t hsh = hash32(key ^ hash32(static_cast<uint32_t>(i) * 0x9E3779B9U));
      const float uu = (static_cast<float>(hsh >> 8) + 0.5f) * (1.f / 16777216.f);
      score = y - __logf(-__logf(uu));
    }
    if (score > bv) { bv = score; bi = i; by = y; }
  });
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(bv, o, 64), y2 = __shfl_xor(by, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    if (v2 > bv || (v2 == bv && i2 < bi)) { bv = v2; bi = i2; by = y2; }
  }
  __shared__ float rv[samp::NT / 64], ry[samp::NT / 64];
  __shared__ int ri[samp::NT / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { rv[wid] = bv; ri[wid] = bi; ry[wid] = by; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < samp::NT / 64; ++w)
      if (rv[w] > rv[0] || (rv[w] == rv[0] && ri[w] < ri[0])) { rv[0] = rv[w]; ri[0] = ri[w]; ry[0] = ry[w]; }
    st16_sc1(&r.draw[p][0], f32x4_t{rv[0], __int_as_float(ri[0]), ry[0], 0.f});
  }
  if (!samp_ticket(&r.tickets[3], P - 1)) return;
  if (threadIdx.x < 64) {  // wave 0 merges the P chunk winners (max score, lowest index)
    const int l = threadIdx.x;
    float v = -INFINITY, y = -INFINITY;
    int idx = 0x7fffffff;
    if (l < P) {
      const float4 d = *reinterpret_cast<const float4*>(&r.draw[l][0]);
      v = d.x; idx = __float_as_int(d.y); y = d.z;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float v2 = __shfl_xor(v, o, 64), y2 = __shfl_xor(y, o, 64);
      const int i2 = __shfl_xor(idx, o, 64);
      if (v2 > v || (v2 == v && i2 < idx)) { v = v2; idx = i2; y = y2; }
    }
    if (l == 0) {
      out_tok[b] = idx;
      if (out_lp) out_lp[b] = y - logZ;  // logprob under the temperature-scaled distribution
    }
  }
}

template <typename T>
static void launch_sample_v2(const T* logits, int64_t stride, int B, int V, const float* temps, const float* top_ps,
                             const int32_t* top_ks, const uint64_t* seeds, uint64_t step, int32_t* tok, float* lp,
                             samp::Row* ws, hipStream_t st) {
  // ~2 workgroups per CU over the whole batch, >= 2048 logits per workgroup
  int P = std::max(1, std::min(samp::PMAX, (512 + B - 1) / B));
  P = std::max(1, std::min(P, (V + 2047) / 2048));
  const dim3 grid(P, B);
  hipLaunchKernelGGL(samp_stats_kernel<T>, grid, dim3(samp::NT), 0, st, logits, stride, V, temps, ws);
  if (top_ps != nullptr || top_ks != nullptr) {
    hipLaunchKernelGGL((samp_hist_kernel<T, 1>), grid, dim3(samp::NT), 0, st, logits, stride, V, temps, top_ps,
                       top_ks, ws);
    hipLaunchKernelGGL((samp_hist_kernel<T, 2>), grid, dim3(samp::NT), 0, st, logits, stride, V, temps, top_ps,
                       top_ks, ws);
  }
  hipLaunchKernelGGL(samp_draw_kernel<T>, grid, dim3(samp::NT), 0, st, logits, stride, V, temps, top_ps, top_ks,
                     seeds, step, ws, tok, lp);
}

// Split-row greedy path: ARG_PARTS workgroups of 256 threads per row each reduce a
// contiguous slice (one batch of loads per thread at V = 128K), publish their (max,
// argmax, log-sum-exp) write-through and take a ticket on the row; the row's last
// arriver merges the slices in slice order (deterministic) and writes the token and its
// logprob. One 1024-thread workgroup per row was latency-bound: 13.7 us per step at
// batch 1 for a 256 KB row (128 exps per thread, two dependent load rounds).
constexpr int ARG_PARTS = 8;
template <typename T>
__global__ void __launch_bounds__(256) argmax_split_kernel(const T* __restrict__ logits, int64_t stride, int V,
                                                           int32_t* __restrict__ out_tok, float* __restrict__ out_lp,
                                                           float4* __restrict__ ws, int* __restrict__ cnt) {
  constexpr int W = VecW<T>::W;
  constexpr int U = 8;
  const int row = blockIdx.x / ARG_PARTS, part = blockIdx.x % ARG_PARTS;
  const T* rp = logits + row * stride;
  const int nv = V / W;
  const int v0 = static_cast<int>(static_cast<int64_t>(nv) * part / ARG_PARTS);
  const int v1 = static_cast<int>(static_cast<int64_t>(nv) * (part + 1) / ARG_PARTS);
  ArgLse a{-INFINITY, 0x7fffffff, -INFINITY, 0.f};
  for (int c0 = v0 + threadIdx.x; c0 < v1; c0 += U * blockDim.x) {
    uint4 raw[U];
#pragma unroll
    for (int u = 0; u < U; ++u) raw[u] = ld16(rp + static_cast<int64_t>(min(c0 + u * (int)blockDim.x, v1 - 1)) * W);
    float f[U][W];
    float bm = -INFINITY;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (W == 8) {
        unpack8(raw[u], f[u]);
      } else {
        f[u][0] = __uint_as_float(raw[u].x); f[u][1] = __uint_as_float(raw[u].y);
        f[u][2] = __uint_as_float(raw[u].z); f[u][3] = __uint_as_float(raw[u].w);
      }
      const bool ok = c0 + u * (int)blockDim.x < v1;
#pragma unroll
      for (int k = 0; k < W; ++k) {
        if (!ok) f[u][k] = -INFINITY;
        const float x = f[u][k];
        if (x > a.v) { a.v = x; a.i = (c0 + u * (int)blockDim.x) * W + k; }
        bm = fmaxf(bm, x);
      }
    }
    if (bm == -INFINITY) continue;
    const float mn = fmaxf(a.m, bm);
    float bs = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < W; ++k) bs += __expf(f[u][k] - mn);
    a.s = (a.m == -INFINITY ? 0.f : a.s * __expf(a.m - mn)) + bs;
    a.m = mn;
  }
  if (part == ARG_PARTS - 1) {  // the scalar tail past the last full vector
    for (int i = nv * W + threadIdx.x; i < V; i += blockDim.x) {
      const float x = scalar_at<T>(rp, i);
      if (x > a.v) { a.v = x; a.i = i; }
      if (x > a.m) { a.s = a.s * __expf(a.m - x) + 1.f; a.m = x; } else { a.s += __expf(x - a.m); }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgLse b{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64), __shfl_xor(a.m, o, 64), __shfl_xor(a.s, o, 64)};
    a = merge(a, b);
  }
  __shared__ ArgLse red[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = a;
  __syncthreads();
  if (threadIdx.x != 0) return;
  ArgLse r = red[0];
  for (int w = 1; w < 4; ++w) r = merge(r, red[w]);
  st16_sc1(reinterpret_cast<float*>(ws + row * ARG_PARTS + part),
           f32x4_t{r.v, __int_as_float(r.i), r.m, r.s});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (__hip_atomic_fetch_add(cnt + row, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ARG_PARTS - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  ArgLse m{-INFINITY, 0x7fffffff, -INFINITY, 0.f};
  for (int q = 0; q < ARG_PARTS; ++q) {
    const float4 v = ws[row * ARG_PARTS + q];
    m = merge(m, ArgLse{v.x, __float_as_int(v.y), v.z, v.w});
  }
  __hip_atomic_store(cnt + row, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed for the next launch
  out_tok[row] = m.i;
  if (out_lp) out_lp[row] = m.v - (m.m + __logf(m.s));
}

int argmax_ws_floats_per_row() { return 4 * ARG_PARTS; }

void argmax_logprob(const void* logits, int is_f32, int64_t stride, int B, int V, int32_t* tok, float* lp,
                    hipStream_t st, float* ws, int* cnt) {
  if (B <= 0) return;
  if (ws != nullptr && cnt != nullptr) {  // ws: B x ARG_PARTS float4; cnt: B zeroed ints
    if (is_f32)
      hipLaunchKernelGGL(argmax_split_kernel<float>, dim3(B * ARG_PARTS), dim3(256), 0, st, (const float*)logits,
                         stride, V, tok, lp, reinterpret_cast<float4*>(ws), cnt);
    else
      hipLaunchKernelGGL(argmax_split_kernel<uint16_t>, dim3(B * ARG_PARTS), dim3(256), 0, st,
                         (const uint16_t*)logits, stride, V, tok, lp, reinterpret_cast<float4*>(ws), cnt);
    return;
  }
  if (is_f32)
    hipLaunchKernelGGL(argmax_kernel<float>, dim3(B), dim3(1024), 0, st, (const float*)logits, stride, V, tok, lp);
  else
    hipLaunchKernelGGL(argmax_kernel<uint16_t>, dim3(B), dim3(1024), 0, st, (const uint16_t*)logits, stride, V,
                       tok, lp);
}

void sample_tokens(const void* logits, int is_f32, int64_t stride, int B, int V, const float* temps,
                   const float* top_ps, const int32_t* top_ks, const uint64_t* seeds, uint64_t step, int32_t* tok,
                   float* lp, void* ws, hipStream_t st) {
  if (B <= 0) return;
  if (ws != nullptr) {  // split-row sampler; ws: B zeroed rows of sample_ws_row_bytes()
    if (is_f32)
      launch_sample_v2<float>(static_cast<const float*>(logits), stride, B, V, temps, top_ps, top_ks, seeds, step,
                              tok, lp, static_cast<samp::Row*>(ws), st);
    else
      launch_sample_v2<uint16_t>(static_cast<const uint16_t*>(logits), stride, B, V, temps, top_ps, top_ks, seeds,
                                 step, tok, lp, static_cast<samp::Row*>(ws), st);
    return;
  }
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
