// pybind11 entry points of xgserve._kernels. Every op takes raw device pointers
// (tensor.data_ptr()) and the hipStream_t of the caller's current torch stream,
// so launches are graph-capturable and there is no dependence on torch's C++ ABI.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>
#include <cstring>
#include <pybind11/stl.h>

namespace py = pybind11;

namespace xgk {
void rmsnorm(const uint16_t*, const uint16_t*, uint16_t*, int, int, float, int64_t, int64_t, hipStream_t);
void fused_add_rmsnorm(const uint16_t*, uint16_t*, const uint16_t*, uint16_t*, int, int, float, hipStream_t);
void layernorm(const uint16_t*, const uint16_t*, const uint16_t*, uint16_t*, int, int, float, hipStream_t);
void silu_and_mul(const uint16_t*, uint16_t*, int, int, int, hipStream_t);
int skinny_gemm(const uint16_t*, int, int, const uint16_t*, int, float*, uint16_t*, int, int, hipStream_t);
int skinny_slab_kmax(int);
int gemm_m64g(const uint16_t*, int, int, const uint16_t*, int, float*, uint16_t*, int, int, int, int, hipStream_t);
int gemm_m64g_ex(const uint16_t*, int, int, const uint16_t*, int, float*, uint16_t*, int, int, int, int, const float*,
                 int, int, float, uint16_t*, float*, int*, hipStream_t);
int gemm_mw(const uint16_t*, int, int, const uint16_t*, int, float*, uint16_t*, int, int, int, hipStream_t);
int gemm_m64g_ar(const uint16_t*, int, int, const uint16_t*, int, float*, int, int, int, uint16_t*, float*, int*,
                 const void*, hipStream_t);
int m64g_ar_desc_bytes();
int gemm_pf_grouped(const uint16_t*, const int32_t*, const int32_t*, int, int, int, const uint16_t*, int, int, float*,
                    uint16_t*, int, int, int, hipStream_t);
int gemm_pf(const uint16_t*, int, int, const uint16_t*, int, float*, uint16_t*, int, int, int, hipStream_t);
void set_pf_krot(int);
void set_k_rotation(int mode);
void add_partials_resid(const float*, int, int, uint16_t*, float*, int, hipStream_t, uint64_t);
void row_sumsq(const uint16_t*, int, int, float*, hipStream_t);
void embed_gather(const int32_t*, int, const uint16_t*, int, int, uint16_t*, float*, hipStream_t);
void mean_l2norm_rows(float*, const int32_t*, const int32_t*, float*, int, int, hipStream_t);
int decode_attention_fq(const float*, int, const int32_t*, const float*, const int32_t*, uint16_t*, uint16_t*,
                        const int32_t*, int, const int32_t*, float*, float*, uint16_t*, int64_t, int, int, int, int,
                        int, float, int, int, hipStream_t, int);
struct MoeResidEpi {
  const int32_t* dest;
  const float* w;
  uint16_t* resid;
  float* ss_out;
  int* counters;
  int T;
  int k;
};
int moe_gemm_m64g(const uint16_t*, const int32_t*, const int32_t*, int, int, const uint16_t*, int, int, float*,
                  uint16_t*, int, int, int, int, int, hipStream_t, const int32_t*, const MoeResidEpi* = nullptr,
                  int pairs = 0);
void add_partials_rmsnorm(const float*, int, int, uint16_t*, const uint16_t*, uint16_t*, int, float, hipStream_t);
void reduce_partials(const float*, int, int64_t, uint16_t*, hipStream_t);
int rope_cache_partials(const float*, int, uint16_t*, int64_t, const int32_t*, const float*, uint16_t*, uint16_t*,
                        const int32_t*, int, int, int, int, int, int, hipStream_t);
void gelu_tanh(const uint16_t*, uint16_t*, int64_t, hipStream_t);
int rope_cache(uint16_t*, int64_t, const int32_t*, const float*, uint16_t*, uint16_t*, const int32_t*, int, int, int,
               int, int, int, hipStream_t);
int decode_attention(const uint16_t*, int64_t, const uint16_t*, const uint16_t*, const int32_t*, int, const int32_t*,
                     float*, float*, uint16_t*, int64_t, int, int, int, int, int, float, int, hipStream_t);
int prefill_attention(const uint16_t*, int64_t, const uint16_t*, const uint16_t*, const int32_t*, int, const int32_t*,
                      const int32_t*, uint16_t*, int64_t, int, int, int, int, int, int, float, hipStream_t, int);
void argmax_logprob(const void*, int, int64_t, int, int, int32_t*, float*, hipStream_t, float* ws = nullptr,
                    int* cnt = nullptr);
int argmax_ws_floats_per_row();
void sample_tokens(const void*, int, int64_t, int, int, const float*, const float*, const int32_t*, const uint64_t*,
                   uint64_t, int32_t*, float*, void*, hipStream_t);
size_t sample_ws_row_bytes();
void segment_sum(const uint16_t*, int, const int32_t*, const int32_t*, float*, int, hipStream_t);
void subst_tokens(int32_t*, const int32_t*, const int32_t*, int, hipStream_t);
int gemm_w8(const uint16_t*, int, int, const uint8_t*, const float*, int, float*, uint16_t*, int, int, int,
            hipStream_t, int);
void moe_topk_softmax(const void*, int, int, int, int, int, float*, int32_t*, hipStream_t);
void moe_align(const int32_t*, int, int, int, int, int, int32_t*, int32_t*, int32_t*, hipStream_t);
int moe_combine(const void*, int, int, const int32_t*, const float*, void*, int, int, int, hipStream_t, int);
int moe_route(const uint16_t*, const uint16_t*, int, int, int, int, int, float*, int32_t*, hipStream_t,
              const uint16_t*, float, uint16_t*, int32_t*, int32_t*, int32_t*, int, int, int);
int moe_combine_resid(const float*, int, int, const int32_t*, const float*, uint16_t*, float*, int, int, int,
                      hipStream_t);
int ep_plan(const int32_t*, int, int, int, int, int, int32_t*, int32_t*, int32_t*, hipStream_t);
int ep_scatter(const uint16_t*, int64_t, int, const int32_t*, int, int, uint16_t*, hipStream_t);
int custom_allreduce(const void*, void*, int64_t, int64_t, const uintptr_t*, const uintptr_t*, int, int, uint32_t*,
                     uint32_t*, hipStream_t);
int custom_allreduce_2shot(const void*, void*, int64_t, int64_t, const uintptr_t*, const uintptr_t*, int, int,
                           uint32_t*, uint32_t*, hipStream_t);
int custom_allreduce_resid(const float*, int, int, uint16_t*, float*, int, int64_t, const uintptr_t*,
                           const uintptr_t*, int, int, uint32_t*, uint32_t*, hipStream_t);
int custom_allgather_lastdim(const void*, void*, int64_t, int64_t, int64_t, const uintptr_t*, const uintptr_t*, int,
                             int, uint32_t*, uint32_t*, hipStream_t);
int custom_allreduce_ll(const void*, void*, int64_t, int64_t, const uintptr_t*, int, int, uint32_t*, uint32_t*,
                        hipStream_t);
int custom_allreduce_resid_ll(const float*, int, int, uint16_t*, float*, int, int64_t, const uintptr_t*, int, int,
                              uint32_t*, uint32_t*, hipStream_t, int);
int car_ll_max_bytes(int64_t);
int car_max_blocks();
int car_wallclock_khz();
int car_chunk();
int car_max_ranks();
int car_alloc_uncached(int64_t, void**);
int car_ipc_handle(void*, hipIpcMemHandle_t*);
int car_ipc_open(const hipIpcMemHandle_t*, void**);
int car_ipc_close(void*);
int car_free(void*);
}  // namespace xgk

template <typename T>
static T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

static void check(int rc, const char* what) {
  if (rc != 0) throw std::invalid_argument(std::string(what) + ": unsupported shape/config");
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

PYBIND11_MODULE(_kernels, m) {
  m.doc() = "xgserve hand-written CDNA4 (gfx950) HIP kernels";
  m.attr("arch") = "gfx950";

  m.def("rmsnorm", [](uintptr_t x, uintptr_t w, uintptr_t out, int T, int H, float eps, int64_t xs, int64_t os,
                      uintptr_t st) {
    if (H % 8) throw std::invalid_argument("rmsnorm: H % 8 != 0");
    xgk::rmsnorm(P<const uint16_t>(x), P<const uint16_t>(w), P<uint16_t>(out), T, H, eps, xs, os, S(st));
    check(0, "rmsnorm");
  });
  m.def("fused_add_rmsnorm", [](uintptr_t x, uintptr_t res, uintptr_t w, uintptr_t out, int T, int H, float eps,
                                uintptr_t st) {
    if (H % 8) throw std::invalid_argument("fused_add_rmsnorm: H % 8 != 0");
    xgk::fused_add_rmsnorm(P<const uint16_t>(x), P<uint16_t>(res), P<const uint16_t>(w), P<uint16_t>(out), T, H,
                           eps, S(st));
    check(0, "fused_add_rmsnorm");
  });
  m.def("layernorm", [](uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t out, int T, int H, float eps,
                        uintptr_t st) {
    if (H % 8) throw std::invalid_argument("layernorm: H % 8 != 0");
    xgk::layernorm(P<const uint16_t>(x), P<const uint16_t>(w), P<const uint16_t>(b), P<uint16_t>(out), T, H, eps,
                   S(st));
    check(0, "layernorm");
  });
  m.def("silu_and_mul", [](uintptr_t in, uintptr_t out, int T, int F, int interleave16, uintptr_t st) {
    if (F % 8) throw std::invalid_argument("silu_and_mul: F % 8 != 0");
    if (interleave16 && F % 16) throw std::invalid_argument("silu_and_mul: interleaved F % 16 != 0");
    xgk::silu_and_mul(P<const uint16_t>(in), P<uint16_t>(out), T, F, interleave16, S(st));
    check(0, "silu_and_mul");
  });
  m.def("skinny_gemm", [](uintptr_t x, int M, int K, uintptr_t w, int N, uintptr_t part, uintptr_t out, int split_k,
                          int mode, uintptr_t st) {
    check(xgk::skinny_gemm(P<const uint16_t>(x), M, K, P<const uint16_t>(w), N, P<float>(part), P<uint16_t>(out),
                           split_k, mode, S(st)),
          "skinny_gemm");
  });
  m.def("skinny_slab_kmax", &xgk::skinny_slab_kmax);
  m.def("add_partials_rmsnorm", [](uintptr_t part, int S_, int T, uintptr_t res, uintptr_t w, uintptr_t out, int H,
                                   float eps, uintptr_t st) {
    if (H % 8) throw std::invalid_argument("add_partials_rmsnorm: H % 8 != 0");
    xgk::add_partials_rmsnorm(P<const float>(part), S_, T, P<uint16_t>(res), P<const uint16_t>(w), P<uint16_t>(out),
                              H, eps, S(st));
    check(0, "add_partials_rmsnorm");
  });
  m.def("reduce_partials", [](uintptr_t part, int S_, int64_t n, uintptr_t out, uintptr_t st) {
    if (n % 4) throw std::invalid_argument("reduce_partials: n % 4 != 0");
    xgk::reduce_partials(P<const float>(part), S_, n, P<uint16_t>(out), S(st));
    check(0, "reduce_partials");
  });
  m.def("rope_cache_partials", [](uintptr_t part, int S_, uintptr_t q_out, int64_t q_stride, uintptr_t pos,
                                  uintptr_t cs, uintptr_t kc, uintptr_t vc, uintptr_t slots, int T, int Hq, int Hkv,
                                  int D, int bs, int apply_rope, uintptr_t st) {
    check(xgk::rope_cache_partials(P<const float>(part), S_, P<uint16_t>(q_out), q_stride, P<const int32_t>(pos),
                                   P<const float>(cs), P<uint16_t>(kc), P<uint16_t>(vc), P<const int32_t>(slots), T,
                                   Hq, Hkv, D, bs, apply_rope, S(st)),
          "rope_cache_partials");
  });
  m.def("gelu_tanh", [](uintptr_t in, uintptr_t out, int64_t n, uintptr_t st) {
    if (n % 8) throw std::invalid_argument("gelu_tanh: n % 8 != 0");
    xgk::gelu_tanh(P<const uint16_t>(in), P<uint16_t>(out), n, S(st));
    check(0, "gelu_tanh");
  });
  m.def("rope_cache", [](uintptr_t qkv, int64_t row_stride, uintptr_t pos, uintptr_t cs, uintptr_t kc, uintptr_t vc,
                         uintptr_t slots, int T, int Hq, int Hkv, int D, int bs, int apply_rope, uintptr_t st) {
    check(xgk::rope_cache(P<uint16_t>(qkv), row_stride, P<const int32_t>(pos), P<const float>(cs), P<uint16_t>(kc),
                          P<uint16_t>(vc), P<const int32_t>(slots), T, Hq, Hkv, D, bs, apply_rope, S(st)),
          "rope_cache");
  });
  m.def("decode_attention", [](uintptr_t q, int64_t qs, uintptr_t kc, uintptr_t vc, uintptr_t bt, int bts,
                               uintptr_t sl, uintptr_t po, uintptr_t pl, uintptr_t out, int64_t os, int B, int Hq,
                               int Hkv, int D, int bs, float scale, int splits, uintptr_t st) {
    check(xgk::decode_attention(P<const uint16_t>(q), qs, P<const uint16_t>(kc), P<const uint16_t>(vc),
                                P<const int32_t>(bt), bts, P<const int32_t>(sl), P<float>(po), P<float>(pl),
                                P<uint16_t>(out), os, B, Hq, Hkv, D, bs, scale, splits, S(st)),
          "decode_attention");
  });
  m.def("prefill_attention", [](uintptr_t q, int64_t qs, uintptr_t kc, uintptr_t vc, uintptr_t bt, int bts,
                                uintptr_t qsl, uintptr_t sl, uintptr_t out, int64_t os, int ns, int maxq, int Hq,
                                int Hkv, int D, int bs, float scale, uintptr_t st, int gh) {
    check(xgk::prefill_attention(P<const uint16_t>(q), qs, P<const uint16_t>(kc), P<const uint16_t>(vc),
                                 P<const int32_t>(bt), bts, P<const int32_t>(qsl), P<const int32_t>(sl),
                                 P<uint16_t>(out), os, ns, maxq, Hq, Hkv, D, bs, scale, S(st), gh),
          "prefill_attention");
  }, py::arg("q"), py::arg("qs"), py::arg("kc"), py::arg("vc"), py::arg("bt"), py::arg("bts"), py::arg("qsl"),
     py::arg("sl"), py::arg("out"), py::arg("os"), py::arg("ns"), py::arg("maxq"), py::arg("Hq"), py::arg("Hkv"),
     py::arg("D"), py::arg("bs"), py::arg("scale"), py::arg("st"), py::arg("gh") = 0);
  // ws / cnt (optional): the split-row form -- B x argmax_ws_floats_per_row() floats and B zeroed
  // ints (re-armed by every launch)
  m.def("argmax_logprob", [](uintptr_t logits, int is_f32, int64_t stride, int B, int V, uintptr_t tok, uintptr_t lp,
                             uintptr_t st, uintptr_t ws, uintptr_t cnt) {
    xgk::argmax_logprob(P<const void>(logits), is_f32, stride, B, V, P<int32_t>(tok), P<float>(lp), S(st), P<float>(ws),
                        P<int>(cnt));
    check(0, "argmax_logprob");
  }, py::arg("logits"), py::arg("is_f32"), py::arg("stride"), py::arg("B"), py::arg("V"), py::arg("tok"), py::arg("lp"),
     py::arg("st"), py::arg("ws") = 0, py::arg("cnt") = 0);
  m.def("argmax_ws_floats_per_row", []() { return xgk::argmax_ws_floats_per_row(); });
  m.def("sample_tokens", [](uintptr_t logits, int is_f32, int64_t stride, int B, int V, uintptr_t temps,
                            uintptr_t top_ps, uintptr_t top_ks, uintptr_t seeds, uint64_t step, uintptr_t tok,
                            uintptr_t lp, uintptr_t st, uintptr_t ws, int ws_rows) {
    if (ws != 0 && ws_rows < B) throw std::invalid_argument("sample_tokens: workspace holds fewer rows than B");
    xgk::sample_tokens(P<const void>(logits), is_f32, stride, B, V, P<const float>(temps), P<const float>(top_ps),
                       P<const int32_t>(top_ks), P<const uint64_t>(seeds), step, P<int32_t>(tok), P<float>(lp),
                       P<void>(ws), S(st));
    check(0, "sample_tokens");
  }, py::arg("logits"), py::arg("is_f32"), py::arg("stride"), py::arg("B"), py::arg("V"), py::arg("temps"),
     py::arg("top_ps"), py::arg("top_ks"), py::arg("seeds"), py::arg("step"), py::arg("tok"), py::arg("lp"),
     py::arg("st"), py::arg("ws") = 0, py::arg("ws_rows") = 0);
  m.def("sample_ws_row_bytes", []() { return static_cast<int64_t>(xgk::sample_ws_row_bytes()); });
  m.def("gemm_w8", [](uintptr_t x, int M, int K, uintptr_t w, uintptr_t scale, int N, uintptr_t part, uintptr_t out,
                      int splits, int mode, int cfg, uintptr_t st, int fmt) {
    check(xgk::gemm_w8(P<const uint16_t>(x), M, K, P<const uint8_t>(w), P<const float>(scale), N, P<float>(part),
                       P<uint16_t>(out), splits, mode, cfg, S(st), fmt),
          "gemm_w8");
  }, py::arg("x"), py::arg("M"), py::arg("K"), py::arg("w"), py::arg("scale"), py::arg("N"), py::arg("part"),
     py::arg("out"), py::arg("splits"), py::arg("mode"), py::arg("cfg"), py::arg("st"), py::arg("fmt") = 0);
  m.def("subst_tokens", [](uintptr_t ids, uintptr_t src, uintptr_t prev, int n, uintptr_t st) {
    xgk::subst_tokens(P<int32_t>(ids), P<const int32_t>(src), P<const int32_t>(prev), n, S(st));
    check(0, "subst_tokens");
  });
  m.def("segment_sum", [](uintptr_t hidden, int H, uintptr_t cu, uintptr_t rows, uintptr_t out, int nseg,
                          uintptr_t st) {
    if (H % 8) throw std::invalid_argument("segment_sum: H % 8 != 0");
    xgk::segment_sum(P<const uint16_t>(hidden), H, P<const int32_t>(cu), P<const int32_t>(rows), P<float>(out), nseg,
                     S(st));
    check(0, "segment_sum");
  });
  m.def("moe_topk_softmax", [](uintptr_t logits, int is_f32, int T, int E, int k, int renorm, uintptr_t w,
                               uintptr_t ids, uintptr_t st) {
    // the kernel keeps the router row and the selection in fixed local arrays (v[64], sel[16])
    if (E < 1 || E > 64) throw std::invalid_argument("moe_topk_softmax: 1 <= E <= 64");
    if (k < 1 || k > 16 || k > E) throw std::invalid_argument("moe_topk_softmax: 1 <= k <= min(16, E)");
    if (T < 0) throw std::invalid_argument("moe_topk_softmax: T < 0");
    xgk::moe_topk_softmax(P<const void>(logits), is_f32, T, E, k, renorm, P<float>(w), P<int32_t>(ids), S(st));
    check(0, "moe_topk_softmax");
  });
  m.def("moe_align", [](uintptr_t ids, int T, int k, int E, int expert_offset, int block_m, uintptr_t sorted_rows,
                        uintptr_t expert_offsets, uintptr_t dest, uintptr_t st) {
    if (E < 1 || E > 256) throw std::invalid_argument("moe_align: 1 <= E <= 256");
    xgk::moe_align(P<const int32_t>(ids), T, k, E, expert_offset, block_m, P<int32_t>(sorted_rows),
                   P<int32_t>(expert_offsets), P<int32_t>(dest), S(st));
    check(0, "moe_align");
  });
  m.def("gemm_m64g", [](uintptr_t x, int M, int K, uintptr_t w, int N, uintptr_t part, uintptr_t out, int splits,
                        int mode, int nw, int cfg, uintptr_t st) {
    check(xgk::gemm_m64g(P<uint16_t>(x), M, K, P<uint16_t>(w), N, P<float>(part), P<uint16_t>(out), splits, mode, nw,
                         cfg, S(st)),
          "gemm_m64g");
  });
  // mid-M weight-streaming GEMM (gemm_mw.hip): 64 < M <= 256 mixed / prompt steps
  m.def("gemm_mw", [](uintptr_t x, int M, int K, uintptr_t w, int N, uintptr_t part, uintptr_t out, int splits,
                      int mode, int cfg, uintptr_t st) {
    check(xgk::gemm_mw(P<uint16_t>(x), M, K, P<uint16_t>(w), N, P<float>(part), P<uint16_t>(out), splits, mode, cfg,
                       S(st)),
          "gemm_mw");
  });
  // prompt-sized MFMA GEMM (gemm_pf.hip): mixed steps above gemm_mw's range, prefill
  m.def("gemm_pf", [](uintptr_t x, int M, int K, uintptr_t w, int N, uintptr_t part, uintptr_t out, int splits,
                      int mode, int cfg, uintptr_t st) {
    check(xgk::gemm_pf(P<uint16_t>(x), M, K, P<uint16_t>(w), N, P<float>(part), P<uint16_t>(out), splits, mode, cfg,
                       S(st)),
          "gemm_pf");
  });
  // grouped form over moe_align's expert-sorted rows (the prompt-sized expert GEMMs)
  m.def("gemm_pf_grouped", [](uintptr_t x, uintptr_t rows, uintptr_t offs, int E, int n_rows, int K, uintptr_t w, int N,
                              int max_pairs, uintptr_t part, uintptr_t out, int splits, int mode, int cfg,
                              uintptr_t st) {
    check(xgk::gemm_pf_grouped(P<uint16_t>(x), P<int32_t>(rows), P<int32_t>(offs), E, n_rows, K, P<uint16_t>(w), N,
                               max_pairs, P<float>(part), P<uint16_t>(out), splits, mode, cfg, S(st)),
          "gemm_pf_grouped");
  });
  m.def("set_pf_krot", [](int on) { xgk::set_pf_krot(on); });
  m.def("set_k_rotation", [](int mode) { xgk::set_k_rotation(mode); });
  m.def("gemm_m64g_ex", [](uintptr_t x, int M, int K, uintptr_t w, int N, uintptr_t part, uintptr_t out, int splits,
                           int mode, int nw, int cfg, uintptr_t ss_in, int ss_n, int ss_stride, float eps,
                           uintptr_t resid, uintptr_t ss_out, uintptr_t counters, uintptr_t st) {
    check(xgk::gemm_m64g_ex(P<uint16_t>(x), M, K, P<uint16_t>(w), N, P<float>(part), P<uint16_t>(out), splits, mode,
                            nw, cfg, P<const float>(ss_in), ss_n, ss_stride, eps, P<uint16_t>(resid),
                            P<float>(ss_out), P<int>(counters), S(st)),
          "gemm_m64g_ex");
  });
  // TP row-parallel GEMM with the all-reduce + residual + statistics in the launch
  // (gemm_m64g.hip GG_AR); data = each rank's LL receive region (loop: this rank's own)
  m.def("gemm_m64g_ar", [](uintptr_t x, int M, int K, uintptr_t w, int N, uintptr_t part, int splits, int nw,
                           int cfg, uintptr_t resid, uintptr_t ss_out, uintptr_t counters, uintptr_t desc,
                           uintptr_t st) {
    check(xgk::gemm_m64g_ar(P<const uint16_t>(x), M, K, P<const uint16_t>(w), N, P<float>(part), splits, nw, cfg,
                            P<uint16_t>(resid), P<float>(ss_out), P<int>(counters), P<const void>(desc), S(st)),
          "gemm_m64g_ar");
  });
  m.def("m64g_ar_desc_bytes", &xgk::m64g_ar_desc_bytes);
  m.def("add_partials_resid", [](uintptr_t part, int S_, int T, uintptr_t res, uintptr_t ss_part, int H,
                                 uintptr_t st, uint64_t sim_ticks) {
    if (H % 1024) throw std::invalid_argument("add_partials_resid: H % 1024 != 0");
    xgk::add_partials_resid(P<const float>(part), S_, T, P<uint16_t>(res), P<float>(ss_part), H, S(st), sim_ticks);
    check(0, "add_partials_resid");
  }, py::arg("part"), py::arg("S"), py::arg("T"), py::arg("res"), py::arg("ss_part"), py::arg("H"), py::arg("st"),
     py::arg("sim_ticks") = 0);
  m.def("embed_gather", [](uintptr_t ids, int T, uintptr_t table, int V, int H, uintptr_t out, uintptr_t ss,
                           uintptr_t st) {
    if (H % 8 || T < 0 || V < 1) throw std::invalid_argument("embed_gather: H % 8 != 0 or bad sizes");
    xgk::embed_gather(P<const int32_t>(ids), T, P<const uint16_t>(table), V, H, P<uint16_t>(out), P<float>(ss), S(st));
    check(0, "embed_gather");
  });
  m.def("mean_l2norm_rows", [](uintptr_t acc, uintptr_t rows, uintptr_t counts, uintptr_t out, int n, int H,
                               uintptr_t st) {
    if (n < 0 || H < 1) throw std::invalid_argument("mean_l2norm_rows: bad sizes");
    xgk::mean_l2norm_rows(P<float>(acc), P<const int32_t>(rows), P<const int32_t>(counts), P<float>(out), n, H, S(st));
    check(0, "mean_l2norm_rows");
  });
  m.def("row_sumsq", [](uintptr_t x, int T, int H, uintptr_t ss, uintptr_t st) {
    if (H % 8) throw std::invalid_argument("row_sumsq: H % 8 != 0");
    xgk::row_sumsq(P<const uint16_t>(x), T, H, P<float>(ss), S(st));
    check(0, "row_sumsq");
  });
  m.def("decode_attention_fq", [](uintptr_t part, int S_, uintptr_t pos, uintptr_t cs, uintptr_t slots, uintptr_t kc,
                                  uintptr_t vc, uintptr_t bt, int bts, uintptr_t sl, uintptr_t po, uintptr_t pl,
                                  uintptr_t out, int64_t os, int B, int Hq, int Hkv, int D, int bs, float scale,
                                  int splits, int apply_rope, uintptr_t st, int depth) {
    check(xgk::decode_attention_fq(P<const float>(part), S_, P<const int32_t>(pos), P<const float>(cs),
                                   P<const int32_t>(slots), P<uint16_t>(kc), P<uint16_t>(vc), P<const int32_t>(bt),
                                   bts, P<const int32_t>(sl), P<float>(po), P<float>(pl), P<uint16_t>(out), os, B, Hq,
                                   Hkv, D, bs, scale, splits, apply_rope, S(st), depth),
          "decode_attention_fq");
  }, py::arg("part"), py::arg("S"), py::arg("pos"), py::arg("cs"), py::arg("slots"), py::arg("kc"), py::arg("vc"),
     py::arg("bt"), py::arg("bts"), py::arg("sl"), py::arg("po"), py::arg("pl"), py::arg("out"), py::arg("os"),
     py::arg("B"), py::arg("Hq"), py::arg("Hkv"), py::arg("D"), py::arg("bs"), py::arg("scale"), py::arg("splits"),
     py::arg("apply_rope"), py::arg("st"), py::arg("depth") = 2);
  m.def("moe_gemm_m64g", [](uintptr_t x, uintptr_t rows, uintptr_t offs, int E, int K, uintptr_t w, int N, int P_,
                            uintptr_t part, uintptr_t out, int splits, int mode, int nw, int cfg, uintptr_t st) {
    check(xgk::moe_gemm_m64g(P<const uint16_t>(x), P<const int32_t>(rows), P<const int32_t>(offs), E, K,
                             P<const uint16_t>(w), N, P_, P<float>(part), P<uint16_t>(out), splits, mode, nw, cfg,
                             64, S(st), nullptr),
          "moe_gemm_m64g");
  });
  // same, with a host-known bound on the real rows of any expert (<= 16: one-x-tile kernel)
  // valid: the sorted rows (-1 = pad) -> per-workgroup 16/32/64-row body; 0: all rows
  m.def("moe_gemm_m64g_rows", [](uintptr_t x, uintptr_t rows, uintptr_t offs, int E, int K, uintptr_t w, int N, int P_,
                                 uintptr_t part, uintptr_t out, int splits, int mode, int nw, int cfg, int max_rows,
                                 uintptr_t st, uintptr_t valid, int pairs) {
    check(xgk::moe_gemm_m64g(P<const uint16_t>(x), P<const int32_t>(rows), P<const int32_t>(offs), E, K,
                             P<const uint16_t>(w), N, P_, P<float>(part), P<uint16_t>(out), splits, mode, nw, cfg,
                             max_rows, S(st), P<const int32_t>(valid), nullptr, pairs),
          "moe_gemm_m64g_rows");
  }, py::arg("x"), py::arg("rows"), py::arg("offs"), py::arg("E"), py::arg("K"), py::arg("w"), py::arg("N"),
     py::arg("P"), py::arg("part"), py::arg("out"), py::arg("splits"), py::arg("mode"), py::arg("nw"), py::arg("cfg"),
     py::arg("max_rows"), py::arg("st"), py::arg("valid") = 0, py::arg("pairs") = 0);
  // w2 of the fused MoE decode layer with the weighted combine + residual add in the
  // launch (GG_MOE_RESID = 4): resid[T, N] += sum_j w[t, j] * (sum_s part[s, dest[t, j]]),
  // ss_out[N / cols, T] = per-column-tile sum of squares of the new residual
  m.def("moe_gemm_m64g_resid", [](uintptr_t x, uintptr_t rows, uintptr_t offs, int E, int K, uintptr_t w, int N,
                                  int P_, uintptr_t part, int splits, int nw, int cfg, int max_rows, uintptr_t st,
                                  uintptr_t valid, uintptr_t dest, uintptr_t wts, uintptr_t resid, uintptr_t ss_out,
                                  uintptr_t counters, int T, int k, int pairs) {
    const xgk::MoeResidEpi e{P<const int32_t>(dest), P<const float>(wts), P<uint16_t>(resid), P<float>(ss_out),
                             P<int>(counters), T, k};
    check(xgk::moe_gemm_m64g(P<const uint16_t>(x), P<const int32_t>(rows), P<const int32_t>(offs), E, K,
                             P<const uint16_t>(w), N, P_, P<float>(part), nullptr, splits, 4, nw, cfg, max_rows,
                             S(st), P<const int32_t>(valid), &e, pairs),
          "moe_gemm_m64g_resid");
  }, py::arg("x"), py::arg("rows"), py::arg("offs"), py::arg("E"), py::arg("K"), py::arg("w"), py::arg("N"),
     py::arg("P"), py::arg("part"), py::arg("splits"), py::arg("nw"), py::arg("cfg"), py::arg("max_rows"),
     py::arg("st"), py::arg("valid"), py::arg("dest"), py::arg("wts"), py::arg("resid"), py::arg("ss_out"),
     py::arg("counters"), py::arg("T"), py::arg("k"), py::arg("pairs") = 0);
  m.def("moe_route", [](uintptr_t h, uintptr_t wr, int T, int H, int E, int k, int renorm, uintptr_t w, uintptr_t ids,
                        uintptr_t st, uintptr_t norm_w, float eps, uintptr_t hn, uintptr_t al_rows, uintptr_t al_offs,
                        uintptr_t al_dest, int al_E, int al_eoff, int al_bm) {
    // norm_w / hn != 0: h is the raw residual stream, normalised in-kernel (fused decode layer);
    // al_rows != 0 (T == 1): also moe_align's layout of this rank's al_E experts
    check(xgk::moe_route(P<const uint16_t>(h), P<const uint16_t>(wr), T, H, E, k, renorm, P<float>(w),
                         P<int32_t>(ids), S(st), P<const uint16_t>(norm_w), eps, P<uint16_t>(hn), P<int32_t>(al_rows),
                         P<int32_t>(al_offs), P<int32_t>(al_dest), al_E, al_eoff, al_bm),
          "moe_route");
  }, py::arg("h"), py::arg("wr"), py::arg("T"), py::arg("H"), py::arg("E"), py::arg("k"), py::arg("renorm"),
     py::arg("w"), py::arg("ids"), py::arg("st"), py::arg("norm_w") = 0, py::arg("eps") = 0.f, py::arg("hn") = 0,
     py::arg("al_rows") = 0, py::arg("al_offs") = 0, py::arg("al_dest") = 0, py::arg("al_E") = 0,
     py::arg("al_eoff") = 0, py::arg("al_bm") = 64);
  m.def("moe_combine_resid", [](uintptr_t part, int splits, int P_, uintptr_t dest, uintptr_t w, uintptr_t resid,
                                uintptr_t ss, int T, int k, int H, uintptr_t st) {
    if (H % 1024 || H > 8192) throw std::invalid_argument("moe_combine_resid: H % 1024 == 0, H <= 8192");
    check(xgk::moe_combine_resid(P<const float>(part), splits, P_, P<const int32_t>(dest), P<const float>(w),
                                 P<uint16_t>(resid), P<float>(ss), T, k, H, S(st)),
          "moe_combine_resid");
  });
  m.def("ep_plan", [](uintptr_t ids, int n_pairs, int E_local, int tp, int cap, int packed, uintptr_t slot,
                      uintptr_t send_eid, uintptr_t counts, uintptr_t st) {
    if (tp < 1 || tp > 8) throw std::invalid_argument("ep_plan: 1 <= tp <= 8");
    if (E_local < 1 || n_pairs < 0) throw std::invalid_argument("ep_plan: E_local >= 1, n_pairs >= 0");
    if (!packed && cap < n_pairs)  // every pair may go to one rank: no slot may overflow
      throw std::invalid_argument("ep_plan: capacity layout needs cap >= n_pairs");
    check(xgk::ep_plan(P<const int32_t>(ids), n_pairs, E_local, tp, cap, packed, P<int32_t>(slot),
                       P<int32_t>(send_eid), P<int32_t>(counts), S(st)),
          "ep_plan");
  });
  m.def("ep_scatter", [](uintptr_t x, int64_t x_stride, int k, uintptr_t slot, int n_pairs, int H, uintptr_t send,
                         uintptr_t st) {
    check(xgk::ep_scatter(P<const uint16_t>(x), x_stride, k, P<const int32_t>(slot), n_pairs, H, P<uint16_t>(send),
                          S(st)),
          "ep_scatter");
  });
  m.def("moe_combine", [](uintptr_t y, int splits, int P_, uintptr_t dest, uintptr_t w, uintptr_t out, int T, int k,
                          int H, uintptr_t st, int out_f32) {
    check(xgk::moe_combine(P<const void>(y), splits, P_, P<const int32_t>(dest), P<const float>(w), P<void>(out),
                           T, k, H, S(st), out_f32),
          "moe_combine");
  }, py::arg("y"), py::arg("splits"), py::arg("P"), py::arg("dest"), py::arg("w"), py::arg("out"), py::arg("T"),
     py::arg("k"), py::arg("H"), py::arg("st"), py::arg("out_f32") = 0);
  m.def("device_synchronize", []() {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) throw std::runtime_error(hipGetErrorString(e));
  });

  // ---- custom one-shot xGMI all-reduce (csrc/comm/custom_allreduce.hip)
  m.def("car_wallclock_khz", []() { return xgk::car_wallclock_khz(); });
  // CU-partitioned streams (engine/partition.py): a HIP stream whose dispatches -- kernels
  // and graph launches alike -- run only on the CUs set in `mask` (32 CUs per word)
  m.def("cu_mask_stream_create", [](std::vector<uint32_t> mask) {
    hipStream_t st = nullptr;
    const hipError_t e = hipExtStreamCreateWithCUMask(&st, static_cast<uint32_t>(mask.size()), mask.data());
    if (e != hipSuccess) throw std::runtime_error(std::string("hipExtStreamCreateWithCUMask: ") + hipGetErrorString(e));
    return reinterpret_cast<uintptr_t>(st);
  });
  m.def("cu_mask_stream_get", [](uintptr_t st, int words) {
    std::vector<uint32_t> mask(static_cast<size_t>(words), 0u);
    const hipError_t e = hipExtStreamGetCUMask(reinterpret_cast<hipStream_t>(st), static_cast<uint32_t>(words),
                                               mask.data());
    if (e != hipSuccess) throw std::runtime_error(std::string("hipExtStreamGetCUMask: ") + hipGetErrorString(e));
    return mask;
  });
  m.def("stream_destroy", [](uintptr_t st) { (void)hipStreamDestroy(reinterpret_cast<hipStream_t>(st)); });
  m.def("car_limits", []() { return py::make_tuple(xgk::car_max_ranks(), xgk::car_max_blocks(), xgk::car_chunk()); });
  m.def("car_alloc_uncached", [](int64_t bytes) {
    void* p = nullptr;
    if (xgk::car_alloc_uncached(bytes, &p)) throw std::runtime_error("car_alloc_uncached failed");
    return reinterpret_cast<uintptr_t>(p);
  });
  m.def("car_ipc_handle", [](uintptr_t ptr) {
    hipIpcMemHandle_t h;
    if (xgk::car_ipc_handle(reinterpret_cast<void*>(ptr), &h)) throw std::runtime_error("hipIpcGetMemHandle failed");
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  });
  m.def("car_ipc_open", [](py::bytes handle) {
    std::string s = handle;
    if (s.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("bad IPC handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, s.data(), sizeof(h));
    void* p = nullptr;
    if (xgk::car_ipc_open(&h, &p)) throw std::runtime_error("hipIpcOpenMemHandle failed");
    return reinterpret_cast<uintptr_t>(p);
  });
  m.def("car_ipc_close", [](uintptr_t p) { return xgk::car_ipc_close(reinterpret_cast<void*>(p)) == 0; });
  m.def("car_free", [](uintptr_t p) { return xgk::car_free(reinterpret_cast<void*>(p)) == 0; });
  m.def("custom_allreduce", [](uintptr_t in, uintptr_t out, int64_t nbytes, int64_t slot_bytes,
                               std::vector<uintptr_t> data, std::vector<uintptr_t> sig, int rank, uintptr_t gens,
                               uintptr_t err, uintptr_t st) {
    if (data.size() != sig.size()) throw std::invalid_argument("custom_allreduce: pointer lists differ in size");
    check(xgk::custom_allreduce(P<void>(in), P<void>(out), nbytes, slot_bytes, data.data(), sig.data(), rank,
                                static_cast<int>(data.size()), P<uint32_t>(gens), P<uint32_t>(err), S(st)),
          "custom_allreduce");
  });
  m.def("custom_allreduce_2shot", [](uintptr_t in, uintptr_t out, int64_t nbytes, int64_t slot_bytes,
                                     std::vector<uintptr_t> data, std::vector<uintptr_t> sig, int rank,
                                     uintptr_t gens, uintptr_t err, uintptr_t st) {
    if (data.size() != sig.size()) throw std::invalid_argument("custom_allreduce_2shot: pointer lists differ");
    check(xgk::custom_allreduce_2shot(P<void>(in), P<void>(out), nbytes, slot_bytes, data.data(), sig.data(), rank,
                                      static_cast<int>(data.size()), P<uint32_t>(gens), P<uint32_t>(err), S(st)),
          "custom_allreduce_2shot");
  });
  // push ("LL") protocol: flag-in-payload lines written into the peers' receive regions
  m.def("car_ll_max_bytes", [](int64_t region) { return xgk::car_ll_max_bytes(region); });
  m.def("custom_allreduce_ll", [](uintptr_t in, uintptr_t out, int64_t nbytes, int64_t region,
                                  std::vector<uintptr_t> data, int rank, uintptr_t gens, uintptr_t err, uintptr_t st) {
    check(xgk::custom_allreduce_ll(P<void>(in), P<void>(out), nbytes, region, data.data(), rank,
                                   static_cast<int>(data.size()), P<uint32_t>(gens), P<uint32_t>(err), S(st)),
          "custom_allreduce_ll");
  });
  m.def("custom_allreduce_resid_ll", [](uintptr_t part, int S_, int T, uintptr_t resid, uintptr_t ss_part, int H,
                                        int64_t region, std::vector<uintptr_t> data, int rank, uintptr_t gens,
                                        uintptr_t err, uintptr_t st, int loop) {
    check(xgk::custom_allreduce_resid_ll(P<const float>(part), S_, T, P<uint16_t>(resid), P<float>(ss_part), H,
                                         region, data.data(), rank, static_cast<int>(data.size()), P<uint32_t>(gens),
                                         P<uint32_t>(err), S(st), loop),
          "custom_allreduce_resid_ll");
  }, py::arg("part"), py::arg("S"), py::arg("T"), py::arg("resid"), py::arg("ss_part"), py::arg("H"),
     py::arg("region"), py::arg("data"), py::arg("rank"), py::arg("gens"), py::arg("err"), py::arg("st"),
     py::arg("loop") = 0);
  m.def("custom_allreduce_resid", [](uintptr_t part, int S_, int T, uintptr_t resid, uintptr_t ss_part, int H,
                                     int64_t slot_bytes, std::vector<uintptr_t> data, std::vector<uintptr_t> sig,
                                     int rank, uintptr_t gens, uintptr_t err, uintptr_t st) {
    if (data.size() != sig.size()) throw std::invalid_argument("custom_allreduce_resid: pointer lists differ");
    if (T < 1 || S_ < 1 || H % 1024 || static_cast<int64_t>(T) * (H / 1024) > xgk::car_max_blocks() ||
        static_cast<int64_t>(T) * H * 2 > slot_bytes)
      throw std::invalid_argument("custom_allreduce_resid: T * H/1024 must fit the block table and T * H * 2 the slot");
    check(xgk::custom_allreduce_resid(P<const float>(part), S_, T, P<uint16_t>(resid), P<float>(ss_part), H,
                                      slot_bytes, data.data(), sig.data(), rank, static_cast<int>(data.size()),
                                      P<uint32_t>(gens), P<uint32_t>(err), S(st)),
          "custom_allreduce_resid");
  });
  m.def("custom_allgather_lastdim", [](uintptr_t in, uintptr_t out, int64_t rows, int64_t cb, int64_t slot_bytes,
                                       std::vector<uintptr_t> data, std::vector<uintptr_t> sig, int rank,
                                       uintptr_t gens, uintptr_t err, uintptr_t st) {
    if (data.size() != sig.size()) throw std::invalid_argument("custom_allgather_lastdim: pointer lists differ");
    if (rows < 1 || cb < 16 || cb % 16 || rows * cb > slot_bytes)
      throw std::invalid_argument("custom_allgather_lastdim: row bytes must be a multiple of 16 and fit the slot");
    check(xgk::custom_allgather_lastdim(P<const void>(in), P<void>(out), rows, cb, slot_bytes, data.data(),
                                        sig.data(), rank, static_cast<int>(data.size()), P<uint32_t>(gens),
                                        P<uint32_t>(err), S(st)),
          "custom_allgather_lastdim");
  });

}
