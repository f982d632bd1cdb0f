#!/usr/bin/env python3
"""Micro-benchmarks of the hot kernels at Llama-3-8B decode/prefill shapes on one
MI355X. Reports time and achieved HBM bandwidth (bytes the op must move)."""
import argparse
import json
import math

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xgserve import ops


def timeit(fn, iters=50, warm=10):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0  # us


def paged(B, L, Hkv, D, bs, dev):
    pages = (L + bs - 1) // bs
    NB = B * pages + 16
    kc = torch.randn(NB, Hkv, bs, D, device=dev).bfloat16()
    vc = torch.randn(NB, Hkv, bs, D, device=dev).bfloat16()
    bt = torch.randperm(NB, device=dev)[:B * pages].view(B, pages).int()
    return kc, vc, bt


def bench_decode(res, B, L, splits_list, Hq=32, Hkv=8, D=128, bs=16):
    dev = "cuda"
    kc, vc, bt = paged(B, L, Hkv, D, bs, dev)
    q = torch.randn(B, Hq, D, device=dev).bfloat16()
    sl = torch.full((B,), L, dtype=torch.int32, device=dev)
    ws = ops.attention.DecodeWorkspace(B, Hq, D, 64, dev)
    out = torch.empty(B, Hq, D, device=dev, dtype=torch.bfloat16)
    nbytes = B * L * Hkv * D * 2 * 2
    for s in splits_list:
        us = timeit(lambda: ops.decode_attention(q, kc, vc, bt, sl, 1 / math.sqrt(D), s, ws, out))
        res.append({"op": "decode_attention", "B": B, "L": L, "splits": s, "us": round(us, 2),
                    "TB/s": round(nbytes / us / 1e6, 3)})


def bench_decode_fq(res, B, L, S_qkv, stagger=0, Hq=32, Hkv=8, D=128, bs=16):
    """Fused-QKV decode attention (the dense decode layer's form): QKV split-K
    partials -> RoPE + KV append + attention, next to the plain kernel at the same
    lengths. stagger > 0: sequence b has L - U[0, stagger) keys (a batch in flight)."""
    from xgserve.ops.linear import PendingSum
    dev = "cuda"
    kc, vc, bt = paged(B, L, Hkv, D, bs, dev)
    g = torch.Generator().manual_seed(0)
    lens = (L - torch.randint(0, max(stagger, 1), (B,), generator=g)).int().to(dev)
    pos = (lens - 1).int()
    slots = (bt.gather(1, (pos // bs).long().view(B, 1)).view(B) * bs + pos % bs).int()
    cs = torch.randn(L + 16, D, device=dev)
    part = torch.randn(S_qkv, B, (Hq + 2 * Hkv) * D, device=dev)
    pend = PendingSum(part, S_qkv)
    q = torch.randn(B, Hq, D, device=dev).bfloat16()
    out = torch.empty(B, Hq * D, device=dev, dtype=torch.bfloat16)
    nbytes = int(lens.sum().item()) * Hkv * D * 2 * 2
    sc = 1 / math.sqrt(D)
    us = timeit(lambda: ops.decode_attention_fused(pend, pos, slots, cs, kc, vc, bt, lens, Hq, sc, 1, None,
                                                   out=out))
    res.append({"op": "decode_attention_fq", "B": B, "L": L, "stagger": stagger, "S_qkv": S_qkv, "us": round(us, 2),
                "TB/s": round(nbytes / us / 1e6, 3)})
    o3 = out.view(B, Hq, D)
    us = timeit(lambda: ops.decode_attention(q, kc, vc, bt, lens, sc, 1, None, o3))
    res.append({"op": "decode_attention", "B": B, "L": L, "stagger": stagger, "splits": 1, "us": round(us, 2),
                "TB/s": round(nbytes / us / 1e6, 3)})


def bench_sampling(res, B, V=128256):
    """Greedy argmax and temperature / top-p / top-k sampling over bf16 logits."""
    dev = "cuda"
    logits = (torch.randn(B, V, device=dev) * 3).bfloat16()
    nbytes = B * V * 2
    us = timeit(lambda: ops.argmax_logprob(logits))
    res.append({"op": "argmax", "B": B, "V": V, "us": round(us, 2), "TB/s": round(nbytes / us / 1e6, 3)})
    temps = torch.full((B,), 0.8, device=dev)
    seeds = torch.arange(B, dtype=torch.int64, device=dev)
    for name, tp, tk in (("temp", None, None), ("top_p0.9", torch.full((B,), 0.9, device=dev), None),
                         ("top_k50", None, torch.full((B,), 50, dtype=torch.int32, device=dev)),
                         ("top_p0.9+k50", torch.full((B,), 0.9, device=dev),
                          torch.full((B,), 50, dtype=torch.int32, device=dev))):
        us = timeit(lambda: ops.sample_tokens(logits, temps, tp, tk, seeds, 7), iters=20, warm=3)
        res.append({"op": "sample_" + name, "B": B, "V": V, "us": round(us, 2)})


def bench_prefill(res, T, Hq=32, Hkv=8, D=128, bs=16):
    dev = "cuda"
    kc, vc, bt = paged(1, T, Hkv, D, bs, dev)
    q = torch.randn(T, Hq, D, device=dev).bfloat16()
    qsl = torch.tensor([0, T], dtype=torch.int32, device=dev)
    sl = torch.tensor([T], dtype=torch.int32, device=dev)
    out = torch.empty(T, Hq, D, device=dev, dtype=torch.bfloat16)
    us = timeit(lambda: ops.prefill_attention(q, kc, vc, bt, qsl, sl, T, 1 / math.sqrt(D), out), iters=20)
    flops = 4 * Hq * D * T * T / 2
    res.append({"op": "prefill_attention", "T": T, "us": round(us, 1), "TFLOP/s": round(flops / us / 1e6, 1)})


def bench_gemm(res, M, N, K):
    dev = "cuda"
    x = torch.randn(M, K, device=dev).bfloat16()
    w = torch.randn(N, K, device=dev).bfloat16()
    us = timeit(lambda: torch.nn.functional.linear(x, w))
    res.append({"op": "hipblaslt_linear", "M": M, "N": N, "K": K, "us": round(us, 2),
                "TB/s(weights)": round(N * K * 2 / us / 1e6, 3)})
    if hasattr(ops, "skinny_linear"):
        from xgserve.ops.linear import MODE_PARTIAL, choose_split
        S = choose_split(M, N, K)
        us2 = timeit(lambda: ops.skinny_linear(x, w, S, MODE_PARTIAL))
        res.append({"op": "xgk_skinny_linear(partial)", "M": M, "N": N, "K": K, "S": S, "us": round(us2, 2),
                    "TB/s(weights)": round(N * K * 2 / us2 / 1e6, 3)})


def bench_small(res, T=64, H=4096, F=14336):
    dev = "cuda"
    x = torch.randn(T, H, device=dev).bfloat16()
    r = torch.randn(T, H, device=dev).bfloat16()
    w = torch.randn(H, device=dev).bfloat16()
    res.append({"op": "fused_add_rmsnorm", "T": T, "us": round(timeit(lambda: ops.fused_add_rmsnorm(x, r, w, 1e-5)), 2)})
    gu = torch.randn(T, 2 * F, device=dev).bfloat16()
    res.append({"op": "silu_and_mul", "T": T, "us": round(timeit(lambda: ops.silu_and_mul(gu)), 2)})


def bench_moe_route(res, H=4096, E=8, k=2, layers=32):
    """Mixtral batch-1 router (RMSNorm + router GEMV + top-k + align, one launch) next to a
    trivial one-workgroup kernel at the same shape (the launch floor); router weights
    rotate over `layers` copies as in a decode step."""
    dev = "cuda"
    resid = torch.randn(1, H, device=dev).bfloat16()
    nw = torch.ones(H, device=dev).bfloat16()
    routers = [(torch.randn(E, H, device=dev) * 0.02).bfloat16() for _ in range(layers)]
    i = [0]

    def route():
        i[0] += 1
        return ops.moe.moe_route_norm(resid, nw, 1e-5, routers[i[0] % layers], k, align=(E, 0))

    def graphed(fn, n=64):
        """device time per call: n calls captured in one HIP graph (no host launch cost)"""
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(n):
                    fn()
        torch.cuda.synchronize()
        return timeit(g.replay, iters=20, warm=3) / n

    res.append({"op": "moe_route_norm+align", "T": 1, "E": E, "us_graph": round(graphed(route), 2)})
    res.append({"op": "moe_route(no norm, no align)", "T": 1, "E": E,
                "us_graph": round(graphed(lambda: ops.moe.moe_route(resid, routers[0], k)), 2)})
    res.append({"op": "rmsnorm (launch floor)", "T": 1, "us_graph": round(graphed(lambda: ops.rmsnorm(resid, nw, 1e-5)), 2)})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="all")
    a = ap.parse_args()
    res = []
    if a.what in ("all", "decode"):
        bench_decode(res, 64, 800, [1, 2, 4])
        bench_decode(res, 1, 1024, [1, 8, 16, 32])
        bench_decode(res, 256, 2048, [1, 2])
        bench_decode_fq(res, 64, 768, 4, stagger=256)
        bench_decode_fq(res, 64, 640, 4, stagger=128)
        bench_decode_fq(res, 64, 800, 4)
        bench_decode_fq(res, 64, 2048, 4)
    if a.what in ("all", "prefill"):
        for T in (512, 2048, 8192):
            bench_prefill(res, T)
    if a.what in ("all", "gemm"):
        for (N, K) in ((6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)):
            for M in (1, 64):
                bench_gemm(res, M, N, K)
    if a.what in ("all", "sampling"):
        for B in (1, 64):
            bench_sampling(res, B)
    if a.what in ("all", "small"):
        bench_small(res)
    if a.what in ("all", "moe"):
        bench_moe_route(res)
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
