#!/usr/bin/env python3
"""Decode-GEMM shoot-out on one MI355X: hipBLASLt (F.linear) vs the hand-written
kernels at the Llama-3-8B projection shapes, cold weights (a ring of weight
copies larger than the 256 MB Infinity Cache, as in a real decode step where
every layer's weights are touched once). Also checks numerics vs fp32."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xgserve.ops import linear as L  # noqa: E402
from xgserve.ops._native import kernels  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096),
          # Llama-3-70B (TP1 / TP8) and Llama-3-8B TP2 shards
          "qkv70": (10240, 8192), "o70": (8192, 8192), "gate_up70": (57344, 8192), "down70": (8192, 28672),
          "qkv70t8": (1280, 8192), "o70t8": (8192, 1024), "gate_up70t8": (7168, 8192), "down70t8": (8192, 3584),
          "qkv8t2": (3072, 4096), "o8t2": (4096, 2048), "gate_up8t2": (14336, 4096), "down8t2": (4096, 7168),
          "qkv8t4": (1536, 4096), "o8t4": (4096, 1024), "gate_up8t4": (7168, 4096), "down8t4": (4096, 3584),
          "qkv8t8": (768, 4096), "o8t8": (4096, 512), "gate_up8t8": (3584, 4096), "down8t8": (4096, 1792),
          "qkv70t2": (5120, 8192), "o70t2": (8192, 4096), "gate_up70t2": (28672, 8192), "down70t2": (8192, 14336),
          "qkv70t4": (2560, 8192), "o70t4": (8192, 2048), "gate_up70t4": (14336, 8192), "down70t4": (8192, 7168),
          # gate_up shapes as plain split-K partial GEMMs (what a split SiLU epilogue would stream)
          "gate_up_p": (28672, 4096), "gate_up70_p": (57344, 8192)}


def timeit(fns, iters=30, warm=5):
    """fns: list of zero-arg callables cycled per iteration (distinct weight copies)."""
    for i in range(warm):
        fns[i % len(fns)]()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fns[i % len(fns)]()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[32, 64])
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    ap.add_argument("--moe-sweep", action="store_true",
                    help="sweep the grouped (MoE) gemm_m64g configurations at Mixtral decode shapes")
    ap.add_argument("--w8-sweep", action="store_true",
                    help="every gemm_w8 (fp8 weight) configuration per shape at M <= 16, cold weights")
    ap.add_argument("--m64g-sweep", action="store_true",
                    help="sweep gemm_m64g (nw, split, cfg) configurations instead of the shoot-out")
    ap.add_argument("--mw-sweep", action="store_true",
                    help="sweep gemm_mw (split, cfg) configurations at 64 < M <= 320 against hipBLASLt")
    ap.add_argument("--top", type=int, default=6, help="--mw-sweep: configurations printed per (shape, M)")
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 3, 4, 5, 6, 8],
                    help="--m64g-sweep: split-K values of the partial-sum mode")
    a = ap.parse_args()
    kernels()
    if a.m64g_sweep:
        return m64g_sweep(a)
    if a.mw_sweep:
        return mw_sweep(a)
    if a.w8_sweep:
        return w8_sweep(a)
    if a.moe_sweep:
        return moe_sweep(a)
    dev = "cuda"
    for name in a.shapes:
        N, K = SHAPES[name]
        nbytes = N * K * 2
        copies = max(2, min(8, (1 << 30) // nbytes + 1))
        ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(copies)]
        for M in a.M:
            x = torch.randn(M, K, device=dev).bfloat16()
            ref = x.float() @ ws[0].float().t()
            rows = []
            us = timeit([lambda w=w: F.linear(x, w) for w in ws])
            rows.append(("hipblaslt", us, None))
            mode = L.MODE_SILU if name.startswith("gate_up") and not name.endswith("_p") else (L.MODE_BF16 if name == "lm_head" else L.MODE_PARTIAL)
            if M <= 16:
                for S in ((1,) if mode != L.MODE_PARTIAL else (1, 2, 4, 7, 8, 14, 16)):
                    if K % (S * 256) or (mode == L.MODE_PARTIAL and N % 64):
                        continue
                    fn = lambda w, S=S: L.skinny_linear(x, w, S, mode)  # noqa: E731
                    us3 = timeit([lambda w=w, fn=fn: fn(w) for w in ws])
                    rows.append((f"skinny(S={S},mode={mode})", us3, None))
            plan = L.m64_plan(M, N, K, mode)
            if plan is not None:
                for nw in ((1, 2) if mode == L.MODE_PARTIAL and N % 128 == 0 else (plan[0],)):
                    S = plan[1] if nw == plan[0] else L.m64_plan(M, N, K, mode)[1] * (2 if nw < plan[0] else 1)
                    if mode != L.MODE_PARTIAL:
                        S = 1
                    if K % (S * 256):
                        continue
                    for var in (0,):
                        fn = lambda w, nw=nw, S=S: L.m64_linear(x, w, mode, S, nw)  # noqa: E731
                        us2 = timeit([lambda w=w, fn=fn: fn(w) for w in ws])
                        y = fn(ws[0])
                        if mode == L.MODE_PARTIAL:
                            y = y.part.sum(0)
                            want = ref
                        elif mode == L.MODE_SILU:
                            g, u = L.deinterleave_gate_up(ws[0])
                            want = F.silu(x.float() @ g.float().t()) * (x.float() @ u.float().t())
                        else:
                            want = ref
                        err = float((y.float() - want).norm() / want.norm())
                        rows.append((f"gemm_m64g(nw={nw},S={S},mode={mode},plan)", us2, err))
            if M <= 16 or plan is None:
                pass
            for op, t, err in rows:
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "op": op, "us": round(t, 2),
                                  "TB/s": round(nbytes / t / 1e6, 3), "rel_err": err}), flush=True)
        del ws
        torch.cuda.empty_cache()


def w8_sweep(a):
    """gemm_w8 configurations (split-K x cfg) per shape, cold fp8 weights; prints the
    checked-correct ones, fastest first (TB/s counts the fp8 weight bytes)."""
    for name in a.shapes:
        N, K = SHAPES[name]
        nbytes = N * K
        copies = max(2, min(8, (1 << 30) // nbytes + 1))
        qs = [L.quantize_fp8(torch.randn(N, K, device="cuda") * 0.02) for _ in range(copies)]
        mode = L.MODE_SILU if name.startswith("gate_up") and not name.endswith("_p") else L.MODE_PARTIAL
        for M in a.M:
            if M > L.W8_MAX_M:
                continue
            x = torch.randn(M, K, device="cuda").bfloat16()
            wd = L.dequantize_fp8(*qs[0])
            if mode == L.MODE_SILU:
                g, u = L.deinterleave_gate_up(wd)
                want = F.silu(x.float() @ g.t()) * (x.float() @ u.t())
            else:
                want = x.float() @ wd.t()
            rows = []
            for cfg, (cols, kc) in L.W8_CFGS.items():
                for S in ((1,) if mode == L.MODE_SILU else (1, 2, 4, 8, 16)):
                    if N % cols or K % (S * kc) or (mode == L.MODE_SILU and cfg == 2) or (M > 16 and cfg >= 3):
                        continue

                    def fn(q, S=S, cfg=cfg):
                        return L.w8_linear(x, q[0], q[1], mode, plan=(S, cfg))
                    us = timeit([lambda q=q, fn=fn: fn(q) for q in qs])
                    y = fn(qs[0])
                    y = y.part.sum(0) if mode == L.MODE_PARTIAL else y.float()
                    rows.append((us, S, cfg, float((y - want).norm() / want.norm())))
            for us, S, cfg, err in sorted(rows):
                print(json.dumps({"shape": name, "M": M, "op": f"w8(S={S},cfg={cfg})", "us": round(us, 2),
                                  "TB/s": round(nbytes / us / 1e6, 3), "rel_err": round(err, 6)}), flush=True)
        del qs
        torch.cuda.empty_cache()


def m64g_sweep(a):
    """Every valid gemm_m64g configuration per shape (cold weights); prints the
    checked-correct ones, fastest first."""
    k = kernels()
    waves = {c: v[0] for c, v in L.M64G_CFGS.items()}
    kcs = {c: v[1] for c, v in L.M64G_CFGS.items()}
    for name in a.shapes:
        N, K = SHAPES[name]
        nbytes = N * K * 2
        copies = max(2, min(8, (1 << 30) // nbytes + 1))
        ws = [(torch.randn(N, K, device="cuda") * 0.02).bfloat16() for _ in range(copies)]
        mode = L.MODE_SILU if name.startswith("gate_up") and not name.endswith("_p") else (L.MODE_BF16 if name == "lm_head" else L.MODE_PARTIAL)
        cnt = L.tile_counters(torch.device("cuda"), N)
        for M in a.M:
            x = torch.randn(M, K, device="cuda").bfloat16()
            if mode == L.MODE_SILU:
                g, u = L.deinterleave_gate_up(ws[0])
                want = F.silu(x.float() @ g.float().t()) * (x.float() @ u.float().t())
            else:
                want = x.float() @ ws[0].float().t()
            rows = []
            for cfg in L.M64G_CFGS:
                if cfg in L.M64G_SMALL_ONLY and M > 16:
                    continue
                for nw in ((2,) if mode == L.MODE_SILU else (1, 2)):
                    for S in ((1, 2, 4) if mode == L.MODE_SILU else (1,) if mode != L.MODE_PARTIAL else
                              tuple(a.splits)):
                        cols = 16 * nw * waves[cfg]
                        if N % cols or K % kcs[cfg] or S > K // kcs[cfg] or (mode == L.MODE_SILU and K % (S * kcs[cfg])):
                            continue
                        part = torch.empty(S, M, N, dtype=torch.float32, device="cuda")
                        out = torch.empty(M, N // 2 if mode == L.MODE_SILU else N, dtype=torch.bfloat16,
                                          device="cuda")

                        def fn(w, nw=nw, S=S, cfg=cfg, part=part, out=out):
                            if mode == L.MODE_SILU and S > 1:
                                k.gemm_m64g_ex(x.data_ptr(), M, K, w.data_ptr(), N, part.data_ptr(), out.data_ptr(),
                                               S, mode, nw, cfg, 0, 0, 0, 0.0, 0, 0, cnt.data_ptr(),
                                               torch.cuda.current_stream().cuda_stream)
                                return
                            k.gemm_m64g(x.data_ptr(), M, K, w.data_ptr(), N,
                                        part.data_ptr() if mode == L.MODE_PARTIAL else 0,
                                        out.data_ptr() if mode != L.MODE_PARTIAL else 0, S, mode, nw, cfg,
                                        torch.cuda.current_stream().cuda_stream)
                        us = timeit([lambda w=w, fn=fn: fn(w) for w in ws])
                        fn(ws[0])
                        y = part.sum(0) if mode == L.MODE_PARTIAL else out.float()
                        err = float((y - want).norm() / want.norm())
                        rows.append((us, nw, S, cfg, err))
            for us, nw, S, cfg, err in sorted(rows):
                print(json.dumps({"shape": name, "M": M, "op": f"m64g(nw={nw},S={S},cfg={cfg})", "us": round(us, 2),
                                  "TB/s": round(nbytes / us / 1e6, 3), "wgs": N // (16 * nw * waves[cfg]) * S,
                                  "rel_err": round(err, 6)}), flush=True)
        del ws
        torch.cuda.empty_cache()


def mw_sweep(a):
    """gemm_mw: every valid (split, cfg) per shape and M (cold weights), checked against
    fp32; prints hipBLASLt and the fastest a.top configurations. TB/s counts the weight
    bytes, TF/s the 2 M N K flops."""
    k = kernels()
    st = torch.cuda.current_stream().cuda_stream
    for name in a.shapes:
        N, K = SHAPES[name]
        nbytes = N * K * 2
        copies = max(2, min(8, (1 << 30) // nbytes + 1))
        ws = [(torch.randn(N, K, device="cuda") * 0.02).bfloat16() for _ in range(copies)]
        mode = L.MODE_SILU if name.startswith("gate_up") and not name.endswith("_p") else (
            L.MODE_BF16 if name == "lm_head" else L.MODE_PARTIAL)
        for M in a.M:
            x = torch.randn(M, K, device="cuda").bfloat16()
            if mode == L.MODE_SILU:
                g, u = L.deinterleave_gate_up(ws[0])
                want = F.silu(x.float() @ g.float().t()) * (x.float() @ u.float().t())
            else:
                want = x.float() @ ws[0].float().t()
            flops = 2.0 * M * N * K

            def show(op, us, err, extra=None):
                print(json.dumps({"shape": name, "M": M, "op": op, "us": round(us, 2),
                                  "TB/s": round(nbytes / us / 1e6, 3), "TF/s": round(flops / us / 1e6, 1),
                                  "rel_err": None if err is None else round(err, 6), **(extra or {})}), flush=True)
            show("hipblaslt", timeit([lambda w=w: F.linear(x, w) for w in ws]), None)
            rows = []
            for cfg, (cols, _, _) in L.MW_CFGS.items():
                if N % cols:
                    continue
                splits = (1,) if mode != L.MODE_PARTIAL else tuple(
                    s for s in (1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16) if s <= K // 64 and (N // cols) * s <= 640)
                for S in splits:
                    part = torch.empty(S, M, N, dtype=torch.float32, device="cuda")
                    out = torch.empty(M, N // 2 if mode == L.MODE_SILU else N, dtype=torch.bfloat16, device="cuda")

                    def fn(w, S=S, cfg=cfg, part=part, out=out):
                        k.gemm_mw(x.data_ptr(), M, K, w.data_ptr(), N,
                                  part.data_ptr() if mode == L.MODE_PARTIAL else 0,
                                  out.data_ptr() if mode != L.MODE_PARTIAL else 0, S, mode, cfg, st)
                    try:
                        fn(ws[0])
                    except (RuntimeError, ValueError):
                        continue  # configuration cannot take this M (LDS)
                    torch.cuda.synchronize()
                    y = part.sum(0) if mode == L.MODE_PARTIAL else out.float()
                    err = float((y - want).norm() / want.norm())
                    us = timeit([lambda w=w, fn=fn: fn(w) for w in ws])
                    rows.append((us, S, cfg, err, (N // cols) * S))
            for us, S, cfg, err, wgs in sorted(rows)[:a.top]:
                show(f"mw(S={S},cfg={cfg})", us, err, {"wgs": wgs})
            if M <= 64 and L.m64_plan(M, N, K, mode) is not None:
                fn = lambda w: L.m64_linear(x, w, mode)  # noqa: E731
                show("m64g(plan)", timeit([lambda w=w: fn(w) for w in ws]), None)
        del ws
        torch.cuda.empty_cache()


def moe_sweep(a):
    """Mixtral-8x7B expert GEMMs at decode batch sizes a.M (top-2 of 8, random routing),
    every grouped gemm_m64g configuration, cold weights (2 copies of all experts)."""
    from xgserve.ops import moe as MO
    k = kernels()
    E, H, F = 8, 4096, 14336
    copies = 2
    w13s = [(torch.randn(E, 2 * F, H, device="cuda") * 0.02).bfloat16() for _ in range(copies)]
    w2s = [(torch.randn(E, H, F, device="cuda") * 0.02).bfloat16() for _ in range(copies)]
    st = torch.cuda.current_stream().cuda_stream
    for T in a.M:
        g = torch.Generator(device="cuda").manual_seed(T)
        ids = torch.stack([torch.randperm(E, generator=g, device="cuda")[:2] for _ in range(T)]).int()
        x = torch.randn(T, H, device="cuda").bfloat16()
        rows, offs, dest = MO.moe_align(ids, E, 0)
        P = rows.shape[0]
        act = torch.empty(P, F, dtype=torch.bfloat16, device="cuda")
        res = []
        for cfg in range(7):
            wv = 2 if cfg >= 4 else 4
            if (2 * F) % (32 * wv):
                continue
            for vd in (0, 1):
                fn = lambda w, cfg=cfg, vd=vd: k.moe_gemm_m64g_rows(  # noqa: E731
                    x.data_ptr(), rows.data_ptr(), offs.data_ptr(), E, H, w.data_ptr(), 2 * F, P, 0, act.data_ptr(), 1,
                    2, 2, cfg, 2 * T, st, rows.data_ptr() if vd else 0)
                res.append(("w13" + ("+rowdispatch" if vd else ""), timeit([lambda w=w, fn=fn: fn(w) for w in w13s]),
                            2, 1, cfg))
        for cfg in range(7):
            wv = 2 if cfg >= 4 else 4
            kc = 64 if cfg in (2, 3, 4, 5) else 128
            for nw in (1, 2):
                for S in (1, 2, 4, 8):
                    if H % (16 * nw * wv) or F % (S * kc):
                        continue
                    part = torch.empty(S, P, H, dtype=torch.float32, device="cuda")
                    for vd in (0, 1):
                        fn = lambda w, cfg=cfg, nw=nw, S=S, part=part, vd=vd: k.moe_gemm_m64g_rows(  # noqa: E731
                            act.data_ptr(), 0, offs.data_ptr(), E, F, w.data_ptr(), H, P, part.data_ptr(), 0, S, 1, nw,
                            cfg, 2 * T, st, rows.data_ptr() if vd else 0)
                        res.append(("w2" + ("+rowdispatch" if vd else ""),
                                    timeit([lambda w=w, fn=fn: fn(w) for w in w2s]), nw, S, cfg))
        for name in ("w13", "w13+rowdispatch", "w2", "w2+rowdispatch"):
            for us, nw, S, cfg in sorted((r[1], r[2], r[3], r[4]) for r in res if r[0] == name)[:8]:
                print(json.dumps({"moe": name, "T": T, "P": P, "nw": nw, "S": S, "cfg": cfg, "us": round(us, 2)}),
                      flush=True)


if __name__ == "__main__":
    main()
