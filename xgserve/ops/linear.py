"""Decode-regime projections on the skinny HIP GEMM (csrc/kernels/skinny_gemm.hip).

`PendingSum` is a value that exists only as fp32 split-K partial sums; the
kernels that consume it (add_partials_rmsnorm, rope_cache_partials) reduce it
in their prologue, so a split-K GEMM costs no extra reduction launch.
"""
from __future__ import annotations

import functools

from dataclasses import dataclass
from typing import Optional

import torch

from .. import tune
from ._native import kernels, stream_ptr, use_native

MODE_BF16, MODE_PARTIAL, MODE_SILU = 0, 1, 2
_SPLITS = (1, 2, 4, 7, 8, 14, 16)


@dataclass
class PendingSum:
    part: torch.Tensor  # [S, M, N] fp32
    S: int

    @property
    def shape(self):
        return self.part.shape[1:]

    def materialize(self) -> torch.Tensor:
        S, M, N = self.part.shape
        out = torch.empty(M, N, dtype=torch.bfloat16, device=self.part.device)
        kernels().reduce_partials(self.part.data_ptr(), S, M * N, out.data_ptr(), stream_ptr())
        return out


def pick_split(N: int, K: int, target_wgs: int = 512) -> int:
    """Smallest split-K giving >= target_wgs workgroups of 32 columns (K % (S*256) == 0).
    512 (two per CU) measured best at M <= 16 on MI355X: Llama-3-8B down_proj 25.2 -> 22.9 us,
    QKV / O unchanged (bench/gemm_bench.py --M 1 4)."""
    nb = N // 32
    best = None
    for s in _SPLITS:
        if K % (s * 256):
            continue
        best = s
        if nb * s >= target_wgs:
            break
    return best or 0


_SLAB_KMAX = {}


def choose_split(M: int, N: int, K: int, target_wgs: int = 512) -> int:
    """Split-K for a given batch size: the slab kernel (16 < M <= 64) needs K/S to fit
    its LDS slab and 64-column tiles; the streaming kernel needs K % (S*256) == 0."""
    if 16 < M <= 64 and N % 64 == 0:
        kmax = _SLAB_KMAX.get(M)
        if kmax is None:
            kmax = _SLAB_KMAX[M] = kernels().skinny_slab_kmax(M)
        if K % kmax == 0:  # the slab kernel takes exactly kmax of K per workgroup
            return K // kmax
    return pick_split(N, K, target_wgs)


def skinny_linear(x: torch.Tensor, w: torch.Tensor, split_k: Optional[int] = None, mode: int = MODE_BF16,
                  out: Optional[torch.Tensor] = None):
    """x [M, K] bf16, w [N, K] bf16 -> bf16 [M, N] (MODE_BF16), PendingSum (MODE_PARTIAL),
    or silu(gate)*up [M, N/2] for a block-16 interleaved gate|up weight (MODE_SILU)."""
    M, K = x.shape
    N = w.shape[0]
    if mode == MODE_PARTIAL:
        S = split_k or choose_split(M, N, K)
        part = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
        kernels().skinny_gemm(x.data_ptr(), M, K, w.data_ptr(), N, part.data_ptr(), 0, S, MODE_PARTIAL, stream_ptr())
        return PendingSum(part, S)
    ncol = N // 2 if mode == MODE_SILU else N
    if out is None:
        out = torch.empty(M, ncol, dtype=torch.bfloat16, device=x.device)
    kernels().skinny_gemm(x.data_ptr(), M, K, w.data_ptr(), N, 0, out.data_ptr(), 1, mode, stream_ptr())
    return out


# gemm_m64g launch configurations (csrc/kernels/gemm_m64g.hip launch_m64g):
# cfg -> (waves per workgroup, k chunk, non-temporal weight DMA)
# 8-10: deep LDS rings (5 / 4 / 6 slots) for M <= 16 -- more weight bytes in flight per CU
M64G_CFGS = {0: (4, 128, False), 1: (4, 128, True), 2: (4, 64, False), 3: (4, 64, True),
             4: (2, 64, False), 5: (2, 64, True), 6: (2, 128, True), 7: (8, 64, True),
             8: (2, 128, True), 9: (4, 128, True), 10: (2, 64, True)}
# (Deep four-x-tile rings -- KC 64, 4-6 slots at M = 64 -- ran the 8B gate_up at 38.1
# vs 41.7 us in isolation but +0.1 % end to end (10,756 vs 10,742 tok/s, 400 steps,
# profiles/r6/r6s_m64g_sweep.md), and were not kept.)
M64G_SMALL_ONLY = (8, 9, 10)

# Measured on MI355X with cold weights (bench/gemm_bench.py --m64g-sweep,
# profiles/r1_m64g_sweep.jsonl; bucket 16 re-swept with the MT=1 kernel: r1_m64g_mt1_sweep.jsonl): (N, K, mode) -> {M bucket: (nw, split_k, cfg)}.
# Bucket 64 serves 40 < M <= 64, bucket 32 serves 16 < M <= 40 (falls back to 64),
# bucket 16 serves M <= 16 -- only shapes that have one take gemm_m64g at M <= 16
# (it beats the register-streaming skinny kernel there: 8B batch 1 QKV 12.3 -> 9.8 us,
# down 22.9 -> 19.2 us); the rest keep the skinny kernel.
_M64_TUNED = {
    # Llama-3-8B / Mixtral attention, TP1
    # 16 / 32 re-swept with K rotation in round 4 (profiles/r4_m64g_sweep_m1.jsonl; 64: r4_m64g_sweep_rot.jsonl)
    (6144, 4096, MODE_PARTIAL): {64: (2, 5, 3), 32: (1, 5, 7), 16: (1, 2, 9)},
    (4096, 4096, MODE_PARTIAL): {64: (1, 4, 0), 32: (1, 4, 0), 16: (1, 3, 0)},
    # bucket 16: the fused (row-scaled) form's sweep, r6/r6_fused_plans.md (batch 1 +3 %)
    (28672, 4096, MODE_SILU): {64: (2, 1, 1), 32: (2, 1, 3), 16: (2, 1, 3)},
    (4096, 14336, MODE_PARTIAL): {64: (2, 8, 3), 32: (1, 4, 1), 16: (1, 4, 9)},
    # Llama-3-70B TP1
    # buckets 16 / 64 of qkv / o / down: the fused-form sweep (r6/r6_fused_plans.md; batch 1 23.2 -> 22.5 ms,
    # 64 concurrent 38.1 -> 37.9 ms)
    (10240, 8192, MODE_PARTIAL): {64: (1, 3, 7), 16: (1, 1, 9)},
    (8192, 8192, MODE_PARTIAL): {64: (1, 2, 1), 32: (2, 8, 7), 16: (1, 1, 9)},  # 8-wave tile: 23.3 vs 24.8-25.7 us
    (57344, 8192, MODE_SILU): {64: (2, 1, 7), 32: (2, 1, 7), 16: (2, 1, 7)},  # 8-wave tile: 148 vs 166-178 us
    (8192, 28672, MODE_PARTIAL): {64: (2, 4, 1), 16: (1, 2, 1)},
    # 70B shards re-swept with K rotation in round 4 at M = 1 / 64 (profiles/r4_m64g_sweep_tp.jsonl)
    # TP shards (Llama-3-8B / Mixtral attention TP2/4/8, Llama-3-70B TP2/4/8), re-swept at
    # M = 1 / 16 (bucket 16: best sum), 32, 64 (profiles/r2_tp_shard_sweep.jsonl); gate_up
    # shards with split-K SiLU (S > 1) and the 8-wave cfg 7: profiles/r2_silu_split_sweep.jsonl
    (8192, 14336, MODE_PARTIAL): {64: (2, 4, 1), 32: (2, 4, 1), 16: (1, 2, 9)},  # down70t2
    (8192, 7168, MODE_PARTIAL): {64: (2, 4, 1), 32: (2, 4, 1), 16: (1, 4, 6)},  # down70t4
    (8192, 3584, MODE_PARTIAL): {64: (1, 4, 7), 32: (1, 2, 1), 16: (2, 4, 6)},  # down70t8
    (4096, 7168, MODE_PARTIAL): {64: (2, 8, 3), 32: (1, 4, 1), 16: (1, 8, 5)},  # down8t2
    (4096, 3584, MODE_PARTIAL): {64: (1, 4, 2), 32: (1, 8, 4), 16: (1, 8, 5)},  # down8t4
    (4096, 1792, MODE_PARTIAL): {64: (1, 4, 2), 32: (1, 4, 4), 16: (1, 2, 2)},  # down8t8
    (28672, 8192, MODE_SILU): {64: (2, 1, 1), 32: (2, 1, 3), 16: (2, 1, 3)},  # gate_up70t2
    (14336, 8192, MODE_SILU): {64: (2, 1, 6), 32: (2, 2, 5), 16: (2, 1, 6)},  # gate_up70t4
    (7168, 8192, MODE_SILU): {64: (2, 2, 6), 32: (2, 2, 6), 16: (2, 2, 6)},  # gate_up70t8
    (14336, 4096, MODE_SILU): {64: (2, 1, 6), 32: (2, 1, 6), 16: (2, 4, 7)},  # gate_up8t2
    (7168, 4096, MODE_SILU): {64: (2, 2, 6), 32: (2, 4, 3), 16: (2, 4, 1)},  # gate_up8t4
    (3584, 4096, MODE_SILU): {64: (2, 4, 6), 32: (2, 4, 0), 16: (2, 4, 0)},  # gate_up8t8
    (8192, 4096, MODE_PARTIAL): {64: (2, 4, 3), 32: (2, 4, 3), 16: (2, 4, 1)},  # o70t2
    (8192, 2048, MODE_PARTIAL): {64: (1, 2, 0), 32: (1, 2, 0), 16: (1, 2, 0)},  # o70t4
    (8192, 1024, MODE_PARTIAL): {64: (1, 2, 2), 32: (2, 2, 4), 16: (1, 1, 0)},  # o70t8 (16: fused-form sweep)
    (4096, 2048, MODE_PARTIAL): {64: (1, 4, 2), 32: (1, 4, 4), 16: (1, 2, 0)},  # o8t2
    (4096, 1024, MODE_PARTIAL): {64: (1, 4, 2), 32: (2, 4, 4), 16: (1, 4, 5)},  # o8t4
    (4096, 512, MODE_PARTIAL): {64: (2, 2, 6), 32: (1, 2, 3), 16: (2, 1, 6)},  # o8t8
    (5120, 8192, MODE_PARTIAL): {64: (2, 6, 1), 32: (2, 8, 5), 16: (1, 6, 6)},  # qkv70t2
    (2560, 8192, MODE_PARTIAL): {64: (1, 6, 1), 32: (2, 8, 1), 16: (1, 6, 0)},  # qkv70t4
    (1280, 8192, MODE_PARTIAL): {64: (1, 8, 0), 32: (1, 8, 0), 16: (1, 8, 0)},  # qkv70t8 (16: fused-form sweep)
    (3072, 4096, MODE_PARTIAL): {64: (1, 8, 4), 32: (1, 4, 2), 16: (1, 8, 6)},  # qkv8t2
    (1536, 4096, MODE_PARTIAL): {64: (1, 8, 2), 32: (1, 4, 1), 16: (1, 8, 4)},  # qkv8t4
    (768, 4096, MODE_PARTIAL): {64: (1, 8, 5), 32: (1, 8, 2), 16: (2, 8, 0)},  # qkv8t8
    # Llama-3 LM head, bf16 logits (profiles/r2_lmhead_sweep.jsonl)
    (128256, 4096, MODE_BF16): {64: (2, 1, 3), 16: (1, 1, 3)},
}


def _apply_plan_overrides(spec: str) -> None:
    """XGS_TUNE m64_plans="NxKxMODE@BUCKET=nw,S,cfg;..." replaces tuned plans (A/B sweeps)."""
    for item in filter(None, (t.strip() for t in spec.split(";"))):
        key, plan = item.split("=")
        shape, bucket = key.split("@")
        n, k, mode = (int(v) for v in shape.split("x"))
        _M64_TUNED.setdefault((n, k, mode), {})[int(bucket)] = tuple(int(v) for v in plan.split(","))


_apply_plan_overrides(tune.get_str("m64_plans", ""))


def _m64_valid(N: int, K: int, mode: int, nw: int, S: int, cfg: int, M: int = 1) -> bool:
    if cfg in M64G_SMALL_ONLY and M > 16:
        return False
    wv, kc, _ = M64G_CFGS[cfg]
    if N % (16 * nw * wv) or K % kc or S > K // kc:  # uneven split-K ranges are fine
        return False
    # split-K SiLU reduces its slabs in the GEMM's tail (m64g_silu_tail): NW = 2 pairs only
    return not (mode == MODE_SILU and nw != 2) and not (mode == MODE_BF16 and S != 1)


def m64_plan(M: int, N: int, K: int, mode: int = MODE_PARTIAL):
    """(nw, split_k, cfg) for gemm_m64g, or None if unsupported. Measured shapes come
    from _M64_TUNED; otherwise split-K 4 whenever K allows (the partials are reduced
    by the consumer kernel for free), 128-column tiles once they give >= 192
    workgroups, else 64; bf16 / SiLU epilogues need split 1 (SiLU: nt weight DMA)."""
    if not (1 <= M <= 64) or K % 256:
        return None
    t = _M64_TUNED.get((N, K, mode))
    if M <= 16:
        p = t.get(16) if t is not None else None
        return p if (p is not None and _m64_valid(N, K, mode, *p, M=M)) else None
    if t is not None:
        p = t.get(32) if (M <= 40 and 32 in t) else t.get(64)
        if p is not None and _m64_valid(N, K, mode, *p, M=M):
            return p
    if mode == MODE_SILU:
        return (2, 1, 1) if N % 128 == 0 else None
    if mode == MODE_BF16:
        nw = 2 if N % 128 == 0 else 1
        return (nw, 1, 0) if N % (64 * nw) == 0 else None
    S = next(s for s in (4, 2, 1) if K % (s * 256) == 0)
    nw = 2 if (N % 128 == 0 and (N // 128) * S >= 192) else 1
    if N % (64 * nw):
        return None
    return nw, S, 0


def m64_linear(x: torch.Tensor, w: torch.Tensor, mode: int = MODE_PARTIAL, split_k: Optional[int] = None,
               nw: Optional[int] = None, out: Optional[torch.Tensor] = None, cfg: Optional[int] = None):
    """gemm_m64g (csrc/kernels/gemm_m64g.hip, LDS-DMA weight streaming) for M <= 64:
    bf16 [M, N], PendingSum (MODE_PARTIAL) or silu(gate)*up [M, N/2] (MODE_SILU,
    interleaved gate|up weight)."""
    M, K = x.shape
    N = w.shape[0]
    plan = m64_plan(M, N, K, mode)
    if plan is None and None not in (nw, split_k, cfg) and 1 <= M <= 64 and _m64_valid(N, K, mode, nw, split_k,
                                                                                     cfg, M):
        plan = (nw, split_k, cfg)  # a fully explicit configuration (sweeps, tests) needs no measured plan
    if plan is None:
        raise ValueError(f"gemm_m64: unsupported shape M={M} N={N} K={K} mode={mode}")
    if nw is None and split_k is None and cfg is None:
        nw, S, cfg = plan
    else:
        nw = nw or plan[0]
        S = split_k or plan[1]
        cfg = plan[2] if cfg is None else cfg
        if not _m64_valid(N, K, mode, nw, S, cfg, M):
            cfg = 0
    k = kernels()
    if mode == MODE_PARTIAL:
        part = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
        k.gemm_m64g(x.data_ptr(), M, K, w.data_ptr(), N, part.data_ptr(), 0, S, MODE_PARTIAL, nw, cfg, stream_ptr())
        return PendingSum(part, S)
    ncol = N // 2 if mode == MODE_SILU else N
    if out is None:
        out = torch.empty(M, ncol, dtype=torch.bfloat16, device=x.device)
    if mode == MODE_SILU and S > 1:  # split-K SiLU: slabs + tile tickets, reduced in the GEMM tail
        part = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
        k.gemm_m64g_ex(x.data_ptr(), M, K, w.data_ptr(), N, part.data_ptr(), out.data_ptr(), S, mode, nw, cfg,
                       0, 0, 0, 0.0, 0, 0, tile_counters(x.device, N).data_ptr(), stream_ptr())
    else:
        k.gemm_m64g(x.data_ptr(), M, K, w.data_ptr(), N, 0, out.data_ptr(), 1, mode, nw, cfg, stream_ptr())
    return out


# ---------------------------------------------------------------------------- gemm_mw (64 < M <= 256)
# csrc/kernels/gemm_mw.hip: one 8-wave workgroup per CU owns a 128- or 256-column
# weight tile and every x row (x bytes per weight byte = M / columns), W and x both
# by LDS-DMA, split-K partials for grids that would not fill the chip.
# cfg -> (columns per workgroup, weight ring depth, non-temporal weight DMA)
# (0-4: 4 x 2 waves as N x M; 5-6: 2 x 4 waves -- fewer LDS fragment reads per MFMA.
# The split-role and software-pipelined families of round 4 (cfg 7-21) never won a
# default plan and were removed in round 5; their sweeps stay in profiles/r4_mw*.)
MW_CFGS = {0: (256, 2, True), 1: (128, 3, True), 2: (128, 2, True), 3: (256, 2, False), 4: (128, 3, False),
           5: (128, 3, True), 6: (256, 2, True)}
MW_MAX_M = 320   # M > 256 (a 320-row x tile) fits the LDS on cfg 2 only
# (N, K, mode) -> {M bucket (128 / 192 / 256 / 320): (split_k, cfg)}, measured on MI355X with cold
# weights (bench/gemm_bench.py --mw-sweep); other shapes take the default rule in mw_plan
_MW_TUNED = {
    # Llama-3 LM head, bf16 logits (profiles/r4_mw_sweep_rot.jsonl, K-chunk rotation on):
    # 64 rows 170.4 us (hipBLASLt 212), 128 rows 175.5 (237), 192 219.5 (257), 256 267 (299)
    (128256, 4096, MODE_BF16): {128: (1, 0), 192: (1, 6), 256: (1, 6)},
}
LM_HEAD_MW_MIN_M = 17  # batch <= 16 keeps the library GEMM (not swept)


def _mw_bucket(M: int) -> int:
    return 128 if M <= 128 else (192 if M <= 192 else (256 if M <= 256 else 320))


def mw_plan(M: int, N: int, K: int, mode: int = MODE_PARTIAL):
    """(split_k, cfg) for gemm_mw, or None when the shape is unsupported. Default: the
    128-column, 3-deep tile; split-K (PARTIAL only) to the split nearest 256 workgroups."""
    if not (1 <= M <= MW_MAX_M) or K % 64:
        return None
    t = _MW_TUNED.get((N, K, mode), {}).get(_mw_bucket(M))
    if t is not None:
        return t
    cfg = 1 if M <= 256 else 2
    cols = MW_CFGS[cfg][0]
    if N % cols:
        return None
    if mode != MODE_PARTIAL:
        return 1, cfg
    tiles = N // cols
    S = max(1, min(K // 64, round(256 / tiles)))
    return S, cfg


def mw_linear(x: torch.Tensor, w: torch.Tensor, mode: int = MODE_PARTIAL, plan=None,
              out: Optional[torch.Tensor] = None):
    """gemm_mw for 1 <= M <= 320 (built for the mixed decode + prefill-chunk step):
    PendingSum (MODE_PARTIAL, reduced by the consumer), bf16 [M, N] (MODE_BF16) or
    silu(gate) * up [M, N / 2] of a block-16 interleaved gate|up weight (MODE_SILU)."""
    M, K = x.shape
    N = w.shape[0]
    p = plan or mw_plan(M, N, K, mode)
    if p is None or not x.is_contiguous():
        raise ValueError(f"gemm_mw: unsupported M={M} N={N} K={K} mode={mode}")
    S, cfg = p
    if mode == MODE_PARTIAL:
        part = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
        kernels().gemm_mw(x.data_ptr(), M, K, w.data_ptr(), N, part.data_ptr(), 0, S, MODE_PARTIAL, cfg,
                          stream_ptr())
        return PendingSum(part, S)
    if out is None:
        out = torch.empty(M, N // 2 if mode == MODE_SILU else N, dtype=torch.bfloat16, device=x.device)
    kernels().gemm_mw(x.data_ptr(), M, K, w.data_ptr(), N, 0, out.data_ptr(), S, mode, cfg, stream_ptr())
    return out


# ---------------------------------------------------------------------------- gemm_pf (prompt-sized M)
# csrc/kernels/gemm_pf.hip: BM x 256 output tiles on 8 waves, 64-deep K tiles consumed
# in phases with the next tiles' LDS-DMA in flight across the barriers, waves 4-7 one
# barrier behind waves 0-3 (MFMA / load ping-pong per SIMD). (A stream-K form measured
# 164 vs 121 us at the 575-row gate_up and was removed, profiles/r5_pf_gemm.md.)
# cfg -> (BM, m tiles per wave per phase): 0 (256, 2) 1 (192, 2) 2 (128, 2) 3 (256, 4)
# 4 (192, 3) 5 (288, 3).
PF_CFG_BM = {0: 256, 1: 192, 2: 128, 3: 256, 4: 192, 5: 288, 6: 288, 7: 256, 8: 192}
# The planner's cost model, fitted to bench/pf_gemm_bench.py at the 8B mixed-step
# shapes (profiles/r5_pf_gemm.md): a workgroup costs PF_WG_US + its output bytes at
# PF_WG_OUT_GBS (fp32 partials or bf16) + K tiles x the per-K-tile time of its cfg;
# one workgroup per CU, so a grid of G costs ceil(G / CUs) of those.
_PF_CFG_KT_US = {2: 1.07, 4: 1.34, 8: 1.37, 3: 1.75, 7: 1.51, 6: 1.77}   # cfg -> us per 64-deep K tile
_PF_CFG_BM_ = {2: 128, 4: 192, 8: 192, 3: 256, 7: 256, 6: 288}
PF_WG_US = 5.0
PF_WG_OUT_GBS = 60.0


def pf_bm(M: int) -> int:
    """The tile height that pads M least (ties -> the taller tile)."""
    return min((256, 192, 128), key=lambda b: (-(-M // b) * b, -b))


_CU_COUNT = {}


def cu_count(device=None) -> int:
    d = torch.cuda.current_device() if device is None else torch.device(device).index or 0
    n = _CU_COUNT.get(d)
    if n is None:
        n = _CU_COUNT[d] = torch.cuda.get_device_properties(d).multi_processor_count
    return n


@functools.lru_cache(maxsize=4096)  # (eager mixed steps call it per projection: ~10 us of host time)
def pf_plan(M: int, N: int, K: int, mode: int = MODE_PARTIAL, cus: int = 256):
    """(split_k, cfg) for gemm_pf, or None when the shape is unsupported. Every cfg of
    _PF_CFG_KT_US is priced with the model above (PARTIAL: with split-K up to one
    round of workgroups; the fp32 partials' round trip through the consumer is
    added)."""
    if M < 1 or N % 256 or K % 64 or K < 64:
        return None
    nk = K // 64
    best = None
    for cfg, kt in _PF_CFG_KT_US.items():
        bm = _PF_CFG_BM_[cfg]
        tiles = -(-M // bm) * (N // 256)
        ob = bm * 256 * (4 if mode == MODE_PARTIAL else 2)      # output bytes per workgroup
        wg = PF_WG_US + ob / (PF_WG_OUT_GBS * 1e3)
        cands = []
        if mode == MODE_PARTIAL:
            S = 1
            while tiles * (S + 1) <= cus and (S + 1) <= K // 256:
                S += 1
            # + the consumer's read of the extra fp32 slabs (~7 TB/s; their writes are in wg)
            cands.append(((-(-tiles * S // cus)) * (wg + -(-nk // S) * kt) + (S - 1) * M * N * 4 / 7e6, S))
        else:
            cands.append((-(-tiles // cus) * (wg + nk * kt), 1))
        for t, S_ in cands:
            if best is None or t < best[0]:
                best = (t, S_, cfg)
    return best[1], best[2]


def pf_linear(x: torch.Tensor, w: torch.Tensor, mode: int = MODE_BF16, plan=None,
              out: Optional[torch.Tensor] = None):
    """gemm_pf: bf16 [M, N] (MODE_BF16), PendingSum (MODE_PARTIAL, reduced by the
    consumer) or silu(gate) * up [M, N / 2] of a block-16 interleaved gate|up weight
    (MODE_SILU)."""
    M, K = x.shape
    N = w.shape[0]
    p = plan or pf_plan(M, N, K, mode, cu_count(x.device) if x.is_cuda else 256)
    if p is None or not x.is_contiguous() or not w.is_contiguous():
        raise ValueError(f"gemm_pf: unsupported M={M} N={N} K={K} mode={mode}")
    S, cfg = p[0], p[1]
    k = kernels()
    if mode == MODE_PARTIAL:
        part = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
        k.gemm_pf(x.data_ptr(), M, K, w.data_ptr(), N, part.data_ptr(), 0, S, MODE_PARTIAL, cfg, stream_ptr())
        return PendingSum(part, S)
    if out is None:
        out = torch.empty(M, N // 2 if mode == MODE_SILU else N, dtype=torch.bfloat16, device=x.device)
    k.gemm_pf(x.data_ptr(), M, K, w.data_ptr(), N, 0, out.data_ptr(), S, mode, cfg, stream_ptr())
    return out


def lm_head_linear(h: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """bf16 logits h . w^T for the LM head: gemm_mw where the sweep measured a plan for
    this row bucket (_MW_TUNED, mode bf16), else hipBLASLt."""
    M, K = h.shape
    N = w.shape[0]
    if (h.is_cuda and LM_HEAD_MW_MIN_M <= M <= MW_MAX_M and h.is_contiguous() and w.is_contiguous()
            and _mw_bucket(M) in _MW_TUNED.get((N, K, MODE_BF16), {})):
        return mw_linear(h, w, MODE_BF16)
    return torch.nn.functional.linear(h, w)


def _apply_mw_overrides(spec: str) -> None:
    """XGS_TUNE mw_plans="NxKxMODE@BUCKET=S,cfg;..." replaces gemm_mw plans (A/B sweeps)."""
    for item in filter(None, (t.strip() for t in spec.split(";"))):
        key, plan = item.split("=")
        shape, bucket = key.split("@")
        n, k, mode = (int(v) for v in shape.split("x"))
        _MW_TUNED.setdefault((n, k, mode), {})[int(bucket)] = tuple(int(v) for v in plan.split(","))


_apply_mw_overrides(tune.get_str("mw_plans", ""))


# ---------------------------------------------------------------------------- fused decode layer
MODE_RESID = 3
# (A cooperative in-launch reduce of the larger slabs -- every split workgroup of a
# tile reducing M / S rows after the splits meet -- measured 2-8 % slower end to end,
# profiles/r2_resid_coop.md, and was removed.)
# GG_RESID (residual add + next-norm statistics inside the GEMM launch) reduces a
# column tile in-launch while its split-K slab (S x M x columns fp32) is at most
# this many bytes -- the tile's last arriver reads it serially (~1 us per 16 KB,
# cdna_hip_programming.md §5); larger slabs (M ~ 64) go through the wide
# add_partials_resid kernel instead. XGS_TUNE resid_inlaunch_kb overrides (A/B of the
# batched last-arriver reduce at M = 64, whose slabs are 64-256 KB).
RESID_INLAUNCH_MAX_BYTES = tune.get_int("resid_inlaunch_kb", 32) << 10


@dataclass
class RowStats:
    """RMSNorm statistics of the rows of a residual stream: `n` partial sums of
    squares per row at ss[j * stride + m], added in order by the consuming GEMM."""
    ss: torch.Tensor
    n: int
    stride: int


class ResidWorkspace:
    """Scratch of the fused decode layer, sized once per model (graph-capture safe).
    Statistics site 0 is the embedding; sites 2i+1 / 2i+2 follow layer i's
    attention / MLP residual adds."""

    MAX_TILES = 64  # per-tile statistics a consumer can combine (ss_n <= 64) at any M
    # ... and at M <= 16 (gemm_m64g's wide statistics path; XGS_TUNE small_m_tiles A/B)
    MAX_TILES_SMALL_M = tune.get_int("small_m_tiles", 128)
    IN_LAUNCH_MAX_M = 64

    def __init__(self, n_sites: int, max_m: int, H: int, device):
        self.max_m = max_m
        rows = max(self.MAX_TILES * self.IN_LAUNCH_MAX_M, max(1, H // 1024) * max_m)
        self.ss = torch.zeros(n_sites, rows, dtype=torch.float32, device=device)
        # arrival tickets (GG_RESID: one word per tile): zero here, and every launch
        # re-arms the words it used
        self.counters = torch.zeros(n_sites, 2 * self.MAX_TILES, dtype=torch.int32, device=device)
        # GG_AR (TP decode, all-reduce in the GEMM launch): tile-pair statistics tickets
        # and per-tile row sums for grids of more than MAX_TILES column tiles
        self.ar_pair = torch.zeros(self.MAX_TILES, dtype=torch.int32, device=device)
        self.ar_ss_tmp = torch.zeros(2 * self.MAX_TILES * self.IN_LAUNCH_MAX_M, dtype=torch.float32, device=device)
        self._ar_descs = {}

    def max_tiles(self, M: int) -> int:
        return self.MAX_TILES_SMALL_M if M <= 16 else self.MAX_TILES

    def ar_desc(self, ar, group: int) -> torch.Tensor:
        """Device copy of gemm_m64g's ArDesc for these all-reduce operands (built once;
        captured graphs keep pointing at it)."""
        key = (id(ar), group)
        d = self._ar_descs.get(key)
        if d is None:
            import struct
            ptrs = list(ar.data) + [0] * (8 - len(ar.data))
            raw = struct.pack("<8Qq4i4Q", *ptrs, ar.region, ar.rank, ar.world, ar.loop, group, ar.gens.data_ptr(),
                              ar.err.data_ptr(), self.ar_ss_tmp.data_ptr(), self.ar_pair.data_ptr())
            assert len(raw) == kernels().m64g_ar_desc_bytes(), "ArDesc layout"
            d = (torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.ss.device), ar)  # (keeps ar alive)
            self._ar_descs[key] = d
        return d[0]


# Prefill-sized down projections (K = 3.5 N) have too few output tiles for the chip at
# M ~ 512-1536 (N = 4096: 66-160 library tiles); a K-split strided-batched GEMM with
# fp32 outputs doubles them and its partials are reduced for free by the consumer
# (add_partials_rmsnorm). bench/splitk_prefill_bench.py, profiles/r2_splitk_prefill.md:
# 8B down at M 575 87.8 -> 70.3 us (+3.3 us of fp32 slab traffic in the consumer).
SPLITK_PREFILL_MAX_M = 1536
SPLITK_PREFILL_S = 4


def splitk_linear(x: torch.Tensor, w: torch.Tensor, S: int) -> PendingSum:
    """x [M, K] . w[N, K]^T as S fp32 K-slice partials [S, M, N] from ONE strided
    batched library GEMM (no copies: both operands are strided views)."""
    M, K = x.shape
    N = w.shape[0]
    a = x.view(M, S, K // S).permute(1, 0, 2)
    b = w.view(N, S, K // S).permute(1, 2, 0)
    return PendingSum(torch.bmm(a, b, out_dtype=torch.float32), S)


def splitk_prefill_ok(x: torch.Tensor, w: torch.Tensor, min_ratio: int = 3) -> bool:
    M, K = x.shape
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous()
            and 64 < M <= SPLITK_PREFILL_MAX_M and K >= min_ratio * w.shape[0] and K % 512 == 0)


_TILE_COUNTERS = {}
_TILE_COUNTERS_RETIRED = []


def tile_counters(device, n: int) -> torch.Tensor:
    """Zeroed int32 arrival tickets (one per column tile, >= n / 16 words) shared by the
    split-K SiLU launches of a device: every ticket winner re-arms its word, so each
    launch leaves them zero for the next one on the stream."""
    key = str(device)
    t = _TILE_COUNTERS.get(key)
    need = max(4096, n // 16)
    if t is None or t.numel() < need:
        if t is not None:  # captured HIP graphs may hold the old words: keep them alive
            _TILE_COUNTERS_RETIRED.append(t)
        t = _TILE_COUNTERS[key] = torch.zeros(need, dtype=torch.int32, device=device)
    return t


def m64_norm_linear(x: torch.Tensor, w: torch.Tensor, mode: int, stats: RowStats, eps: float,
                    out: Optional[torch.Tensor] = None, plan=None):
    """gemm_m64g on the raw residual stream x with its RMSNorm applied as a per-row
    epilogue scale rsqrt(sum_sq / K + eps) (norm weight folded into w): PendingSum
    (MODE_PARTIAL) or bf16 silu(gate) * up (MODE_SILU). plan: (nw, S, cfg) override
    (sweeps)."""
    M, K = x.shape
    N = w.shape[0]
    plan = plan or m64_plan(M, N, K, mode)
    if plan is None:
        raise ValueError(f"gemm_m64g: unsupported shape M={M} N={N} K={K} mode={mode}")
    nw, S, cfg = plan
    k = kernels()
    st = (stats.ss.data_ptr(), stats.n, stats.stride, float(eps))
    if mode == MODE_PARTIAL:
        part = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
        k.gemm_m64g_ex(x.data_ptr(), M, K, w.data_ptr(), N, part.data_ptr(), 0, S, MODE_PARTIAL, nw, cfg, *st,
                       0, 0, 0, stream_ptr())
        return PendingSum(part, S)
    if out is None:
        out = torch.empty(M, N // 2 if mode == MODE_SILU else N, dtype=torch.bfloat16, device=x.device)
    if mode == MODE_SILU and S > 1:  # split-K SiLU: slabs + tile tickets, reduced in the GEMM tail
        part = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
        k.gemm_m64g_ex(x.data_ptr(), M, K, w.data_ptr(), N, part.data_ptr(), out.data_ptr(), S, mode, nw, cfg, *st,
                       0, 0, tile_counters(x.device, N).data_ptr(), stream_ptr())
        return out
    k.gemm_m64g_ex(x.data_ptr(), M, K, w.data_ptr(), N, 0, out.data_ptr(), 1, mode, nw, cfg, *st, 0, 0, 0,
                   stream_ptr())
    return out


def m64_resid_linear(x, w: torch.Tensor, resid: torch.Tensor, ws: ResidWorkspace, site: int,
                     eps: float, plan=None) -> RowStats:
    """resid += x . w^T (bf16 residual stream, in place) on gemm_m64g; returns the
    new residual's RMSNorm statistics. Small split-K slabs are reduced inside the
    GEMM launch (GG_RESID), large ones by the wide add_partials_resid kernel.
    x: bf16 [M, K]."""
    M, K = x.shape
    xp = x.data_ptr()
    N = w.shape[0]
    plan = plan or m64_plan(M, N, K, MODE_PARTIAL)
    if plan is None or N % 1024 or tuple(resid.shape) != (M, N):
        raise ValueError(f"gemm_m64g resid: unsupported shape M={M} N={N} K={K}")
    nw, S, cfg = plan
    k = kernels()
    part = torch.empty(S, M, N, dtype=torch.float32, device=resid.device)
    ss = ws.ss[site]
    cols = 16 * nw * M64G_CFGS[cfg][0]
    ntiles = N // cols
    if (S * M * cols * 4 <= RESID_INLAUNCH_MAX_BYTES and ntiles <= ws.max_tiles(M)
            and M <= ws.IN_LAUNCH_MAX_M):
        k.gemm_m64g_ex(xp, M, K, w.data_ptr(), N, part.data_ptr(), 0, S, MODE_RESID, nw, cfg, 0, 0, 0,
                       float(eps), resid.data_ptr(), ss.data_ptr(), ws.counters[site].data_ptr(), stream_ptr())
        return RowStats(ss, ntiles, M)  # one partial sum per column tile
    k.gemm_m64g(xp, M, K, w.data_ptr(), N, part.data_ptr(), 0, S, MODE_PARTIAL, nw, cfg, stream_ptr())
    k.add_partials_resid(part.data_ptr(), S, M, resid.data_ptr(), ss.data_ptr(), N, stream_ptr())
    return RowStats(ss, N // 1024, M)  # one partial sum per 1024-column chunk


def m64_ar_resid_linear(x: torch.Tensor, w: torch.Tensor, resid: torch.Tensor, ws: ResidWorkspace, site: int,
                        ar) -> RowStats:
    """TP row-parallel projection of the fused decode layer in ONE launch: resid +=
    all-reduce over the TP group of x . w^T (this rank's K shard), with the new
    residual's statistics (gemm_m64g GG_AR: the tile's last arriver pushes its bf16
    contribution to every peer as LL lines and folds the peers' lines in rank order).
    `ar` = comm.GemmArArgs (the custom all-reduce's GEMM region, or the one-process
    loopback of a --tp-shard simulation). x: bf16 [M, K], M <= 64."""
    M, K = x.shape
    N = w.shape[0]
    plan = m64_plan(M, N, K, MODE_PARTIAL)
    if plan is None or M > ws.IN_LAUNCH_MAX_M or tuple(resid.shape) != (M, N):
        raise ValueError(f"gemm_m64g_ar: unsupported shape M={M} N={N} K={K}")
    nw, S, cfg = plan
    ntiles = N // (16 * nw * M64G_CFGS[cfg][0])
    # more column tiles than the consumer combines: statistics per pair of tiles
    group = 1 if ntiles <= ws.max_tiles(M) else 2
    if ntiles > 2 * ws.MAX_TILES:
        raise ValueError(f"gemm_m64g_ar: {ntiles} column tiles")
    part = torch.empty(S, M, N, dtype=torch.float32, device=resid.device)
    ss = ws.ss[site]
    kernels().gemm_m64g_ar(x.data_ptr(), M, K, w.data_ptr(), N, part.data_ptr(), S, nw, cfg, resid.data_ptr(),
                           ss.data_ptr(), ws.counters[site].data_ptr(), ws.ar_desc(ar, group).data_ptr(), stream_ptr())
    return RowStats(ss, ntiles // group, M)


def interleave_gate_up(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """[F, H] x2 -> [2F, H] in blocks of 16 rows: g0..g15 u0..u15 g16.. (F % 16 == 0)."""
    F, H = gate.shape
    return torch.stack([gate.reshape(F // 16, 16, H), up.reshape(F // 16, 16, H)], 1).reshape(2 * F, H)


def deinterleave_gate_up(w: torch.Tensor):
    F2, H = w.shape
    v = w.reshape(F2 // 32, 2, 16, H)
    return v[:, 0].reshape(F2 // 2, H), v[:, 1].reshape(F2 // 2, H)


# ---------------------------------------------------------------------------- FP8 weights
# Weight-only FP8 (OCP E4M3 + one fp32 scale per output channel) for batch <= 16
# decode: csrc/kernels/gemm_w8.hip streams half the bytes of the bf16 kernels.
W8_MAX_M = 64
# cfg -> (columns per workgroup, k chunk)
W8_CFGS = {0: (128, 128), 1: (64, 128), 2: (64, 128), 3: (64, 256), 4: (128, 256)}
# (N, K, mode) -> (split_k, cfg), measured at M = 1 / 16 with cold weights
# (bench/gemm_bench.py --w8-sweep, profiles/r1_w8_sweep.jsonl)
_W8_TUNED = {
    (6144, 4096, MODE_PARTIAL): (4, 4), (4096, 4096, MODE_PARTIAL): (4, 4),
    (28672, 4096, MODE_SILU): (1, 3), (4096, 14336, MODE_PARTIAL): (8, 2),
    (10240, 8192, MODE_PARTIAL): (4, 2), (8192, 8192, MODE_PARTIAL): (4, 2),
    (57344, 8192, MODE_SILU): (1, 3), (8192, 28672, MODE_PARTIAL): (4, 2),
}
# 16 < M <= 64 (four 16-row x tiles, KC 128 configurations 0-2 only), measured at M = 64
# (profiles/r1_w8_sweep_m64.jsonl)
_W8_TUNED64 = {
    (6144, 4096, MODE_PARTIAL): (4, 1), (4096, 4096, MODE_PARTIAL): (4, 2),
    (28672, 4096, MODE_SILU): (1, 0), (4096, 14336, MODE_PARTIAL): (8, 0),
    (10240, 8192, MODE_PARTIAL): (8, 0), (8192, 8192, MODE_PARTIAL): (4, 0),
    (57344, 8192, MODE_SILU): (1, 0), (8192, 28672, MODE_PARTIAL): (4, 0),
}
# Projections below this many weight elements keep bf16 (gemm_m64g) in the fp8
# decode chain. 0: in isolation the 8B QKV / O are latency-bound either way (fp8
# 9.4 / 9.0 us vs bf16 9.5 / 7.3 us), but end to end all-fp8 measured faster
# (8B batch 1: 387 vs 375 tok/s with QKV / O on bf16).
W8_MIN_ELEMS = 0


def quantize_fp8(w: torch.Tensor):
    """[N, K] -> (uint8 E4M3 codes [N, K], fp32 per-row scales [N]) with
    scale = max|w_row| / 448 (the E4M3 finite maximum)."""
    wf = w.float()
    scale = (wf.abs().amax(dim=1) / 448.0).clamp_min(1e-12)
    q = (wf / scale[:, None]).clamp(-448.0, 448.0).to(torch.float8_e4m3fn)
    return q.view(torch.uint8).contiguous(), scale.contiguous()


def dequantize_fp8(q: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    return q.view(torch.float8_e4m3fn).float() * scale.float()[:, None]


# ---------------------------------------------------------------------------- INT8 / INT4 weights
# Req 10.3 quantization levels (the reference's Q8_0 / Q4_0 of llama.cpp, design.md:326-332),
# weight-only on the same gemm_w8 pipeline (csrc/kernels/gemm_w8.hip, FMT):
#   int8: symmetric, one fp32 scale per output channel (scale = max|w_row| / 127);
#   int4: symmetric, one fp32 scale per 128-k group and output channel
#         (scale = max|w_group| / 7, codes -8..7), packed two per byte.
WQ_FP8, WQ_INT8, WQ_INT4 = 0, 1, 2
WQ_FORMATS = {"fp8": WQ_FP8, "int8": WQ_INT8, "int4": WQ_INT4}
WQ_GROUP = 128
WQ_SC_FLOATS = 4096  # int4 scales one workgroup stages in LDS (groups x columns)


def quantize_int8(w: torch.Tensor):
    """[N, K] -> (int8 codes as uint8 [N, K], fp32 per-row scales [N])."""
    wf = w.float()
    scale = (wf.abs().amax(dim=1) / 127.0).clamp_min(1e-12)
    q = torch.round(wf / scale[:, None]).clamp(-127, 127).to(torch.int8)
    return q.view(torch.uint8).contiguous(), scale.contiguous()


def dequantize_int8(q: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    return q.view(torch.int8).float() * scale.float()[:, None]


def quantize_int4(w: torch.Tensor):
    """[N, K] -> (packed uint8 [N, K / 2], fp32 group scales [K / 128, N]). Codes
    q = round(w / s) in -8..7 are stored offset-binary (u = q + 8); each 32-bit word
    holds 8 consecutive k, element 2j at bits 4j and element 2j + 1 at bits 16 + 4j
    (the pair layout the kernel widens with one and_or per bf16 pair)."""
    N, K = w.shape
    if K % WQ_GROUP:
        raise ValueError(f"int4 weights need K % {WQ_GROUP} == 0, got K={K}")
    wf = w.float().view(N, K // WQ_GROUP, WQ_GROUP)
    scale = (wf.abs().amax(dim=2) / 7.0).clamp_min(1e-12)  # [N, G]
    u = (torch.round(wf / scale[:, :, None]).clamp(-8, 7) + 8).to(torch.int32).view(N, K // 8, 4, 2)
    word = torch.zeros(N, K // 8, dtype=torch.int32, device=w.device)
    for j in range(4):
        word |= u[:, :, j, 0] << (4 * j)
        word |= u[:, :, j, 1] << (16 + 4 * j)
    packed = word.view(torch.uint8).view(N, K // 2)  # little-endian words
    return packed.contiguous(), scale.t().contiguous()


def dequantize_int4(packed: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    N = packed.shape[0]
    K = packed.shape[1] * 2
    word = packed.contiguous().view(torch.int32).view(N, K // 8)
    u = torch.empty(N, K // 8, 4, 2, dtype=torch.int32, device=packed.device)
    for j in range(4):
        u[:, :, j, 0] = (word >> (4 * j)) & 15
        u[:, :, j, 1] = (word >> (16 + 4 * j)) & 15
    q = (u.view(N, K) - 8).float()
    return q * scale.t().repeat_interleave(WQ_GROUP, dim=1).float()


def quantize_weight(w: torch.Tensor, fmt: int):
    return {WQ_FP8: quantize_fp8, WQ_INT8: quantize_int8, WQ_INT4: quantize_int4}[fmt](w)


def dequantize_weight(q: torch.Tensor, scale: torch.Tensor, fmt: int) -> torch.Tensor:
    return {WQ_FP8: dequantize_fp8, WQ_INT8: dequantize_int8, WQ_INT4: dequantize_int4}[fmt](q, scale)


def _w8_fits(N: int, K: int, mode: int, S: int, cfg: int, M: int, fmt: int) -> bool:
    cols, kc = W8_CFGS[cfg]
    if N % cols or K % (S * kc) or (M > 16 and cfg >= 3) or (mode == MODE_SILU and (S != 1 or cfg == 2)):
        return False
    return fmt != WQ_INT4 or ((K // S) % WQ_GROUP == 0 and (K // S // WQ_GROUP) * cols <= WQ_SC_FLOATS)


def w8_plan(M: int, N: int, K: int, mode: int, fmt: int = WQ_FP8):
    """(split_k, cfg) for gemm_w8, or None. SiLU needs split 1 and two 16-column
    tiles per wave; otherwise the smallest split-K giving >= 256 workgroups. int4:
    the measured plan with the split raised (or the tile narrowed) until the
    workgroup's group scales fit its LDS stage."""
    if not (1 <= M <= W8_MAX_M):
        return None
    t = (_W8_TUNED if M <= 16 else _W8_TUNED64).get((N, K, mode))
    if t is None:
        cfg = 1
        cols, kc = W8_CFGS[cfg]
        if N % cols or K % kc:
            return None
        if mode == MODE_SILU:
            t = (1, cfg)
        else:
            S = 1
            for s in (1, 2, 4, 8, 16):
                if K % (s * kc):
                    break
                S = s
                if (N // cols) * s >= 256:
                    break
            t = (S, cfg)
    if _w8_fits(N, K, mode, t[0], t[1], M, fmt):
        return t
    S0, cfg0 = t
    for cfg in (cfg0, 1, 3, 0, 4, 2):
        for S in ((S0, 2 * S0, 4 * S0, 8 * S0) if mode != MODE_SILU else (1,)):
            if _w8_fits(N, K, mode, S, cfg, M, fmt):
                return S, cfg
    return None


def w8_linear(x: torch.Tensor, q: torch.Tensor, scale: torch.Tensor, mode: int = MODE_PARTIAL,
              plan=None, out: Optional[torch.Tensor] = None, fmt: int = WQ_FP8):
    """x [M <= 64, K] bf16 . W^T with W the dequantized weight (fmt WQ_FP8 / WQ_INT8:
    diag(scale) q; WQ_INT4: group scales): PendingSum (MODE_PARTIAL) or bf16
    silu(gate) * up [M, N/2] from block-16 interleaved gate|up rows (MODE_SILU)."""
    M, K = x.shape
    N = q.shape[0]
    p = plan or w8_plan(M, N, K, mode, fmt)
    kq = K // 2 if fmt == WQ_INT4 else K
    if (p is None or not x.is_contiguous() or q.dtype != torch.uint8 or scale.dtype != torch.float32
            or tuple(q.shape) != (N, kq) or scale.numel() != (N * (K // WQ_GROUP) if fmt == WQ_INT4 else N)):
        raise ValueError(f"gemm_w8: unsupported M={M} N={N} K={K} mode={mode} fmt={fmt}")
    S, cfg = p
    k = kernels()
    if mode == MODE_PARTIAL:
        part = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
        k.gemm_w8(x.data_ptr(), M, K, q.data_ptr(), scale.data_ptr(), N, part.data_ptr(), 0, S, MODE_PARTIAL, cfg,
                  stream_ptr(), fmt)
        return PendingSum(part, S)
    if out is None:
        out = torch.empty(M, N // 2, dtype=torch.bfloat16, device=x.device)
    k.gemm_w8(x.data_ptr(), M, K, q.data_ptr(), scale.data_ptr(), N, 0, out.data_ptr(), 1, MODE_SILU, cfg,
              stream_ptr(), fmt)
    return out
