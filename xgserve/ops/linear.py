"""Decode-regime projections on the skinny HIP GEMM (csrc/kernels/skinny_gemm.hip).

`PendingSum` is a value that exists only as fp32 split-K partial sums; the
kernels that consume it (add_partials_rmsnorm, rope_cache_partials) reduce it
in their prologue, so a split-K GEMM costs no extra reduction launch.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from ._native import kernels, stream_ptr, use_native

MODE_BF16, MODE_PARTIAL, MODE_SILU = 0, 1, 2
SKINNY_MAX_M = 128
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


def skinny_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    M, K = x.shape
    N = w.shape[0]
    return (use_native(x) and M <= SKINNY_MAX_M and N % 64 == 0 and K % 256 == 0
            and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.is_contiguous())


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


def m64_plan(M: int, N: int, K: int, mode: int = MODE_PARTIAL):
    """(nw, split_k) for gemm_m64 / gemm_m64g, or None if unsupported. Measured on
    MI355X (bench/gemm_bench.py, profiles/r1_gemm_*): split-K 4 whenever K allows
    (the partials are reduced by the consumer kernel for free), 128-column tiles
    once they give >= 192 workgroups, else 64; bf16 / SiLU epilogues need split 1."""
    if not (16 < M <= 64) or K % 256:
        return None
    if mode == MODE_SILU:
        return (2, 1) if N % 128 == 0 else None
    if mode == MODE_BF16:
        nw = 2 if N % 128 == 0 else 1
        return (nw, 1) if N % (64 * nw) == 0 else None
    S = next(s for s in (4, 2, 1) if K % (s * 256) == 0)
    nw = 2 if (N % 128 == 0 and (N // 128) * S >= 192) else 1
    if N % (64 * nw):
        return None
    return nw, S


# 4: LDS-DMA staging (gemm_m64g.hip, fastest on every measured shape); 0-3: register-ring gemm_m64
# (bit0: two W chunks in flight; bit1: default cache policy for W, else non-temporal)
M64_VARIANT = 4


def m64_linear(x: torch.Tensor, w: torch.Tensor, mode: int = MODE_PARTIAL, split_k: Optional[int] = None,
               nw: Optional[int] = None, out: Optional[torch.Tensor] = None, variant: Optional[int] = None):
    """gemm_m64 (csrc/kernels/gemm_m64.hip) for 16 < M <= 64: bf16 [M, N], PendingSum
    (MODE_PARTIAL) or silu(gate)*up [M, N/2] (MODE_SILU, interleaved gate|up weight)."""
    M, K = x.shape
    N = w.shape[0]
    plan = m64_plan(M, N, K, mode)
    if plan is None:
        raise ValueError(f"gemm_m64: unsupported shape M={M} N={N} K={K} mode={mode}")
    nw = nw or plan[0]
    S = split_k or plan[1]
    var = M64_VARIANT if variant is None else variant
    k = kernels()
    if mode == MODE_PARTIAL:
        part = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
        if var == 4:  # LDS-DMA staging (gemm_m64g.hip)
            k.gemm_m64g(x.data_ptr(), M, K, w.data_ptr(), N, part.data_ptr(), 0, S, MODE_PARTIAL, nw, stream_ptr())
        else:
            k.gemm_m64(x.data_ptr(), M, K, w.data_ptr(), N, part.data_ptr(), 0, S, MODE_PARTIAL, nw, var, stream_ptr())
        return PendingSum(part, S)
    ncol = N // 2 if mode == MODE_SILU else N
    if out is None:
        out = torch.empty(M, ncol, dtype=torch.bfloat16, device=x.device)
    if var == 4:
        k.gemm_m64g(x.data_ptr(), M, K, w.data_ptr(), N, 0, out.data_ptr(), 1, mode, nw, stream_ptr())
    else:
        k.gemm_m64(x.data_ptr(), M, K, w.data_ptr(), N, 0, out.data_ptr(), 1, mode, nw, var, stream_ptr())
    return out


def interleave_gate_up(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """[F, H] x2 -> [2F, H] in blocks of 16 rows: g0..g15 u0..u15 g16.. (F % 16 == 0)."""
    F, H = gate.shape
    return torch.stack([gate.reshape(F // 16, 16, H), up.reshape(F // 16, 16, H)], 1).reshape(2 * F, H)


def deinterleave_gate_up(w: torch.Tensor):
    F2, H = w.shape
    v = w.reshape(F2 // 32, 2, 16, H)
    return v[:, 0].reshape(F2 // 2, H), v[:, 1].reshape(F2 // 2, H)
