"""K1: RMSNorm / fused residual-add RMSNorm / LayerNorm."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._native import kernels, stream_ptr, use_native


def rmsnorm_ref(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    return (xf * torch.rsqrt(var + eps) * w.float()).to(x.dtype)


def fused_add_rmsnorm_ref(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                          eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    r = (x.float() + residual.float()).to(x.dtype)
    return rmsnorm_ref(r, w, eps), r


def layernorm_ref(x, w, b, eps):
    return torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x * rsqrt(mean(x^2) + eps) * w over the last dim. x may be row-strided."""
    if not use_native(x):
        r = rmsnorm_ref(x, w, eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    H = x.shape[-1]
    x2 = x.reshape(-1, H) if x.is_contiguous() else x
    T = x2.shape[0]
    assert x2.stride(-1) == 1 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
    if out is None:
        out = torch.empty((T, H), dtype=x.dtype, device=x.device)
    kernels().rmsnorm(x2.data_ptr(), w.data_ptr(), out.data_ptr(), T, H, float(eps), x2.stride(0),
                      out.stride(0) if out.dim() > 1 else H, stream_ptr())
    return out.view(*x.shape[:-1], H) if out.dim() == 2 and x.dim() != 2 else out


def fused_add_rmsnorm(x, residual: torch.Tensor, w: torch.Tensor, eps: float,
                      out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """residual <- x + residual (in place); returns (rmsnorm(residual) * w, residual).
    `x` may be a PendingSum (split-K partials): they are reduced in the kernel prologue."""
    from .linear import PendingSum
    if isinstance(x, PendingSum):
        S, T, H = x.part.shape
        if out is None:
            out = torch.empty(T, H, dtype=residual.dtype, device=residual.device)
        kernels().add_partials_rmsnorm(x.part.data_ptr(), S, T, residual.data_ptr(), w.data_ptr(), out.data_ptr(),
                                       H, float(eps), stream_ptr())
        return out, residual
    if not use_native(x):
        y, r = fused_add_rmsnorm_ref(x, residual, w, eps)
        residual.copy_(r)
        if out is not None:
            out.copy_(y)
            return out, residual
        return y, residual
    H = x.shape[-1]
    T = x.numel() // H
    assert x.is_contiguous() and residual.is_contiguous()
    if out is None:
        out = torch.empty_like(x)
    kernels().fused_add_rmsnorm(x.data_ptr(), residual.data_ptr(), w.data_ptr(), out.data_ptr(), T, H,
                                float(eps), stream_ptr())
    return out, residual


def row_sumsq(x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out.view(-1)[t] = sum_k x[t, k]^2 (fp32) for bf16 rows [T, H]: the RMSNorm
    statistic the fused decode GEMMs apply as an epilogue row scale."""
    T, H = x.shape
    if not use_native(x):
        out.view(-1)[:T] = x.float().pow(2).sum(-1)
        return out
    assert x.is_contiguous() and x.dtype == torch.bfloat16 and out.dtype == torch.float32
    kernels().row_sumsq(x.data_ptr(), T, H, out.data_ptr(), stream_ptr())
    return out


def layernorm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    if not use_native(x):
        return layernorm_ref(x, w, b, eps)
    H = x.shape[-1]
    x = x.contiguous()
    out = torch.empty_like(x)
    kernels().layernorm(x.data_ptr(), w.data_ptr(), b.data_ptr(), out.data_ptr(), x.numel() // H, H, float(eps),
                        stream_ptr())
    return out
