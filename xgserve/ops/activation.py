"""K3: SiLU-gate and GELU-tanh."""
from __future__ import annotations

from typing import Optional

import torch

from ._native import kernels, stream_ptr, use_native


def silu_and_mul_ref(x: torch.Tensor, interleave16: bool = False) -> torch.Tensor:
    F = x.shape[-1] // 2
    xf = x.float()
    if interleave16:
        v = xf.reshape(*xf.shape[:-1], F // 16, 2, 16)
        g, u = v[..., 0, :].reshape(*xf.shape[:-1], F), v[..., 1, :].reshape(*xf.shape[:-1], F)
        return (torch.nn.functional.silu(g) * u).to(x.dtype)
    return (torch.nn.functional.silu(xf[..., :F]) * xf[..., F:]).to(x.dtype)


def gelu_tanh_ref(x: torch.Tensor) -> torch.Tensor:
    return torch.nn.functional.gelu(x.float(), approximate="tanh").to(x.dtype)


def silu_and_mul(x: torch.Tensor, out: Optional[torch.Tensor] = None, interleave16: bool = False) -> torch.Tensor:
    """[.., 2F] (gate | up, or block-16 interleaved) -> silu(gate) * up  [.., F]."""
    if not use_native(x):
        r = silu_and_mul_ref(x, interleave16)
        if out is not None:
            out.copy_(r)
            return out
        return r
    F = x.shape[-1] // 2
    T = x.numel() // (2 * F)
    assert x.is_contiguous() and x.dtype == torch.bfloat16
    if out is None:
        out = torch.empty((*x.shape[:-1], F), dtype=x.dtype, device=x.device)
    kernels().silu_and_mul(x.data_ptr(), out.data_ptr(), T, F, 1 if interleave16 else 0, stream_ptr())
    return out


def gelu_tanh(x: torch.Tensor) -> torch.Tensor:
    if not use_native(x):
        return gelu_tanh_ref(x)
    x = x.contiguous()
    out = torch.empty_like(x)
    kernels().gelu_tanh(x.data_ptr(), out.data_ptr(), x.numel(), stream_ptr())
    return out
