"""K2 + K4: rotary embedding fused with the paged KV-cache append."""
from __future__ import annotations

import math
from typing import Optional

import torch

from ._native import kernels, stream_ptr, use_native


def _llama3_inv_freq(inv_freq: torch.Tensor, scaling: dict) -> torch.Tensor:
    # Llama-3.1 "llama3" rope scaling (frequency-dependent interpolation).
    factor = scaling.get("factor", 8.0)
    low = scaling.get("low_freq_factor", 1.0)
    high = scaling.get("high_freq_factor", 4.0)
    old_ctx = scaling.get("original_max_position_embeddings", 8192)
    low_wl, high_wl = old_ctx / low, old_ctx / high
    wl = 2 * math.pi / inv_freq
    out = torch.where(wl > low_wl, inv_freq / factor, inv_freq)
    smooth = (old_ctx / wl - low) / (high - low)
    mid = (1 - smooth) * out / factor + smooth * out
    is_mid = (wl <= low_wl) & (wl >= high_wl)
    return torch.where(is_mid, mid, out)


def build_cos_sin(head_dim: int, max_pos: int, theta: float, scaling: Optional[dict] = None,
                  device="cpu") -> torch.Tensor:
    """fp32 table [max_pos, head_dim] = [cos(pos*f) | sin(pos*f)] over the head_dim/2 freqs."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        inv = _llama3_inv_freq(inv, scaling)
    pos = torch.arange(max_pos, dtype=torch.float64)
    ang = torch.outer(pos, inv)
    return torch.cat([ang.cos(), ang.sin()], dim=-1).float().to(device)


class RotaryCache:
    def __init__(self, head_dim: int, max_pos: int, theta: float, scaling: Optional[dict] = None, device="cpu"):
        self.head_dim = head_dim
        self.table = build_cos_sin(head_dim, max_pos, theta, scaling, device)


def _rotate(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    h = x.shape[-1] // 2
    x1, x2 = x[..., :h], x[..., h:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


def rope_cache_ref(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor, k_cache: torch.Tensor,
                   v_cache: torch.Tensor, slot_mapping: torch.Tensor, Hq: int, Hkv: int, D: int,
                   apply_rope: bool = True) -> None:
    """Reference: in-place rope on q (qkv[:, :Hq*D]); rope(k), v -> paged cache [NB, Hkv, bs, D]."""
    T = qkv.shape[0]
    if T == 0:
        return
    bs = k_cache.shape[2]
    q = qkv[:, :Hq * D].float().view(T, Hq, D)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].float().view(T, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].view(T, Hkv, D)
    if apply_rope:
        cs = cos_sin[positions.long()]
        cos, sin = cs[:, None, :D // 2], cs[:, None, D // 2:]
        q = _rotate(q, cos, sin)
        k = _rotate(k, cos, sin)
        qkv[:, :Hq * D] = q.reshape(T, Hq * D).to(qkv.dtype)
    valid = slot_mapping >= 0
    sl = slot_mapping[valid].long()
    pages, offs = sl // bs, sl % bs
    k_cache[pages, :, offs] = k[valid].to(k_cache.dtype)
    v_cache[pages, :, offs] = v[valid].to(v_cache.dtype)


def rope_cache_partials(pend, q_out: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor,
                        k_cache: torch.Tensor, v_cache: torch.Tensor, slot_mapping: torch.Tensor, Hq: int, Hkv: int,
                        D: int, apply_rope: bool = True) -> torch.Tensor:
    """QKV given as split-K partial sums (PendingSum [S, T, (Hq+2Hkv)D]); q -> q_out [T, Hq*D]."""
    S, T, W = pend.part.shape
    assert W == (Hq + 2 * Hkv) * D and q_out.stride(-1) == 1
    kernels().rope_cache_partials(pend.part.data_ptr(), S, q_out.data_ptr(), q_out.stride(0), positions.data_ptr(),
                                  cos_sin.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), slot_mapping.data_ptr(),
                                  T, Hq, Hkv, D, k_cache.shape[2], 1 if apply_rope else 0, stream_ptr())
    return q_out


def rope_cache(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor, k_cache: torch.Tensor,
               v_cache: torch.Tensor, slot_mapping: torch.Tensor, Hq: int, Hkv: int, D: int,
               apply_rope: bool = True) -> None:
    if not use_native(qkv):
        return rope_cache_ref(qkv, positions, cos_sin, k_cache, v_cache, slot_mapping, Hq, Hkv, D, apply_rope)
    T = qkv.shape[0]
    assert qkv.stride(-1) == 1 and positions.dtype == torch.int32 and slot_mapping.dtype == torch.int32
    assert cos_sin.dtype == torch.float32 and k_cache.is_contiguous() and v_cache.is_contiguous()
    assert qkv.shape[1] >= (Hq + 2 * Hkv) * D
    bs = k_cache.shape[2]
    kernels().rope_cache(qkv.data_ptr(), qkv.stride(0), positions.data_ptr(), cos_sin.data_ptr(),
                         k_cache.data_ptr(), v_cache.data_ptr(), slot_mapping.data_ptr(), T, Hq, Hkv, D, bs,
                         1 if apply_rope else 0, stream_ptr())
