"""K12: Mixture-of-Experts routing, layout, grouped GEMM, combine."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._native import kernels, stream_ptr, use_native
from .activation import silu_and_mul

BLOCK_M = 64


def moe_topk_softmax(router_logits: torch.Tensor, k: int, renorm: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    T, E = router_logits.shape
    if not use_native(router_logits):
        p = torch.softmax(router_logits.float(), -1)
        w, ids = torch.topk(p, k, dim=-1)
        if renorm:
            w = w / w.sum(-1, keepdim=True)
        return w, ids.to(torch.int32)
    assert E <= 64 and k <= 16
    w = torch.empty(T, k, dtype=torch.float32, device=router_logits.device)
    ids = torch.empty(T, k, dtype=torch.int32, device=router_logits.device)
    rl = router_logits.contiguous()
    kernels().moe_topk_softmax(rl.data_ptr(), 1 if rl.dtype == torch.float32 else 0, T, E, k, 1 if renorm else 0,
                               w.data_ptr(), ids.data_ptr(), stream_ptr())
    return w, ids


def moe_align(ids: torch.Tensor, num_experts: int, block_m: int = BLOCK_M):
    """-> (sorted_rows [cap], expert_offsets [E+1], tile_expert [cap/block_m], dest [T*k])"""
    T, k = ids.shape
    cap = T * k + num_experts * (block_m - 1)
    cap = (cap + block_m - 1) // block_m * block_m
    dev = ids.device
    sorted_rows = torch.empty(cap, dtype=torch.int32, device=dev)
    offs = torch.empty(num_experts + 1, dtype=torch.int32, device=dev)
    tile_expert = torch.empty(cap // block_m, dtype=torch.int32, device=dev)
    dest = torch.empty(T * k, dtype=torch.int32, device=dev)
    kernels().moe_align(ids.data_ptr(), T, k, num_experts, block_m, sorted_rows.data_ptr(), offs.data_ptr(),
                        tile_expert.data_ptr(), dest.data_ptr(), stream_ptr())
    return sorted_rows, offs, tile_expert, dest


def moe_grouped_gemm(x: torch.Tensor, rows: Optional[torch.Tensor], w: torch.Tensor, tile_expert: torch.Tensor,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[p] = x[rows[p]] @ w[e(p)]^T for padded expert-sorted rows p. w: [E, N, K]."""
    E, N, K = w.shape
    n_tiles = tile_expert.shape[0]
    P = n_tiles * BLOCK_M
    if out is None:
        out = torch.zeros(P, N, dtype=x.dtype, device=x.device)
    kernels().moe_grouped_gemm(x.data_ptr(), rows.data_ptr() if rows is not None else 0, w.data_ptr(),
                               out.data_ptr(), 0, tile_expert.data_ptr(), n_tiles, N, K, 1 if rows is not None else 0,
                               x.shape[0], E, stream_ptr())
    return out


def moe_combine(y: torch.Tensor, dest: torch.Tensor, weights: torch.Tensor, T: int, k: int) -> torch.Tensor:
    H = y.shape[1]
    out = torch.empty(T, H, dtype=y.dtype, device=y.device)
    kernels().moe_combine(y.data_ptr(), dest.data_ptr(), weights.data_ptr(), out.data_ptr(), T, k, H, stream_ptr())
    return out


def moe_forward_ref(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
                    topk_ids: torch.Tensor, expert_offset: int = 0) -> torch.Tensor:
    """fp32 reference. w13: [E_local, 2F, H], w2: [E_local, H, F]; experts outside
    [expert_offset, expert_offset+E_local) contribute nothing."""
    T, H = x.shape
    E = w13.shape[0]
    out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
    xf = x.float()
    for e in range(E):
        ge = e + expert_offset
        mask = (topk_ids == ge)
        tok = mask.any(-1).nonzero()[:, 0]
        if tok.numel() == 0:
            continue
        wt = (topk_w * mask).sum(-1)[tok]
        h = xf[tok] @ w13[e].float().t()
        F = h.shape[1] // 2
        a = torch.nn.functional.silu(h[:, :F]) * h[:, F:]
        a = a.to(x.dtype).float()
        y = a @ w2[e].float().t()
        out[tok] += wt[:, None] * y
    return out.to(x.dtype)


def fused_moe(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
              topk_ids: torch.Tensor, expert_offset: int = 0) -> torch.Tensor:
    """Local-expert MoE FFN: sum_j w_j * FFN_{e_j}(x) over choices owned locally
    (ids in [expert_offset, expert_offset + E_local)); others are skipped."""
    if not use_native(x):
        return moe_forward_ref(x, w13, w2, topk_w, topk_ids, expert_offset)
    T, k = topk_ids.shape
    E = w13.shape[0]
    local = topk_ids - expert_offset
    in_range = (local >= 0) & (local < E)
    # out-of-range choices are routed to a dummy expert id E (dropped tiles) with weight 0
    ids = torch.where(in_range, local, torch.full_like(local, E)).to(torch.int32).contiguous()
    wts = torch.where(in_range, topk_w, torch.zeros_like(topk_w)).float().contiguous()
    sorted_rows, offs, tile_expert, dest = moe_align(ids, E + 1)
    # tiles of the dummy expert are skipped by the GEMM (tile_expert == E -> mark -1)
    tile_expert = torch.where(tile_expert >= E, torch.full_like(tile_expert, -1), tile_expert)
    h = moe_grouped_gemm(x.contiguous(), sorted_rows, w13, tile_expert)
    a = silu_and_mul(h)
    y = moe_grouped_gemm(a, None, w2, tile_expert)
    return moe_combine(y, dest, wts, T, k)
