"""K5 / K6: paged attention (prefill varlen-causal and decode split-K)."""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch

from ._native import kernels, stream_ptr, use_native

# register K/V tiles in flight per wave of the fused decode attention (2 or 3; 3 only
# for G <= 4): XGS_TUNE decode_depth A/B (bench/decode_cold.py --depth)
DECODE_DEPTH = __import__("xgserve.tune", fromlist=["get_int"]).get_int("decode_depth", 2)


def choose_num_splits(batch: int, num_kv_heads: int, max_seq_len: int, num_cus: int = 256) -> int:
    """Split-K factor so the decode grid has >= ~2 workgroups per CU, but every
    split still owns >= 256 keys (16 pages)."""
    wgs = max(1, batch * num_kv_heads)
    want = max(1, (2 * num_cus + wgs - 1) // wgs)
    cap = max(1, (max_seq_len + 255) // 256)
    return int(max(1, min(want, cap, 64)))


def _gather_kv(cache: torch.Tensor, bt_row: torch.Tensor, L: int) -> torch.Tensor:
    """[NB, Hkv, bs, D] paged -> [L, Hkv, D] for one sequence."""
    bs = cache.shape[2]
    n = (L + bs - 1) // bs
    pages = cache[bt_row[:n].long()]  # [n, Hkv, bs, D]
    return pages.permute(0, 2, 1, 3).reshape(n * bs, cache.shape[1], cache.shape[3])[:L]


def _attend(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, q_pos: torch.Tensor, scale: float) -> torch.Tensor:
    """q [n, Hq, D], k/v [L, Hkv, D]; causal by absolute positions q_pos. fp32."""
    Hq, Hkv = q.shape[1], k.shape[1]
    G = Hq // Hkv
    kf = k.float().repeat_interleave(G, dim=1)
    vf = v.float().repeat_interleave(G, dim=1)
    s = torch.einsum("nhd,lhd->hnl", q.float(), kf) * scale
    L = k.shape[0]
    mask = torch.arange(L, device=q.device)[None, :] > q_pos[:, None].to(q.device)
    s = s.masked_fill(mask[None], float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("hnl,lhd->nhd", p, vf)


def decode_attention_ref(q, k_cache, v_cache, block_tables, seq_lens, scale) -> torch.Tensor:
    B, Hq, D = q.shape
    out = torch.zeros(B, Hq, D, dtype=q.dtype, device=q.device)
    for b in range(B):
        L = int(seq_lens[b])
        if L == 0:
            continue
        k = _gather_kv(k_cache, block_tables[b], L)
        v = _gather_kv(v_cache, block_tables[b], L)
        out[b] = _attend(q[b:b + 1], k, v, torch.tensor([L - 1]), scale)[0].to(q.dtype)
    return out


def prefill_attention_ref(q, k_cache, v_cache, block_tables, query_start_loc, seq_lens, scale) -> torch.Tensor:
    T, Hq, D = q.shape
    out = torch.zeros(T, Hq, D, dtype=q.dtype, device=q.device)
    S = seq_lens.shape[0]
    for s in range(S):
        a, b = int(query_start_loc[s]), int(query_start_loc[s + 1])
        if b == a:
            continue
        L = int(seq_lens[s])
        ctx = L - (b - a)
        k = _gather_kv(k_cache, block_tables[s], L)
        v = _gather_kv(v_cache, block_tables[s], L)
        pos = torch.arange(ctx, L)
        out[a:b] = _attend(q[a:b], k, v, pos, scale).to(q.dtype)
    return out


class DecodeWorkspace:
    """Split-K partial buffers, sized once (graph-capture safe)."""

    def __init__(self, max_batch: int, num_q_heads: int, head_dim: int, max_splits: int, device):
        self.part_out = torch.empty(max_batch * num_q_heads * max_splits * head_dim, dtype=torch.float32,
                                    device=device)
        self.part_lse = torch.empty(max_batch * num_q_heads * max_splits, dtype=torch.float32, device=device)
        self.max_splits = max_splits


def decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                     seq_lens: torch.Tensor, scale: float, num_splits: int = 1,
                     workspace: Optional[DecodeWorkspace] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """q: [B, Hq, D] (rows may be strided, e.g. a view into the QKV buffer).
    k/v_cache: [NB, Hkv, bs, D]; block_tables [B, W] int32; seq_lens [B] int32."""
    if not use_native(q):
        r = decode_attention_ref(q, k_cache, v_cache, block_tables, seq_lens, scale)
        if out is not None:
            out.copy_(r.view_as(out))
            return out
        return r
    B, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    bs = k_cache.shape[2]
    assert q.stride(2) == 1 and q.stride(1) == D, "q heads must be contiguous within a row"
    assert block_tables.dtype == torch.int32 and seq_lens.dtype == torch.int32 and block_tables.stride(1) == 1
    if out is None:
        out = torch.empty(B, Hq, D, dtype=q.dtype, device=q.device)
    if num_splits > 1:
        if workspace is None or workspace.max_splits < num_splits or workspace.part_lse.numel() < B * Hq * num_splits:
            workspace = DecodeWorkspace(B, Hq, D, num_splits, q.device)
        po, pl = workspace.part_out.data_ptr(), workspace.part_lse.data_ptr()
    else:
        po = pl = 0
    kernels().decode_attention(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                               block_tables.data_ptr(), block_tables.stride(0), seq_lens.data_ptr(), po, pl,
                               out.data_ptr(), out.stride(0), B, Hq, Hkv, D, bs, float(scale), int(num_splits),
                               stream_ptr())
    return out


def decode_attention_fused(pend, positions: torch.Tensor, slot_mapping: torch.Tensor, cos_sin: torch.Tensor,
                           k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                           seq_lens: torch.Tensor, num_heads: int, scale: float, num_splits: int = 1,
                           workspace: Optional[DecodeWorkspace] = None, apply_rope: bool = True,
                           out: Optional[torch.Tensor] = None, depth: Optional[int] = None):
    """Paged decode attention on the QKV projection's split-K partials (PendingSum
    [S, B, (Hq + 2 Hkv) D]): each workgroup's prologue reduces its (sequence, kv
    head) slice, applies RoPE and appends the new K/V row to the cache -- the work
    of rope_cache_partials without its launch or the q round trip. -> [B, Hq * D]."""
    S, B, W = pend.part.shape
    Hkv, bs, D = k_cache.shape[1], k_cache.shape[2], k_cache.shape[3]
    Hq = num_heads
    assert W == (Hq + 2 * Hkv) * D and pend.part.is_contiguous()
    assert block_tables.dtype == torch.int32 and seq_lens.dtype == torch.int32 and block_tables.stride(1) == 1
    assert positions.dtype == torch.int32 and slot_mapping.dtype == torch.int32 and cos_sin.dtype == torch.float32
    if out is None:
        out = torch.empty(B, Hq * D, dtype=torch.bfloat16, device=pend.part.device)
    po = pl = 0
    if num_splits > 1:
        if workspace is None or workspace.max_splits < num_splits or workspace.part_lse.numel() < B * Hq * num_splits:
            workspace = DecodeWorkspace(B, Hq, D, num_splits, pend.part.device)
        po, pl = workspace.part_out.data_ptr(), workspace.part_lse.data_ptr()
    kernels().decode_attention_fq(pend.part.data_ptr(), S, positions.data_ptr(), cos_sin.data_ptr(),
                                  slot_mapping.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                  block_tables.data_ptr(), block_tables.stride(0), seq_lens.data_ptr(), po, pl,
                                  out.data_ptr(), out.stride(0), B, Hq, Hkv, D, bs, float(scale), int(num_splits),
                                  1 if apply_rope else 0, stream_ptr(), DECODE_DEPTH if depth is None else depth)
    return out


def prefill_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                      query_start_loc: torch.Tensor, seq_lens: torch.Tensor, max_q_len: int, scale: float,
                      out: Optional[torch.Tensor] = None, gh: Optional[int] = None) -> torch.Tensor:
    """q: [T, Hq, D] packed varlen (rows may be strided); causal w.r.t. absolute
    positions ctx+i where ctx = seq_len - q_len; keys read from the paged cache.
    gh (tests / A/B sweeps; None = the kernel's own choice): > 0 runs the 16-row
    kernel with gh query heads per workgroup; < 0 forces a D = 128 prefill_attn2_kernel
    configuration -gh = 1000 (KS - 1) + 100 NSLOT + 10 NW + GH (key phases, ring
    slots, waves, heads per workgroup; NSLOT 0 = default), e.g. -82 or -1284."""
    if not use_native(q):
        r = prefill_attention_ref(q, k_cache, v_cache, block_tables, query_start_loc, seq_lens, scale)
        if out is not None:
            out.copy_(r.view_as(out))
            return out
        return r
    T, Hq, D = q.shape
    Hkv, bs = k_cache.shape[1], k_cache.shape[2]
    assert q.stride(2) == 1 and q.stride(1) == D
    if out is None:
        out = torch.empty(T, Hq, D, dtype=q.dtype, device=q.device)
    S = seq_lens.shape[0]
    kernels().prefill_attention(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                block_tables.data_ptr(), block_tables.stride(0), query_start_loc.data_ptr(),
                                seq_lens.data_ptr(), out.data_ptr(), out.stride(0), S, int(max_q_len), Hq, Hkv, D,
                                bs, float(scale), stream_ptr(), 0 if gh is None else int(gh))
    return out
