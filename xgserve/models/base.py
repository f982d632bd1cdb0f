"""Shared model plumbing: attention metadata for a packed step, the paged
attention layer, and TP-sharded parameter helpers."""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from .. import ops
from ..ops.attention import DecodeWorkspace
from ..parallel.state import get_state

@dataclass
class AttnMeta:
    """Metadata of one packed engine step: [decode tokens (1/seq)] ++ [prefill/verify chunks].

    All index tensors are int32 on the model's device.
    """
    num_tokens: int
    num_decodes: int
    positions: torch.Tensor
    slot_mapping: torch.Tensor
    dec_block_tables: Optional[torch.Tensor] = None
    dec_seq_lens: Optional[torch.Tensor] = None
    num_splits: int = 1
    workspace: Optional[DecodeWorkspace] = None
    pre_block_tables: Optional[torch.Tensor] = None
    pre_qsl: Optional[torch.Tensor] = None
    pre_seq_lens: Optional[torch.Tensor] = None
    pre_max_q: int = 0

    @property
    def num_prefill_tokens(self) -> int:
        return self.num_tokens - self.num_decodes


def shard(t: torch.Tensor, dim: int, tp: int, rank: int) -> torch.Tensor:
    if tp == 1:
        return t
    n = t.shape[dim]
    assert n % tp == 0, f"dim {dim} of size {n} not divisible by tp={tp}"
    c = n // tp
    return t.narrow(dim, rank * c, c)


def init_weight(shape, std: float, device, dtype, gen: Optional[torch.Generator] = None) -> torch.Tensor:
    t = torch.empty(shape, device=device, dtype=dtype)
    if gen is not None and t.device.type == "cpu":
        t.normal_(0.0, std, generator=gen)
    else:
        t.normal_(0.0, std)
    return t


class PagedAttention:
    """q/k/v from a fused QKV row -> rope + paged KV append -> ragged attention."""

    def __init__(self, num_heads: int, num_kv_heads: int, head_dim: int, use_rope: bool = True):
        self.Hq = num_heads
        self.Hkv = num_kv_heads
        self.D = head_dim
        self.scale = 1.0 / math.sqrt(head_dim)
        self.use_rope = use_rope

    def __call__(self, qkv: torch.Tensor, meta: AttnMeta, kv: Tuple[torch.Tensor, torch.Tensor],
                 cos_sin: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        T = qkv.shape[0]
        kc, vc = kv
        ops.rope_cache(qkv, meta.positions, cos_sin, kc, vc, meta.slot_mapping, self.Hq, self.Hkv, self.D,
                       self.use_rope)
        q = qkv[:, :self.Hq * self.D].view(T, self.Hq, self.D)
        return self.attend(q, meta, kv, out)

    def from_partials(self, pend, meta: AttnMeta, kv: Tuple[torch.Tensor, torch.Tensor],
                      cos_sin: torch.Tensor) -> torch.Tensor:
        """QKV as split-K partial sums (decode skinny GEMM): reduce + rope + KV append in one kernel."""
        T = meta.num_tokens
        q = torch.empty(T, self.Hq * self.D, dtype=torch.bfloat16, device=pend.part.device)
        ops.rope_cache_partials(pend, q, meta.positions, cos_sin, kv[0], kv[1], meta.slot_mapping, self.Hq,
                                self.Hkv, self.D, self.use_rope)
        return self.attend(q.view(T, self.Hq, self.D), meta, kv)

    def fused_decode(self, pend, meta: AttnMeta, kv: Tuple[torch.Tensor, torch.Tensor],
                     cos_sin: torch.Tensor) -> torch.Tensor:
        """Pure-decode step on QKV split-K partials: the attention kernel's prologue
        reduces them, applies RoPE and appends K/V (ops.decode_attention_fused)."""
        return ops.decode_attention_fused(pend, meta.positions, meta.slot_mapping, cos_sin, kv[0], kv[1],
                                          meta.dec_block_tables, meta.dec_seq_lens, self.Hq, self.scale,
                                          meta.num_splits, meta.workspace, self.use_rope)

    def attend(self, q: torch.Tensor, meta: AttnMeta, kv: Tuple[torch.Tensor, torch.Tensor],
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
        T = q.shape[0]
        kc, vc = kv
        if out is None:
            out = torch.empty(T, self.Hq, self.D, dtype=q.dtype, device=q.device)
        nd = meta.num_decodes
        # (decode rows' attention on a side stream under the prefill chunk's attention
        # measured within noise, profiles/r2_mixed_attn_overlap.md)
        if nd > 0:
            ops.decode_attention(q[:nd], kc, vc, meta.dec_block_tables, meta.dec_seq_lens, self.scale,
                                 meta.num_splits, meta.workspace, out=out[:nd])
        if T > nd:
            ops.prefill_attention(q[nd:], kc, vc, meta.pre_block_tables, meta.pre_qsl, meta.pre_seq_lens,
                                  meta.pre_max_q, self.scale, out=out[nd:])
        return out.view(T, self.Hq * self.D)


def local_heads(cfg, tp: int) -> Tuple[int, int]:
    if cfg.num_heads % tp:
        raise ValueError(f"{cfg.num_heads} heads not divisible by tp={tp}")
    hkv = cfg.num_kv_heads // tp if cfg.num_kv_heads >= tp else 1
    if cfg.num_kv_heads >= tp and cfg.num_kv_heads % tp:
        raise ValueError(f"{cfg.num_kv_heads} kv heads not divisible by tp={tp}")
    return cfg.num_heads // tp, hkv


def kv_head_range(cfg, tp: int, rank: int) -> Tuple[int, int]:
    """Global kv heads owned by `rank` (replicated when num_kv_heads < tp)."""
    if cfg.num_kv_heads >= tp:
        n = cfg.num_kv_heads // tp
        return rank * n, n
    per = tp // cfg.num_kv_heads
    return rank // per, 1
