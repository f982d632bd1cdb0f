"""GPT-2 (small) on the paged-KV engine -- BASELINE config 1 (CPU eager
plumbing through the HTTP server); also runs on the GPU in bf16.

Learned absolute positions, pre-LayerNorm blocks, MHA with biases, GELU-tanh
MLP, tied LM head. The paged KV append reuses K2/K4 with rotation disabled.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..parallel.state import get_state
from .base import AttnMeta, PagedAttention
from .config import ModelConfig


def _p(t):
    return nn.Parameter(t, requires_grad=False)


class GPT2Layer(nn.Module):
    def __init__(self, cfg: ModelConfig, device, dtype):
        super().__init__()
        H, Fd = cfg.hidden_size, cfg.intermediate_size
        e = lambda *s: torch.empty(*s, device=device, dtype=dtype)  # noqa: E731
        self.ln1_w, self.ln1_b = _p(torch.ones(H, device=device, dtype=dtype)), _p(torch.zeros(H, device=device, dtype=dtype))
        self.ln2_w, self.ln2_b = _p(torch.ones(H, device=device, dtype=dtype)), _p(torch.zeros(H, device=device, dtype=dtype))
        self.qkv_w, self.qkv_b = _p(e(3 * H, H)), _p(torch.zeros(3 * H, device=device, dtype=dtype))
        self.o_w, self.o_b = _p(e(H, H)), _p(torch.zeros(H, device=device, dtype=dtype))
        self.fc_w, self.fc_b = _p(e(Fd, H)), _p(torch.zeros(Fd, device=device, dtype=dtype))
        self.proj_w, self.proj_b = _p(e(H, Fd)), _p(torch.zeros(H, device=device, dtype=dtype))
        self.attn = PagedAttention(cfg.num_heads, cfg.num_heads, cfg.head_dim, use_rope=False)
        self.eps = cfg.norm_eps

    def forward(self, x, meta: AttnMeta, kv, cos_sin):
        h = ops.layernorm(x, self.ln1_w, self.ln1_b, self.eps)
        qkv = F.linear(h, self.qkv_w, self.qkv_b)
        a = self.attn(qkv, meta, kv, cos_sin)
        x = x + F.linear(a, self.o_w, self.o_b)
        h = ops.layernorm(x, self.ln2_w, self.ln2_b, self.eps)
        h = ops.gelu_tanh(F.linear(h, self.fc_w, self.fc_b))
        return x + F.linear(h, self.proj_w, self.proj_b)


class GPT2ForCausalLM(nn.Module):
    def __init__(self, cfg: ModelConfig, device="cpu", dtype=torch.float32, tp: Optional[int] = None,
                 rank: Optional[int] = None):
        super().__init__()
        tp = get_state().tp_size if tp is None else tp
        if tp != 1:
            raise ValueError("GPT-2 runs with tp=1 (use DP replicas to scale)")
        self.cfg = cfg
        self.tp, self.rank = 1, 0
        self.device = torch.device(device)
        self.dtype = dtype
        H = cfg.hidden_size
        self.wte = _p(torch.empty(cfg.vocab_size, H, device=device, dtype=dtype))
        self.wpe = _p(torch.empty(cfg.max_position, H, device=device, dtype=dtype))
        self.layers = nn.ModuleList([GPT2Layer(cfg, device, dtype) for _ in range(cfg.num_layers)])
        self.lnf_w = _p(torch.ones(H, device=device, dtype=dtype))
        self.lnf_b = _p(torch.zeros(H, device=device, dtype=dtype))
        self.cos_sin = torch.zeros(1, cfg.head_dim, device=device, dtype=torch.float32)  # unused (no rope)
        self.num_kv_heads_local = cfg.num_heads

    @torch.no_grad()
    def random_init(self, seed: int = 0, std: float = 0.02):
        g = torch.Generator(device=self.device).manual_seed(seed) if self.device.type == "cuda" \
            else torch.Generator().manual_seed(seed)
        for name, p in self.named_parameters():
            if name.endswith("_b") or "ln" in name:
                continue
            p.normal_(0.0, std, generator=g)

    def forward(self, input_ids: torch.Tensor, meta: AttnMeta, kv_caches: List[Tuple[torch.Tensor, torch.Tensor]]):
        pos = meta.positions.long().clamp(max=self.cfg.max_position - 1)
        x = F.embedding(input_ids, self.wte) + F.embedding(pos, self.wpe)
        for i, layer in enumerate(self.layers):
            x = layer(x, meta, kv_caches[i], self.cos_sin)
        return ops.layernorm(x, self.lnf_w, self.lnf_b, self.cfg.norm_eps)

    def compute_logits(self, h: torch.Tensor) -> torch.Tensor:
        return F.linear(h, self.wte)

    def set_moe_comm(self, mode: str):
        pass
