"""Plain-PyTorch fp32 reference forward (dense, unpaged, one sequence) for the
model-numerics tests: the engine's greedy tokens / logits are checked against
this with the same weights."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ..ops.linear import deinterleave_gate_up
from ..ops.rope import build_cos_sin


def _rot(x, cos, sin):
    h = x.shape[-1] // 2
    return torch.cat([x[..., :h] * cos - x[..., h:] * sin, x[..., h:] * cos + x[..., :h] * sin], -1)


@torch.no_grad()
def reference_logits(model, tokens) -> torch.Tensor:
    """Logits [len(tokens), V] of a TP=1 model on one sequence, fp32 math."""
    cfg = model.cfg
    ids = torch.tensor(tokens, dtype=torch.long, device=model.device)
    T = ids.shape[0]
    D = cfg.head_dim
    causal = torch.ones(T, T, dtype=torch.bool, device=ids.device).tril()
    if cfg.arch == "gpt2":
        x = model.wte.float()[ids] + model.wpe.float()[torch.arange(T, device=ids.device)]
        for L in model.layers:
            h = F.layer_norm(x, (x.shape[-1],), L.ln1_w.float(), L.ln1_b.float(), cfg.norm_eps)
            qkv = h @ L.qkv_w.float().t() + L.qkv_b.float()
            q, k, v = qkv.split(cfg.hidden_size, -1)
            q, k, v = (t.view(T, cfg.num_heads, D).transpose(0, 1) for t in (q, k, v))
            s = (q @ k.transpose(-1, -2)) / math.sqrt(D)
            s = s.masked_fill(~causal, float("-inf"))
            a = (torch.softmax(s, -1) @ v).transpose(0, 1).reshape(T, -1)
            x = x + a @ L.o_w.float().t() + L.o_b.float()
            h = F.layer_norm(x, (x.shape[-1],), L.ln2_w.float(), L.ln2_b.float(), cfg.norm_eps)
            h = F.gelu(h @ L.fc_w.float().t() + L.fc_b.float(), approximate="tanh")
            x = x + h @ L.proj_w.float().t() + L.proj_b.float()
        x = F.layer_norm(x, (x.shape[-1],), model.lnf_w.float(), model.lnf_b.float(), cfg.norm_eps)
        return x @ model.wte.float().t()

    cs = build_cos_sin(D, max(T, 1), cfg.rope_theta, cfg.rope_scaling, device=ids.device)
    cos, sin = cs[:, None, :D // 2], cs[:, None, D // 2:]
    eps = cfg.norm_eps

    def rms(x, w):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w.float()

    x = model.embed.float()[ids]
    Hq, Hkv = cfg.num_heads, cfg.num_kv_heads
    for L in model.layers:
        h = rms(x, L.input_norm)
        qkv = h @ L.qkv.float().t()
        q = qkv[:, :Hq * D].view(T, Hq, D)
        k = qkv[:, Hq * D:(Hq + Hkv) * D].view(T, Hkv, D)
        v = qkv[:, (Hq + Hkv) * D:].view(T, Hkv, D)
        q, k = _rot(q, cos, sin), _rot(k, cos, sin)
        G = Hq // Hkv
        k = k.repeat_interleave(G, 1)
        v = v.repeat_interleave(G, 1)
        s = torch.einsum("thd,shd->hts", q, k) / math.sqrt(D)
        s = s.masked_fill(~causal[None], float("-inf"))
        a = torch.einsum("hts,shd->thd", torch.softmax(s, -1), v).reshape(T, Hq * D)
        x = x + a @ L.o.float().t()
        h = rms(x, L.post_norm)
        if L.moe:
            p = torch.softmax(h @ L.router.float().t(), -1)
            w, e = torch.topk(p, cfg.experts_per_token, -1)
            w = w / w.sum(-1, keepdim=True)
            out = torch.zeros_like(h)
            Fd = cfg.intermediate_size
            for t in range(T):
                for j in range(cfg.experts_per_token):
                    ei = int(e[t, j])
                    gw, uw = deinterleave_gate_up(L.w13[ei])  # block-16 interleaved per expert
                    a = F.silu(h[t] @ gw.float().t()) * (h[t] @ uw.float().t())
                    out[t] += w[t, j] * (a @ L.w2[ei].float().t())
            x = x + out
        else:
            gw, uw = deinterleave_gate_up(L.gate_up)  # stored block-16 interleaved
            x = x + (F.silu(h @ gw.float().t()) * (h @ uw.float().t())) @ L.down.float().t()
    x = rms(x, model.norm)
    w = model.embed if model.lm_head is None else model.lm_head[:cfg.vocab_size]
    return x @ w.float().t()


@torch.no_grad()
def reference_greedy(model, prompt, n: int):
    toks = list(prompt)
    for _ in range(n):
        toks.append(int(reference_logits(model, toks)[-1].argmax()))
    return toks[len(prompt):]
