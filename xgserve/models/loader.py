"""Model construction + safetensors checkpoint loading with per-rank TP/EP slicing.

Checkpoints: a HF-layout directory (config.json + model.safetensors or
model-XXXXX-of-YYYYY.safetensors + model.safetensors.index.json). Each rank
reads ONLY its shard through safetensors' lazy `get_slice` (row slices for
column-parallel weights, column slices for row-parallel ones, whole experts for
EP), converts to the serving dtype on the host and copies to HBM. q/k/v and
gate/up are fused on load. `save_checkpoint` writes the same HF layout from a
TP=1 model (tests, and to materialise random-init checkpoints).
"""
from __future__ import annotations

import json
import os
from typing import Callable, Dict, Optional

import torch

from ..ops.linear import deinterleave_gate_up, interleave_gate_up
from .base import kv_head_range
from .config import ModelConfig, get_config
from .gpt2 import GPT2ForCausalLM
from .llama import LlamaForCausalLM


def model_class(cfg: ModelConfig):
    return GPT2ForCausalLM if cfg.arch == "gpt2" else LlamaForCausalLM


def build_model(cfg: ModelConfig, device="cpu", dtype: Optional[torch.dtype] = None,
                checkpoint: Optional[str] = None, seed: int = 0, tp: Optional[int] = None,
                rank: Optional[int] = None, weight_dtype: Optional[str] = None):
    """weight_dtype "fp8" / "int8" / "int4": also keep quantized weight copies for
    decode batches <= 64 (LlamaForCausalLM.quantize_weights); activations and
    everything else stay `dtype`."""
    if dtype is None:
        dtype = torch.float32 if (cfg.dtype == "float32" and torch.device(device).type == "cpu") else torch.bfloat16
    m = model_class(cfg)(cfg, device=device, dtype=dtype, tp=tp, rank=rank)
    if checkpoint:
        load_checkpoint(m, checkpoint)
    else:
        m.random_init(seed)
    if hasattr(m, "fold_norms"):
        m.fold_norms()  # RMSNorm weights into the projections (fused decode layer)
    if weight_dtype in ("fp8", "int8", "int4"):
        if not (hasattr(m, "quantize_weights") and m.quantize_weights(weight_dtype)):
            raise ValueError(f"{weight_dtype} weights are not supported for {cfg.name} on {device}")
    elif weight_dtype not in (None, "bf16", "fp16", "fp32"):
        raise ValueError(f"unknown weight_dtype {weight_dtype!r}")
    m.eval()
    return m


class _Reader:
    def __init__(self, path: str):
        from safetensors import safe_open
        self.path = path
        idx = os.path.join(path, "model.safetensors.index.json")
        files = {}
        if os.path.exists(idx):
            with open(idx) as f:
                wm = json.load(f)["weight_map"]
            for name, fn in wm.items():
                files.setdefault(fn, []).append(name)
        else:
            for fn in sorted(os.listdir(path)):
                if fn.endswith(".safetensors"):
                    files[fn] = None
        self.handles = {fn: safe_open(os.path.join(path, fn), framework="pt") for fn in files}
        self.where: Dict[str, str] = {}
        for fn, h in self.handles.items():
            for k in h.keys():
                self.where[k] = fn

    def has(self, name: str) -> bool:
        return name in self.where

    def get(self, name: str, dim: Optional[int] = None, start: int = 0, length: Optional[int] = None) -> torch.Tensor:
        if name not in self.where:
            raise KeyError(f"missing tensor {name!r} in checkpoint {self.path}")
        sl = self.handles[self.where[name]].get_slice(name)
        if dim is None:
            return sl[:]
        shape = sl.get_shape()
        end = start + (length if length is not None else shape[dim] - start)
        idx = [slice(None)] * len(shape)
        idx[dim] = slice(start, end)
        return sl[tuple(idx)]


def _copy(dst: torch.nn.Parameter, src: torch.Tensor, name: str):
    if tuple(dst.shape) != tuple(src.shape):
        raise ValueError(f"shape mismatch for {name}: model {tuple(dst.shape)} vs checkpoint {tuple(src.shape)}")
    dst.data.copy_(src.to(dst.dtype))


@torch.no_grad()
def load_checkpoint(model, path: str) -> None:
    r = _Reader(path)
    cfg = model.cfg
    if cfg.arch == "gpt2":
        _load_gpt2(model, r)
    else:
        _load_llama(model, r)


def _pre(r: _Reader) -> str:
    return "model." if r.has("model.embed_tokens.weight") else ""


def _load_llama(m, r: _Reader):
    cfg, tp, rank = m.cfg, m.tp, m.rank
    D, H = cfg.head_dim, cfg.hidden_size
    p = _pre(r)
    _copy(m.embed, r.get(f"{p}embed_tokens.weight"), "embed")
    _copy(m.norm, r.get(f"{p}norm.weight"), "norm")
    if m.lm_head is not None:
        name = "lm_head.weight" if r.has("lm_head.weight") else f"{p}embed_tokens.weight"
        V = cfg.vocab_size
        per = m.V_pad // tp
        lo = rank * per
        n = max(0, min(per, V - lo))
        w = torch.zeros(per, H)
        if n > 0:
            w[:n] = r.get(name, 0, lo, n).float()
        _copy(m.lm_head, w, "lm_head")
    Hq_l = cfg.num_heads // tp
    kv0, nkv = kv_head_range(cfg, tp, rank)
    for i, L in enumerate(m.layers):
        b = f"{p}layers.{i}."
        _copy(L.input_norm, r.get(b + "input_layernorm.weight"), "input_norm")
        _copy(L.post_norm, r.get(b + "post_attention_layernorm.weight"), "post_norm")
        q = r.get(b + "self_attn.q_proj.weight", 0, rank * Hq_l * D, Hq_l * D)
        k = r.get(b + "self_attn.k_proj.weight", 0, kv0 * D, nkv * D)
        v = r.get(b + "self_attn.v_proj.weight", 0, kv0 * D, nkv * D)
        _copy(L.qkv, torch.cat([q, k, v], 0), f"layer{i}.qkv")
        _copy(L.o, r.get(b + "self_attn.o_proj.weight", 1, rank * Hq_l * D, Hq_l * D), f"layer{i}.o")
        if L.moe:
            _copy(L.router, r.get(b + "block_sparse_moe.gate.weight"), "router")
            for el in range(L.E_local):
                e = L.expert_offset + el
                eb = b + f"block_sparse_moe.experts.{e}."
                L.w13.data[el].copy_(interleave_gate_up(r.get(eb + "w1.weight"), r.get(eb + "w3.weight")).to(L.w13.dtype))
                L.w2.data[el].copy_(r.get(eb + "w2.weight").to(L.w2.dtype))
        else:
            Fl = cfg.intermediate_size // tp
            g = r.get(b + "mlp.gate_proj.weight", 0, rank * Fl, Fl)
            u = r.get(b + "mlp.up_proj.weight", 0, rank * Fl, Fl)
            _copy(L.gate_up, interleave_gate_up(g, u), f"layer{i}.gate_up")
            _copy(L.down, r.get(b + "mlp.down_proj.weight", 1, rank * Fl, Fl), f"layer{i}.down")


def _load_gpt2(m, r: _Reader):
    p = "transformer." if r.has("transformer.wte.weight") else ""
    _copy(m.wte, r.get(p + "wte.weight"), "wte")
    _copy(m.wpe, r.get(p + "wpe.weight"), "wpe")
    _copy(m.lnf_w, r.get(p + "ln_f.weight"), "ln_f")
    _copy(m.lnf_b, r.get(p + "ln_f.bias"), "ln_f.b")
    for i, L in enumerate(m.layers):
        b = f"{p}h.{i}."
        _copy(L.ln1_w, r.get(b + "ln_1.weight"), "ln1")
        _copy(L.ln1_b, r.get(b + "ln_1.bias"), "ln1b")
        _copy(L.ln2_w, r.get(b + "ln_2.weight"), "ln2")
        _copy(L.ln2_b, r.get(b + "ln_2.bias"), "ln2b")
        # HF GPT-2 uses Conv1D ([in, out]) -> transpose to the nn.Linear layout
        _copy(L.qkv_w, r.get(b + "attn.c_attn.weight").t(), "c_attn")
        _copy(L.qkv_b, r.get(b + "attn.c_attn.bias"), "c_attn.b")
        _copy(L.o_w, r.get(b + "attn.c_proj.weight").t(), "c_proj")
        _copy(L.o_b, r.get(b + "attn.c_proj.bias"), "c_proj.b")
        _copy(L.fc_w, r.get(b + "mlp.c_fc.weight").t(), "c_fc")
        _copy(L.fc_b, r.get(b + "mlp.c_fc.bias"), "c_fc.b")
        _copy(L.proj_w, r.get(b + "mlp.c_proj.weight").t(), "mlp.c_proj")
        _copy(L.proj_b, r.get(b + "mlp.c_proj.bias"), "mlp.c_proj.b")


@torch.no_grad()
def save_checkpoint(model, path: str) -> None:
    """Write a TP=1 model in HF layout (safetensors + config.json)."""
    from safetensors.torch import save_file
    assert model.tp == 1, "save from a TP=1 model"
    cfg = model.cfg
    os.makedirs(path, exist_ok=True)
    t: Dict[str, torch.Tensor] = {}
    if cfg.arch == "gpt2":
        t["transformer.wte.weight"] = model.wte
        t["transformer.wpe.weight"] = model.wpe
        t["transformer.ln_f.weight"] = model.lnf_w
        t["transformer.ln_f.bias"] = model.lnf_b
        for i, L in enumerate(model.layers):
            b = f"transformer.h.{i}."
            t[b + "ln_1.weight"], t[b + "ln_1.bias"] = L.ln1_w, L.ln1_b
            t[b + "ln_2.weight"], t[b + "ln_2.bias"] = L.ln2_w, L.ln2_b
            t[b + "attn.c_attn.weight"], t[b + "attn.c_attn.bias"] = L.qkv_w.t(), L.qkv_b
            t[b + "attn.c_proj.weight"], t[b + "attn.c_proj.bias"] = L.o_w.t(), L.o_b
            t[b + "mlp.c_fc.weight"], t[b + "mlp.c_fc.bias"] = L.fc_w.t(), L.fc_b
            t[b + "mlp.c_proj.weight"], t[b + "mlp.c_proj.bias"] = L.proj_w.t(), L.proj_b
        hf = {"model_type": "gpt2", "n_embd": cfg.hidden_size, "n_layer": cfg.num_layers, "n_head": cfg.num_heads,
              "n_inner": cfg.intermediate_size, "vocab_size": cfg.vocab_size, "n_positions": cfg.max_position,
              "layer_norm_epsilon": cfg.norm_eps, "bos_token_id": cfg.bos_token_id,
              "eos_token_id": cfg.eos_token_ids[0]}
    else:
        D = cfg.head_dim
        qs, ks = cfg.num_heads * D, cfg.num_kv_heads * D
        t["model.embed_tokens.weight"] = model.embed
        t["model.norm.weight"] = model.norm
        if model.lm_head is not None:
            t["lm_head.weight"] = model.lm_head[:cfg.vocab_size]
        for i, L in enumerate(model.layers):
            b = f"model.layers.{i}."
            t[b + "input_layernorm.weight"] = L.input_norm
            t[b + "post_attention_layernorm.weight"] = L.post_norm
            t[b + "self_attn.q_proj.weight"] = L.qkv[:qs]
            t[b + "self_attn.k_proj.weight"] = L.qkv[qs:qs + ks]
            t[b + "self_attn.v_proj.weight"] = L.qkv[qs + ks:]
            t[b + "self_attn.o_proj.weight"] = L.o
            if L.moe:
                Fd = cfg.intermediate_size
                t[b + "block_sparse_moe.gate.weight"] = L.router
                for e in range(cfg.num_experts):
                    eb = b + f"block_sparse_moe.experts.{e}."
                    t[eb + "w1.weight"], t[eb + "w3.weight"] = deinterleave_gate_up(L.w13[e])
                    t[eb + "w2.weight"] = L.w2[e]
            else:
                Fd = cfg.intermediate_size
                gw, uw = deinterleave_gate_up(L.gate_up)
                t[b + "mlp.gate_proj.weight"] = gw
                t[b + "mlp.up_proj.weight"] = uw
                t[b + "mlp.down_proj.weight"] = L.down
        hf = {"model_type": "mixtral" if cfg.arch == "mixtral" else "llama", "hidden_size": cfg.hidden_size,
              "num_hidden_layers": cfg.num_layers, "num_attention_heads": cfg.num_heads,
              "num_key_value_heads": cfg.num_kv_heads, "head_dim": cfg.head_dim,
              "intermediate_size": cfg.intermediate_size, "vocab_size": cfg.vocab_size,
              "max_position_embeddings": cfg.max_position, "rope_theta": cfg.rope_theta,
              "rope_scaling": cfg.rope_scaling, "rms_norm_eps": cfg.norm_eps,
              "tie_word_embeddings": cfg.tie_embeddings, "bos_token_id": cfg.bos_token_id,
              "eos_token_id": cfg.eos_token_ids}
        if cfg.arch == "mixtral":
            hf["num_local_experts"] = cfg.num_experts
            hf["num_experts_per_tok"] = cfg.experts_per_token
    save_file({k: v.detach().contiguous().cpu() for k, v in t.items()}, os.path.join(path, "model.safetensors"))
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(hf, f, indent=1)
