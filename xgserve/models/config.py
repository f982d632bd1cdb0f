"""Model registry: architecture hyper-parameters of the supported families.

BASELINE.json names Llama-3 8B / 70B, Mixtral 8x7B and GPT-2-small; the
registry also carries Llama-3.2-1B (speculative-decoding draft) and tiny
variants of every family for CPU tests. `from_hf_config` maps a HF
config.json onto the same dataclass (safetensors checkpoints).
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field, replace
from typing import Dict, List, Optional


@dataclass
class ModelConfig:
    name: str
    arch: str                      # "llama" | "mixtral" | "gpt2"
    hidden_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate_size: int
    vocab_size: int
    max_position: int = 8192
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    norm_eps: float = 1e-5
    tie_embeddings: bool = False
    num_experts: int = 0
    experts_per_token: int = 0
    bos_token_id: int = 1
    eos_token_ids: List[int] = field(default_factory=lambda: [2])
    dtype: str = "bfloat16"

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    def num_params(self) -> int:
        H, F, V, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_layers
        attn = H * (self.q_size + 2 * self.kv_size) + self.q_size * H
        if self.arch == "mixtral":
            mlp = self.num_experts * 3 * H * F + H * self.num_experts
        elif self.arch == "gpt2":
            mlp = 2 * H * F
        else:
            mlp = 3 * H * F
        emb = V * H * (1 if self.tie_embeddings else 2)
        return L * (attn + mlp + 2 * H) + emb + H

    def kv_bytes_per_token(self, tp: int = 1, dtype_bytes: int = 2) -> int:
        kvh = max(1, self.num_kv_heads // tp)
        return 2 * self.num_layers * kvh * self.head_dim * dtype_bytes

    def to_dict(self) -> dict:
        return asdict(self)


_REGISTRY: Dict[str, ModelConfig] = {}


def register(cfg: ModelConfig) -> ModelConfig:
    _REGISTRY[cfg.name] = cfg
    return cfg


register(ModelConfig("llama3-8b", "llama", 4096, 32, 32, 8, 128, 14336, 128256, 8192, 500000.0,
                     bos_token_id=128000, eos_token_ids=[128001, 128009]))
register(ModelConfig("llama3-70b", "llama", 8192, 80, 64, 8, 128, 28672, 128256, 8192, 500000.0,
                     bos_token_id=128000, eos_token_ids=[128001, 128009]))
register(ModelConfig("llama3.2-1b", "llama", 2048, 16, 32, 8, 64, 8192, 128256, 8192, 500000.0,
                     rope_scaling={"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
                                   "high_freq_factor": 4.0, "original_max_position_embeddings": 8192},
                     tie_embeddings=True, bos_token_id=128000, eos_token_ids=[128001, 128009]))
register(ModelConfig("mixtral-8x7b", "mixtral", 4096, 32, 32, 8, 128, 14336, 32000, 32768, 1000000.0,
                     num_experts=8, experts_per_token=2, bos_token_id=1, eos_token_ids=[2]))
register(ModelConfig("gpt2", "gpt2", 768, 12, 12, 12, 64, 3072, 50257, 1024, 0.0, norm_eps=1e-5,
                     tie_embeddings=True, bos_token_id=50256, eos_token_ids=[50256], dtype="float32"))
# tiny variants for CPU / unit tests (same code paths, small dims)
register(ModelConfig("llama-tiny", "llama", 256, 2, 4, 2, 64, 512, 512, 1024, 10000.0,
                     bos_token_id=1, eos_token_ids=[2]))
register(ModelConfig("llama-tiny-draft", "llama", 128, 1, 2, 1, 64, 256, 512, 1024, 10000.0,
                     bos_token_id=1, eos_token_ids=[2]))
register(ModelConfig("llama-tiny-gqa8", "llama", 512, 2, 8, 8, 64, 1024, 512, 1024, 10000.0,
                     bos_token_id=1, eos_token_ids=[2]))
register(ModelConfig("mixtral-tiny", "mixtral", 256, 2, 4, 2, 64, 256, 512, 1024, 1000000.0,
                     num_experts=8, experts_per_token=2, bos_token_id=1, eos_token_ids=[2]))
register(ModelConfig("gpt2-tiny", "gpt2", 128, 2, 2, 2, 64, 512, 512, 256, 0.0, tie_embeddings=True,
                     bos_token_id=0, eos_token_ids=[0], dtype="float32"))


def get_config(name: str) -> ModelConfig:
    if name in _REGISTRY:
        return replace(_REGISTRY[name])
    if os.path.isdir(name) and os.path.exists(os.path.join(name, "config.json")):
        return from_hf_config(os.path.join(name, "config.json"), name=name)
    raise KeyError(f"unknown model {name!r}; known: {sorted(_REGISTRY)} or a HF checkpoint directory")


def list_models() -> List[str]:
    return sorted(_REGISTRY)


def from_hf_config(path: str, name: Optional[str] = None) -> ModelConfig:
    with open(path) as f:
        c = json.load(f)
    mt = c.get("model_type", "llama")
    eos = c.get("eos_token_id", 2)
    eos = eos if isinstance(eos, list) else [eos]
    if mt == "gpt2":
        H = c["n_embd"]
        return ModelConfig(name or "gpt2", "gpt2", H, c["n_layer"], c["n_head"], c["n_head"], H // c["n_head"],
                           c.get("n_inner") or 4 * H, c["vocab_size"], c.get("n_positions", 1024), 0.0,
                           norm_eps=c.get("layer_norm_epsilon", 1e-5), tie_embeddings=True,
                           bos_token_id=c.get("bos_token_id", 50256), eos_token_ids=eos, dtype="float32")
    H = c["hidden_size"]
    nh = c["num_attention_heads"]
    arch = "mixtral" if mt == "mixtral" else "llama"
    return ModelConfig(
        name or mt, arch, H, c["num_hidden_layers"], nh, c.get("num_key_value_heads", nh),
        c.get("head_dim", H // nh), c["intermediate_size"], c["vocab_size"],
        c.get("max_position_embeddings", 8192), float(c.get("rope_theta", 10000.0)), c.get("rope_scaling"),
        c.get("rms_norm_eps", 1e-5), bool(c.get("tie_word_embeddings", False)),
        c.get("num_local_experts", 0), c.get("num_experts_per_tok", 0), c.get("bos_token_id", 1), eos)
