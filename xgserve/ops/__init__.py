"""Operator layer: thin dispatchers over the gfx950 HIP kernels (GPU tensors)
and PyTorch reference implementations (CPU tensors, tests).

Every GPU op here launches a hand-written kernel from csrc/kernels; the
`*_ref` functions are the fp32 PyTorch references the kernel tests compare to.
"""
from .norm import rmsnorm, fused_add_rmsnorm, layernorm, rmsnorm_ref, fused_add_rmsnorm_ref, layernorm_ref, row_sumsq
from .activation import silu_and_mul, gelu_tanh, silu_and_mul_ref, gelu_tanh_ref
from .rope import RotaryCache, rope_cache, rope_cache_ref, build_cos_sin, rope_cache_partials
from . import linear
from .linear import skinny_linear, PendingSum
from .attention import (decode_attention, decode_attention_fused, prefill_attention, decode_attention_ref,
                        prefill_attention_ref, choose_num_splits)
from .sampling import argmax_logprob, sample_tokens, argmax_logprob_ref, segment_sum, subst_tokens
from .embedding import embed_gather, mean_l2norm_rows
from .moe import (moe_topk_softmax, moe_route, moe_route_norm, moe_align, moe_forward_ref, fused_moe, ep_plan,
                  ep_scatter, ep_combine)
from ._native import available as native_available

__all__ = [
    "rmsnorm", "fused_add_rmsnorm", "layernorm", "row_sumsq", "rmsnorm_ref", "fused_add_rmsnorm_ref", "layernorm_ref",
    "silu_and_mul", "gelu_tanh", "silu_and_mul_ref", "gelu_tanh_ref",
    "RotaryCache", "rope_cache", "rope_cache_ref", "build_cos_sin",
    "decode_attention", "decode_attention_fused", "prefill_attention", "decode_attention_ref", "prefill_attention_ref", "choose_num_splits",
    "argmax_logprob", "sample_tokens", "argmax_logprob_ref", "segment_sum", "subst_tokens",
    "embed_gather", "mean_l2norm_rows",
    "moe_topk_softmax", "moe_route", "moe_route_norm", "moe_align", "moe_forward_ref", "fused_moe", "ep_plan", "ep_scatter", "ep_combine",
    "native_available",
]
