"""Measurement knobs: the A/B switches and plan overrides the profiles in
`profiles/` were measured with, behind ONE environment variable instead of one
variable per knob:

  XGS_TUNE="key=value|key=value|..."      e.g.  XGS_TUNE="krot=0|decode_depth=3"

Keys (default in brackets; every default is the production setting):
  fused_decode [1]         fused decode layer (GEMM epilogue norms / residuals)
  async_sched [1]          plan + launch step N+1 before step N's tokens reach the host
  early_release [config]   release length-finishing rows at lookahead
  spin_wait [1]            host polls the step event instead of blocking
  pf [1]                   gemm_pf projections of prompt-sized mixed steps: 1 = the measured windows,
                           0 = library GEMMs, or a list "qkv,o,gate_up,down" of those allowed
  pf_windows [gate_up:448-576/down:513-576]   step sizes (tokens) per projection that take gemm_pf
  moe_pf [1]               prompt-sized expert GEMMs (> 256 token-expert pairs) on gemm_pf's grouped form
  argmax_split [1]         greedy argmax over large vocabularies: 8 workgroups per row
  moe_w2_small [1]         decode-sized w2 on 64-column tiles (<= 8 and 64-256 token-expert pairs)
  krot [1]                 K-chunk rotation of the weight-streaming GEMMs (0 / 1 / 2)
  m64_plans / mw_plans     gemm_m64g / gemm_mw plan overrides, "NxKxMODE@BUCKET=...;..."
  mw_max_tokens [320]      largest step on gemm_mw
  resid_inlaunch_kb [32]   in-launch residual reduce bound of the fused decode GEMMs
  decode_depth [2]         decode attention K/V register pipeline depth (4: depth 2 with the classic QKV prologue)
  decode_max_splits [16]   split-K cap of decode attention
  gemm_ar [1]              TP decode: all-reduce inside the row-parallel O / down GEMM launches
  gemm_ar_shared [0]       test-only: GG_AR also for <= 4 ranks sharing one GPU (one-GPU boxes)
  small_m_tiles [128]      column-tile statistics a M <= 16 consumer combines (64: pair combine above)
  ar_ll_max [262144]       push (LL) all-reduce up to this many bytes (0: pull kernels)
  sim_ar_us [0]            --tp-shard simulation: stand-in all-reduce latency
  tp_overlap_chunks [2]    TP prefill: all-reduces pipelined over this many chunks
  tp_overlap_min_tokens [256]
  ep_exact_min_pairs [256] EP all_to_all: count-exact splits from this many pairs
Unknown keys are an error (a typo must not silently measure the default).
"""
from __future__ import annotations

import os
from typing import Dict

KEYS = {"fused_decode", "async_sched", "early_release", "spin_wait", "pf", "pf_windows", "moe_pf", "moe_w2_small", "argmax_split", "gemm_ar", "gemm_ar_shared", "small_m_tiles", "krot", "m64_plans", "mw_plans",
        "mw_max_tokens", "resid_inlaunch_kb", "decode_depth", "decode_max_splits", "ar_ll_max", "sim_ar_us",
        "tp_overlap_chunks", "tp_overlap_min_tokens", "ep_exact_min_pairs"}


def _parse(spec: str) -> Dict[str, str]:
    out = {}
    for item in filter(None, (t.strip() for t in spec.split("|"))):
        if "=" not in item:
            raise ValueError(f"XGS_TUNE: expected key=value, got {item!r}")
        k, v = item.split("=", 1)
        k = k.strip()
        if k not in KEYS:
            raise ValueError(f"XGS_TUNE: unknown key {k!r} (known: {sorted(KEYS)})")
        out[k] = v.strip()
    return out


def knobs() -> Dict[str, str]:
    return _parse(os.environ.get("XGS_TUNE", ""))


def get_str(key: str, default: str) -> str:
    assert key in KEYS, key
    return knobs().get(key, default)


def get_int(key: str, default: int) -> int:
    return int(float(get_str(key, str(default))))


def get_float(key: str, default: float) -> float:
    return float(get_str(key, str(default)))


def get_bool(key: str, default: bool) -> bool:
    return get_str(key, "1" if default else "0") not in ("0", "false", "False", "off", "")
