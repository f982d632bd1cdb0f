"""Llama-3 (8B / 70B / 3.2-1B) and Mixtral-8x7B decoders on the paged-KV engine.

Tensor parallelism (Megatron layout, one process per GPU, RCCL/xGMI):
  * fused QKV and gate_up projections are column-parallel (heads / FFN split),
  * o_proj and down_proj are row-parallel followed by one all-reduce each,
  * the LM head is vocab-parallel (logits all-gathered), the embedding is
    replicated (2 GB for 70B -- negligible in 288 GB of HBM).
Expert parallelism (Mixtral): EP == TP group, rank r owns experts
[r*E/tp, (r+1)*E/tp). Two exchange forms, chosen per step by moe_comm "auto" (the
default: allreduce for decode-sized steps on the custom IPC all-reduce, all_to_all
for prefill-sized ones) or forced with "alltoall" / "allreduce":
  * "alltoall" (prefill steps under "auto"; BASELINE config 5): each rank routes its
    token slice, packs (token, choice) rows for the expert owners with the HIP
    ep_plan / ep_scatter kernels (count-exact splits on eager prefill steps,
    fixed capacity under graph capture), runs its local experts as one grouped
    GEMM, returns rows with a second all_to_all, combines them with ep_combine
    and all-gathers the slices;
  * "allreduce": every rank runs its local experts on all tokens and one
    all-reduce sums the partial outputs.
Per layer the hot path is: fused_add_rmsnorm (K1) -> QKV GEMM -> rope+KV append
(K2/K4) -> paged decode / varlen prefill attention (K6/K5) -> o GEMM -> AR ->
fused_add_rmsnorm -> gate_up GEMM -> SiLU-gate (K3) -> down GEMM -> AR.
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops, tune
from ..parallel import comm
from ..parallel.state import get_state
from ..ops import linear as linear_mod
from ..ops.linear import (MODE_PARTIAL, MODE_SILU, MW_MAX_M, W8_MAX_M, W8_MIN_ELEMS, ResidWorkspace, RowStats,
                          lm_head_linear, m64_ar_resid_linear, m64_linear, m64_norm_linear, m64_plan,
                          m64_resid_linear,
                          mw_linear, mw_plan, pf_linear, pf_plan, pick_split,
                          quantize_fp8, quantize_weight, skinny_linear, splitk_linear, splitk_prefill_ok, w8_linear,
                          w8_plan, WQ_FORMATS)
from .base import AttnMeta, PagedAttention, init_weight, kv_head_range, local_heads, shard
from .config import ModelConfig



FAST_M_SMALL = 16   # tokens per step handled entirely by the streaming skinny GEMM
FAST_M_SLAB = 64    # tokens per step for the O-projection slab kernel
# Fused decode layer (dense Llama, TP=1, pure-decode steps of <= 64 tokens): the
# RMSNorms become GEMM epilogue row scales (norm weights folded into W), the
# residual adds + norm statistics run inside the O / down GEMM launches and the
# QKV reduce + RoPE + KV append inside the attention prologue: 4 GEMM launches +
# 1 attention launch per layer instead of 9. Under TP the O / down GEMMs emit
# split-K partials and ONE custom all-reduce launch per projection reduces them,
# sums across ranks over xGMI, adds the residual and writes the next norm's
# statistics (comm.tp_allreduce_resid): 6 launches + attention per layer instead
# of 11. XGS_TUNE fused_decode=0 restores the unfused chain (A/B measurements, tests).
FUSED_DECODE = tune.get_bool("fused_decode", True)
# 64 < T <= this many tokens (the mixed step: decode rows + one bounded prefill chunk)
# run every projection on gemm_mw (csrc/kernels/gemm_mw.hip): weight-stream-bound
# MFMA GEMMs whose split-K partials go to the consumers, SiLU-gate in gate_up.
# 0 = hipBLASLt for every step above 64 tokens.
MW_MAX_TOKENS = min(MW_MAX_M, tune.get_int("mw_max_tokens", MW_MAX_M))
# Prompt-sized mixed steps on TP = 1: each projection takes gemm_pf
# (csrc/kernels/gemm_pf.hip) for the step sizes where it measured faster than the
# tuned library GEMM (profiles/r6/r6p_pf_vs_library.md, cold weights, the engine's
# library forms) -- QKV / O / down as split-K partials into their consumers, gate_up
# with the SiLU gate in its epilogue:
#   gate_up 448-576 rows: 4-5 % ahead of the library's GEMM + SiLU-gate pair at 448 / 512
#     rows, 22 % at 575 -- its tile-quantisation cliff (GEMM 103 us at 512 rows, 135 at
#     575), where two 288-row tiles cover the step; within +-1 % or behind elsewhere;
#   down 513-576 rows: 5-11 % ahead of the library's split-4 GEMM in isolation at every
#     measured size from 320 to 576 rows, but its 8 fp32 slabs (vs the library's 4) cost
#     the consumer more than that below 513: 447-row steps (--prompt-len 384) ran 11,603
#     vs 11,694 tok/s with down on pf (r6p_pf_vs_library.md);
#   QKV / O: never -- pf's isolated lead is smaller than the fp32 partial slabs it adds
#     to their consumers (r5: -0.5 % end to end with every projection on pf).
# XGS_TUNE pf: "1" = these windows, "0" = library everywhere, or a comma list of
# projections to allow; pf_windows overrides the table ("gate_up:513-576/down:321-576").
PF_WINDOWS_DEFAULT = "gate_up:448-576/down:513-576"


def _parse_pf_windows(spec: str):
    out = {"qkv": (), "o": (), "gate_up": (), "down": ()}
    for item in filter(None, (t.strip() for t in spec.split("/"))):
        name, rng = item.split(":")
        assert name in out, f"XGS_TUNE pf_windows: {name!r}"
        out[name] = tuple(tuple(int(v) for v in r.split("-")) for r in rng.split("+"))
    return out


_pf_spec = tune.get_str("pf", "1")
PF_SET = frozenset() if _pf_spec in ("0", "") else frozenset(
    ("qkv,o,gate_up,down" if _pf_spec == "1" else _pf_spec).replace("+", ",").split(","))
assert PF_SET <= {"qkv", "o", "gate_up", "down"}, f"XGS_TUNE pf: {sorted(PF_SET)}"
PF_WINDOWS = {k: (v if k in PF_SET else ())
              for k, v in _parse_pf_windows(tune.get_str("pf_windows", PF_WINDOWS_DEFAULT)).items()}
PF_MAX_M = max([hi for ws in PF_WINDOWS.values() for _, hi in ws] or [0])


def pf_projections(T: int) -> frozenset:
    """The projections that run on gemm_pf at a T-token step."""
    return frozenset(k for k, ws in PF_WINDOWS.items() if any(lo <= T <= hi for lo, hi in ws))


# TP > 1 prefill-sized steps: the row-parallel all-reduces are pipelined over this
# many token chunks and overlapped with the next chunk's GEMMs (RCCL stream); a
# 2k-token 8B step moves 16 MiB per all-reduce -- ~100 us on 7 xGMI links, a
# GEMM-sized share of the layer. XGS_TUNE tp_overlap_chunks=1 disables it.
TP_OVERLAP_CHUNKS = tune.get_int("tp_overlap_chunks", 2)
TP_OVERLAP_MIN_TOKENS = tune.get_int("tp_overlap_min_tokens", 256)
# EP all_to_all: steps with at least this many (token, choice) pairs (and not under
# graph capture) exchange exact per-destination counts first and send only real rows
EP_EXACT_MIN_PAIRS = tune.get_int("ep_exact_min_pairs", 256)
# moe_comm "auto": steps of at most this many tokens use the allreduce form when the
# custom IPC all-reduce can take the [T, H] message
EP_AR_MAX_TOKENS = 64


@torch.no_grad()
def _fold_norm(w: torch.Tensor, norm: torch.Tensor) -> None:
    """W[:, k] *= norm[k] (one bf16 rounding), norm <- 1: rmsnorm(x, g) @ W^T ==
    rmsnorm(x, 1) @ (W diag(g))^T exactly in real arithmetic."""
    if bool((norm == 1).all()):
        return
    w.copy_((w.float() * norm.float()[None, :]).to(w.dtype))
    norm.fill_(1.0)


def _p(t: torch.Tensor) -> nn.Parameter:
    return nn.Parameter(t, requires_grad=False)


class LlamaLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, tp: int, rank: int, device, dtype):
        super().__init__()
        self.cfg = cfg
        self.tp, self.rank = tp, rank
        Hq, Hkv = local_heads(cfg, tp)
        D, H = cfg.head_dim, cfg.hidden_size
        self.Hq, self.Hkv = Hq, Hkv
        z = lambda *s: torch.empty(*s, device=device, dtype=dtype)  # noqa: E731
        self.input_norm = _p(torch.ones(H, device=device, dtype=dtype))
        self.post_norm = _p(torch.ones(H, device=device, dtype=dtype))
        self.qkv = _p(z((Hq + 2 * Hkv) * D, H))
        self.o = _p(z(H, Hq * D))
        self.moe = cfg.arch == "mixtral"
        if self.moe:
            E = cfg.num_experts
            if E % tp:
                raise ValueError(f"{E} experts not divisible by ep={tp}")
            self.E_local = E // tp
            self.expert_offset = rank * self.E_local
            self.router = _p(z(E, H))
            self.w13 = _p(z(self.E_local, 2 * cfg.intermediate_size, H))
            self.w2 = _p(z(self.E_local, H, cfg.intermediate_size))
        else:
            Fl = cfg.intermediate_size // tp
            self.gate_up = _p(z(2 * Fl, H))
            self.down = _p(z(H, Fl))
        self.attn = PagedAttention(Hq, Hkv, D)
        # the decode attention kernel's fused-QKV form (D = 128, GQA groups of 1/2/4/8)
        self.attn_fq_ok = (torch.device(device).type == "cuda" and D == 128 and Hq % Hkv == 0
                           and Hq // Hkv in (1, 2, 4, 8))
        self.moe_comm = "auto"
        # decode fast path: skinny split-K GEMMs whose partial sums are reduced by
        # the consuming kernel (rope_cache / add+rmsnorm); SiLU fused in gate_up.
        Nqkv = (Hq + 2 * Hkv) * D
        self.split_qkv = pick_split(Nqkv, H)
        self.split_o = pick_split(H, Hq * D)
        dims_ok = (H % 256 == 0 and (Hq * D) % 256 == 0 and Nqkv % 64 == 0 and H % 64 == 0
                   and self.split_qkv and self.split_o)
        if not self.moe:
            Fl = cfg.intermediate_size // tp
            self.split_down = pick_split(H, Fl)
            dims_ok = dims_ok and Fl % 256 == 0 and (2 * Fl) % 64 == 0 and self.split_down
        self.fast_ok = bool(dims_ok) and torch.device(device).type == "cuda"
        # 16 < M <= 64: gemm_m64g for QKV / O / down (split-K partials into the consumers)
        # and the fused SiLU-gate gate_up (measured: bench/gemm_bench.py)
        self.m64_ok = self.fast_ok and all(
            m64_plan(64, n, k, MODE_PARTIAL) is not None
            for n, k in ((Nqkv, H), (H, Hq * D)) + (() if self.moe else ((H, cfg.intermediate_size // tp),)))
        self.m64_silu_ok = self.m64_ok and not self.moe and m64_plan(64, 2 * (cfg.intermediate_size // tp), H,
                                                                     MODE_SILU) is not None
        # 64 < M <= MW_MAX_TOKENS: gemm_mw for every projection (MoE layers: the attention
        # projections; the experts stay on the grouped gemm_m64g)
        mw_shapes = ((Nqkv, H, MODE_PARTIAL), (H, Hq * D, MODE_PARTIAL))
        if not self.moe:
            mw_shapes += ((2 * (cfg.intermediate_size // tp), H, MODE_SILU),
                          (H, cfg.intermediate_size // tp, MODE_PARTIAL))
        self.mw_ok = self.fast_ok and MW_MAX_TOKENS > FAST_M_SLAB and all(
            mw_plan(MW_MAX_TOKENS, n, k, mode) is not None and mw_plan(FAST_M_SLAB + 1, n, k, mode) is not None
            for n, k, mode in mw_shapes)
        # T > MW_MAX_TOKENS on TP = 1: gemm_pf for every projection (MoE layers: attention)
        self.pf_ok = self.fast_ok and PF_MAX_M > 0 and tp == 1 and all(
            pf_plan(PF_MAX_M, n, k, mode) is not None for n, k, mode in mw_shapes)
        # M <= 16 too, when every projection has a measured small-M plan
        self.w8 = None  # fp8 / int8 / int4 weight copies for decode (LlamaForCausalLM.quantize_weights)
        self.m64_small_ok = self.m64_ok and all(
            m64_plan(1, n, k, MODE_PARTIAL) is not None
            for n, k in ((Nqkv, H), (H, Hq * D)) + (() if self.moe else ((H, cfg.intermediate_size // tp),))) and (
            self.moe or m64_plan(1, 2 * (cfg.intermediate_size // tp), H, MODE_SILU) is not None)

    def _w8_or_m64(self, x: torch.Tensor, name: str, mode: int):
        """One projection of the fp8 decode chain: the E4M3 copy when the layer has
        one, else the bf16 weight on gemm_m64g (same PendingSum / SiLU outputs)."""
        q = self.w8.get(name)
        if q is not None:
            return w8_linear(x, q[0], q[1], mode, fmt=q[2])
        return m64_linear(x, getattr(self, name), mode)

    def _ar(self, x: torch.Tensor) -> torch.Tensor:
        # keyed on the layer's own TP degree: a TP=1 draft model may live in a TP>1 process
        return x if self.tp == 1 else comm.tp_all_reduce(x)

    # ------------------------------------------------------------------ MoE
    def _moe_allreduce(self, h: torch.Tensor) -> torch.Tensor:
        w, ids = ops.moe_route(h, self.router, self.cfg.experts_per_token)
        out = ops.fused_moe(h, self.w13, self.w2, w, ids, self.expert_offset,
                              experts_total=self.router.shape[0])
        return self._ar(out)

    def _moe_alltoall(self, h: torch.Tensor) -> torch.Tensor:
        """Expert-parallel MoE with an all_to_all dispatch on the replicated [T, H]
        input: this rank's token slice goes through `_moe_alltoall_rows`, and an
        all_gather rebuilds the replicated output. (Prefill-sized steps take the
        sequence-parallel form instead, `forward_sp`, which never gathers it.)"""
        T = h.shape[0]
        per = (T + self.tp - 1) // self.tp
        lo, hi = min(T, self.rank * per), min(T, (self.rank + 1) * per)
        out_slice = self._moe_alltoall_rows(h[lo:hi], T, per)
        return comm.tp_all_gather_rows(out_slice)[:T].contiguous()

    def _moe_alltoall_rows(self, hs: torch.Tensor, T: int, per: int) -> torch.Tensor:
        """The all_to_all MoE on this rank's rows hs [Ts <= per, H] of a T-token step
        (rank r owns tokens [r * per, r * per + Ts)) -> [per, H], rows >= Ts zero.
        ep_plan/ep_scatter (HIP) pack each (token, choice) row for the rank that owns
        the expert, the owners run their experts as one grouped GEMM (send_eid = -1
        rows are skipped by the align), the rows travel back and ep_combine (HIP)
        applies the routing weights.
        Split policy: count-exact (packed layout, splits exchanged first: one host
        sync per layer) for eager steps of >= EP_EXACT_MIN_PAIRS pairs; fixed
        capacity (per * k rows per destination, no host sync) otherwise, which is
        what a captured decode graph needs."""
        tp = self.tp
        Ts, H = hs.shape
        k = self.cfg.experts_per_token
        cap = per * k
        if Ts > 0:
            w, ids = ops.moe_route(hs, self.router, k)
        else:
            w = torch.empty(0, k, dtype=torch.float32, device=hs.device)
            ids = torch.empty(0, k, dtype=torch.int32, device=hs.device)
        capturing = hs.is_cuda and torch.cuda.is_current_stream_capturing()
        packed = not capturing and T * k >= EP_EXACT_MIN_PAIRS
        slot, send_eid, counts = ops.ep_plan(ids, self.E_local, tp, cap, packed)
        rows = Ts * k if packed else tp * cap
        send = ops.ep_scatter(hs, k, slot, rows)
        if packed:
            recv_counts = comm.tp_exchange_counts(counts)
            send_splits, recv_splits = counts.tolist(), recv_counts.tolist()
        else:
            send_splits = recv_splits = [cap] * tp
        recv = comm.tp_all_to_all(send, send_splits, recv_splits)
        recv_eid = comm.tp_all_to_all(send_eid.view(-1, 1), send_splits, recv_splits).view(-1, 1)
        ones = torch.ones(recv.shape[0], 1, dtype=torch.float32, device=hs.device)
        y = ops.fused_moe(recv, self.w13, self.w2, ones, recv_eid, 0)    # unused slots (eid -1) -> 0 rows
        back = comm.tp_all_to_all(y, recv_splits, send_splits)            # rows in this rank's send order
        out_slice = torch.zeros(per, H, dtype=hs.dtype, device=hs.device)
        ops.ep_combine(back, slot, w, out_slice)
        return out_slice

    def forward_sp(self, x: torch.Tensor, residual: Optional[torch.Tensor], meta: AttnMeta,
                   kv: Tuple[torch.Tensor, torch.Tensor], cos_sin: torch.Tensor, T: int, per: int):
        """Sequence-parallel TP + EP layer (MoE layers on the all_to_all exchange): the
        residual stream stays token-sliced, [per, H] per rank (rank r holds tokens
        [r * per, r * per + per), zero-padded). The head-parallel attention reads
        the all-gathered normed input; its row-parallel output is reduce-scattered
        (half the bytes of the all-reduce) straight into this rank's rows, whose
        post-attention norm feeds the expert dispatch, and the combined expert output
        stays sliced. Per layer: all_gather(h) + reduce_scatter(o) + 2 all_to_all,
        against all_reduce(o) + 2 all_to_all + all_gather(out) in the replicated form
        (VERDICT r2 #8)."""
        eps = self.cfg.norm_eps
        Ts = max(0, min(T, (self.rank + 1) * per) - self.rank * per)
        if residual is None:
            residual = x
            hs = ops.rmsnorm(x, self.input_norm, eps)
        else:
            hs, residual = ops.fused_add_rmsnorm(x, residual, self.input_norm, eps)
        h = comm.tp_all_gather_rows(hs)[:T]
        a = self.attn(F.linear(h, self.qkv), meta, kv, cos_sin)
        o = F.linear(a, self.o)
        if o.shape[0] < self.tp * per:
            o = torch.cat([o, o.new_zeros(self.tp * per - o.shape[0], o.shape[1])])
        hs, residual = ops.fused_add_rmsnorm(comm.tp_reduce_scatter_rows(o), residual, self.post_norm, eps)
        return self._moe_alltoall_rows(hs[:Ts], T, per), residual

    def _moe_use_alltoall(self, h: torch.Tensor) -> bool:
        """Exchange choice for a TP > 1 MoE layer. "auto" (default): the activations
        are replicated after the head-parallel attention, so the allreduce form needs
        no dispatch at all -- each rank runs its experts on the tokens routed to them
        and one all-reduce sums the partial outputs. For decode-sized steps that
        all-reduce is ONE launch of the custom IPC kernel (~latency of one xGMI hop),
        where the all_to_all form costs three RCCL all_to_alls + an all_gather of tiny
        messages per layer; prefill-sized steps take the all_to_all, which moves only
        the routed rows (count-exact) instead of the whole [T, H] partial."""
        if self.moe_comm == "alltoall":
            return True
        if self.moe_comm == "allreduce":
            return False
        if get_state().tp_size == 1:  # a simulated TP shard (bench --tp-shard): collectives are local
            return False
        ar = comm.custom_allreduce()
        # the partial output is a fresh contiguous [T, H] bf16 tensor like h
        return not (h.shape[0] <= EP_AR_MAX_TOKENS and ar is not None and ar.can_run(h.contiguous()))

    def mlp(self, h: torch.Tensor) -> torch.Tensor:
        if self.moe:
            if self.tp > 1 and self._moe_use_alltoall(h):
                return self._moe_alltoall(h)
            return self._moe_allreduce(h)
        gu = F.linear(h, self.gate_up)
        a = ops.silu_and_mul(gu, interleave16=True)
        if self.tp == 1 and splitk_prefill_ok(a, self.down):
            return splitk_linear(a, self.down, linear_mod.SPLITK_PREFILL_S)  # reduced by the next add + norm
        return self._ar(F.linear(a, self.down))

    def _row_parallel_fast(self, a: torch.Tensor, w: torch.Tensor, split: int):
        pend = skinny_linear(a, w, None, MODE_PARTIAL)
        if self.tp == 1:
            return pend  # reduced by the consumer's prologue
        return self._ar(pend.materialize())

    def forward(self, x, residual: Optional[torch.Tensor], meta: AttnMeta,
                kv: Tuple[torch.Tensor, torch.Tensor], cos_sin: torch.Tensor):
        eps = self.cfg.norm_eps
        if residual is None:
            residual = x
            h = ops.rmsnorm(x, self.input_norm, eps)
        else:
            h, residual = ops.fused_add_rmsnorm(x, residual, self.input_norm, eps)
        T = meta.num_tokens
        if self.w8 is not None and T <= W8_MAX_M:
            # FP8 weights (gemm_w8): half the weight bytes of the bf16 decode chain; the
            # split-K partials go to the same consumers (rope_cache / add+rmsnorm)
            pqkv = self._w8_or_m64(h, "qkv", MODE_PARTIAL)
            a = self.attn.from_partials(pqkv, meta, kv, cos_sin)
            o = self._w8_or_m64(a, "o", MODE_PARTIAL)
            if self.tp > 1:
                o = self._ar(o.materialize())
            h, residual = ops.fused_add_rmsnorm(o, residual, self.post_norm, eps)
            act = self._w8_or_m64(h, "gate_up", MODE_SILU)
            d = self._w8_or_m64(act, "down", MODE_PARTIAL)
            return (d if self.tp == 1 else self._ar(d.materialize())), residual
        if self.fast_ok and T <= FAST_M_SMALL and not self.m64_small_ok:
            # M <= 16: every projection on the streaming skinny kernel (1.7x hipBLASLt
            # on QKV/O at batch 1), split-K partials reduced by the consumers
            pqkv = skinny_linear(h, self.qkv, None, MODE_PARTIAL)
            a = self.attn.from_partials(pqkv, meta, kv, cos_sin)
            o = self._row_parallel_fast(a, self.o, self.split_o)
            h, residual = ops.fused_add_rmsnorm(o, residual, self.post_norm, eps)
            if self.moe:
                return self.mlp(h), residual
            act = skinny_linear(h, self.gate_up, mode=MODE_SILU)
            return self._row_parallel_fast(act, self.down, self.split_down), residual
        if self.m64_ok and T <= FAST_M_SLAB:
            # gemm_m64g (LDS-DMA weight streaming) for every projection: split-K partials
            # go to the consumers (rope_cache / add+rmsnorm), SiLU-gate fused in gate_up;
            # pure-decode steps reduce the QKV partials + RoPE + KV append in the
            # attention prologue (one launch instead of two; MoE layers, TP fallback)
            pqkv = m64_linear(h, self.qkv, MODE_PARTIAL)
            if T == meta.num_decodes and self.attn_fq_ok:
                a = self.attn.fused_decode(pqkv, meta, kv, cos_sin)
            else:
                a = self.attn.from_partials(pqkv, meta, kv, cos_sin)
            o = m64_linear(a, self.o, MODE_PARTIAL)
            if self.tp > 1:
                o = self._ar(o.materialize())
            h, residual = ops.fused_add_rmsnorm(o, residual, self.post_norm, eps)
            if self.moe:
                return self.mlp(h), residual
            if self.m64_silu_ok:
                act = m64_linear(h, self.gate_up, MODE_SILU)
            else:
                act = ops.silu_and_mul(F.linear(h, self.gate_up), interleave16=True)
            d = m64_linear(act, self.down, MODE_PARTIAL)
            return (d if self.tp == 1 else self._ar(d.materialize())), residual
        if self.mw_ok and T <= MW_MAX_TOKENS:
            # 64 < M <= 320 (decode rows + a prefill chunk): gemm_mw streams each weight
            # once with the MFMA work under the stream; split-K partials go to the
            # consumers (rope_cache_partials / add + rmsnorm), SiLU-gate in gate_up
            pqkv = mw_linear(h, self.qkv, MODE_PARTIAL)
            a = self.attn.from_partials(pqkv, meta, kv, cos_sin)
            o = mw_linear(a, self.o, MODE_PARTIAL)
            if self.tp > 1:
                o = self._ar(o.materialize())
            h, residual = ops.fused_add_rmsnorm(o, residual, self.post_norm, eps)
            if self.moe:
                return self.mlp(h), residual
            act = mw_linear(h, self.gate_up, MODE_SILU)
            d = mw_linear(act, self.down, MODE_PARTIAL)
            return (d if self.tp == 1 else self._ar(d.materialize())), residual
        use_pf = pf_projections(T) if self.pf_ok else frozenset()
        if use_pf:
            # prompt-sized mixed steps: gemm_pf for the projections whose measured window
            # holds T (split-K partials into the consumers: rope_cache_partials / add +
            # rmsnorm; the SiLU gate in the gate_up epilogue), the library GEMMs for the others
            if "qkv" in use_pf:
                a = self.attn.from_partials(pf_linear(h, self.qkv, MODE_PARTIAL), meta, kv, cos_sin)
            else:
                a = self.attn(F.linear(h, self.qkv), meta, kv, cos_sin)
            o = pf_linear(a, self.o, MODE_PARTIAL) if "o" in use_pf else F.linear(a, self.o)
            h, residual = ops.fused_add_rmsnorm(o, residual, self.post_norm, eps)
            if self.moe:
                return self.mlp(h), residual
            if "gate_up" in use_pf:
                act = pf_linear(h, self.gate_up, MODE_SILU)
            else:
                act = ops.silu_and_mul(F.linear(h, self.gate_up), interleave16=True)
            if "down" in use_pf:
                return pf_linear(act, self.down, MODE_PARTIAL), residual
            if splitk_prefill_ok(act, self.down):
                return splitk_linear(act, self.down, linear_mod.SPLITK_PREFILL_S), residual
            return F.linear(act, self.down), residual
        if self.fast_ok and T <= FAST_M_SLAB:
            # 16 < M <= 64: measured per shape on MI355X -- only the O projection
            # (N = H) is faster on the LDS-slab kernel; its split-K partials are
            # reduced inside add+rmsnorm. QKV / gate_up / down stay on hipBLASLt.
            qkv = F.linear(h, self.qkv)
            a = self.attn(qkv, meta, kv, cos_sin)
            o = self._row_parallel_fast(a, self.o, self.split_o)
            h, residual = ops.fused_add_rmsnorm(o, residual, self.post_norm, eps)
            return self.mlp(h), residual
        a = self.attn(F.linear(h, self.qkv), meta, kv, cos_sin)
        if self.tp > 1 and not self.moe and T >= TP_OVERLAP_MIN_TOKENS and TP_OVERLAP_CHUNKS > 1:
            return self._forward_tp_overlap(a, residual)
        o = self._ar(F.linear(a, self.o))
        h, residual = ops.fused_add_rmsnorm(o, residual, self.post_norm, eps)
        return self.mlp(h), residual

    def _forward_tp_overlap(self, a: torch.Tensor, residual: torch.Tensor):
        """Row-parallel half of a TP layer for prefill-sized steps, pipelined over
        token chunks so every all-reduce runs (on RCCL's stream) under the GEMMs of
        the following chunk: O GEMM(c) -> AR(c) async; then per chunk: wait AR(c)
        -> add + post-norm -> gate_up -> SiLU-gate -> down(c) -> AR(c) async. Only
        the last chunk's down all-reduce is exposed. Everything after attention is
        per-token, so the chunked result equals the unchunked one exactly."""
        T, H = residual.shape
        eps = self.cfg.norm_eps
        n = TP_OVERLAP_CHUNKS
        step = (T + n - 1) // n
        if step > 64:
            step = (step + 63) // 64 * 64  # GEMM-friendly row blocks
        bounds = [(lo, min(T, lo + step)) for lo in range(0, T, step)]
        o = torch.empty(T, H, dtype=a.dtype, device=a.device)
        works = []
        for lo, hi in bounds:
            torch.mm(a[lo:hi], self.o.t(), out=o[lo:hi])
            works.append(comm.tp_all_reduce_async(o[lo:hi]))
        d = torch.empty(T, H, dtype=a.dtype, device=a.device)
        dworks = []
        for (lo, hi), w in zip(bounds, works):
            w.wait()
            hc, _ = ops.fused_add_rmsnorm(o[lo:hi], residual[lo:hi], self.post_norm, eps)
            act = ops.silu_and_mul(F.linear(hc, self.gate_up), interleave16=True)
            torch.mm(act, self.down.t(), out=d[lo:hi])
            dworks.append(comm.tp_all_reduce_async(d[lo:hi]))
        for w in dworks:
            w.wait()
        return d, residual

    def forward_fused(self, resid: torch.Tensor, stats: RowStats, meta: AttnMeta,
                      kv: Tuple[torch.Tensor, torch.Tensor], cos_sin: torch.Tensor, ws: ResidWorkspace,
                      site: int) -> RowStats:
        """Fused decode layer: QKV GEMM (input norm as a row scale) -> attention (QKV
        reduce + RoPE + KV append in its prologue) -> O GEMM (+ residual, + post-norm
        statistics) -> gate_up GEMM (post-norm row scale, SiLU-gate) -> down GEMM
        (+ residual, + next statistics). `resid` (bf16 [T, H]) is updated in place;
        returns the statistics of the new residual for the next layer."""
        eps = self.cfg.norm_eps
        pqkv = m64_norm_linear(resid, self.qkv, MODE_PARTIAL, stats, eps)
        a = self.attn.fused_decode(pqkv, meta, kv, cos_sin)
        if self.moe:
            return self._fused_moe_tail(a, resid, ws, site)
        if self.tp > 1:
            return self._fused_tp_tail(a, resid, ws, site)
        st = m64_resid_linear(a, self.o, resid, ws, site, eps)
        act = m64_norm_linear(resid, self.gate_up, MODE_SILU, st, eps)
        return m64_resid_linear(act, self.down, resid, ws, site + 1, eps)

    def _fused_moe_tail(self, a, resid: torch.Tensor, ws: ResidWorkspace, site: int) -> RowStats:
        """MoE half of the fused decode layer: O GEMM (+ residual; under TP the custom
        all-reduce with the residual) -> router with the post-attention RMSNorm in its
        prologue (writes the normalised rows for the experts) -> align -> grouped w13
        (SiLU-gate) -> grouped w2 -> combine + residual + next-norm statistics (under
        TP: this rank's experts' partial through the residual all-reduce -- the
        activations are replicated, so no dispatch). 7 launches instead of 9."""
        T, H = resid.shape
        eps = self.cfg.norm_eps
        if self.tp > 1:
            po = m64_linear(a, self.o, MODE_PARTIAL)
            comm.tp_allreduce_resid(po.part, resid, ws.ss[site], self.tp)
        else:
            m64_resid_linear(a, self.o, resid, ws, site, eps)  # its statistics go unused: the router renorms
        # one token (batch 1): the router launch also writes the expert layout
        hn, w, ids, layout = ops.moe_route_norm(resid, self.post_norm, eps, self.router, self.cfg.experts_per_token,
                                                align=(self.E_local, self.expert_offset))
        ss = ws.ss[site + 1]
        if self.tp > 1:
            part = ops.fused_moe(hn, self.w13, self.w2, w, ids, self.expert_offset, out_f32=True, layout=layout,
                                 experts_total=self.router.shape[0])
            comm.tp_allreduce_resid(part.unsqueeze(0), resid, ss, self.tp)
        else:
            return RowStats(ss, ops.fused_moe(hn, self.w13, self.w2, w, ids, self.expert_offset, resid=resid, ss=ss,
                                              layout=layout, counters=ws.counters[site + 1]), T)
        return RowStats(ss, H // 1024, T)

    def _fused_tp_tail(self, a: torch.Tensor, resid: torch.Tensor, ws: ResidWorkspace, site: int) -> RowStats:
        """Row-parallel half of the fused decode layer under TP: O GEMM partials ->
        all-reduce + residual + statistics (one launch) -> gate_up (norm row scale,
        SiLU-gate) -> down GEMM partials -> all-reduce + residual + statistics."""
        T, H = resid.shape
        eps = self.cfg.norm_eps
        ar = comm.gemm_ar_args(self.tp, T, H, resid.device)
        if ar is not None:
            # the all-reduce inside the O / down launches (gemm_m64g GG_AR): 2 launches fewer
            st = m64_ar_resid_linear(a, self.o, resid, ws, site, ar)
            act = m64_norm_linear(resid, self.gate_up, MODE_SILU, st, eps)
            return m64_ar_resid_linear(act, self.down, resid, ws, site + 1, ar)
        po = m64_linear(a, self.o, MODE_PARTIAL)
        comm.tp_allreduce_resid(po.part, resid, ws.ss[site], self.tp)
        st = RowStats(ws.ss[site], H // 1024, T)
        act = m64_norm_linear(resid, self.gate_up, MODE_SILU, st, eps)
        pd = m64_linear(act, self.down, MODE_PARTIAL)
        comm.tp_allreduce_resid(pd.part, resid, ws.ss[site + 1], self.tp)
        return RowStats(ws.ss[site + 1], H // 1024, T)


class LlamaForCausalLM(nn.Module):
    def __init__(self, cfg: ModelConfig, device="cpu", dtype=torch.bfloat16, tp: Optional[int] = None,
                 rank: Optional[int] = None):
        super().__init__()
        st = get_state()
        self.cfg = cfg
        self.tp = st.tp_size if tp is None else tp
        self.rank = st.tp_rank if rank is None else rank
        self.device = torch.device(device)
        self.dtype = dtype
        H, V = cfg.hidden_size, cfg.vocab_size
        self.V_pad = (V + self.tp - 1) // self.tp * self.tp
        self.embed = _p(torch.empty(V, H, device=device, dtype=dtype))
        self.layers = nn.ModuleList([LlamaLayer(cfg, self.tp, self.rank, device, dtype)
                                     for _ in range(cfg.num_layers)])
        self.norm = _p(torch.ones(H, device=device, dtype=dtype))
        self.lm_head = None if (cfg.tie_embeddings and self.tp == 1) else \
            _p(torch.empty(self.V_pad // self.tp, H, device=device, dtype=dtype))
        self.cos_sin = ops.build_cos_sin(cfg.head_dim, cfg.max_position, cfg.rope_theta, cfg.rope_scaling,
                                         device=device)
        self.num_kv_heads_local = self.layers[0].Hkv
        l0 = self.layers[0]
        self.norms_folded = False
        self.weight_dtype = "bf16"
        self._fused_ok = (self.device.type == "cuda" and l0.m64_ok and (l0.moe or l0.m64_silu_ok)
                          and cfg.head_dim == 128 and l0.Hq % l0.Hkv == 0
                          and l0.Hq // l0.Hkv in (1, 2, 4, 8) and H % 1024 == 0 and H // 1024 <= 8)
        self._fused_small_ok = self._fused_ok and l0.m64_small_ok
        # every layer on gemm_mw for 64 < T <= MW_MAX_TOKENS (the runner's mixed-step graphs)
        self._mw_ok = self.device.type == "cuda" and all(l.mw_ok for l in self.layers)
        self._fused_ws = ResidWorkspace(2 * cfg.num_layers + 1, FAST_M_SLAB, H, device) if self._fused_ok else None

    @torch.no_grad()
    def fold_norms(self):
        """Fold every RMSNorm weight into the input columns of the projection that
        consumes it and reset the norm to 1, so the decode GEMMs can apply the norm
        as a per-row epilogue scale of the raw residual stream. Exact in real
        arithmetic: every other path (prefill, TP, the fp32 reference) computes the
        same function. MoE post-attention norms stay (router and experts read them)."""
        for l in self.layers:
            _fold_norm(l.qkv, l.input_norm)
            if not l.moe:
                _fold_norm(l.gate_up, l.post_norm)
        self.norms_folded = True

    @torch.no_grad()
    def quantize_fp8(self) -> bool:
        return self.quantize_weights("fp8")

    @torch.no_grad()
    def quantize_weights(self, kind: str = "fp8") -> bool:
        """Weight-only quantization for decode batches <= 64 (Req 10.3): per dense
        layer, copies of the QKV / O / gate_up / down weights (after the RMSNorm
        folding) as fp8 (E4M3, per-channel scale), int8 (per-channel scale) or int4
        (per 128-k group scales), run by gemm_w8. Prefill and larger batches keep
        the bf16 weights (MFMA-bound there); the fused bf16 decode layer is
        disabled. Returns False (and changes nothing) when a shape has no gemm_w8
        plan or the model is MoE."""
        fmt = WQ_FORMATS[kind]
        if self.device.type != "cuda" or any(l.moe for l in self.layers):
            return False
        l0 = self.layers[0]
        names = ("qkv", "o", "gate_up", "down")
        for n in names:
            w = getattr(l0, n)
            mode = MODE_SILU if n == "gate_up" else MODE_PARTIAL
            if any(w8_plan(m, w.shape[0], w.shape[1], mode, fmt) is None for m in (1, W8_MAX_M)):
                return False
        def use_q(n):  # small projections stay bf16 where gemm_m64g has a plan
            w = getattr(l0, n)
            mode = MODE_SILU if n == "gate_up" else MODE_PARTIAL
            return w.numel() >= W8_MIN_ELEMS or not (l0.m64_small_ok and
                                                     m64_plan(1, w.shape[0], w.shape[1], mode) is not None)
        chosen = [n for n in names if use_q(n)]
        for l in self.layers:
            l.w8 = {n: quantize_weight(getattr(l, n), fmt) + (fmt,) for n in chosen}
        self._fused_ok = self._fused_small_ok = False
        self.weight_dtype = kind
        return True

    def fused_decode_ok(self, meta: AttnMeta) -> bool:
        T = meta.num_tokens
        if not (FUSED_DECODE and self._fused_ok and self.norms_folded) or T != meta.num_decodes or not 0 < T <= 64:
            return False
        l0 = self.layers[0]
        if l0.moe and self.tp > 1 and l0.moe_comm == "alltoall":  # the fused MoE tail is the allreduce form
            return False
        if self.tp > 1 and not comm.resid_allreduce_ok(T, self.cfg.hidden_size):
            return False
        return T > FAST_M_SMALL or self._fused_small_ok

    def _forward_fused(self, input_ids: torch.Tensor, meta: AttnMeta,
                       kv_caches: List[Tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
        ws = self._fused_ws
        resid = ops.embed_gather(input_ids, self.embed, ws.ss[0])  # gather + first norm statistic, one launch
        st = RowStats(ws.ss[0], 1, meta.num_tokens)
        for i, layer in enumerate(self.layers):
            st = layer.forward_fused(resid, st, meta, kv_caches[i], self.cos_sin, ws, 2 * i + 1)
        return ops.rmsnorm(resid, self.norm, self.cfg.norm_eps)

    def set_moe_comm(self, mode: str):
        for l in self.layers:
            l.moe_comm = mode

    # ------------------------------------------------------------------ init
    @torch.no_grad()
    def random_init(self, seed: int = 0, std: float = 0.02):
        g = torch.Generator(device=self.device).manual_seed(seed + 1000 * self.rank) \
            if self.device.type == "cuda" else torch.Generator().manual_seed(seed + 1000 * self.rank)
        for name, p in self.named_parameters():
            if "norm" in name:
                p.fill_(1.0)
            else:
                p.normal_(0.0, std, generator=g)
        # replicated parameters must agree across TP ranks
        ge = torch.Generator(device=self.device).manual_seed(seed) if self.device.type == "cuda" \
            else torch.Generator().manual_seed(seed)
        self.embed.normal_(0.0, std, generator=ge)
        for l in self.layers:
            if l.moe:
                l.router.normal_(0.0, std, generator=ge)

    # ------------------------------------------------------------------ forward
    def forward(self, input_ids: torch.Tensor, meta: AttnMeta,
                kv_caches: List[Tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
        if self.fused_decode_ok(meta):
            return self._forward_fused(input_ids, meta, kv_caches)
        x = ops.embed_gather(input_ids, self.embed) if input_ids.dtype == torch.int32 else \
            F.embedding(input_ids, self.embed)
        residual = None
        l0 = self.layers[0]
        if self.tp > 1 and l0.moe and l0._moe_use_alltoall(x):
            return self._forward_sp(x, meta, kv_caches)
        for i, layer in enumerate(self.layers):
            x, residual = layer(x, residual, meta, kv_caches[i], self.cos_sin)
        if residual is None:
            return ops.rmsnorm(x, self.norm, self.cfg.norm_eps)
        h, _ = ops.fused_add_rmsnorm(x, residual, self.norm, self.cfg.norm_eps)
        return h

    def _forward_sp(self, x: torch.Tensor, meta: AttnMeta, kv_caches) -> torch.Tensor:
        """Every layer in the sequence-parallel form (LlamaLayer.forward_sp): the
        residual stream stays token-sliced from the embedding to the final norm,
        whose rows are gathered once for the LM head."""
        T, H = x.shape
        per = (T + self.tp - 1) // self.tp
        lo = min(T, self.rank * per)
        xs = x.new_zeros(per, H)
        xs[:min(T, lo + per) - lo] = x[lo:lo + per]
        residual = None
        for i, layer in enumerate(self.layers):
            xs, residual = layer.forward_sp(xs, residual, meta, kv_caches[i], self.cos_sin, T, per)
        hs, _ = ops.fused_add_rmsnorm(xs, residual, self.norm, self.cfg.norm_eps)
        return comm.tp_all_gather_rows(hs)[:T]

    def compute_logits(self, h: torch.Tensor) -> torch.Tensor:
        w = self.embed if self.lm_head is None else self.lm_head
        logits = lm_head_linear(h, w)
        if self.tp > 1:
            logits = comm.tp_all_gather_lastdim(logits)
        return logits[:, :self.cfg.vocab_size]

    def hidden_size(self) -> int:
        return self.cfg.hidden_size
