"""K9 sampling + K11 pooling helpers."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._native import kernels, stream_ptr, use_native, ptr


def argmax_logprob_ref(logits: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    lf = logits.float()
    tok = lf.argmax(-1)
    lp = torch.log_softmax(lf, -1).gather(-1, tok[:, None])[:, 0]
    return tok.to(torch.int32), lp


_ARGMAX_WS = {}
_ARGMAX_WS_RETIRED = []
# below this a row is one workgroup's work anyway; XGS_TUNE argmax_split=0: always the
# one-workgroup-per-row kernel (A/B)
ARGMAX_SPLIT_MIN_V = 16384 if __import__("xgserve.tune", fromlist=["get_bool"]).get_bool("argmax_split", True) else 1 << 62


def _argmax_ws(device, B: int):
    """Split-row argmax scratch: per-slice partials and zeroed per-row tickets (every
    launch's last arriver re-arms its row), grown on demand, kept alive for captured graphs."""
    key = str(device)
    ws = _ARGMAX_WS.get(key)
    if ws is None or ws[1].numel() < B:
        if ws is not None:
            _ARGMAX_WS_RETIRED.append(ws)
        n = max(B, 64)
        ws = _ARGMAX_WS[key] = (torch.empty(n * kernels().argmax_ws_floats_per_row(), dtype=torch.float32,
                                            device=device),
                                torch.zeros(n, dtype=torch.int32, device=device))
    return ws


def argmax_logprob(logits: torch.Tensor, out_tok: Optional[torch.Tensor] = None,
                   out_lp: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Greedy token + its log-probability per row of a [B, V] logits matrix. Large
    vocabularies take the split-row kernel (8 workgroups per row, last arriver merges)."""
    if not use_native(logits):
        t, lp = argmax_logprob_ref(logits)
        return t, lp
    B, V = logits.shape
    assert logits.stride(1) == 1
    if out_tok is None:
        out_tok = torch.empty(B, dtype=torch.int32, device=logits.device)
    if out_lp is None:
        out_lp = torch.empty(B, dtype=torch.float32, device=logits.device)
    ws = cnt = 0
    if V >= ARGMAX_SPLIT_MIN_V:
        w, c = _argmax_ws(logits.device, B)
        ws, cnt = w.data_ptr(), c.data_ptr()
    kernels().argmax_logprob(logits.data_ptr(), 1 if logits.dtype == torch.float32 else 0, logits.stride(0), B, V,
                             out_tok.data_ptr(), out_lp.data_ptr(), stream_ptr(), ws, cnt)
    return out_tok, out_lp


def _sample_ref(logits, temps, top_ps, top_ks, gen: Optional[torch.Generator]):
    lf = logits.float()
    B, V = lf.shape
    toks = torch.empty(B, dtype=torch.int32, device=lf.device)
    lps = torch.empty(B, dtype=torch.float32, device=lf.device)
    for i in range(B):
        t = float(temps[i])
        if t <= 0:
            toks[i] = int(lf[i].argmax())
            lps[i] = torch.log_softmax(lf[i], -1)[toks[i]]
            continue
        x = lf[i] / t
        logp = torch.log_softmax(x, -1)
        keep = torch.ones(V, dtype=torch.bool, device=lf.device)
        k = int(top_ks[i]) if top_ks is not None else 0
        if 0 < k < V:
            kth = torch.topk(x, k).values[-1]
            keep &= x >= kth
        p = float(top_ps[i]) if top_ps is not None else 1.0
        if p < 1.0:
            sp, si = torch.sort(logp.exp(), descending=True)
            c = torch.cumsum(sp, 0)
            n = int((c < p).sum()) + 1
            m = torch.zeros(V, dtype=torch.bool, device=lf.device)
            m[si[:n]] = True
            keep &= m
        probs = torch.where(keep, logp.exp(), torch.zeros_like(logp))
        j = int(torch.multinomial(probs / probs.sum(), 1, generator=gen))
        toks[i] = j
        lps[i] = logp[j]
    return toks, lps


def sample_tokens(logits: torch.Tensor, temps: torch.Tensor, top_ps: Optional[torch.Tensor] = None,
                  top_ks: Optional[torch.Tensor] = None, seeds: Optional[torch.Tensor] = None, step: int = 0,
                  generator: Optional[torch.Generator] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-row temperature / top-k / top-p sampling (temps <= 0 -> greedy)."""
    if not use_native(logits):
        return _sample_ref(logits, temps, top_ps, top_ks, generator)
    B, V = logits.shape
    tok = torch.empty(B, dtype=torch.int32, device=logits.device)
    lp = torch.empty(B, dtype=torch.float32, device=logits.device)
    ws = _sample_workspace(logits.device, B) if SAMPLE_SPLIT else None
    kernels().sample_tokens(logits.data_ptr(), 1 if logits.dtype == torch.float32 else 0, logits.stride(0), B, V,
                            temps.data_ptr(), ptr(top_ps), ptr(top_ks), ptr(seeds), int(step) & ((1 << 64) - 1),
                            tok.data_ptr(), lp.data_ptr(), stream_ptr(), ptr(ws),
                            0 if ws is None else ws.shape[0])
    return tok, lp


# Split-row sampler (csrc/kernels/sampling.hip "sample v2": several workgroups per row,
# histogram thresholds instead of a 24-pass bisection); False selects the
# one-workgroup-per-row kernel (the tests' cross-check; A/B in profiles/r2_sampling.md).
SAMPLE_SPLIT = True
_SAMPLE_WS = {}


def _sample_workspace(device, B: int) -> torch.Tensor:
    """Per-device zeroed scratch of the split-row sampler, one row per batch row; the
    kernels leave it zero after every call (ticket winners re-zero what they used), so
    one allocation serves eager calls and captured graphs. Grown (never shrunk, never
    freed) to the largest batch seen."""
    key = (device.type, device.index)
    wss = _SAMPLE_WS.setdefault(key, [])
    if not wss or wss[-1].shape[0] < B:
        row = kernels().sample_ws_row_bytes()
        # earlier (smaller) workspaces stay alive: captured graphs may still use them
        wss.append(torch.zeros(max(B, 256), row // 8, dtype=torch.int64, device=device))
    return wss[-1]


def segment_sum(hidden: torch.Tensor, cu: torch.Tensor, out: torch.Tensor,
                out_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[rows[s]] += sum(hidden[cu[s]:cu[s+1]]) (fp32)."""
    S = cu.shape[0] - 1
    if not use_native(hidden):
        for s in range(S):
            r = int(out_rows[s]) if out_rows is not None else s
            if r < 0:
                continue
            out[r] += hidden[int(cu[s]):int(cu[s + 1])].float().sum(0)
        return out
    H = hidden.shape[-1]
    kernels().segment_sum(hidden.data_ptr(), H, cu.data_ptr(), ptr(out_rows), out.data_ptr(), S, stream_ptr())
    return out


def subst_tokens(ids: torch.Tensor, src: torch.Tensor, prev: torch.Tensor) -> torch.Tensor:
    """ids[i] <- prev[src[i]] where src[i] >= 0 (int32, in place): the decode rows of
    a step planned before the previous step's tokens reached the host."""
    n = ids.shape[0]
    assert ids.dtype == src.dtype == prev.dtype == torch.int32 and src.shape[0] >= n
    if not use_native(ids):
        s = src[:n].long()
        m = s >= 0
        ids[m] = prev[s[m]]
        return ids
    kernels().subst_tokens(ids.data_ptr(), src.data_ptr(), prev.data_ptr(), n, stream_ptr())
    return ids
