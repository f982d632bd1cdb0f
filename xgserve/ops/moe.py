"""K12: Mixture-of-Experts routing, layout, grouped GEMM, combine."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._native import kernels, stream_ptr, use_native
from .activation import silu_and_mul

BLOCK_M = 64
# gemm_m64g launch configurations for the expert GEMMs (see ops/linear.py M64G_CFGS);
# measured with bench/gemm_bench.py --moe-sweep
# (Mixtral 8x7B; profiles/r1_moe_sweep_v2.jsonl, per-row-tile grid + MT=1: w13 cfg 5 = 324 us at
# T=64 (cfg 3: 338), 81 us at T=1; w2 nw 2 + cfg 1 = 153 us at T=64)
MOE_CFG_W13 = 5  # (2 waves, KC 64, nt): best at T = 1..64 with the per-row-tile grid (bench --moe-sweep)
MOE_CFG_W2 = 1
# prefill-sized steps (> 256 token-expert pairs): w2 on a KC-64 config so the grouped
# kernel can run 128-row tile pairs (each expert's weights streamed once per 128 rows
# instead of per 64; profiles/r2_moe_pairs_ab.md). A per-expert hipBLASLt path for
# these steps measured slower than the grouped kernel (2,638 vs 2,680 tok/s) and was
# removed.
MOE_PREFILL_PAIRS = 256
MOE_CFG_W2_PREFILL = 3
# waves per workgroup of each gemm_m64g cfg (csrc/kernels/gemm_m64g.hip m64g_cfg_waves)
M64G_CFG_WAVES = {0: 4, 1: 4, 2: 4, 3: 4, 4: 2, 5: 2, 6: 2, 7: 8}
MOE_CFG_W13_PREFILL = 3
# prefill-sized steps on gemm_pf's grouped form instead (csrc/kernels/gemm_pf.hip
# gemm_pf_grouped): one MFMA tile of 192-288 rows covers an expert's rows, so each
# expert's weights stream once per step (profiles/r5_moe_pf.md). XGS_TUNE moe_pf=0: off.
MOE_PF = __import__("xgserve.tune", fromlist=["get_bool"]).get_bool("moe_pf", True)
# decode-sized w2 in its fused form (combine into the residual in the launch) on 64-column
# tiles with the 4-wave nt config: steps of <= 8 token-expert pairs (2 K splits) and of
# 64-256 pairs (1 split). bench/moe_fused_bench.py, profiles/r6/r6_moe_w2.md: T = 1 / 4 /
# 32 / 64 at 39.1 / 109.3 / 144.8 / 156.6 us vs 40.5 / 114+ / 153.0 / 166.6 for the
# 128-column tiles; end to end Mixtral batch 1 5.12 -> 5.07 ms, 64 concurrent 19.83 ->
# 19.53 ms (with w13 on cfg 3 from 64 pairs: 19.41 ms). 16 pairs (batch 8) measured
# 0.4 % slower, so 9-63 pairs keep the 128-column tiles. XGS_TUNE moe_w2_small=0:
# the 128-column tiles everywhere and w13 on cfg 5 (A/B).
MOE_W2_SMALL = __import__("xgserve.tune", fromlist=["get_bool"]).get_bool("moe_w2_small", True)
MOE_W2_SMALL_LOW = 8     # <= this many pairs
MOE_W2_SMALL_HIGH = 64   # >= this many pairs (and <= MOE_PREFILL_PAIRS)
# w13 of decode-sized steps from this many pairs up on cfg 3 (swept fastest at T = 64:
# 290.5 vs 297.0 us for cfg 5)
MOE_W13_BIG_PAIRS = 64
MOE_CFG_W13_BIG = 3


def _moe_pf_cfg(pairs: int, E: int) -> int:
    """gemm_pf lag-2 tile (cfg 8 / 7 / 6 = 192 / 256 / 288 rows) covering the average
    expert's 64-padded segment."""
    seg = -(-max(1, pairs // max(1, E)) // BLOCK_M) * BLOCK_M
    return 8 if seg <= 192 else 7 if seg <= 256 else 6


def _moe_pf_ok(H: int, F: int) -> bool:
    return H % 256 == 0 and (2 * F) % 256 == 0 and F % 64 == 0 and H >= 256


def moe_topk_softmax(router_logits: torch.Tensor, k: int, renorm: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    T, E = router_logits.shape
    if not use_native(router_logits):
        p = torch.softmax(router_logits.float(), -1)
        w, ids = torch.topk(p, k, dim=-1)
        if renorm:
            w = w / w.sum(-1, keepdim=True)
        return w, ids.to(torch.int32)
    assert E <= 64 and k <= 16
    w = torch.empty(T, k, dtype=torch.float32, device=router_logits.device)
    ids = torch.empty(T, k, dtype=torch.int32, device=router_logits.device)
    rl = router_logits.contiguous()
    kernels().moe_topk_softmax(rl.data_ptr(), 1 if rl.dtype == torch.float32 else 0, T, E, k, 1 if renorm else 0,
                               w.data_ptr(), ids.data_ptr(), stream_ptr())
    return w, ids


def moe_route(h: torch.Tensor, router: torch.Tensor, k: int, renorm: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """Router logits (fp32) + softmax + top-k in one kernel: h [T, H] bf16, router [E, H] bf16."""
    if not use_native(h):
        return moe_topk_softmax(h.float() @ router.float().t(), k, renorm)
    T, H = h.shape
    E = router.shape[0]
    w = torch.empty(T, k, dtype=torch.float32, device=h.device)
    ids = torch.empty(T, k, dtype=torch.int32, device=h.device)
    hc = h.contiguous()
    kernels().moe_route(hc.data_ptr(), router.data_ptr(), T, H, E, k, 1 if renorm else 0, w.data_ptr(),
                        ids.data_ptr(), stream_ptr())
    return w, ids


def moe_route_norm(resid: torch.Tensor, norm_w: torch.Tensor, eps: float, router: torch.Tensor, k: int,
                   renorm: bool = True, align: Optional[Tuple[int, int]] = None):
    """Fused decode layer: RMSNorm of the raw residual stream + router + top-k in one
    launch -> (hn = bf16 normalised rows for the experts, weights, expert ids).
    align = (E_local, expert_offset) and a single token: the same launch also writes
    moe_align's expert layout, returned as a fourth value (fused_moe(layout=...))."""
    T, H = resid.shape
    if not use_native(resid):
        rf = resid.float()
        hn = (rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + eps) * norm_w.float()).to(resid.dtype)
        w, ids = moe_route(hn, router, k, renorm)
        return (hn, w, ids) if align is None else (hn, w, ids, None)  # CPU: fused_moe runs the reference
    E = router.shape[0]
    hn = torch.empty_like(resid)
    w = torch.empty(T, k, dtype=torch.float32, device=resid.device)
    ids = torch.empty(T, k, dtype=torch.int32, device=resid.device)
    fuse = align is not None and T == 1 and E <= 8 and align[0] <= 8
    if fuse:
        El, eoff = align
        cap = (T * k + El * (BLOCK_M - 1) + BLOCK_M - 1) // BLOCK_M * BLOCK_M
        layout = (torch.empty(cap, dtype=torch.int32, device=resid.device),
                  torch.empty(El + 1, dtype=torch.int32, device=resid.device),
                  torch.empty(T * k, dtype=torch.int32, device=resid.device))
        al = dict(al_rows=layout[0].data_ptr(), al_offs=layout[1].data_ptr(), al_dest=layout[2].data_ptr(), al_E=El,
                  al_eoff=eoff, al_bm=BLOCK_M)
    else:
        al = {}
    kernels().moe_route(resid.data_ptr(), router.data_ptr(), T, H, E, k, 1 if renorm else 0, w.data_ptr(),
                        ids.data_ptr(), stream_ptr(), norm_w.data_ptr(), float(eps), hn.data_ptr(), **al)
    if align is None:
        return hn, w, ids
    return hn, w, ids, (layout if fuse else moe_align(ids, align[0], align[1]))


def moe_align(ids: torch.Tensor, num_experts: int, expert_offset: int = 0, block_m: int = BLOCK_M):
    """Expert-sorted, block_m-padded layout of this rank's experts
    [expert_offset, expert_offset + num_experts). -> (sorted_rows [cap] (-1 = pad),
    expert_offsets [E+1], dest [T*k] (padded row of each pair, -1 = another rank's expert))."""
    T, k = ids.shape
    cap = T * k + num_experts * (block_m - 1)
    cap = (cap + block_m - 1) // block_m * block_m
    dev = ids.device
    sorted_rows = torch.empty(cap, dtype=torch.int32, device=dev)
    offs = torch.empty(num_experts + 1, dtype=torch.int32, device=dev)
    dest = torch.empty(T * k, dtype=torch.int32, device=dev)
    kernels().moe_align(ids.contiguous().data_ptr(), T, k, num_experts, expert_offset, block_m, sorted_rows.data_ptr(),
                        offs.data_ptr(), dest.data_ptr(), stream_ptr())
    return sorted_rows, offs, dest


def moe_forward_ref(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
                    topk_ids: torch.Tensor, expert_offset: int = 0) -> torch.Tensor:
    """fp32 reference. w13: [E_local, 2F, H] block-16 interleaved gate|up rows
    (ops.linear.interleave_gate_up per expert), w2: [E_local, H, F]; experts outside
    [expert_offset, expert_offset+E_local) contribute nothing."""
    from .linear import deinterleave_gate_up
    T, H = x.shape
    E = w13.shape[0]
    out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
    xf = x.float()
    for e in range(E):
        ge = e + expert_offset
        mask = (topk_ids == ge)
        tok = mask.any(-1).nonzero()[:, 0]
        if tok.numel() == 0:
            continue
        wt = (topk_w * mask).sum(-1)[tok]
        g, u = deinterleave_gate_up(w13[e])
        a = torch.nn.functional.silu(xf[tok] @ g.float().t()) * (xf[tok] @ u.float().t())
        a = a.to(x.dtype).float()
        y = a @ w2[e].float().t()
        out[tok] += wt[:, None] * y
    return out.to(x.dtype)


def fused_moe(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
              topk_ids: torch.Tensor, expert_offset: int = 0, resid: Optional[torch.Tensor] = None,
              ss: Optional[torch.Tensor] = None, out_f32: bool = False, layout=None,
              counters: Optional[torch.Tensor] = None, experts_total: Optional[int] = None):
    """Local-expert MoE FFN: sum_j w_j * FFN_{e_j}(x) over choices owned locally
    (ids in [expert_offset, expert_offset + E_local)); others contribute nothing.

    align (one tiny kernel) -> grouped gemm_m64 on w13 with the SiLU-gate fused
    (x gathered through the sorted rows) -> grouped gemm_m64 on w2 (split-K
    partials when few experts are active) -> combine (weights, partial sums).
    resid / ss given (fused decode layer): the combine adds into the bf16 residual
    stream in place and writes the next RMSNorm's per-column-tile statistics
    ss[c * T + t]; returns the number of partial sums per row. With `counters`
    (>= H / 128 zeroed int32 words, re-armed by every launch) and a decode-sized
    step the combine runs inside the w2 launch (GG_MOE_RESID: the last workgroup to
    store into a column tile adds that tile's weighted rows into the residual), one
    launch fewer per layer; otherwise a separate combine kernel with 1024-column
    statistics. experts_total (EP shards): the global expert count, so the prompt-sized
    path sizes its tiles by this rank's expected share of the pairs."""
    if not use_native(x):
        out = moe_forward_ref(x, w13, w2, topk_w, topk_ids, expert_offset)
        if resid is None:
            return out.float() if out_f32 else out
        r = (resid.float() + out.float()).to(resid.dtype)
        resid.copy_(r)
        T, H = r.shape
        ss[: (H // 1024) * T].copy_(r.float().view(T, H // 1024, 1024).pow(2).sum(-1).t().reshape(-1))
        return H // 1024
    T, k = topk_ids.shape
    E, F2, H = w13.shape
    F = F2 // 2
    # layout: moe_align's (sorted_rows, offsets, dest), e.g. from moe_route_norm(align=...)
    sorted_rows, offs, dest = layout if layout is not None else moe_align(topk_ids, E, expert_offset)
    P = sorted_rows.shape[0]
    act = torch.empty(P, F, dtype=x.dtype, device=x.device)
    kn = kernels()
    max_rows = T * k  # no expert holds more rows than (token, choice) pairs
    valid = sorted_rows.data_ptr()  # per-workgroup real-row count -> 16 / 32 / 64-row body

    if MOE_PF and max_rows > MOE_PREFILL_PAIRS and _moe_pf_ok(H, F):
        share = max_rows * E // experts_total if experts_total else max_rows  # this rank's expected pairs
        cfg = _moe_pf_cfg(share, E)
        kn.gemm_pf_grouped(x.contiguous().data_ptr(), sorted_rows.data_ptr(), offs.data_ptr(), E, P, H, w13.data_ptr(),
                           F2, max_rows, 0, act.data_ptr(), 1, 2, cfg, stream_ptr())
        # w2 has H / 256 column tiles per expert: 2 K splits (reduced by the combine)
        S = 2 if F % 128 == 0 else 1
        part = torch.empty(S, P, H, dtype=torch.float32, device=x.device)
        kn.gemm_pf_grouped(act.data_ptr(), 0, offs.data_ptr(), E, P, F, w2.data_ptr(), H, max_rows, part.data_ptr(), 0,
                           S, 1, cfg, stream_ptr())
        return _moe_combine(kn, part, S, P, dest, topk_w, resid, ss, T, k, H, x, out_f32)

    # pairs = T * k bounds the real row tiles (they lead the padded layout): the grid
    # stops there instead of at the capacity P / 64
    def gemm(*a, cfg=0):
        kn.moe_gemm_m64g_rows(*a[:-1], cfg, max_rows, a[-1], valid, T * k)
    cfg13 = ((MOE_CFG_W13_PREFILL if T * k > MOE_PREFILL_PAIRS else
              MOE_CFG_W13_BIG if MOE_W2_SMALL and T * k >= MOE_W13_BIG_PAIRS else MOE_CFG_W13)
             if (H % 64 == 0 and F2 % 128 == 0) else 0)
    gemm(x.contiguous().data_ptr(), sorted_rows.data_ptr(), offs.data_ptr(), E, H, w13.data_ptr(), F2, P, 0,
         act.data_ptr(), 1, 2, 2, stream_ptr(), cfg=cfg13)
    # w2 has only H/128 column tiles per expert: split K while few experts are active
    nw2 = 2 if H % 128 == 0 else 1
    cfg2 = (MOE_CFG_W2_PREFILL if T * k > MOE_PREFILL_PAIRS else MOE_CFG_W2) if nw2 == 2 else 0
    kc2 = 128
    S = 1
    small = (MOE_W2_SMALL and (T * k <= MOE_W2_SMALL_LOW or MOE_W2_SMALL_HIGH <= T * k <= MOE_PREFILL_PAIRS)
             and H % 64 == 0 and H // 64 <= 64)
    if small:
        nw2, cfg2 = 1, MOE_CFG_W2
    for sk in (((2,) if T * k <= 8 else ()) if small else (4, 2) if T * k <= 4 else (2,) if T * k <= 16 else ()):
        if F % (sk * kc2) == 0 and F % (sk * 256) == 0:
            S = sk
            break
    cols2 = 16 * nw2 * M64G_CFG_WAVES[cfg2]
    if S == 1 and (H // cols2) * E < 192 and F % (2 * kc2) == 0 and F % 512 == 0:
        # few column tiles x local experts (EP shards: 4 experts x 32 tiles = 128
        # workgroups on 256 CUs): 2 K splits fill the chip
        S = 2
    part = torch.empty(S, P, H, dtype=torch.float32, device=x.device)
    if (resid is not None and counters is not None and max_rows <= MOE_PREFILL_PAIRS and H // cols2 <= 64
            and H // cols2 <= counters.numel()
            and (H // cols2) * T <= ss.numel()):
        kn.moe_gemm_m64g_resid(act.data_ptr(), 0, offs.data_ptr(), E, F, w2.data_ptr(), H, P, part.data_ptr(), S, nw2,
                               cfg2, max_rows, stream_ptr(), valid, dest.data_ptr(),
                               topk_w.float().contiguous().data_ptr(), resid.data_ptr(), ss.data_ptr(),
                               counters.data_ptr(), T, k, T * k)
        return H // cols2
    gemm(act.data_ptr(), 0, offs.data_ptr(), E, F, w2.data_ptr(), H, P, part.data_ptr(), 0, S, 1, nw2, stream_ptr(),
         cfg=cfg2)
    return _moe_combine(kn, part, S, P, dest, topk_w, resid, ss, T, k, H, x, out_f32)


def _moe_combine(kn, part, S, P, dest, topk_w, resid, ss, T, k, H, x, out_f32):
    """Weighted unpermute of the w2 partials: into the residual stream (+ statistics,
    returns the partial-sum count) or a fresh [T, H] output."""
    if resid is not None:
        kn.moe_combine_resid(part.data_ptr(), S, P, dest.data_ptr(), topk_w.float().contiguous().data_ptr(),
                             resid.data_ptr(), ss.data_ptr(), T, k, H, stream_ptr())
        return H // 1024
    out = torch.empty(T, H, dtype=torch.float32 if out_f32 else x.dtype, device=x.device)
    kn.moe_combine(part.data_ptr(), S, P, dest.data_ptr(), topk_w.float().contiguous().data_ptr(), out.data_ptr(), T,
                   k, H, stream_ptr(), 1 if out_f32 else 0)
    return out


def ep_plan(ids: torch.Tensor, E_local: int, tp: int, cap: int, packed: bool):
    """Dispatch plan for expert parallelism (csrc/kernels/moe.hip ep_plan): pair
    i = (t, j) of ids [Ts, k] goes to rank d = ids[i] // E_local at a stable slot
    base[d] + (earlier pairs bound for d), base[d] = d * cap (fixed capacity: equal
    all_to_all splits, graph-capturable) or the exclusive prefix of the counts
    (packed: the count-exact all_to_all). -> (slot [Ts*k] int32, send_eid [rows]
    int32 = the owner's local expert id (-1 = unused capacity slot), counts [tp])."""
    n = ids.numel()
    rows = n if packed else tp * cap
    if not use_native(ids):
        flat = ids.reshape(-1).long()
        dest = flat // E_local
        onehot = torch.nn.functional.one_hot(dest, tp)
        pos = (torch.cumsum(onehot, 0) - onehot).gather(1, dest[:, None])[:, 0]
        counts = onehot.sum(0)
        base = (torch.cumsum(counts, 0) - counts) if packed else torch.arange(tp) * cap
        slot = base[dest] + pos
        send_eid = torch.full((rows,), -1, dtype=torch.int32)
        send_eid[slot] = (flat - dest * E_local).to(torch.int32)
        return slot.to(torch.int32), send_eid, counts.to(torch.int32)
    dev = ids.device
    slot = torch.empty(n, dtype=torch.int32, device=dev)
    send_eid = torch.empty(rows, dtype=torch.int32, device=dev)
    counts = torch.empty(tp, dtype=torch.int32, device=dev)
    kernels().ep_plan(ids.contiguous().data_ptr(), n, E_local, tp, cap, 1 if packed else 0, slot.data_ptr(),
                      send_eid.data_ptr(), counts.data_ptr(), stream_ptr())
    return slot, send_eid, counts


def ep_scatter(x: torch.Tensor, k: int, slot: torch.Tensor, rows: int) -> torch.Tensor:
    """send [rows, H]: send[slot[i]] = x[i // k] (unused capacity rows are left
    uninitialised: their expert id is -1, so no kernel reads them)."""
    T, H = x.shape
    send = torch.empty(rows, H, dtype=x.dtype, device=x.device)
    if not use_native(x):
        src = torch.arange(slot.numel()) // k
        send[slot.long()] = x[src]
        return send
    kernels().ep_scatter(x.data_ptr(), x.stride(0), k, slot.data_ptr(), slot.numel(), H, send.data_ptr(),
                         stream_ptr())
    return send


def ep_combine(back: torch.Tensor, slot: torch.Tensor, topk_w: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """Source-side unpermute + weighted sum: out[t] = sum_j w[t, j] * back[slot[t*k+j]]
    (fp32 accumulation, one bf16 rounding), written into out[:T]."""
    T, k = topk_w.shape
    if T == 0:
        return out
    H = back.shape[1]
    if not use_native(back):
        contrib = back[slot.long()].float() * topk_w.reshape(-1, 1).float()
        out[:T] = contrib.view(T, k, H).sum(1).to(out.dtype)
        return out
    kernels().moe_combine(back.data_ptr(), 0, back.shape[0], slot.data_ptr(), topk_w.float().contiguous().data_ptr(),
                          out.data_ptr(), T, k, H, stream_ptr())
    return out
