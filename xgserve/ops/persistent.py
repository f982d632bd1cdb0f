"""Persistent batch-1 decode (csrc/kernels/decode_b1.hip): every dense layer plus the
final RMSNorm of a Llama-family model in one launch of 256 workgroups.

The kernel streams the weights through a per-CU LDS ring without stopping at the
data dependencies, and hands activations between workgroups as tagged 8-byte
granules. This wrapper owns what the launch needs beside the step metadata: the
per-layer weight / KV-cache pointer tables, the granule area (zeroed by a memset
node before every launch, so graph replays are self-contained) and the wait-limit /
timeout word (`ctl`, same contract as the custom all-reduce's: captured graphs read
the current limit at replay; a timeout is counted and the step fails on the host).
"""
from __future__ import annotations

import weakref
from typing import List, Optional, Sequence, Tuple

import torch

from ._native import kernels, stream_ptr

SERVE_TIMEOUT_S = 1.0
WARMUP_TIMEOUT_S = 20.0

_LIVE: "weakref.WeakSet[B1Decoder]" = weakref.WeakSet()


class PersistentDecodeTimeout(RuntimeError):
    pass


def b1_plan(L: int, H: int, F: int, Hq: int, Hkv: int) -> Optional[List[int]]:
    """Kernel plan (granules, S_att, ring lines, LDS offsets, ...) or None if unsupported."""
    p = list(kernels().decode_b1_plan(L, H, F, Hq, Hkv))
    return p if p[0] > 0 else None


class B1Decoder:
    """One model's persistent batch-1 decode launch."""

    def __init__(self, layers: Sequence, final_norm: torch.Tensor, H: int, F: int, Hq: int, Hkv: int,
                 eps: float, scale: float, use_rope: bool = True):
        dev = final_norm.device
        self.k = kernels()
        self.L, self.H, self.F, self.Hq, self.Hkv = len(layers), H, F, Hq, Hkv
        self.plan = b1_plan(self.L, H, F, Hq, Hkv)
        if self.plan is None:
            raise ValueError(f"decode_b1: unsupported shape L={self.L} H={H} F={F} Hq={Hq} Hkv={Hkv}")
        self.eps, self.scale, self.use_rope = float(eps), float(scale), bool(use_rope)
        self.final_norm = final_norm
        self.wptr = torch.tensor([[l.qkv.data_ptr(), l.o.data_ptr(), l.gate_up.data_ptr(), l.down.data_ptr()]
                                  for l in layers], dtype=torch.int64, device=dev)
        self._layers = list(layers)  # keeps the weights (and so the pointers) alive
        # the loaders' schedule: each workgroup's weight lines as contiguous runs (built once)
        self.runs = torch.zeros(256 * self.plan[13] * 2, dtype=torch.int64, device=dev)
        overflow = torch.zeros(1, dtype=torch.int32, device=dev)
        self.k.decode_b1_build_runs(self.wptr.data_ptr(), self.L, H, F, Hq, Hkv, self.runs.data_ptr(),
                                    overflow.data_ptr(), stream_ptr())
        if int(overflow.item()):
            raise RuntimeError("decode_b1: run table overflow")
        self.gran = torch.empty(self.plan[0], dtype=torch.int64, device=dev)
        self.ctl = torch.zeros(4, dtype=torch.int32, device=dev)  # timeouts, limit, fault injection
        self.h_err = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self.out = torch.empty(1, H, dtype=torch.bfloat16, device=dev)
        self._kv_key: Optional[Tuple[int, ...]] = None
        self.kvptr: Optional[torch.Tensor] = None
        self._khz = self.k.car_wallclock_khz()
        self.stamps: Optional[torch.Tensor] = None  # diagnostics: enable_stamps()
        self.set_timeout(WARMUP_TIMEOUT_S)
        _LIVE.add(self)

    # ------------------------------------------------------------------ errors
    def set_timeout(self, seconds: float) -> None:
        ticks = int(min(max(seconds, 1e-3) * self._khz * 1000, 0x7FFFFFFF))
        self.ctl[1].fill_(ticks)

    def poll_async(self) -> None:
        self.h_err.copy_(self.ctl[:1], non_blocking=True)

    def check(self) -> None:
        n = int(self.h_err[0])
        if n:
            raise PersistentDecodeTimeout(f"persistent decode: {n} wait(s) timed out (a workgroup was not "
                                          "resident or stalled); failing the step")

    def timeouts(self) -> int:
        return int(self.ctl[0].item())

    # ------------------------------------------------------------------ diagnostics
    NSTAMP = 18
    PHASES = ("resid gather + norm", "QKV rows", "attention + combine", "attn gather", "O rows",
              "post gather + norm", "gate_up rows", "act gather", "down rows")

    def enable_stamps(self) -> None:
        """Record per-(workgroup, layer) phase clocks on every later launch (wall clock,
        100 MHz) plus per-workgroup loader stall / consumer line-wait totals."""
        n = 256 * self.L * self.NSTAMP + 256 * 4
        self.stamps = torch.zeros(n, dtype=torch.int64, device=self.gran.device)

    def stamp_report(self) -> dict:
        """Phase durations (us) of the last launch: mean / max over workgroups, summed
        over layers; loader ring-full stall and consumer line waits (us, mean over WGs)."""
        st = self.stamps.cpu()
        ph = st[:256 * self.L * self.NSTAMP].view(256, self.L, self.NSTAMP).double()
        tick_us = 1000.0 / self._khz
        att = ph[:32, :, [2, 10, 11, 12, 13, 14, 15, 3]]        # attention sub-phases (splits 0..31)
        ad = ((att[:, :, 1:] - att[:, :, :-1]) * tick_us).sum(1)
        gu_loop = ((ph[:, :, 17] - ph[:, :, 16]) * tick_us).sum(1)
        ph = ph[:, :, :10]
        d = (ph[:, :, 1:] - ph[:, :, :-1]) * tick_us           # [wg, layer, 9]
        nxt = torch.cat([ph[:, 1:, 0], ph[:, -1:, 9]], 1)      # next layer's start
        tail = (nxt - ph[:, :, 9]) * tick_us
        tail[:, -1] = 0
        per = d.sum(1)
        tot = (ph[:, -1, 9] - ph[:, 0, 0]) * tick_us
        extra = st[256 * self.L * self.NSTAMP:].view(256, 4).double() * tick_us
        rep = {name: (float(per[:, i].mean()), float(per[:, i].max())) for i, name in enumerate(self.PHASES)}
        rep["layer tail (down -> next layer)"] = (float(tail.sum(1).mean()), float(tail.sum(1).max()))
        rep["total"] = (float(tot.mean()), float(tot.max()))
        rep["  gate_up item loop (consumer 0)"] = (float(gu_loop.mean()), float(gu_loop.max()))
        rep["loader ring-full stall"] = (float(extra[:, 0].mean()), float(extra[:, 0].max()))
        rep["consumer line wait"] = (float(extra[:, 2].mean()), float(extra[:, 2].max()))
        lspan = (st[256 * self.L * self.NSTAMP:].view(256, 4)[:, 1].double() - ph[:, 0, 0]) * tick_us
        rep["loader span (start -> last line landed)"] = (float(lspan.mean()), float(lspan.max()))
        for i, name in enumerate(("kv prefetch issue", "qkv gather", "rope", "softmax.V", "partials publish",
                                  "combine gather", "combine + publish")):
            rep["  attn: " + name] = (float(ad[:, i].mean()), float(ad[:, i].max()))
        # hand-off edges: producer skew (last - first workgroup to publish) and the time
        # from the last publish to the consumers' completion (mean), summed over layers
        for name, pi, ci in (("post (O -> gate_up)", 5, 6), ("act (gate_up -> down)", 7, 8),
                             ("attn (combine -> O)", 3, 4)):
            prod, cons = ph[:, :, pi], ph[:, :, ci]
            skew = ((prod.max(0).values - prod.min(0).values) * tick_us).sum()
            lat = ((cons.mean(0) - prod.max(0).values) * tick_us).sum()
            rep["  edge " + name + ": skew / after-last"] = (float(skew), float(lat))
        prod, cons = ph[:, :-1, 9], ph[:, 1:, 1]
        rep["  edge resid (down -> next QKV): skew / after-last"] = (
            float(((prod.max(0).values - prod.min(0).values) * tick_us).sum()),
            float(((cons.mean(0) - prod.max(0).values) * tick_us).sum()))
        return rep

    # ------------------------------------------------------------------ launch
    def _kv_table(self, kv_caches: List[Tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
        key = tuple(t.data_ptr() for kv in kv_caches for t in kv)
        if key != self._kv_key:
            self.kvptr = torch.tensor(key, dtype=torch.int64, device=self.gran.device).view(-1, 2)
            self._kv_key = key
        return self.kvptr

    def __call__(self, resid: torch.Tensor, positions: torch.Tensor, slot_mapping: torch.Tensor,
                 block_tables: torch.Tensor, seq_lens: torch.Tensor, cos_sin: torch.Tensor,
                 kv_caches: List[Tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
        """resid: [1, H] bf16 embedding row -> [1, H] bf16 final normalised hidden state.
        The new token's K/V rows are appended to the paged caches."""
        kc = kv_caches[0][0]
        bs = kc.shape[2]
        if block_tables.shape[-1] > 32 * 500:  # the kernel keeps a split's pages (<= 512) in LDS
            raise ValueError("decode_b1: context too long for the persistent kernel")
        kvp = self._kv_table(kv_caches)
        self.k.decode_b1(self.wptr.data_ptr(), kvp.data_ptr(), resid.data_ptr(), self.final_norm.data_ptr(),
                         self.out.data_ptr(), positions.data_ptr(), slot_mapping.data_ptr(), block_tables.data_ptr(),
                         seq_lens.data_ptr(), cos_sin.data_ptr(), self.gran.data_ptr(), self.ctl.data_ptr(),
                         self.runs.data_ptr(), self.L, self.H, self.F, self.Hq, self.Hkv, bs, int(self.use_rope), self.eps, self.scale,
                         0 if self.stamps is None else self.stamps.data_ptr(), stream_ptr())
        return self.out


def poll_all() -> None:
    for d in list(_LIVE):
        d.poll_async()


def check_all() -> None:
    for d in list(_LIVE):
        d.check()


def set_timeout_all(seconds: float) -> None:
    for d in list(_LIVE):
        d.set_timeout(seconds)
