"""Collectives used on the model's hot path (TP all-reduce, vocab all-gather,
EP all-to-all) over RCCL/xGMI, with the custom one-shot xGMI all-reduce
(csrc/comm/custom_allreduce.hip) taking latency-bound decode messages when it
has been registered for the TP group.

Sizing notes for MI355X (7 xGMI links x ~153 GB/s per GPU, point-to-point):
  * decode all-reduces are T*H*2 bytes (8B: 8 KiB/token) -> latency bound;
    the one-shot kernel reads all peers' buffers concurrently over all 7 links
    instead of RCCL's per-link-bound ring;
  * prefill all-reduces (MBs) go to RCCL.
"""
from __future__ import annotations

import os
import pickle
from typing import List, Optional

import torch
import torch.distributed as dist

from .state import get_state

_CUSTOM_AR = None  # set by register_custom_allreduce()


def register_custom_allreduce(ar) -> None:
    global _CUSTOM_AR
    _CUSTOM_AR = ar


def custom_allreduce():
    return _CUSTOM_AR


def tp_all_reduce(x: torch.Tensor) -> torch.Tensor:
    s = get_state()
    if s.tp_size == 1:
        return x
    ar = _CUSTOM_AR
    if ar is not None and ar.can_run(x):
        return ar.all_reduce(x)
    dist.all_reduce(x, group=s.tp_group)
    return x


def resid_allreduce_ok(T: int, H: int) -> bool:
    """Can `tp_allreduce_resid` take a [T, H] message in one launch? True with the
    custom all-reduce registered, and for a simulated TP shard (a model built
    with tp > 1 in a single-rank process: the collective is a local reduction)."""
    s = get_state()
    if s.tp_size == 1:
        return True
    return _CUSTOM_AR is not None and _CUSTOM_AR.can_resid(T, H)


# Simulated TP all-reduce (bench.py --tp-shard: one rank of a TP group in one process):
# XGS_TUNE sim_ar_us > 0 makes the local stand-in wait that long (the peer round trip of the
# one-shot xGMI all-reduce), so the simulation exposes collective latency
# (profiles/r3_tp_ar_overlap.md). A measurement knob.
# TP decode: the row-parallel O / down GEMMs all-reduce inside their own launch, for
# steps of at most GEMM_AR_MAX_T rows. Above that one tail workgroup per column tile
# has too many lines to push and poll; the separate LL kernel spreads them over
# T x H / 1024 workgroups. One simulated 70B TP8 rank (profiles/r5_gemm_ar.md):
# batch 1 6.14 vs 6.30 ms, 16 rows 7.91 vs 7.74, 64 rows 13.6 vs 11.0.
GEMM_AR = __import__("xgserve.tune", fromlist=["get_bool"]).get_bool("gemm_ar", True)
GEMM_AR_MAX_T = 4
_SIM_AR_TICKS = int(__import__("xgserve.tune", fromlist=["get_float"]).get_float("sim_ar_us", 0.0) * 100)  # 100 MHz


def tp_allreduce_resid(part: torch.Tensor, resid: torch.Tensor, ss: torch.Tensor, sim_world: int = 1) -> None:
    """Row-parallel projection epilogue of the fused decode layer:
    resid += all-reduce(sum_s part[s]) in place (bf16), ss[chunk * T + t] <- the new
    residual's sum of squares per 1024 columns. `part` is this rank's fp32 split-K
    partials [S, T, H]. One launch on the custom all-reduce. A simulated TP shard
    (single-rank process, layers built for sim_world > 1 ranks) runs the same LL
    kernel in its loopback form (pushes / polls of sim_world ranks through its own
    region, numerics of one rank; XGS_TUNE sim_ar_us adds a link latency)."""
    from ..ops._native import kernels, stream_ptr
    S, T, H = part.shape
    s = get_state()
    if s.tp_size == 1 and sim_world > 1 and H % 1024 == 0 and T * (H // 1024) <= 512 and T * H * 4 <= (32 << 20) // 16:
        a = _loopback_args(sim_world, part.device)
        kernels().custom_allreduce_resid_ll(part.data_ptr(), S, T, resid.data_ptr(), ss.data_ptr(), H, a.region,
                                            a.data2, 0, a.gens2.data_ptr(), a.err.data_ptr(), stream_ptr(), a.loop)
        return
    if s.tp_size == 1:
        kernels().add_partials_resid(part.data_ptr(), S, T, resid.data_ptr(), ss.data_ptr(), H, stream_ptr(),
                                     _SIM_AR_TICKS)
        return
    _CUSTOM_AR.all_reduce_resid(part, resid, ss)


class GemmArArgs:
    """Operands of the all-reduce inside a row-parallel GEMM launch (gemm_m64g GG_AR):
    each rank's LL receive region, this rank, the group size, one generation word per
    column tile and the timeout control words. loop = 1: a one-process --tp-shard
    simulation whose "peers" are its own region (the waits and traffic of `world`
    ranks, the numerics of one)."""

    REGION = 32 << 20

    def __init__(self, data, region, rank, world, loop, gens, err):
        self.data, self.region, self.rank, self.world, self.loop = data, region, rank, world, loop
        self.gens, self.err = gens, err


_LOOPBACK = {}


def _loopback_args(world: int, device) -> GemmArArgs:
    key = (str(device), world)
    a = _LOOPBACK.get(key)
    if a is None:
        from ..ops._native import kernels
        buf = torch.zeros(GemmArArgs.REGION, dtype=torch.uint8, device=device)
        gens = torch.zeros(4096, dtype=torch.int32, device=device)
        # [timeouts, wait limit in wall-clock ticks]: 20 s
        khz = max(1, int(kernels().car_wallclock_khz()) or 100_000)
        err = torch.tensor([0, min(2**31 - 1, 20 * khz * 1000)], dtype=torch.int32, device=device)
        # loop = 1 + the simulated link latency (XGS_TUNE sim_ar_us) in wall-clock ticks
        a = GemmArArgs([buf.data_ptr()] * world, GemmArArgs.REGION, 0, world, 1 + _SIM_AR_TICKS, gens, err)
        a._buf = buf
        # the unfused path's LL residual all-reduce: its own region and block generations
        a._buf2 = torch.zeros(GemmArArgs.REGION, dtype=torch.uint8, device=device)
        a.gens2 = torch.zeros(1024, dtype=torch.int32, device=device)
        a.data2 = [a._buf2.data_ptr()] * world
        _LOOPBACK[key] = a
    return a


def gemm_ar_args(layer_tp: int, T: int, H: int, device) -> Optional[GemmArArgs]:
    """The GG_AR operands for a decode step of T rows, or None (the GEMM + all-reduce
    launches then run as before): the verified custom all-reduce of a real TP group,
    or the loopback of a simulated shard (tp_size 1, layer built for layer_tp ranks)."""
    if not GEMM_AR or T > GEMM_AR_MAX_T or T * H * 4 > GemmArArgs.REGION // 16:
        return None
    s = get_state()
    if s.tp_size == 1:
        return _loopback_args(layer_tp, device) if layer_tp > 1 else None
    if _CUSTOM_AR is None or not getattr(_CUSTOM_AR, "gemm_ar", None) or not _CUSTOM_AR.gemm_ar_allowed():
        return None
    return _CUSTOM_AR.gemm_ar


class _Done:
    def wait(self):
        return True


def tp_all_reduce_async(x: torch.Tensor):
    """In-place all-reduce of x over the TP group without blocking the compute
    stream: RCCL runs it on its own stream behind an event on the current one;
    `.wait()` on the returned handle makes the current stream (not the host)
    wait for it. Used to overlap prefill-sized all-reduces with the GEMMs of the
    next token chunk (LlamaLayer._forward_tp_overlap)."""
    s = get_state()
    if s.tp_size == 1:
        return _Done()
    return dist.all_reduce(x, group=s.tp_group, async_op=True)


def tp_all_gather_lastdim(x: torch.Tensor) -> torch.Tensor:
    """[.., n] sharded over TP ranks -> [.., n*tp] (rank-major)."""
    s = get_state()
    if s.tp_size == 1:
        return x
    x = x.contiguous()
    ar = _CUSTOM_AR
    if ar is not None and ar.can_gather(x):
        return ar.all_gather_lastdim(x)  # IPC peer reads, graph capturable
    # flat [tp*rows, ...] output (the layout every backend accepts), viewed as [tp, ...]
    out = torch.empty((s.tp_size * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=s.tp_group)
    out = out.view((s.tp_size,) + tuple(x.shape))
    return out.movedim(0, -2).reshape(*x.shape[:-1], s.tp_size * x.shape[-1])


def tp_all_gather_rows(x: torch.Tensor) -> torch.Tensor:
    """[n, ..] per rank -> [n*tp, ..] (rank-major rows)."""
    s = get_state()
    if s.tp_size == 1:
        return x
    x = x.contiguous()
    out = torch.empty((s.tp_size * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=s.tp_group)
    return out


def tp_reduce_scatter_rows(x: torch.Tensor) -> torch.Tensor:
    """[tp * n, ..] partial sums per rank -> this rank's [n, ..] block of the sum
    (rank-major rows). gloo builds without reduce_scatter: all-reduce + slice."""
    s = get_state()
    if s.tp_size == 1:
        return x
    x = x.contiguous()
    n = x.shape[0] // s.tp_size
    if s.backend == "gloo":
        dist.all_reduce(x, group=s.tp_group)
        return x[s.tp_rank * n:(s.tp_rank + 1) * n]
    out = torch.empty((n,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, x, group=s.tp_group)
    return out


def tp_all_to_all(x: torch.Tensor, send_splits: List[int], recv_splits: List[int]) -> torch.Tensor:
    s = get_state()
    out = torch.empty((sum(recv_splits),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    if s.tp_size == 1:
        out.copy_(x)
        return out
    dist.all_to_all_single(out, x.contiguous(), recv_splits, send_splits, group=s.tp_group)
    return out


def tp_exchange_counts(counts: torch.Tensor) -> torch.Tensor:
    """counts[r] = rows this rank sends to rank r -> rows this rank receives from each r."""
    s = get_state()
    if s.tp_size == 1:
        return counts.clone()
    out = torch.empty_like(counts)
    dist.all_to_all_single(out, counts.contiguous(), group=s.tp_group)
    return out


PLAN_TIMEOUT_S = 600.0


def tp_broadcast_object(obj, src: int = 0):
    """Leader -> followers object broadcast. Uses the shared-memory plan channel
    when the group has one (one memcpy + an atomic, no TCP round trip); an object
    larger than the channel travels over gloo, announced by an empty message."""
    s = get_state()
    if s.tp_size == 1:
        return obj
    ch = s.plan_channel
    if ch is not None and src == 0:
        if s.tp_rank == 0:
            data = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
            big = len(data) > ch.capacity
            if not ch.publish(b"" if big else data, PLAN_TIMEOUT_S):
                raise RuntimeError("TP follower did not consume the previous plan (dead rank?)")
            if not big:
                return obj
        else:
            data = None
            while data is None:
                data = ch.receive(s.tp_rank - 1, PLAN_TIMEOUT_S)
            if data:
                return pickle.loads(data)
    lst = [obj]
    g = s.tp_cpu_group if s.tp_cpu_group is not None else s.tp_group
    src_global = dist.get_global_rank(g, src) if g is not None and g != dist.group.WORLD else src
    dist.broadcast_object_list(lst, src=src_global, group=g)
    return lst[0]


def barrier() -> None:
    if dist.is_initialized():
        dist.barrier()
