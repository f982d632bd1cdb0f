"""Process-group state for tensor / expert / data parallelism.

One OS process per GPU. A replica is a TP group of `tp` consecutive ranks
(TP groups never span replicas); DP replicas are independent engines that the
router feeds, so no collective is ever issued across replicas on the request
path. Expert parallelism (Mixtral) reuses the TP group: EP degree == TP degree,
each rank owning E/tp experts.

Backends: "nccl" (== RCCL on ROCm, over xGMI) on GPUs, "gloo" for the CPU
tests. Rendezvous always uses 127.0.0.1 unless MASTER_ADDR says otherwise.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class ParallelState:
    world_size: int = 1
    rank: int = 0
    tp_size: int = 1
    tp_rank: int = 0
    dp_size: int = 1
    dp_rank: int = 0
    tp_group: Optional[object] = None
    tp_cpu_group: Optional[object] = None
    backend: str = "none"
    device: torch.device = torch.device("cpu")
    plan_channel: Optional[object] = None  # _runtime.ShmChannel (TP leader writes, followers read)

    @property
    def ep_size(self) -> int:
        return self.tp_size

    @property
    def ep_rank(self) -> int:
        return self.tp_rank

    @property
    def is_tp_leader(self) -> bool:
        return self.tp_rank == 0


_STATE = ParallelState()


def get_state() -> ParallelState:
    return _STATE


def set_state(s: ParallelState) -> None:
    global _STATE
    _STATE = s


def init_distributed(tp_size: int = 1, backend: Optional[str] = None, device: Optional[torch.device] = None,
                     timeout_s: int = 600) -> ParallelState:
    """Initialise torch.distributed from the usual env (RANK/WORLD_SIZE/MASTER_*)
    and build TP groups of `tp_size` consecutive ranks."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device is None:
        if torch.cuda.is_available():
            torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
            device = torch.device("cuda", torch.cuda.current_device())
        else:
            device = torch.device("cpu")
    if world == 1 and tp_size == 1:
        s = ParallelState(device=device)
        set_state(s)
        return s
    if world % tp_size:
        raise ValueError(f"world size {world} not divisible by tp {tp_size}")
    if backend is None:
        backend = "nccl" if device.type == "cuda" else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    if not dist.is_initialized():
        import datetime
        kw = {}
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    tp_group = tp_cpu = None
    my = None
    for start in range(0, world, tp_size):
        ranks = list(range(start, start + tp_size))
        g = dist.new_group(ranks, backend=backend) if tp_size < world else dist.group.WORLD
        gc = dist.new_group(ranks, backend="gloo") if backend != "gloo" else g
        if rank in ranks:
            tp_group, tp_cpu, my = g, gc, ranks
    s = ParallelState(world_size=world, rank=rank, tp_size=tp_size, tp_rank=my.index(rank),
                      dp_size=world // tp_size, dp_rank=rank // tp_size, tp_group=tp_group,
                      tp_cpu_group=tp_cpu, backend=backend, device=device)
    if tp_size > 1:
        s.plan_channel = _open_plan_channel(s, my)
    set_state(s)
    return s


PLAN_CHANNEL_BYTES = 32 << 20  # sparse: only the pages a plan touches are ever backed


def _open_plan_channel(s: ParallelState, ranks):
    """Per-step plan broadcast over POSIX shared memory.

    The TP leader creates the segment, the name travels once over the gloo
    group, every follower maps it, and the leader unlinks the name as soon as
    all ranks hold a mapping, so a crashed group leaves nothing in /dev/shm.
    TP groups are always node-local (one process per GPU of one node).
    Disabled with XGS_SHM_PLAN=0 (plans then go over gloo)."""
    if os.environ.get("XGS_SHM_PLAN", "1") == "0":
        return None
    try:
        from .. import _runtime as R
    except ImportError:
        return None
    g = s.tp_cpu_group
    src = ranks[0]
    ch, err = None, None
    if s.tp_rank == 0:
        name = f"xgs_plan_{os.getpid()}_{s.dp_rank}_{os.environ.get('MASTER_PORT', '0')}"
        try:
            ch = R.ShmChannel(name, PLAN_CHANNEL_BYTES, s.tp_size - 1, True)
        except Exception as e:  # noqa: BLE001 - fall back to gloo below
            name, err = None, e
        box = [name]
    else:
        box = [None]
    dist.broadcast_object_list(box, src=src, group=g)
    name = box[0]
    ok = 1
    if name is not None and s.tp_rank != 0:
        try:
            ch = R.ShmChannel(name, 0, s.tp_size - 1, False)
        except Exception as e:  # noqa: BLE001
            ch, ok, err = None, 0, e
    flag = torch.tensor([ok if name is not None else 0], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=g)
    if s.tp_rank == 0 and ch is not None:
        ch.unlink()
    if not int(flag.item()):
        if err is not None:
            import logging
            logging.getLogger("xgserve").warning("shm plan channel unavailable (%s); using gloo", err)
        return None
    return ch


def destroy_distributed() -> None:
    _STATE.plan_channel = None
    if dist.is_initialized():
        dist.destroy_process_group()
    set_state(ParallelState())
