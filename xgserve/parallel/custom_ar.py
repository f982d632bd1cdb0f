"""Custom one-shot / two-shot all-reduce over xGMI peer memory (csrc/comm/custom_allreduce.hip).

Each TP rank allocates one uncached HBM buffer (2 slots x max_bytes) and one
signal array, exports both with hipIpcGetMemHandle, and exchanges the handles
over the CPU (gloo) group; every rank then maps all peers' buffers. The kernel
is graph capturable, so TP decode graphs contain the all-reduce.

Path choice, bf16 messages of 16-byte multiples:
  * one-shot (each rank reads every peer's whole message; lowest latency) up to
    `two_shot_min` bytes, or up to `max_bytes` when TP < 4 (at 2 ranks the
    two-shot moves the same bytes per link plus a second synchronisation);
  * two-shot (reduce-scatter + all-gather through peer memory, ~2n/W bytes per
    xGMI link) from `two_shot_min` to `two_shot_max` bytes at TP >= 4;
  * RCCL above that (comm.tp_all_reduce falls back automatically).
"""
from __future__ import annotations

import logging
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops._native import kernels, stream_ptr

log = logging.getLogger("xgserve.comm")


class CustomAllReduce:
    def __init__(self, rank: int, world: int, device: torch.device, cpu_group=None, max_bytes: int = 8 << 20,
                 two_shot_min: Optional[int] = None, two_shot_max: int = 32 << 20):
        k = kernels()
        max_ranks, self.max_blocks, chunk = k.car_limits()
        if not (2 <= world <= max_ranks):
            raise ValueError(f"custom all-reduce supports 2..{max_ranks} ranks, got {world}")
        self.rank, self.world, self.device = rank, world, device
        self.slot = min(max_bytes, self.max_blocks * chunk) // chunk * chunk
        if two_shot_min is None:
            two_shot_min = (512 << 10) if world >= 4 else self.slot + 1
        # a two-shot shard of n/W bytes must fit max_blocks chunks
        self.slot2 = min(two_shot_max, self.max_blocks * chunk * world) // chunk * chunk
        self.two_shot_min = two_shot_min
        nsig = max_ranks * self.max_blocks * 4  # bytes per phase
        self._k = k
        self.data = self.sig = 0
        self._opened: List[int] = []
        # phase 1 (local): allocate + export; every rank reports success so a
        # failure anywhere disables the path everywhere instead of hanging peers
        mine = None
        try:
            # [one-shot 2 x slot | two-shot 2 x slot2] and [one-shot | two-shot phase 0 | phase 1] signals
            self.data = k.car_alloc_uncached(2 * self.slot + 2 * self.slot2)
            self.sig = k.car_alloc_uncached(3 * nsig)
            mine = (k.car_ipc_handle(self.data), k.car_ipc_handle(self.sig))
        except RuntimeError as e:
            log.warning("custom all-reduce: local setup failed: %s", e)
        handles: List = [None] * world
        dist.all_gather_object(handles, mine, group=cpu_group)
        if any(h is None for h in handles):
            self.close()
            raise RuntimeError("custom all-reduce setup failed on some rank")
        # phase 2: map the peers
        ok = 1
        self.data_ptrs, self.sig_ptrs = [], []
        try:
            for r in range(world):
                if r == rank:
                    self.data_ptrs.append(self.data)
                    self.sig_ptrs.append(self.sig)
                    continue
                d = k.car_ipc_open(handles[r][0])
                self._opened.append(d)
                s_ = k.car_ipc_open(handles[r][1])
                self._opened.append(s_)
                self.data_ptrs.append(d)
                self.sig_ptrs.append(s_)
        except RuntimeError as e:
            log.warning("custom all-reduce: mapping peers failed: %s", e)
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=cpu_group)
        if int(flag.item()) == 0:
            self.close()
            raise RuntimeError("custom all-reduce: peer mapping failed on some rank")
        self.data_ptrs2 = [d + 2 * self.slot for d in self.data_ptrs]
        self.sig_ptrs2 = [s_ + nsig for s_ in self.sig_ptrs]
        self.gens = torch.zeros(self.max_blocks + 1, dtype=torch.int32, device=device)
        self.gens2 = torch.zeros(self.max_blocks + 1, dtype=torch.int32, device=device)
        log.info("custom all-reduce ready: rank %d/%d, one-shot <= %d KiB, two-shot <= %d MiB", rank, world,
                 min(self.slot, self.two_shot_min) >> 10, self.slot2 >> 20)

    def _two_shot(self, n: int) -> bool:
        return self.two_shot_min <= n <= self.slot2

    def can_run(self, x: torch.Tensor) -> bool:
        n = x.numel() * x.element_size()
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and n > 0 and n % 16 == 0
                and (n <= self.slot or self._two_shot(n)))

    def all_reduce(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        out = x if out is None else out
        n = x.numel() * x.element_size()
        if self._two_shot(n):
            self._k.custom_allreduce_2shot(x.data_ptr(), out.data_ptr(), n, self.slot2, self.data_ptrs2,
                                           self.sig_ptrs2, self.rank, self.gens2.data_ptr(), stream_ptr())
        else:
            self._k.custom_allreduce(x.data_ptr(), out.data_ptr(), n, self.slot, self.data_ptrs, self.sig_ptrs,
                                     self.rank, self.gens.data_ptr(), stream_ptr())
        return out

    def timeouts(self) -> int:
        """Peer-wait timeouts recorded by the kernels (0 when healthy)."""
        return int(self.gens[self.max_blocks].item()) + int(self.gens2[self.max_blocks].item())

    def close(self) -> None:
        for p in self._opened:
            self._k.car_ipc_close(p)
        self._opened = []
        for p in (self.data, self.sig):
            if p:
                self._k.car_free(p)
        self.data = self.sig = 0


def maybe_enable(state, device: torch.device) -> Optional[CustomAllReduce]:
    """Register the custom all-reduce for this TP group (GPU, 2..8 ranks), unless
    XGS_CUSTOM_AR=0. Falls back to RCCL on any setup failure."""
    import os
    from . import comm
    if state.tp_size < 2 or device.type != "cuda" or os.environ.get("XGS_CUSTOM_AR", "1") == "0":
        return None
    try:
        ar = CustomAllReduce(state.tp_rank, state.tp_size, device, cpu_group=state.tp_cpu_group)
    except Exception as e:  # noqa: BLE001 - RCCL remains correct
        log.warning("custom all-reduce unavailable (%s); using RCCL", e)
        return None
    comm.register_custom_allreduce(ar)
    return ar
