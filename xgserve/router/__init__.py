"""Replica router: the spec's Adaptive Scheduler (Req 6, requirements.md:88-98;
design.md:269-308). Selection runs in the C++ ReplicaRouter
(csrc/runtime/router.cpp); this wrapper maps strategy names and adds the
Python-side views used by /server/stats."""
from __future__ import annotations

import time
from typing import List

from .. import _runtime as R

STRATEGIES = {"round_robin": R.Strategy.RoundRobin, "least_loaded": R.Strategy.LeastLoaded,
              "memory_aware": R.Strategy.MemoryAware}
_NAMES = {v: k for k, v in STRATEGIES.items()}


class Router:
    def __init__(self, strategy: str = "least_loaded"):
        self._r = R.ReplicaRouter(STRATEGIES[strategy])

    def set_strategy(self, name: str) -> None:
        self._r.set_strategy(STRATEGIES[name])

    @property
    def strategy(self) -> str:
        return _NAMES[self._r.strategy()]

    def register(self, rid: int, memory_available: int = 0) -> None:
        self._r.register_worker(rid, int(memory_available))

    def unregister(self, rid: int) -> bool:
        return self._r.unregister_worker(rid)

    def update(self, rid: int, active: int, memory_used: int, memory_available: int) -> None:
        self._r.update(rid, int(active), int(memory_used), int(memory_available), time.monotonic())

    def set_healthy(self, rid: int, healthy: bool) -> None:
        self._r.set_healthy(rid, healthy, time.monotonic())

    def add_active(self, rid: int, delta: int) -> None:
        self._r.add_active(rid, delta)

    def select(self, estimated_memory: int = 0) -> int:
        return self._r.select(int(estimated_memory))

    def num_healthy(self) -> int:
        return self._r.num_healthy()

    def statuses(self) -> List[dict]:
        return self._r.statuses()
