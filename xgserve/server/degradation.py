"""Graceful degradation ladder (Req 9.3/9.5, requirements.md:132,134;
design.md:921-944).

Memory pressure = fraction of KV-cache pages in use on the *least* loaded
healthy replica (if any replica still has room the system is not saturated).
Levels, with the spec's thresholds (configurable):
  < 0.70 Normal; < 0.80 ReducedBatchSize (max batch halved on every replica);
  < 0.90 AggressiveCacheEviction (prefix caches flushed); < 0.95
  RejectLowPriority (Low-priority requests get 503); else Emergency (all new
  requests get 503).
"""
from __future__ import annotations

import enum


class DegradationLevel(enum.IntEnum):
    Normal = 0
    ReducedBatchSize = 1
    AggressiveCacheEviction = 2
    RejectLowPriority = 3
    Emergency = 4

    @classmethod
    def from_memory_pressure(cls, p: float, reduce_at: float = 0.70, evict_at: float = 0.80,
                             reject_low_at: float = 0.90, emergency_at: float = 0.95) -> "DegradationLevel":
        if p < reduce_at:
            return cls.Normal
        if p < evict_at:
            return cls.ReducedBatchSize
        if p < reject_low_at:
            return cls.AggressiveCacheEviction
        if p < emergency_at:
            return cls.RejectLowPriority
        return cls.Emergency

    def admits(self, priority: int) -> bool:
        """Whether a new request of `priority` (0 Low, 1 Normal, 2 High) is admitted."""
        if self == DegradationLevel.Emergency:
            return False
        if self == DegradationLevel.RejectLowPriority:
            return priority > 0
        return True
