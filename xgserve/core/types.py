"""ID aliases and Priority (reference `crates/core/src/types.rs:7-28`).

* RequestID / BatchId are UUIDs (types.rs:7,9).
* WorkerId is a small int (the replica index) -- the reference comment at
  types.rs:10 and design.md:676 say u32 while the alias says Uuid; we take the
  int form.
* CacheKey is a token-id sequence (types.rs:13).
* Priority is Low=0 < Normal=1 < High=2, default Normal (types.rs:17-28). Its
  serde representation is PascalCase ("Low"/"Normal"/"High"); we also accept
  lowercase as a strict superset.
"""
from __future__ import annotations

import enum
import uuid
from typing import List

RequestID = uuid.UUID
BatchId = uuid.UUID
WorkerId = int
CacheKey = List[int]


def new_request_id() -> str:
    return str(uuid.uuid4())


class Priority(enum.IntEnum):
    Low = 0
    Normal = 1
    High = 2

    @classmethod
    def default(cls) -> "Priority":
        return cls.Normal

    @classmethod
    def parse(cls, value) -> "Priority":
        """Parse the wire representation. Raises ValueError on unknown variants."""
        if isinstance(value, Priority):
            return value
        if isinstance(value, str):
            table = {"Low": cls.Low, "Normal": cls.Normal, "High": cls.High,
                     "low": cls.Low, "normal": cls.Normal, "high": cls.High}
            if value in table:
                return table[value]
            raise ValueError(f"unknown variant `{value}`, expected one of `Low`, `Normal`, `High`")
        raise ValueError(f"invalid type: {type(value).__name__}, expected a priority string")
