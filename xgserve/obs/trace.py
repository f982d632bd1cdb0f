"""Lightweight tracing: request-lifecycle spans (Req 8.5, requirements.md:122).

`span(name, **attrs)` is a context manager that records start/end/duration and
parent linkage through contextvars (request -> validate -> queue -> engine ->
stream). Finished spans go to an in-memory ring (served at /debug/traces) and,
when XGS_TRACE_FILE is set, are appended as JSON lines -- the OpenTelemetry
span shape (trace_id, span_id, parent_span_id, name, start/end ns, attributes)
so an OTel collector can ingest the file. Kernel-level profiling is
rocprofv3 (bench/profile.sh: kernel table + step-gap analysis); `XGS_TORCH_PROFILE=N` wraps N engine steps in
torch.profiler.
"""
from __future__ import annotations

import contextlib
import contextvars
import json
import os
import random
import threading
import time
from collections import deque
from typing import Any, Dict, Optional

_current: contextvars.ContextVar = contextvars.ContextVar("xgs_span", default=None)
_ring: deque = deque(maxlen=2048)
_lock = threading.Lock()
_enabled = True
_sample_rate = 1.0


def configure(enabled: bool = True, sample_rate: float = 1.0):
    global _enabled, _sample_rate
    _enabled, _sample_rate = enabled, sample_rate


class Span:
    __slots__ = ("name", "trace_id", "span_id", "parent", "start_ns", "end_ns", "attrs", "sampled")

    def __init__(self, name: str, parent: Optional["Span"], attrs: Dict[str, Any]):
        self.name = name
        self.parent = parent
        self.trace_id = parent.trace_id if parent else "%032x" % random.getrandbits(128)
        self.span_id = "%016x" % random.getrandbits(64)
        self.sampled = parent.sampled if parent else (random.random() < _sample_rate)
        self.start_ns = time.time_ns()
        self.end_ns = 0
        self.attrs = dict(attrs)

    def set(self, **kw):
        self.attrs.update(kw)

    def to_dict(self) -> dict:
        return {"trace_id": self.trace_id, "span_id": self.span_id,
                "parent_span_id": self.parent.span_id if self.parent else None, "name": self.name,
                "start_time_unix_nano": self.start_ns, "end_time_unix_nano": self.end_ns,
                "duration_ms": (self.end_ns - self.start_ns) / 1e6, "attributes": self.attrs}


def _emit(s: Span):
    if not s.sampled:
        return
    d = s.to_dict()
    with _lock:
        _ring.append(d)
        path = os.environ.get("XGS_TRACE_FILE")
        if path:
            with open(path, "a") as f:
                f.write(json.dumps(d) + "\n")


@contextlib.contextmanager
def span(name: str, **attrs):
    if not _enabled:
        yield None
        return
    parent = _current.get()
    s = Span(name, parent, attrs)
    tok = _current.set(s)
    try:
        yield s
    except Exception as e:
        s.set(error=repr(e))
        raise
    finally:
        s.end_ns = time.time_ns()
        _current.reset(tok)
        _emit(s)


def start_span(name: str, parent: Optional[Span] = None, **attrs) -> Span:
    """Manual span (crosses async boundaries); finish with end_span()."""
    return Span(name, parent if parent is not None else _current.get(), attrs)


def end_span(s: Optional[Span], **attrs):
    if s is None or not _enabled:
        return
    s.set(**attrs)
    s.end_ns = time.time_ns()
    _emit(s)


def recent(n: int = 100):
    with _lock:
        return list(_ring)[-n:]
