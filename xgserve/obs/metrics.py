"""Metrics collector + Prometheus text exposition.

Realises the reference's spec'd MetricsCollector / MetricsSnapshot
(design.md:461-492; Req 8.1-8.4): request counts / latency histograms by
endpoint and status, TTFT and inter-token latency, prompt vs generation token
throughput, batch sizes, cache hit rate, queue depth by priority, replica
health, speculative-decoding acceptance. `/metrics` renders Prometheus text
format 0.0.4 (hand-rolled: no dependency), `/server/stats` the JSON snapshot.
"""
from __future__ import annotations

import bisect
import itertools
import math
import threading
import time
from collections import defaultdict, deque
from typing import Dict, List, Optional, Tuple

_LAT_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60, 120)
_TTFT_BUCKETS = (0.001, 0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5, 1, 2, 5, 10, 30)
_ITL_BUCKETS = (0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.25, 0.5, 1)
_DELIVERY_BUCKETS = (0.0005, 0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.5)
_BATCH_BUCKETS = (1, 2, 4, 8, 16, 32, 64, 128, 256, 512)


class Histogram:
    def __init__(self, buckets):
        self.buckets = tuple(buckets)
        self.counts = [0] * (len(self.buckets) + 1)
        self.sum = 0.0
        self.n = 0

    def observe(self, v: float, n: int = 1):
        self.counts[bisect.bisect_left(self.buckets, v)] += n
        self.sum += v * n
        self.n += n


def _labels(d: Dict[str, str]) -> str:
    if not d:
        return ""
    return "{" + ",".join(f'{k}="{v}"' for k, v in sorted(d.items())) + "}"


def _pcts(xs) -> dict:
    if not xs:
        return {"p50": None, "p99": None, "max": None, "n": 0}
    v = sorted(xs)
    pick = lambda q: 1000 * v[min(len(v) - 1, int(math.ceil(q * len(v))) - 1)]  # noqa: E731
    return {"p50": pick(0.5), "p99": pick(0.99), "max": 1000 * v[-1], "n": len(v)}


class MetricsCollector:
    def __init__(self, window_s: float = 60.0):
        self._lock = threading.Lock()
        self.start = time.time()
        self.window_s = window_s
        self.requests_total: Dict[Tuple[str, int], int] = defaultdict(int)
        self.latency: Dict[Tuple[str, int], Histogram] = {}
        self.requests_active = 0
        self.ttft = Histogram(_TTFT_BUCKETS)
        self.itl = Histogram(_ITL_BUCKETS)
        self.delivery = Histogram(_DELIVERY_BUCKETS)
        self._recent_delivery: deque = deque(maxlen=1 << 16)
        self._recent_loop_lag: deque = deque(maxlen=4096)
        self.batch = Histogram(_BATCH_BUCKETS)
        self.padding_ratio_sum = 0.0
        self.prompt_tokens_total = 0
        self.generation_tokens_total = 0
        self.errors_total: Dict[str, int] = defaultdict(int)
        self.cache_hits = 0
        self.cache_misses = 0
        self.queue_depth = (0, 0, 0)
        self.workers: Dict[int, dict] = {}
        self.spec_proposed = 0
        self.spec_accepted = 0
        self.spec_speedup: Optional[float] = None
        self._recent_lat: deque = deque(maxlen=4096)
        self._tok_events: deque = deque()  # (t, prompt, gen)
        self.rejected_total: Dict[str, int] = defaultdict(int)

    # ---- recorders (design.md:467-476) ------------------------------------
    def record_request(self, endpoint: str, status: int, duration_s: float):
        with self._lock:
            key = (endpoint, int(status))
            self.requests_total[key] += 1
            h = self.latency.get(key)
            if h is None:
                h = self.latency[key] = Histogram(_LAT_BUCKETS)
            h.observe(duration_s)
            if status < 400:
                self._recent_lat.append(duration_s)

    def request_started(self):
        with self._lock:
            self.requests_active += 1

    def request_finished(self):
        with self._lock:
            self.requests_active = max(0, self.requests_active - 1)

    def record_batch(self, size: int, padding_ratio: float = 0.0):
        with self._lock:
            self.batch.observe(size)
            self.padding_ratio_sum += padding_ratio

    def record_inference(self, prompt_tokens: int, generation_tokens: int):
        with self._lock:
            now = time.time()
            self.prompt_tokens_total += prompt_tokens
            self.generation_tokens_total += generation_tokens
            self._tok_events.append((now, prompt_tokens, generation_tokens))
            while self._tok_events and self._tok_events[0][0] < now - self.window_s:
                self._tok_events.popleft()

    def record_ttft(self, s: float):
        with self._lock:
            self.ttft.observe(s)

    def record_delivery(self, s: float, n: int = 1):
        """Req 5.1: token delivery delay -- from the token reaching the host (after
        the engine step) to its SSE event being written to the client socket; n
        events written together (one engine step's tokens) share the delay."""
        with self._lock:
            self.delivery.observe(s, n)
            self._recent_delivery.extend(itertools.repeat(s, n))

    def record_loop_lag(self, s: float):
        """Event-loop responsiveness: how late a periodic wake-up fired."""
        with self._lock:
            self._recent_loop_lag.append(s)

    def record_itl(self, s: float):
        with self._lock:
            self.itl.observe(s)

    def record_itl_many(self, xs) -> None:
        """One engine step's inter-token latencies (one lock, one pass)."""
        h = self.itl
        b, counts = h.buckets, h.counts
        bl = bisect.bisect_left
        with self._lock:
            for v in xs:
                counts[bl(b, v)] += 1
            h.sum += sum(xs)
            h.n += len(xs)

    def record_cache_access(self, hit: bool, n: int = 1):
        with self._lock:
            if hit:
                self.cache_hits += n
            else:
                self.cache_misses += n

    def set_cache_counts(self, hits: int, misses: int):
        with self._lock:
            self.cache_hits, self.cache_misses = hits, misses

    def record_queue_depth(self, high: int, normal: int, low: int):
        with self._lock:
            self.queue_depth = (high, normal, low)

    def record_worker_status(self, wid: int, status: dict):
        with self._lock:
            self.workers[wid] = dict(status)

    def record_error(self, kind: str):
        with self._lock:
            self.errors_total[kind] += 1

    def record_rejection(self, reason: str):
        with self._lock:
            self.rejected_total[reason] += 1

    def set_spec_totals(self, proposed: int, accepted: int, speedup: Optional[float] = None):
        """Absolute draft-token counters (summed over replicas' heartbeats) and the
        measured speculation speedup factor (mean over replicas that report one)."""
        with self._lock:
            self.spec_proposed, self.spec_accepted = proposed, accepted
            self.spec_speedup = speedup

    # ---- snapshot (design.md:480-491) -------------------------------------
    def snapshot(self) -> dict:
        with self._lock:
            now = time.time()
            span = min(self.window_s, max(1e-6, now - self.start))
            p_tok = sum(e[1] for e in self._tok_events if e[0] >= now - span)
            g_tok = sum(e[2] for e in self._tok_events if e[0] >= now - span)
            lat = sorted(self._recent_lat)
            avg_lat = sum(lat) / len(lat) if lat else 0.0
            p99 = lat[min(len(lat) - 1, int(math.ceil(0.99 * len(lat))) - 1)] if lat else 0.0
            total = sum(self.requests_total.values())
            acc = self.cache_hits + self.cache_misses
            return {
                "requests_total": total,
                "requests_active": self.requests_active,
                "tokens_per_second": g_tok / span,
                "prompt_tokens_per_second": p_tok / span,
                "generation_tokens_per_second": g_tok / span,
                "prompt_tokens_total": self.prompt_tokens_total,
                "generation_tokens_total": self.generation_tokens_total,
                "avg_ttft_ms": 1000 * self.ttft.sum / self.ttft.n if self.ttft.n else 0.0,
                "avg_latency_ms": 1000 * avg_lat,
                "p99_latency_ms": 1000 * p99,
                "batch_size_avg": self.batch.sum / self.batch.n if self.batch.n else 0.0,
                "padding_overhead_avg": self.padding_ratio_sum / self.batch.n if self.batch.n else 0.0,
                "cache_hit_rate": self.cache_hits / acc if acc else 0.0,
                "queue_depth": {"high": self.queue_depth[0], "normal": self.queue_depth[1],
                                "low": self.queue_depth[2], "total": sum(self.queue_depth)},
                "workers": [dict(v, id=k) for k, v in sorted(self.workers.items())],
                "errors": dict(self.errors_total),
                "rejections": dict(self.rejected_total),
                "speculative": {"proposed": self.spec_proposed, "accepted": self.spec_accepted,
                                "acceptance_rate": self.spec_accepted / self.spec_proposed
                                if self.spec_proposed else 0.0, "speedup_factor": self.spec_speedup},
                "token_delivery_ms": _pcts(self._recent_delivery),
                "event_loop_lag_ms": _pcts(self._recent_loop_lag),
                "uptime_s": now - self.start,
            }

    # ---- Prometheus exposition ----------------------------------------------
    def prometheus(self) -> str:
        out: List[str] = []
        with self._lock:
            def counter(name, help_, samples):
                out.append(f"# HELP {name} {help_}")
                out.append(f"# TYPE {name} counter")
                for lab, v in samples:
                    out.append(f"{name}{_labels(lab)} {v}")

            def gauge(name, help_, samples):
                out.append(f"# HELP {name} {help_}")
                out.append(f"# TYPE {name} gauge")
                for lab, v in samples:
                    out.append(f"{name}{_labels(lab)} {v}")

            def hist(name, help_, items):
                out.append(f"# HELP {name} {help_}")
                out.append(f"# TYPE {name} histogram")
                for lab, h in items:
                    cum = 0
                    for b, c in zip(h.buckets, h.counts):
                        cum += c
                        out.append(f"{name}_bucket{_labels(dict(lab, le=repr(float(b))))} {cum}")
                    cum += h.counts[-1]
                    out.append(f"{name}_bucket{_labels(dict(lab, le='+Inf'))} {cum}")
                    out.append(f"{name}_sum{_labels(lab)} {h.sum}")
                    out.append(f"{name}_count{_labels(lab)} {h.n}")

            counter("xgs_requests_total", "HTTP requests by endpoint and status",
                    [({"endpoint": e, "status": str(s)}, n) for (e, s), n in sorted(self.requests_total.items())])
            hist("xgs_request_latency_seconds", "end-to-end request latency",
                 [({"endpoint": e, "status": str(s)}, h) for (e, s), h in sorted(self.latency.items())])
            gauge("xgs_requests_active", "requests in flight", [({}, self.requests_active)])
            hist("xgs_ttft_seconds", "time to first token", [({}, self.ttft)])
            hist("xgs_itl_seconds", "inter-token latency", [({}, self.itl)])
            hist("xgs_token_delivery_seconds", "token on host -> SSE event written (Req 5.1: <= 10 ms)",
                 [({}, self.delivery)])
            hist("xgs_batch_size", "sequences per engine step", [({}, self.batch)])
            counter("xgs_prompt_tokens_total", "prompt tokens processed", [({}, self.prompt_tokens_total)])
            counter("xgs_generation_tokens_total", "tokens generated", [({}, self.generation_tokens_total)])
            counter("xgs_errors_total", "errors by type", [({"type": k}, v) for k, v in sorted(self.errors_total.items())])
            counter("xgs_rejections_total", "admission rejections by reason",
                    [({"reason": k}, v) for k, v in sorted(self.rejected_total.items())])
            counter("xgs_prefix_cache_hit_tokens_total", "prefix-cache hit tokens", [({}, self.cache_hits)])
            counter("xgs_prefix_cache_miss_tokens_total", "prefix-cache miss tokens", [({}, self.cache_misses)])
            gauge("xgs_queue_depth", "admission queue depth by priority",
                  [({"priority": p}, v) for p, v in zip(("high", "normal", "low"), self.queue_depth)])
            gauge("xgs_worker_healthy", "replica health (1 healthy)",
                  [({"worker": str(k)}, int(bool(v.get("healthy", True)))) for k, v in sorted(self.workers.items())])
            gauge("xgs_worker_kv_usage", "replica KV-cache page usage",
                  [({"worker": str(k)}, v.get("kv_usage", 0.0)) for k, v in sorted(self.workers.items())])
            counter("xgs_spec_proposed_tokens_total", "draft tokens proposed", [({}, self.spec_proposed)])
            counter("xgs_spec_accepted_tokens_total", "draft tokens accepted", [({}, self.spec_accepted)])
            if self.spec_speedup is not None:
                gauge("xgs_spec_speedup_factor", "measured speculative-decoding speedup (tokens/s per sequence "
                      "with speculation / without)", [({}, self.spec_speedup)])
        return "\n".join(out) + "\n"
