"""Server configuration: one dataclass tree with the reference's component
defaults, loaded with precedence  file < environment < CLI  (Req 10.1,
requirements.md:142), validated as a whole (Req 10.4: every error is reported,
startup exits non-zero), and partially hot-reloadable (Req 10.5: batch limits,
queue thresholds, scheduling strategy).

Defaults mirror the reference: QueueConfig (queue.rs:24-33), ValidatorConfig
(validator.rs:17-28), ApiConfig (design.md:131-136), BatcherConfig
(design.md:233-238, 50 ms / 32), SchedulerConfig (design.md:283-287),
WorkerConfig (design.md:316-322), CacheConfig (design.md:369-373, 0.8).

File formats: JSON, YAML (SafeLoader), or a flat TOML subset
([section] + key = value). Environment: XGS_<SECTION>__<KEY>=value, e.g.
XGS_QUEUE__HIGH_WATERMARK=800. CLI: --set section.key=value (repeatable) plus
the common shortcuts of xgserve.cli.
"""
from __future__ import annotations

import copy
import dataclasses
import json
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, List, Optional

from ..core.errors import ConfigError


@dataclass
class ApiConfig:
    host: str = "127.0.0.1"
    port: int = 8000
    grpc_addr: Optional[str] = None
    max_request_size: int = 4 * 1024 * 1024
    request_timeout_s: float = 300.0
    # HTTP front-end processes (SO_REUSEPORT) over the one orchestrator process;
    # 1 = HTTP on the orchestrator's own event loop (server/frontend.py); 0 = auto:
    # 2 when GPU process replicas serve (one replica's ~10k token events/s: delivery
    # p99 12.4 ms on one loop, 6.9 ms on two, profiles/r3_frontend.md), else 1
    frontends: int = 0

    def resolved_frontends(self, worker) -> int:
        if self.frontends > 0:
            return self.frontends
        gpu = not worker.mock and not worker.in_process and (worker.device or "cuda") != "cpu"
        return 2 if gpu else 1


@dataclass
class QueueSection:
    high_watermark: int = 1000
    low_watermark: int = 500
    request_timeout_s: float = 30.0
    max_queue_size: int = 2000
    aging_s: float = 0.0
    retry_after_s: float = 1.0


@dataclass
class ValidatorSection:
    max_context_tokens: int = 8192
    max_output_tokens: int = 4096
    min_temperature: float = 0.0
    max_temperature: float = 2.0
    min_top_p: float = 0.0
    max_top_p: float = 1.0


@dataclass
class BatcherSection:
    mode: str = "continuous"          # continuous | static
    max_batch_size: int = 32
    batch_timeout_ms: float = 50.0
    max_sequence_length: int = 8192
    padding_token_id: int = 0
    # continuous mode: admission window over prompt admission (1: off); see
    # EngineConfig.prompt_coalesce
    coalesce_prompts: int = 1
    coalesce_max_wait_steps: int = 4


@dataclass
class SchedulerSection:
    strategy: str = "least_loaded"    # round_robin | least_loaded | memory_aware
    health_check_interval_s: float = 1.0
    heartbeat_timeout_s: float = 5.0
    max_inflight_per_replica: int = 512
    restart_failed: bool = True
    max_restarts: int = 3


@dataclass
class WorkerSection:
    model: str = "llama3-8b"
    checkpoint: Optional[str] = None
    random_init: bool = True
    replicas: int = 1                 # data-parallel replicas
    tp: int = 1                       # tensor-parallel degree per replica
    gpus: Optional[str] = None        # e.g. "0,1,2,3"; default 0..replicas*tp-1
    device: Optional[str] = None      # "cpu" forces the CPU path
    # bf16 | fp16 | fp32 | fp8 | int8 | int4: fp8 (E4M3, per-channel scale), int8 (per-channel)
    # and int4 (per 128-k group scales) are weight-only copies for decode batches <= 64,
    # bf16 activations (Req 10.3; the reference's Q8_0 / Q4_0 levels)
    quantization: str = "bf16"
    block_size: int = 16
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    max_model_len: Optional[int] = None
    gpu_memory_utilization: float = 0.90
    num_blocks: Optional[int] = None
    use_graphs: bool = True
    in_process: bool = False          # run the engine in a thread of the server process
    mock: bool = False                # deterministic MockEngine (tests / plumbing)
    mock_latency_ms: float = 1.0
    mock_kv_seqs: int = 0             # mock KV capacity in sequences (memory pressure model; 0 = max_num_seqs)
    moe_comm: str = "auto"
    seed: int = 0


@dataclass
class CacheSection:
    enable_prefix_cache: bool = True
    memory_threshold: float = 0.8
    ttl_s: Optional[float] = None


@dataclass
class DegradationSection:
    reduce_batch_at: float = 0.70
    aggressive_evict_at: float = 0.80
    reject_low_priority_at: float = 0.90
    emergency_at: float = 0.95


@dataclass
class SpecSection:
    draft_model: Optional[str] = None
    num_speculative_tokens: int = 0
    min_acceptance_rate: float = 0.5


@dataclass
class ObservabilitySection:
    metrics: bool = True
    tracing: bool = True
    trace_sample_rate: float = 1.0
    log_level: str = "INFO"
    otel_endpoint: Optional[str] = None


@dataclass
class ServerConfig:
    api: ApiConfig = field(default_factory=ApiConfig)
    queue: QueueSection = field(default_factory=QueueSection)
    validator: ValidatorSection = field(default_factory=ValidatorSection)
    batcher: BatcherSection = field(default_factory=BatcherSection)
    scheduler: SchedulerSection = field(default_factory=SchedulerSection)
    worker: WorkerSection = field(default_factory=WorkerSection)
    cache: CacheSection = field(default_factory=CacheSection)
    degradation: DegradationSection = field(default_factory=DegradationSection)
    spec: SpecSection = field(default_factory=SpecSection)
    observability: ObservabilitySection = field(default_factory=ObservabilitySection)

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    def validate(self) -> List[str]:
        e: List[str] = []
        q = self.queue
        if q.high_watermark <= 0:
            e.append("queue.high_watermark must be > 0")
        if q.low_watermark < 0 or q.low_watermark > q.high_watermark:
            e.append("queue.low_watermark must be in [0, high_watermark]")
        if q.max_queue_size < q.high_watermark:
            e.append("queue.max_queue_size must be >= high_watermark")
        if q.request_timeout_s <= 0:
            e.append("queue.request_timeout_s must be > 0")
        v = self.validator
        if v.max_context_tokens <= 0 or v.max_output_tokens <= 0:
            e.append("validator token limits must be > 0")
        if v.min_temperature > v.max_temperature or v.min_top_p > v.max_top_p:
            e.append("validator ranges must satisfy min <= max")
        if self.api.frontends < 0:
            e.append("api.frontends must be >= 0 (0: auto)")
        b = self.batcher
        if b.mode not in ("continuous", "static"):
            e.append(f"batcher.mode must be continuous|static, got {b.mode!r}")
        if b.max_batch_size <= 0:
            e.append("batcher.max_batch_size must be > 0")
        if b.batch_timeout_ms < 0:
            e.append("batcher.batch_timeout_ms must be >= 0")
        if b.coalesce_prompts < 1 or b.coalesce_max_wait_steps < 0:
            e.append("batcher.coalesce_prompts must be >= 1 and batcher.coalesce_max_wait_steps >= 0")
        s = self.scheduler
        if s.strategy not in ("round_robin", "least_loaded", "memory_aware"):
            e.append(f"scheduler.strategy must be round_robin|least_loaded|memory_aware, got {s.strategy!r}")
        if s.health_check_interval_s <= 0:
            e.append("scheduler.health_check_interval_s must be > 0")
        w = self.worker
        if w.replicas <= 0 or w.tp <= 0:
            e.append("worker.replicas and worker.tp must be > 0")
        if w.quantization not in ("bf16", "fp16", "fp32", "fp8", "int8", "int4"):
            e.append(f"worker.quantization {w.quantization!r} not supported (bf16|fp16|fp32|fp8|int8|int4)")
        if not (0.0 < w.gpu_memory_utilization <= 1.0):
            e.append("worker.gpu_memory_utilization must be in (0, 1]")
        if w.block_size % 16:
            e.append("worker.block_size must be a multiple of 16")
        if not w.mock and not w.random_init and not w.checkpoint:
            e.append("worker.checkpoint is required unless random_init or mock")
        if w.checkpoint and w.checkpoint.startswith(("http://", "https://")) and not w.mock:
            e.append(f"worker.checkpoint {w.checkpoint!r}: remote checkpoints are fetched by load_config")
        elif w.checkpoint and not w.checkpoint.startswith(("http://", "https://")) and not os.path.isdir(w.checkpoint):
            e.append(f"worker.checkpoint {w.checkpoint!r} is not a directory")
        if not w.mock:
            try:
                from ..models.config import get_config
                get_config(w.checkpoint or w.model)
            except KeyError as ex:
                e.append(str(ex))
        c = self.cache
        if not (0.0 < c.memory_threshold <= 1.0):
            e.append("cache.memory_threshold must be in (0, 1]")
        d = self.degradation
        if not (0 < d.reduce_batch_at <= d.aggressive_evict_at <= d.reject_low_priority_at <= d.emergency_at <= 1):
            e.append("degradation thresholds must be increasing in (0, 1]")
        if self.spec.num_speculative_tokens < 0:
            e.append("spec.num_speculative_tokens must be >= 0")
        return e


HOT_RELOADABLE = {
    "queue": {"high_watermark", "low_watermark", "request_timeout_s", "max_queue_size", "aging_s"},
    "batcher": {"max_batch_size", "batch_timeout_ms"},
    "scheduler": {"strategy", "health_check_interval_s"},
    "worker": {"max_num_seqs", "max_num_batched_tokens"},
    "validator": {"max_context_tokens", "max_output_tokens"},
}


def _base_type(typ) -> tuple:
    """(base type name, optional) for a dataclass field annotation (a string under
    `from __future__ import annotations`)."""
    tname = typ if isinstance(typ, str) else getattr(typ, "__name__", str(typ))
    tname = tname.replace("typing.", "")
    optional = tname.startswith("Optional[")
    if optional:
        tname = tname[len("Optional["):-1]
    return tname, optional


def _coerce(value: Any, typ) -> Any:
    base, optional = _base_type(typ)
    if value is None:
        if optional:
            return None
        raise ValueError("null is not allowed")
    if isinstance(value, str):
        s = value.strip()
        if optional and s.lower() in ("none", "null"):
            return None
        if base == "bool":
            if s.lower() in ("1", "true", "yes", "on"):
                return True
            if s.lower() in ("0", "false", "no", "off"):
                return False
            raise ValueError(f"not a boolean: {value!r}")
        if base == "int":
            return int(s)
        if base == "float":
            return float(s)
        return s
    if base == "bool" and not isinstance(value, bool):
        raise ValueError(f"not a boolean: {value!r}")
    if base == "int" and (isinstance(value, bool) or not isinstance(value, int)):
        if isinstance(value, float) and value.is_integer():
            return int(value)
        raise ValueError(f"not an integer: {value!r}")
    if base == "float":
        if isinstance(value, bool) or not isinstance(value, (int, float)):
            raise ValueError(f"not a number: {value!r}")
        return float(value)
    if base == "str" and not isinstance(value, str):
        return str(value)
    return value


def _set(cfg: ServerConfig, section: str, key: str, value: Any, errors: List[str], src: str):
    sec = getattr(cfg, section, None)
    if sec is None or not dataclasses.is_dataclass(sec):
        errors.append(f"{src}: unknown section {section!r}")
        return
    fmap = {f.name: f for f in fields(sec)}
    if key not in fmap:
        errors.append(f"{src}: unknown key {section}.{key}")
        return
    try:
        setattr(sec, key, _coerce(value, fmap[key].type))
    except (TypeError, ValueError) as ex:
        errors.append(f"{src}: invalid value for {section}.{key}: {ex}")


def _parse_toml_lite(text: str) -> Dict[str, Dict[str, Any]]:
    out: Dict[str, Dict[str, Any]] = {}
    sec = None
    for ln, line in enumerate(text.splitlines(), 1):
        s = line.split("#", 1)[0].strip()
        if not s:
            continue
        if s.startswith("[") and s.endswith("]"):
            sec = s[1:-1].strip()
            out.setdefault(sec, {})
            continue
        if "=" not in s or sec is None:
            raise ValueError(f"line {ln}: expected key = value inside a [section]")
        k, v = (x.strip() for x in s.split("=", 1))
        if v.startswith(('"', "'")):
            v = v[1:-1]
        elif v.lower() in ("true", "false"):
            v = v.lower() == "true"
        else:
            try:
                v = int(v)
            except ValueError:
                try:
                    v = float(v)
                except ValueError:
                    pass
        out[sec][k] = v
    return out


def load_file(path: str) -> Dict[str, Dict[str, Any]]:
    with open(path) as f:
        text = f.read()
    if path.endswith(".json"):
        return json.loads(text)
    if path.endswith((".yaml", ".yml")):
        import yaml
        return yaml.load(text, Loader=yaml.SafeLoader) or {}
    return _parse_toml_lite(text)


def load_config(file: Optional[str] = None, env: Optional[Dict[str, str]] = None,
                cli: Optional[List[str]] = None, overrides: Optional[Dict[str, Dict[str, Any]]] = None) -> ServerConfig:
    """file < env < cli < overrides. Raises ConfigError listing every problem."""
    cfg = ServerConfig()
    errors: List[str] = []
    if file:
        try:
            data = load_file(file)
            for sec, kv in (data or {}).items():
                if not isinstance(kv, dict):
                    errors.append(f"file: section {sec!r} must be a table")
                    continue
                for k, v in kv.items():
                    _set(cfg, sec, k, v, errors, "file")
        except (OSError, ValueError) as ex:
            errors.append(f"file {file}: {ex}")
    env = os.environ if env is None else env
    for k, v in env.items():
        if not k.startswith("XGS_") or "__" not in k:
            continue
        sec, key = k[4:].split("__", 1)
        _set(cfg, sec.lower(), key.lower(), v, errors, f"env {k}")
    for item in cli or []:
        if "=" not in item or "." not in item.split("=", 1)[0]:
            errors.append(f"cli: expected section.key=value, got {item!r}")
            continue
        lhs, v = item.split("=", 1)
        sec, key = lhs.split(".", 1)
        _set(cfg, sec, key, v, errors, "cli")
    for sec, kv in (overrides or {}).items():
        for k, v in kv.items():
            if v is not None:
                _set(cfg, sec, k, v, errors, "cli")
    w = cfg.worker
    if not errors and not w.mock and w.checkpoint and w.checkpoint.startswith(("http://", "https://")):
        # Req 10.2: a remote checkpoint directory is fetched once into the local cache
        # and loaded from there; an unreachable URL is a configuration error (exit != 0)
        from ..models.fetch import FetchError, fetch_checkpoint
        try:
            w.checkpoint = fetch_checkpoint(w.checkpoint)
        except FetchError as ex:
            errors.append(f"worker.checkpoint: cannot fetch {w.checkpoint}: {ex}")
    errors += cfg.validate()
    if errors:
        raise ConfigError("; ".join(errors))
    return cfg


def apply_hot_reload(cfg: ServerConfig, patch: Dict[str, Dict[str, Any]]) -> ServerConfig:
    """Return a new config with `patch` applied; only HOT_RELOADABLE keys are accepted."""
    new = copy.deepcopy(cfg)
    errors: List[str] = []
    for sec, kv in patch.items():
        allowed = HOT_RELOADABLE.get(sec, set())
        for k, v in kv.items():
            if k not in allowed:
                errors.append(f"{sec}.{k} is not hot-reloadable")
                continue
            _set(new, sec, k, v, errors, "reload")
    errors += new.validate()
    if errors:
        raise ConfigError("; ".join(errors))
    return new
