"""Error taxonomy.

Behavioural parity with the reference's `crates/core/src/error.rs`:

* ``ServerError``      -> error.rs:6-19   (startup / internal errors, exit != 0)
* ``ApiError``         -> error.rs:22-57  (HTTP status + ``type`` mapping)
* ``ValidationError``  -> error.rs:60-76  (exact Display strings)
* ``QueueError``, ``BatcherError``, ``CacheError``, ``WorkerError``,
  ``StreamError``      -> error.rs:79-141 (declared-but-unused in the reference;
  here each one is raised by a real failure path of the engine/server).

Display strings are byte-identical to the reference's ``#[error(...)]``
attributes so that clients see the same messages.
"""
from __future__ import annotations

from typing import Optional


# ---------------------------------------------------------------------------
# ServerError (error.rs:6-19)
# ---------------------------------------------------------------------------
class ServerError(Exception):
    kind = "server"

    def __init__(self, detail: str = ""):
        self.detail = detail
        super().__init__(self.display())

    def display(self) -> str:  # pragma: no cover - overridden
        return self.detail


class ConfigError(ServerError):
    kind = "config"

    def display(self) -> str:
        return f"Configuration error: {self.detail}"


class ModelLoadError(ServerError):
    kind = "model_load"

    def display(self) -> str:
        return f"Model load error: {self.detail}"


class WorkerServerError(ServerError):
    kind = "worker"

    def display(self) -> str:
        return f"Worker error: {self.detail}"


class IoServerError(ServerError):
    kind = "io"

    def display(self) -> str:
        return f"IO error: {self.detail}"


# ---------------------------------------------------------------------------
# ValidationError (error.rs:60-76)
# ---------------------------------------------------------------------------
class ValidationError(Exception):
    """One of: InvalidJson, MissingField, TokenLimitExceeded, InvalidParameter, EmptyPrompt."""

    def __init__(self, kind: str, message: str, *, field: Optional[str] = None,
                 reason: Optional[str] = None, actual: Optional[int] = None,
                 limit: Optional[int] = None):
        self.kind = kind
        self.field = field
        self.reason = reason
        self.actual = actual
        self.limit = limit
        self.message = message
        super().__init__(message)

    # constructors mirroring the Rust variants --------------------------------
    @classmethod
    def invalid_json(cls, detail: str) -> "ValidationError":
        return cls("invalid_json", f"Invalid JSON: {detail}")

    @classmethod
    def missing_field(cls, name: str) -> "ValidationError":
        return cls("missing_field", f"Missing required field: {name}", field=name)

    @classmethod
    def token_limit_exceeded(cls, actual: int, limit: int) -> "ValidationError":
        return cls("token_limit_exceeded",
                   f"Token limit exceeded: {actual} tokens > {limit} max",
                   actual=actual, limit=limit)

    @classmethod
    def invalid_parameter(cls, field: str, reason: str) -> "ValidationError":
        return cls("invalid_parameter", f"Invalid parameter '{field}': {reason}",
                   field=field, reason=reason)

    @classmethod
    def empty_prompt(cls) -> "ValidationError":
        return cls("empty_prompt", "Empty prompt not allowed")

    @property
    def code(self) -> str:
        return self.kind


# ---------------------------------------------------------------------------
# ApiError (error.rs:22-57)
# ---------------------------------------------------------------------------
class ApiError(Exception):
    status: int = 500
    error_type: str = "server_error"
    code: str = "internal_error"

    def __init__(self, message: str, *, code: Optional[str] = None,
                 retry_after: Optional[float] = None):
        self.message = message
        if code is not None:
            self.code = code
        self.retry_after = retry_after
        super().__init__(message)

    def status_code(self) -> int:
        return self.status

    def to_response(self) -> dict:
        # ErrorResponse / ErrorDetail (models.rs:230-261). We emit "type" per the
        # spec (design.md:637, requirements.md:157) rather than the impl's
        # "error_type" key -- see SURVEY.md 2.6.
        return {"error": {"message": self.message, "type": self.error_type,
                          "code": self.code}}


class ApiValidationError(ApiError):
    status = 400
    error_type = "invalid_request_error"

    def __init__(self, err: ValidationError):
        self.validation = err
        super().__init__(f"Validation error: {err.message}", code=err.kind)


class ApiQueueFull(ApiError):
    status = 503
    error_type = "rate_limit_error"
    code = "queue_full"

    def __init__(self, retry_after: float = 1.0):
        super().__init__("Queue full , server is overloaded", retry_after=retry_after)


class ApiTimeout(ApiError):
    status = 408
    error_type = "timeout_error"
    code = "timeout"

    def __init__(self):
        super().__init__("Request timeout")


class ApiInternal(ApiError):
    status = 500
    error_type = "server_error"
    code = "internal_error"

    def __init__(self, detail: str, code: str = "internal_error"):
        super().__init__(f"Internal server error: {detail}", code=code)


class ApiNotFound(ApiError):
    status = 404
    error_type = "invalid_request_error"
    code = "not_found"

    def __init__(self, what: str):
        super().__init__(f"Not found: {what}")


# ---------------------------------------------------------------------------
# Component errors (error.rs:79-141)
# ---------------------------------------------------------------------------
class QueueError(Exception):
    pass


class QueueFull(QueueError):
    def __init__(self):
        super().__init__("Queue is full")


class QueueNotFound(QueueError):
    def __init__(self, rid: str):
        super().__init__(f"Request not found: {rid}")


class QueueCancelled(QueueError):
    def __init__(self):
        super().__init__("Request cancelled")


class BatcherError(Exception):
    pass


class BatcherTimeout(BatcherError):
    def __init__(self):
        super().__init__("Batch timeout")


class BatcherChannelClosed(BatcherError):
    def __init__(self):
        super().__init__("Channel closed")


class CacheError(Exception):
    pass


class CacheSerialization(CacheError):
    def __init__(self, d: str):
        super().__init__(f"Serialization error: {d}")


class CacheDeserialization(CacheError):
    def __init__(self, d: str):
        super().__init__(f"Deserialization error: {d}")


class CacheFull(CacheError):
    def __init__(self):
        super().__init__("Cache full")


class WorkerError(Exception):
    code = "worker_error"


class WorkerModelNotLoaded(WorkerError):
    code = "model_not_loaded"

    def __init__(self):
        super().__init__("Model not loaded")


class WorkerInferenceFailed(WorkerError):
    code = "inference_failed"

    def __init__(self, d: str):
        super().__init__(f"Inference failed: {d}")


class WorkerShutdown(WorkerError):
    code = "worker_shutdown"

    def __init__(self):
        super().__init__("Worker shutdown")


class WorkerOutOfMemory(WorkerError):
    code = "out_of_memory"

    def __init__(self):
        super().__init__("Out of memory")


class StreamError(Exception):
    pass


class StreamClientDisconnected(StreamError):
    def __init__(self):
        super().__init__("Client disconnected")


class StreamNotFound(StreamError):
    def __init__(self, d: str):
        super().__init__(f"Stream not found: {d}")


class StreamSendFailed(StreamError):
    def __init__(self):
        super().__init__("Send failed")
