"""Wire models: requests, responses, SSE events.

Parity target: reference `crates/core/src/models.rs` (serde structs).

Request parsing reproduces serde_json's strictness (models.rs:55-139):
  * required fields: ``prompt`` (generate), ``messages`` (chat), ``input``
    (embeddings); missing -> ``ValidationError.missing_field``.
  * ``usize`` fields accept only non-negative JSON integers (no floats, no
    bools, no strings); ``f32`` fields accept any JSON number (ints too) and are
    rounded to float32 exactly like serde does; ``bool`` accepts only bools.
  * unknown fields are ignored (serde default).
  * defaults: max_tokens=256, temperature=1.0, top_p=1.0, stop_sequences=[],
    stream=false, priority=None (models.rs:294-322).

Responses serialise to exactly the reference's JSON shapes (models.rs:146-223),
except two documented spec fixes: ErrorDetail emits ``type``
(not ``error_type``) and the SSE error event emits ``message`` (not ``messages``).
Both keys are still accepted when *parsing*.
"""
from __future__ import annotations

import enum
import json
import struct
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Union

from .errors import ValidationError
from .types import Priority, new_request_id

DEFAULT_MAX_TOKENS = 256
DEFAULT_TEMPERATURE = 1.0
DEFAULT_TOP_P = 1.0


def _f32(x: float) -> float:
    """Round a Python float to IEEE float32 (serde parses into f32)."""
    return struct.unpack("f", struct.pack("f", x))[0] if x == x and abs(x) < 3.5e38 else float(x)


# ---------------------------------------------------------------------------
# Small enums (models.rs:8-48)
# ---------------------------------------------------------------------------
@dataclass
class Usage:
    prompt_tokens: int = 0
    completion_tokens: int = 0
    total_tokens: int = 0

    @classmethod
    def new(cls, prompt_tokens: int, completion_tokens: int) -> "Usage":
        return cls(prompt_tokens, completion_tokens, prompt_tokens + completion_tokens)

    def to_dict(self) -> dict:
        return {"prompt_tokens": self.prompt_tokens,
                "completion_tokens": self.completion_tokens,
                "total_tokens": self.total_tokens}

    @classmethod
    def from_dict(cls, d: dict) -> "Usage":
        return cls(_req_usize(d, "prompt_tokens"), _req_usize(d, "completion_tokens"),
                   _req_usize(d, "total_tokens"))


class FinishReason(str, enum.Enum):
    Stop = "stop"
    Length = "length"
    StopSequence = "stop_sequence"


class Role(str, enum.Enum):
    System = "system"
    User = "user"
    Assistant = "assistant"


@dataclass
class ChatMessage:
    role: Role
    content: str

    def to_dict(self) -> dict:
        return {"role": self.role.value, "content": self.content}

    @classmethod
    def from_dict(cls, d: Any) -> "ChatMessage":
        if not isinstance(d, dict):
            raise ValidationError.invalid_json("invalid type: expected struct ChatMessage")
        if "role" not in d:
            raise ValidationError.missing_field("role")
        if "content" not in d:
            raise ValidationError.missing_field("content")
        try:
            role = Role(d["role"])
        except ValueError:
            raise ValidationError.invalid_json(
                f"unknown variant `{d['role']}`, expected one of `system`, `user`, `assistant`")
        return cls(role, _str(d["content"], "content"))


# ---------------------------------------------------------------------------
# strict field helpers (serde_json semantics)
# ---------------------------------------------------------------------------
def _str(v: Any, name: str) -> str:
    if not isinstance(v, str):
        raise ValidationError.invalid_json(f"invalid type for `{name}`: expected a string")
    return v


def _usize(v: Any, name: str) -> int:
    if isinstance(v, bool) or not isinstance(v, int) or v < 0 or v > 2**64 - 1:
        raise ValidationError.invalid_json(
            f"invalid value for `{name}`: expected usize (a non-negative integer)")
    return v


def _req_usize(d: dict, name: str) -> int:
    if name not in d:
        raise ValidationError.missing_field(name)
    return _usize(d[name], name)


def _f32_field(v: Any, name: str) -> float:
    if isinstance(v, bool) or not isinstance(v, (int, float)):
        raise ValidationError.invalid_json(f"invalid type for `{name}`: expected f32")
    return _f32(float(v))


def _bool(v: Any, name: str) -> bool:
    if not isinstance(v, bool):
        raise ValidationError.invalid_json(f"invalid type for `{name}`: expected a boolean")
    return v


def _str_list(v: Any, name: str) -> List[str]:
    if not isinstance(v, list) or not all(isinstance(s, str) for s in v):
        raise ValidationError.invalid_json(f"invalid type for `{name}`: expected a sequence of strings")
    return list(v)


def _obj(body: Union[bytes, str, dict]) -> dict:
    if isinstance(body, dict):
        return body
    try:
        d = json.loads(body)
    except (ValueError, UnicodeDecodeError) as e:
        raise ValidationError.invalid_json(str(e))
    if not isinstance(d, dict):
        raise ValidationError.invalid_json("invalid type: expected a JSON object")
    return d


def _sampling(d: dict) -> dict:
    return {
        "max_tokens": _usize(d["max_tokens"], "max_tokens") if "max_tokens" in d else DEFAULT_MAX_TOKENS,
        "temperature": _f32_field(d["temperature"], "temperature") if "temperature" in d else DEFAULT_TEMPERATURE,
        "top_p": _f32_field(d["top_p"], "top_p") if "top_p" in d else DEFAULT_TOP_P,
        "stop_sequences": _str_list(d["stop_sequences"], "stop_sequences") if "stop_sequences" in d else [],
        "stream": _bool(d["stream"], "stream") if "stream" in d else False,
    }


# ---------------------------------------------------------------------------
# Requests (models.rs:55-139)
# ---------------------------------------------------------------------------
@dataclass
class GenerateRequest:
    prompt: str = ""
    max_tokens: int = DEFAULT_MAX_TOKENS
    temperature: float = DEFAULT_TEMPERATURE
    top_p: float = DEFAULT_TOP_P
    stop_sequences: List[str] = field(default_factory=list)
    stream: bool = False
    priority: Optional[Priority] = None
    # extensions (not in the reference wire format; ignored by it)
    seed: Optional[int] = None
    logprobs: bool = False
    ignore_eos: bool = False

    @classmethod
    def parse(cls, body: Union[bytes, str, dict]) -> "GenerateRequest":
        d = _obj(body)
        if "prompt" not in d:
            raise ValidationError.missing_field("prompt")
        prompt = _str(d["prompt"], "prompt")
        s = _sampling(d)
        pr = d.get("priority", None)
        if pr is not None:
            try:
                pr = Priority.parse(pr)
            except ValueError as e:
                raise ValidationError.invalid_json(str(e))
        return cls(prompt=prompt, priority=pr, seed=_opt_int(d, "seed"),
                   logprobs=bool(d.get("logprobs", False)) if isinstance(d.get("logprobs", False), bool) else False,
                   ignore_eos=d.get("ignore_eos") is True, **s)


def _opt_int(d: dict, name: str) -> Optional[int]:
    v = d.get(name)
    if v is None:
        return None
    return _usize(v, name)


@dataclass
class ChatRequest:
    messages: List[ChatMessage] = field(default_factory=list)
    max_tokens: int = DEFAULT_MAX_TOKENS
    temperature: float = DEFAULT_TEMPERATURE
    top_p: float = DEFAULT_TOP_P
    stop_sequences: List[str] = field(default_factory=list)
    stream: bool = False
    seed: Optional[int] = None
    ignore_eos: bool = False

    @classmethod
    def parse(cls, body: Union[bytes, str, dict]) -> "ChatRequest":
        d = _obj(body)
        if "messages" not in d:
            raise ValidationError.missing_field("messages")
        if not isinstance(d["messages"], list):
            raise ValidationError.invalid_json("invalid type for `messages`: expected a sequence")
        msgs = [ChatMessage.from_dict(m) for m in d["messages"]]
        return cls(messages=msgs, seed=_opt_int(d, "seed"), ignore_eos=d.get("ignore_eos") is True,
                   **_sampling(d))


@dataclass
class EmbeddingsRequest:
    input: Union[str, List[str]] = ""
    model: Optional[str] = None

    @classmethod
    def parse(cls, body: Union[bytes, str, dict]) -> "EmbeddingsRequest":
        d = _obj(body)
        if "input" not in d:
            raise ValidationError.missing_field("input")
        inp = d["input"]
        # serde(untagged): a string or an array of strings (models.rs:127-131)
        if isinstance(inp, str):
            pass
        elif isinstance(inp, list) and all(isinstance(s, str) for s in inp):
            inp = list(inp)
        else:
            raise ValidationError.invalid_json(
                "data did not match any variant of untagged enum EmbeddingsInput")
        model = d.get("model")
        if model is not None and not isinstance(model, str):
            raise ValidationError.invalid_json("invalid type for `model`: expected a string")
        return cls(input=inp, model=model)

    def into_vec(self) -> List[str]:
        return [self.input] if isinstance(self.input, str) else list(self.input)


# ---------------------------------------------------------------------------
# Responses (models.rs:146-223)
# ---------------------------------------------------------------------------
def _now() -> int:
    return int(time.time())


@dataclass
class GenerateChoice:
    text: str
    index: int
    finish_reason: FinishReason

    def to_dict(self) -> dict:
        return {"text": self.text, "index": self.index, "finish_reason": self.finish_reason.value}

    @classmethod
    def from_dict(cls, d: dict) -> "GenerateChoice":
        return cls(d["text"], d["index"], FinishReason(d["finish_reason"]))


@dataclass
class GenerateResponse:
    id: str
    object: str
    created: int
    model: str
    choices: List[GenerateChoice]
    usage: Usage

    @classmethod
    def build(cls, model: str, choices: List[GenerateChoice], usage: Usage,
              rid: Optional[str] = None) -> "GenerateResponse":
        return cls(rid or new_request_id(), "text_completion", _now(), model, choices, usage)

    def to_dict(self) -> dict:
        return {"id": self.id, "object": self.object, "created": self.created,
                "model": self.model, "choices": [c.to_dict() for c in self.choices],
                "usage": self.usage.to_dict()}

    @classmethod
    def from_dict(cls, d: dict) -> "GenerateResponse":
        return cls(d["id"], d["object"], d["created"], d["model"],
                   [GenerateChoice.from_dict(c) for c in d["choices"]], Usage.from_dict(d["usage"]))


@dataclass
class ChatChoice:
    index: int
    message: ChatMessage
    finish_reason: FinishReason

    def to_dict(self) -> dict:
        return {"index": self.index, "message": self.message.to_dict(),
                "finish_reason": self.finish_reason.value}

    @classmethod
    def from_dict(cls, d: dict) -> "ChatChoice":
        return cls(d["index"], ChatMessage.from_dict(d["message"]), FinishReason(d["finish_reason"]))


@dataclass
class ChatResponse:
    id: str
    object: str
    created: int
    model: str
    choices: List[ChatChoice]
    usage: Usage

    @classmethod
    def build(cls, model: str, choices: List[ChatChoice], usage: Usage,
              rid: Optional[str] = None) -> "ChatResponse":
        return cls(rid or new_request_id(), "chat.completion", _now(), model, choices, usage)

    def to_dict(self) -> dict:
        return {"id": self.id, "object": self.object, "created": self.created,
                "model": self.model, "choices": [c.to_dict() for c in self.choices],
                "usage": self.usage.to_dict()}

    @classmethod
    def from_dict(cls, d: dict) -> "ChatResponse":
        return cls(d["id"], d["object"], d["created"], d["model"],
                   [ChatChoice.from_dict(c) for c in d["choices"]], Usage.from_dict(d["usage"]))


@dataclass
class EmbeddingData:
    embedding: List[float]
    index: int
    object: str = "embedding"

    def to_dict(self) -> dict:
        return {"object": self.object, "embedding": list(self.embedding), "index": self.index}

    @classmethod
    def from_dict(cls, d: dict) -> "EmbeddingData":
        return cls(list(d["embedding"]), d["index"], d["object"])


@dataclass
class EmbeddingsResponse:
    data: List[EmbeddingData]
    model: str
    usage: Usage
    object: str = "list"

    def to_dict(self) -> dict:
        return {"object": self.object, "data": [e.to_dict() for e in self.data],
                "model": self.model, "usage": self.usage.to_dict()}

    @classmethod
    def from_dict(cls, d: dict) -> "EmbeddingsResponse":
        return cls([EmbeddingData.from_dict(e) for e in d["data"]], d["model"],
                   Usage.from_dict(d["usage"]), d["object"])


@dataclass
class ErrorDetail:
    message: str
    type: str
    code: str


@dataclass
class ErrorResponse:
    error: ErrorDetail

    @classmethod
    def new(cls, message: str, error_type: str, code: str) -> "ErrorResponse":
        return cls(ErrorDetail(message, error_type, code))

    def to_dict(self) -> dict:
        return {"error": {"message": self.error.message, "type": self.error.type,
                          "code": self.error.code}}

    @classmethod
    def from_dict(cls, d: dict) -> "ErrorResponse":
        e = d["error"]
        t = e["type"] if "type" in e else e["error_type"]
        return cls(ErrorDetail(e["message"], t, e["code"]))


# ---------------------------------------------------------------------------
# Streaming (models.rs:268-288)
# ---------------------------------------------------------------------------
@dataclass
class TokenEvent:
    """Internally tagged union: type in {token, done, error}."""
    type: str
    token: Optional[str] = None
    index: Optional[int] = None
    logprob: Optional[float] = None
    finish_reason: Optional[FinishReason] = None
    usage: Optional[Usage] = None
    message: Optional[str] = None
    code: Optional[str] = None

    @classmethod
    def tok(cls, token: str, index: int, logprob: Optional[float] = None) -> "TokenEvent":
        return cls("token", token=token, index=index, logprob=logprob)

    @classmethod
    def done(cls, finish_reason: FinishReason, usage: Usage) -> "TokenEvent":
        return cls("done", finish_reason=finish_reason, usage=usage)

    @classmethod
    def error(cls, message: str, code: str) -> "TokenEvent":
        return cls("error", message=message, code=code)

    def to_dict(self) -> dict:
        if self.type == "token":
            d = {"type": "token", "token": self.token, "index": self.index}
            if self.logprob is not None:  # skip_serializing_if = "Option::is_none"
                d["logprob"] = self.logprob
            return d
        if self.type == "done":
            return {"type": "done", "finish_reason": self.finish_reason.value,
                    "usage": self.usage.to_dict()}
        return {"type": "error", "message": self.message, "code": self.code}

    @classmethod
    def from_dict(cls, d: dict) -> "TokenEvent":
        t = d["type"]
        if t == "token":
            return cls.tok(d["token"], d["index"], d.get("logprob"))
        if t == "done":
            return cls.done(FinishReason(d["finish_reason"]), Usage.from_dict(d["usage"]))
        if t == "error":
            return cls.error(d.get("message", d.get("messages")), d["code"])
        raise ValueError(f"unknown TokenEvent type {t!r}")

    def sse(self) -> bytes:
        return b"data: " + json.dumps(self.to_dict(), separators=(",", ":")).encode() + b"\n\n"
