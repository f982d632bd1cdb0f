"""KV-cache entry serialisation (Req 4.6, requirements.md:74; design.md:400-401;
Property 12 "deserialize(serialize(entry)) == entry").

A CacheEntry is a page-aligned token prefix plus its KV tensors in the
engine's paged layout, gathered into [L, 2, n_pages, Hkv, block_size, D].
Wire format (little endian):

    b"XGKV" | u32 version | u64 header_len | header JSON | raw tensor bytes

header = {key, token_count, dtype, shape, model, block_size, tp_rank}. The
payload is the tensor's raw memory (bf16/fp16/fp32), so a round trip is
bit-exact. `LLMEngine.export_prefix` / `import_prefix` move entries in and
out of the radix prefix cache (warm restarts, cross-replica prefix sharing).
"""
from __future__ import annotations

import json
import struct
from dataclasses import dataclass, field
from typing import List

import torch

from ..core.errors import CacheDeserialization, CacheSerialization

MAGIC = b"XGKV"
VERSION = 1
_DTYPES = {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32}


@dataclass
class CacheEntry:
    key: List[int]                 # the cached token prefix (page aligned)
    kv: torch.Tensor               # [L, 2, n_pages, Hkv, block_size, D]
    token_count: int
    model: str = ""
    block_size: int = 16
    tp_rank: int = 0
    meta: dict = field(default_factory=dict)

    def equivalent(self, other: "CacheEntry") -> bool:
        """Same key, token count and bit-identical KV."""
        if (self.key, self.token_count, self.model, self.block_size) != \
                (other.key, other.token_count, other.model, other.block_size):
            return False
        if self.kv.dtype != other.kv.dtype or self.kv.shape != other.kv.shape:
            return False
        a, b = self.kv.contiguous().cpu(), other.kv.contiguous().cpu()
        return a.numel() == 0 or torch.equal(a.view(torch.uint8), b.view(torch.uint8))


def serialize(e: CacheEntry) -> bytes:
    dt = str(e.kv.dtype).replace("torch.", "")
    if dt not in _DTYPES:
        raise CacheSerialization(f"unsupported dtype {dt}")
    if len(e.key) != e.token_count:
        raise CacheSerialization("token_count does not match key length")
    hdr = json.dumps({"key": list(map(int, e.key)), "token_count": int(e.token_count), "dtype": dt,
                      "shape": list(e.kv.shape), "model": e.model, "block_size": int(e.block_size),
                      "tp_rank": int(e.tp_rank), "meta": e.meta}, separators=(",", ":")).encode()
    t = e.kv.detach().contiguous().cpu()
    raw = t.view(torch.uint8).numpy().tobytes() if t.numel() else b""
    return MAGIC + struct.pack("<IQ", VERSION, len(hdr)) + hdr + raw


def deserialize(buf: bytes) -> CacheEntry:
    if len(buf) < 16 or buf[:4] != MAGIC:
        raise CacheDeserialization("bad magic")
    ver, hl = struct.unpack_from("<IQ", buf, 4)
    if ver != VERSION:
        raise CacheDeserialization(f"unsupported version {ver}")
    try:
        h = json.loads(buf[16:16 + hl])
        dtype = _DTYPES[h["dtype"]]
    except (ValueError, KeyError) as ex:
        raise CacheDeserialization(f"bad header: {ex}")
    shape = tuple(h["shape"])
    n = 1
    for s in shape:
        n *= s
    nbytes = n * torch.tensor([], dtype=dtype).element_size()
    raw = buf[16 + hl:]
    if len(raw) != nbytes:
        raise CacheDeserialization(f"payload is {len(raw)} bytes, expected {nbytes}")
    kv = torch.frombuffer(bytearray(raw), dtype=torch.uint8).view(dtype).reshape(shape) if n else \
        torch.empty(shape, dtype=dtype)
    return CacheEntry(h["key"], kv, h["token_count"], h.get("model", ""), h.get("block_size", 16),
                      h.get("tp_rank", 0), h.get("meta", {}))
