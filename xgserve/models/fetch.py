"""Remote checkpoints (Req 10.2, `requirements.md:143`): `worker.checkpoint` may be
an http(s):// URL of a checkpoint DIRECTORY in the HF layout. It is fetched once,
with the standard library only, into a local cache directory and the server then
loads the local copy like any other checkpoint:

  <url>/config.json                                   required
  <url>/model.safetensors                             one file, or
  <url>/model.safetensors.index.json + its shards     a sharded checkpoint
  <url>/tokenizer.json                                optional

Each file is streamed to `<name>.part` and renamed when its byte count matches the
response's Content-Length, and a `.complete` marker written last makes a later
start skip the download. A URL that cannot be fetched is a configuration error
with the reason (the server then exits != 0, Req 10.4) instead of a crash at load.

Cache: $XGS_CHECKPOINT_CACHE, default ~/.cache/xgserve/checkpoints, one directory
per URL (sha256 prefix of the URL).
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import urllib.error
import urllib.parse
import urllib.request
from typing import List, Optional

CHUNK = 8 << 20


class FetchError(RuntimeError):
    def __init__(self, msg: str, status: Optional[int] = None):
        super().__init__(msg)
        self.status = status  # the HTTP status when the server answered with an error


def is_url(spec: Optional[str]) -> bool:
    return bool(spec) and spec.startswith(("http://", "https://"))


def cache_root() -> str:
    return os.environ.get("XGS_CHECKPOINT_CACHE", os.path.join(os.path.expanduser("~"), ".cache", "xgserve",
                                                               "checkpoints"))


def _join(base: str, name: str) -> str:
    return base.rstrip("/") + "/" + urllib.parse.quote(name)


def _get(url: str, dest: str, timeout: float) -> int:
    tmp = dest + ".part"
    try:
        try:
            with urllib.request.urlopen(url, timeout=timeout) as r:  # noqa: S310 - http(s) only (is_url)
                want = r.headers.get("Content-Length")
                n = 0
                with open(tmp, "wb") as f:
                    while True:
                        b = r.read(CHUNK)
                        if not b:
                            break
                        f.write(b)
                        n += len(b)
        except urllib.error.HTTPError as e:
            raise FetchError(f"{url}: HTTP {e.code} {e.reason}", status=e.code) from None
        except (urllib.error.URLError, OSError, ValueError) as e:
            raise FetchError(f"{url}: {getattr(e, 'reason', e)}") from None
        if want is not None and int(want) != n:
            raise FetchError(f"{url}: truncated ({n} of {want} bytes)")
    except FetchError:
        try:  # a failed download leaves no partial file behind
            os.remove(tmp)
        except OSError:
            pass
        raise
    os.replace(tmp, dest)
    return n


def fetch_checkpoint(url: str, root: Optional[str] = None, timeout: float = 60.0) -> str:
    """Download the checkpoint directory at `url` (if not cached) and return the
    local directory. Raises FetchError with the reason on any failure."""
    if not is_url(url):
        raise FetchError(f"not an http(s) URL: {url!r}")
    root = root or cache_root()
    d = os.path.join(root, hashlib.sha256(url.encode()).hexdigest()[:16])
    if os.path.exists(os.path.join(d, ".complete")):
        return d
    os.makedirs(d, exist_ok=True)
    files: List[str] = ["config.json"]
    _get(_join(url, "config.json"), os.path.join(d, "config.json"), timeout)
    try:
        _get(_join(url, "model.safetensors.index.json"), os.path.join(d, "model.safetensors.index.json"), timeout)
        with open(os.path.join(d, "model.safetensors.index.json")) as f:
            shards = sorted(set(json.load(f)["weight_map"].values()))
    except FetchError as e:
        # only a missing index means "unsharded": a timeout, 5xx or truncation of the
        # index of a sharded checkpoint is reported as itself
        if e.status != 404:
            raise
        shards = ["model.safetensors"]
    except (ValueError, KeyError) as e:
        raise FetchError(f"{url}: bad model.safetensors.index.json ({e})") from None
    for name in shards:
        if "/" in name or name.startswith("."):
            raise FetchError(f"{url}: refusing shard path {name!r}")
        _get(_join(url, name), os.path.join(d, name), timeout)
        files.append(name)
    try:
        _get(_join(url, "tokenizer.json"), os.path.join(d, "tokenizer.json"), timeout)
    except FetchError:
        pass  # optional: the synthetic tokenizer covers a checkpoint without one
    with open(os.path.join(d, ".complete"), "w") as f:
        json.dump({"url": url, "files": files}, f)
    return d


def clear_cache(url: str, root: Optional[str] = None) -> None:
    d = os.path.join(root or cache_root(), hashlib.sha256(url.encode()).hexdigest()[:16])
    shutil.rmtree(d, ignore_errors=True)
