"""Tokenizers + incremental detokenization + chat templating.

* HFTokenizer: a `tokenizer.json` from the checkpoint directory (HF
  `tokenizers`, no network).
* SyntheticTokenizer: the offline default sized to the model vocab (the GPU
  box has no tokenizer downloads). Text bytes map to ids [base, base+256); any
  other id decodes to a deterministic pseudo-word so random-weight outputs are
  readable text. Round-trips every UTF-8 string.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

_SYL = ["ka", "lo", "mi", "ne", "su", "ta", "ri", "po", "ve", "du", "an", "el", "is", "or", "um", "ya"]


class BaseTokenizer:
    vocab_size: int
    bos_id: Optional[int]
    eos_ids: List[int]

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        raise NotImplementedError

    def decode(self, ids: Sequence[int]) -> str:
        raise NotImplementedError

    def apply_chat_template(self, messages) -> str:
        """Llama-3 style header template (roles: system/user/assistant)."""
        parts = []
        for m in messages:
            role = m.role.value if hasattr(m.role, "value") else m["role"]
            content = m.content if hasattr(m, "content") else m["content"]
            parts.append(f"<|start_header_id|>{role}<|end_header_id|>\n\n{content}<|eot_id|>")
        parts.append("<|start_header_id|>assistant<|end_header_id|>\n\n")
        return "".join(parts)


class SyntheticTokenizer(BaseTokenizer):
    def __init__(self, vocab_size: int, bos_id: Optional[int] = None, eos_ids: Optional[List[int]] = None):
        self.vocab_size = vocab_size
        self.bos_id = bos_id if bos_id is not None and bos_id < vocab_size else None
        self.eos_ids = [e for e in (eos_ids or []) if e < vocab_size]
        specials = set(self.eos_ids) | ({self.bos_id} if self.bos_id is not None else set())
        base = 3
        while any(base <= s < base + 256 for s in specials):
            base += 256
        if base + 256 > vocab_size:
            base = 0
        self.base = base
        self.specials = specials

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        ids = [self.base + b for b in text.encode("utf-8")]
        if add_bos and self.bos_id is not None:
            ids = [self.bos_id] + ids
        return ids

    def _word(self, i: int) -> bytes:
        s, n = [], i
        while True:
            s.append(_SYL[n % 16])
            n //= 16
            if n == 0 or len(s) >= 3:
                break
        return (" " + "".join(s)).encode()

    def token_bytes(self, i: int) -> bytes:
        if i in self.specials:
            return b""
        if self.base <= i < self.base + 256:
            return bytes([i - self.base])
        return self._word(i)

    def decode(self, ids: Sequence[int]) -> str:
        return b"".join(self.token_bytes(int(i)) for i in ids).decode("utf-8", errors="replace")


class HFTokenizer(BaseTokenizer):
    def __init__(self, path: str, bos_id: Optional[int] = None, eos_ids: Optional[List[int]] = None):
        from tokenizers import Tokenizer
        self.tok = Tokenizer.from_file(path)
        self.vocab_size = self.tok.get_vocab_size()
        self.bos_id = bos_id
        self.eos_ids = list(eos_ids or [])

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        ids = self.tok.encode(text, add_special_tokens=False).ids
        if add_bos and self.bos_id is not None:
            ids = [self.bos_id] + ids
        return ids

    def decode(self, ids: Sequence[int]) -> str:
        return self.tok.decode(list(ids), skip_special_tokens=True)


def load_tokenizer(cfg, checkpoint: Optional[str] = None) -> BaseTokenizer:
    if checkpoint:
        p = os.path.join(checkpoint, "tokenizer.json")
        if os.path.exists(p):
            return HFTokenizer(p, cfg.bos_token_id, cfg.eos_token_ids)
    return SyntheticTokenizer(cfg.vocab_size, cfg.bos_token_id, cfg.eos_token_ids)


class IncrementalDetokenizer:
    """O(new tokens) incremental detokenization.

    * synthetic tokenizer: token bytes go through an incremental UTF-8 decoder
      (partial characters are buffered until complete);
    * HF tokenizers: the prefix/read-offset window scheme (decode only the last
      few ids; hold output while it ends in a replacement char);
    * stop strings: only the tail window is searched, and a suffix that could
      still grow into a stop string is held back.
    """

    def __init__(self, tok: BaseTokenizer, stop: Sequence[str] = ()):
        import codecs
        self.tok = tok
        self.ids: List[int] = []
        self.text = ""          # decoded text so far (complete chars only)
        self.emitted = 0        # chars of self.text already handed out
        self.stop = [s for s in stop if s]
        self.max_stop = max((len(s) for s in self.stop), default=0)
        self.stopped = False
        self._synthetic = isinstance(tok, SyntheticTokenizer)
        self._dec = codecs.getincrementaldecoder("utf-8")(errors="replace") if self._synthetic else None
        self._eos = set(tok.eos_ids)
        self._prefix_off = 0
        self._read_off = 0

    def _append(self, new_ids) -> None:
        ids = [int(i) for i in new_ids if int(i) not in self._eos]
        if not ids:
            return
        self.ids.extend(ids)
        if self._synthetic:
            tb = self.tok.token_bytes
            self.text += self._dec.decode(b"".join(tb(i) for i in ids))
            return
        prefix = self.tok.decode(self.ids[self._prefix_off:self._read_off])
        full = self.tok.decode(self.ids[self._prefix_off:])
        if full.endswith("\ufffd"):
            return  # wait for the rest of the character
        if len(full) > len(prefix):
            self.text += full[len(prefix):]
        self._prefix_off = self._read_off
        self._read_off = len(self.ids)

    def add(self, new_ids: Sequence[int]) -> str:
        """Append tokens; return newly available text (stop strings excluded)."""
        if self.stopped:
            return ""
        self._append(new_ids)
        if not self.stop:
            out = self.text[self.emitted:]
            self.emitted = len(self.text)
            return out
        lo = max(0, self.emitted - self.max_stop)
        cut = None
        for st in self.stop:
            j = self.text.find(st, lo)
            if j >= 0 and (cut is None or j < cut):
                cut = j
        if cut is not None:
            self.stopped = True
            out = self.text[self.emitted:cut]
            self.text = self.text[:cut]
            self.emitted = cut
            return out
        safe = len(self.text)
        for k in range(min(self.max_stop - 1, len(self.text)), 0, -1):
            tail = self.text[-k:]
            if any(st.startswith(tail) for st in self.stop):
                safe = len(self.text) - k
                break
        safe = max(safe, self.emitted)
        out = self.text[self.emitted:safe]
        self.emitted = safe
        return out

    def flush(self) -> str:
        if self.stopped:
            return ""
        if self._synthetic:
            self.text += self._dec.decode(b"", final=True)
        out = self.text[self.emitted:]
        self.emitted = len(self.text)
        return out
