"""TokenStreamer: per-request SSE channels (Req 5, requirements.md:76-86;
design.md:415-459).

`create_stream(id)` returns a (sender, stream) pair backed by one asyncio
queue; the engine side pushes TokenEvents through `send_token` from the event
loop thread (the replica reader hops onto the loop with call_soon_threadsafe,
so a token reaches the socket in one loop iteration -- Req 5.1's 10 ms budget
is dominated by the engine step, not by this layer). `close_stream(id,
reason)` emits the final `done` (or `error`) event and ends the stream
(Req 5.3/5.5). A client disconnect surfaces as StreamClientDisconnected in the
HTTP writer, which calls the registered abort hook so the engine frees the
sequence's KV pages (Req 5.4).
"""
from __future__ import annotations

import asyncio
from typing import AsyncIterator, Callable, Dict, Optional

from ..core.errors import StreamNotFound
from ..core.wire import FinishReason, TokenEvent, Usage

_END = object()


class StreamSender:
    def __init__(self, rid: str, q: asyncio.Queue):
        self.rid = rid
        self._q = q
        self.closed = False

    def send(self, ev: TokenEvent) -> None:
        if not self.closed:
            self._q.put_nowait(ev)

    def close(self) -> None:
        if not self.closed:
            self.closed = True
            self._q.put_nowait(_END)


class TokenStream:
    def __init__(self, rid: str, q: asyncio.Queue):
        self.rid = rid
        self._q = q

    def __aiter__(self) -> AsyncIterator[TokenEvent]:
        return self._gen()

    async def _gen(self):
        while True:
            ev = await self._q.get()
            if ev is _END:
                return
            yield ev

    def take_ready(self) -> list:
        """Every event already queued, without waiting (stops at the end marker,
        which it puts back): lets the SSE writer coalesce a backlog into one socket
        write instead of one coroutine wake-up + write per token."""
        out = []
        while True:
            try:
                ev = self._q.get_nowait()
            except asyncio.QueueEmpty:
                return out
            if ev is _END:
                self._q.put_nowait(_END)
                return out
            out.append(ev)


class TokenStreamer:
    def __init__(self):
        self._senders: Dict[str, StreamSender] = {}
        self.on_disconnect: Optional[Callable[[str], None]] = None

    def create_stream(self, rid: str):
        q: asyncio.Queue = asyncio.Queue()
        s = StreamSender(rid, q)
        self._senders[rid] = s
        return s, TokenStream(rid, q)

    def register(self, rid: str, sender) -> None:
        """A sender owned elsewhere (a front-end process's RemoteSender)."""
        self._senders[rid] = sender

    def send_token(self, rid: str, token: str, index: int, logprob: Optional[float] = None) -> None:
        s = self._senders.get(rid)
        if s is None:
            raise StreamNotFound(rid)
        s.send(TokenEvent.tok(token, index, logprob))

    def close_stream(self, rid: str, finish_reason: FinishReason, usage: Usage) -> None:
        s = self._senders.pop(rid, None)
        if s is None:
            raise StreamNotFound(rid)
        s.send(TokenEvent.done(finish_reason, usage))
        s.close()

    def fail_stream(self, rid: str, message: str, code: str) -> None:
        s = self._senders.pop(rid, None)
        if s is None:
            return
        s.send(TokenEvent.error(message, code))
        s.close()

    def discard(self, rid: str) -> None:
        """Drop a channel that never carried anything (request rejected at admission)."""
        self._senders.pop(rid, None)

    def disconnect(self, rid: str) -> None:
        """Client went away: drop the channel and abort generation."""
        s = self._senders.pop(rid, None)
        if s is not None:
            s.closed = True
        if self.on_disconnect is not None:
            self.on_disconnect(rid)

    def active_streams(self) -> int:
        return len(self._senders)
