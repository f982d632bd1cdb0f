"""MockEngine: deterministic stand-in for LLMEngine (same interface) used for
API/plumbing tests and fault injection (the reference's planned
MockInferenceWorker, tasks.md:193).

Token rule: next = (31 * last + 7 + step_of_request) % vocab, so outputs are a
pure function of the prompt. Fault knobs:
  * a prompt containing `fail_marker` fails alone (Property 22: isolation);
  * `crash_after_steps`: raise SystemExit (process replica) after N steps;
  * `step_latency_s`: sleep per step (streaming / timeout tests);
  * `hang`: stop producing (heartbeat-based failure detection tests).
"""
from __future__ import annotations

import threading
import time
from typing import Dict, List, Optional, Sequence

from .request import EngineRequest, RequestOutput, RequestType, SamplingParams
from .tokenizer import IncrementalDetokenizer, SyntheticTokenizer


class _MockModelCfg:
    def __init__(self, name: str, vocab: int, hidden: int):
        self.name = name
        self.vocab_size = vocab
        self.hidden_size = hidden
        self.eos_token_ids = [2]
        self.max_position = 8192


class MockEngine:
    def __init__(self, model_name: str = "mock", vocab_size: int = 1000, hidden_size: int = 16,
                 step_latency_s: float = 0.0, max_num_seqs: int = 256, fail_marker: str = "__FAIL__",
                 crash_after_steps: Optional[int] = None, eos_every: Optional[int] = None, kv_seqs: int = 0):
        self.mcfg = _MockModelCfg(model_name, vocab_size, hidden_size)
        self.tokenizer = SyntheticTokenizer(vocab_size, 1, [2])
        self.step_latency_s = step_latency_s
        self.max_num_seqs = max_num_seqs
        self.kv_seqs = kv_seqs  # memory-pressure model: live sequences / capacity (0: max_num_seqs)
        self.fail_marker_ids = self.tokenizer.encode(fail_marker, add_bos=False)
        self.crash_after_steps = crash_after_steps
        self.eos_every = eos_every
        self.hang = False
        self.fail_collective = False  # fault injection: the next step raises a TP collective timeout
        self.requests: Dict[str, EngineRequest] = {}
        self._order: List[str] = []
        self._lock = threading.Lock()
        self._aborted: List[str] = []
        self._seq = 0
        self.steps = 0
        self.num_blocks = 1000
        self.stats_counters = {"prompt_tokens": 0, "generation_tokens": 0, "steps": 0, "requests_finished": 0}
        self.batch_log: List[int] = []

    # ---- LLMEngine-compatible API -----------------------------------------
    def add_request(self, request_id: str, prompt_ids: Sequence[int], params: SamplingParams, priority: int = 1,
                    kind: RequestType = RequestType.Generate, user_data=None) -> EngineRequest:
        with self._lock:
            self._seq += 1
            r = EngineRequest(request_id, self._seq, list(prompt_ids), params, priority, kind, user_data=user_data)
            r.detok = IncrementalDetokenizer(self.tokenizer, params.stop)
            self.requests[request_id] = r
            self._order.append(request_id)
            self.stats_counters["prompt_tokens"] += len(prompt_ids)
        return r

    def abort(self, request_id: str, reason: int = 4) -> bool:
        with self._lock:
            r = self.requests.pop(request_id, None)
            if r is None:
                return False
            self._order.remove(request_id)
            self._aborted.append(request_id)
            return True

    def has_work(self) -> bool:
        return bool(self.requests) or bool(self._aborted)

    def _contains(self, ids, sub) -> bool:
        n = len(sub)
        return n > 0 and any(ids[i:i + n] == sub for i in range(len(ids) - n + 1))

    def step(self) -> List[RequestOutput]:
        t_hang = time.monotonic()
        while self.hang and time.monotonic() - t_hang < 30.0:  # a wedged step: no outputs, no heartbeats
            time.sleep(0.02)
        if self.hang:
            return []
        if self.fail_collective:
            from ..parallel.custom_ar import CustomAllReduceTimeout
            raise CustomAllReduceTimeout("mock: peer wait timed out (fault injection)")
        if self.step_latency_s:
            time.sleep(self.step_latency_s)
        self.steps += 1
        if self.crash_after_steps is not None and self.steps > self.crash_after_steps:
            raise SystemExit("mock engine crash (fault injection)")
        outs: List[RequestOutput] = []
        with self._lock:
            for rid in self._aborted:
                outs.append(RequestOutput(rid, [], "", True, "abort"))
            self._aborted.clear()
            active = self._order[: self.max_num_seqs]
            self.batch_log.append(len(active))
            self.stats_counters["steps"] += 1
            for rid in list(active):
                r = self.requests[rid]
                if self._contains(r.prompt_ids, self.fail_marker_ids):
                    outs.append(RequestOutput(rid, [], "", True, "error", prompt_tokens=len(r.prompt_ids),
                                              error="Inference failed: injected failure",
                                              error_code="inference_failed"))
                    self._drop(rid)
                    continue
                if r.kind == RequestType.Embeddings:
                    h = self.mcfg.hidden_size
                    v = [((sum(r.prompt_ids) * (i + 3)) % 97) / 97.0 + 0.01 for i in range(h)]
                    nrm = sum(x * x for x in v) ** 0.5
                    outs.append(RequestOutput(rid, [], "", True, "stop", prompt_tokens=len(r.prompt_ids),
                                              embedding=[x / nrm for x in v]))
                    self._drop(rid)
                    continue
                last = r.output_ids[-1] if r.output_ids else (r.prompt_ids[-1] if r.prompt_ids else 1)
                tok = (31 * last + 7 + len(r.output_ids)) % self.mcfg.vocab_size
                if tok in (2,) or tok < 3:
                    tok += 3
                if self.eos_every and len(r.output_ids) + 1 >= self.eos_every and not r.params.ignore_eos:
                    tok = 2
                if r.first_token_time is None:
                    r.first_token_time = time.monotonic()
                r.output_ids.append(tok)
                text = r.detok.add([tok])
                reason = None
                if tok == 2:
                    reason = "stop"
                elif r.detok.stopped:
                    reason = "stop_sequence"
                elif len(r.output_ids) >= r.params.max_tokens:
                    reason = "length"
                if reason is not None and not r.detok.stopped:
                    text += r.detok.flush()
                self.stats_counters["generation_tokens"] += 1
                outs.append(RequestOutput(rid, [tok], text, reason is not None, reason,
                                          prompt_tokens=len(r.prompt_ids), completion_tokens=len(r.output_ids),
                                          t_tokens=time.monotonic()))
                if reason is not None:
                    self._drop(rid)
        return outs

    def _drop(self, rid):
        self.requests.pop(rid, None)
        if rid in self._order:
            self._order.remove(rid)
        self.stats_counters["requests_finished"] += 1

    def kv_usage(self) -> float:
        return min(1.0, len(self.requests) / max(1, self.kv_seqs or self.max_num_seqs))

    def stats(self) -> dict:
        used = len(self.requests)
        return {"model": self.mcfg.name, "waiting": max(0, used - self.max_num_seqs),
                "running": min(used, self.max_num_seqs), "kv_blocks_total": self.num_blocks,
                "kv_blocks_used": used, "kv_blocks_free": self.num_blocks - used, "kv_usage": self.kv_usage(),
                "memory_used": used * 1024, "memory_available": (self.num_blocks - used) * 1024,
                "memory_limit": int(self.num_blocks * 1024 * 0.8),
                "cache": {"entries": 0, "hit_tokens": 0, "miss_tokens": 0, "hit_count": 0, "miss_count": 0,
                          "eviction_count": 0},
                "preemptions": 0, **self.stats_counters}

    def clear_prefix_cache(self):
        pass

    def set_limits(self, max_num_seqs: int, max_num_batched_tokens: int):
        self.max_num_seqs = max_num_seqs

    def generate(self, prompts, params: SamplingParams):
        import copy
        rids = [f"m{i}-{time.monotonic_ns()}" for i in range(len(prompts))]
        for rid, p in zip(rids, prompts):
            self.add_request(rid, p, copy.deepcopy(params))
        res = {r: [] for r in rids}
        while self.has_work():
            for o in self.step():
                if o.request_id in res:
                    res[o.request_id] += o.new_token_ids
        return [res[r] for r in rids]
