"""Speculative decoding (Req 12, requirements.md:160-170; tasks.md:340-354).

A small draft model (same vocabulary, e.g. Llama-3.2-1B for Llama-3-8B) runs on
the TP leader's GPU with its own paged KV cache and ModelRunner (HIP graphs for
its single-token steps). Each engine step:

  propose():  for every running greedy decode sequence, catch the draft's KV
              up to the sequence's tokens (one ragged step), then run k-1
              batched single-token draft steps -> k draft tokens, handed to the
              C++ scheduler (set_draft). The scheduler emits such a sequence as
              a verify row block of q_len = 1 + k.
  verify:     the target runs ONE forward over all rows (the prefill-attention
              kernel handles q_len > 1 against the paged context); the longest
              prefix of draft tokens matching the target's argmax is accepted,
              plus the target's own token at the first mismatch (so every verify
              yields >= 1 token and the output equals plain greedy decoding).

Speedup (Req 12.4, requirements.md:169) is measured, not assumed: the engine
times every step it runs with the draft (propose + verify) and every pure-decode
step without verify rows, and `stats()` reports
  speedup_factor = (tokens per sequence-step when speculating / spec step time)
                 / (1 token per sequence-step / plain decode step time)
from exponential moving averages of both (None until both kinds were seen).

Acceptance is tracked per request and globally; a request whose acceptance rate
stays below `min_acceptance_rate` (0.5, requirements.md:170) after a few
verifies stops speculating (its draft pages are freed). Sampled (temperature >
0) requests are not speculated: greedy verification is exact, and they simply
run as plain decodes in the same batches.

TP > 1: the draft lives only on the leader (TP=1 weights); followers execute the
verify plan broadcast with every other step.
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch

from .request import RequestType
from .runner import ModelRunner, SamplingRows

log = logging.getLogger("xgserve.spec")

MIN_VERIFIES = 3


@dataclass
class _DraftSeq:
    blocks: List[int]
    computed: int = 0        # draft KV valid for positions [0, computed)
    pending_L: int = -1      # len(tokens) at the last proposal (-1: none outstanding)
    pending_k: int = 0
    proposed: int = 0
    accepted: int = 0
    verifies: int = 0
    disabled: bool = False


class SpeculativeDecoder:
    def __init__(self, engine, draft_model: str, k: int, min_acceptance_rate: float = 0.5):
        from ..models import build_model, get_config
        self.engine = engine
        self.k = int(k)
        self.min_acceptance_rate = min_acceptance_rate
        self.enabled = engine.is_driver
        self.proposed = 0
        self.accepted = 0
        self.verifies = 0
        self.seqs: Dict[int, _DraftSeq] = {}
        self.ema_spec_ms: Optional[float] = None   # step time with verify rows (propose + verify)
        self.ema_plain_ms: Optional[float] = None  # pure-decode step time without verify rows
        self.ema_tokens_per_row: Optional[float] = None  # tokens per speculated sequence-step
        if not self.enabled:
            return
        if isinstance(draft_model, str):
            dcfg = get_config(draft_model)
            self.model = build_model(dcfg, device=engine.device, dtype=engine.model.dtype, seed=engine.cfg.seed,
                                     tp=1, rank=0)
        else:  # a pre-built TP=1 model (tests, or a draft sharing memory with something else)
            self.model, dcfg = draft_model, draft_model.cfg
        if dcfg.vocab_size != engine.mcfg.vocab_size:
            raise ValueError(f"draft vocab {dcfg.vocab_size} != target vocab {engine.mcfg.vocab_size}")
        ec = engine.cfg
        bs = ec.block_size
        per_seq = (engine.max_model_len + bs - 1) // bs + 1
        nblocks = int(min(engine.num_blocks, ec.max_num_seqs * per_seq))
        self.bs = bs
        self.runner = ModelRunner(self.model, block_size=bs, num_blocks=nblocks, max_num_seqs=ec.max_num_seqs,
                                  max_num_batched_tokens=ec.max_num_batched_tokens, max_model_len=engine.max_model_len,
                                  use_graphs=ec.use_graphs, graph_batch_sizes=ec.graph_batch_sizes, is_driver=True)
        self.runner.capture_graphs()
        self.free: List[int] = list(range(nblocks - 1, -1, -1))
        log.info("speculative decoding: draft=%s k=%d draft KV pages=%d", draft_model, self.k, nblocks)

    # ------------------------------------------------------------------ bookkeeping
    def _release(self, sid: int) -> None:
        ds = self.seqs.pop(sid, None)
        if ds is not None:
            self.free.extend(ds.blocks)

    def _ensure(self, ds: _DraftSeq, n_tokens: int) -> bool:
        need = (n_tokens + self.bs - 1) // self.bs - len(ds.blocks)
        if need > len(self.free):
            return False
        for _ in range(max(0, need)):
            ds.blocks.append(self.free.pop())
        return True

    EMA = 0.1

    def _ema(self, old: Optional[float], x: float) -> float:
        return x if old is None else (1 - self.EMA) * old + self.EMA * x

    def record_step(self, seconds: float, plan: dict, counts: Optional[np.ndarray]) -> None:
        """Engine hook: wall time of one step run with the draft attached."""
        ns, nd = int(plan["num_seqs"]), int(plan["num_decodes"])
        if ns == 0:
            return
        q, pre = plan["q_lens"], plan["is_prefill"]
        verify = (q > 1) & (pre == 0)
        if verify.any() and counts is not None:
            nrows = int(verify.sum())
            sidx = plan["sample_seq_index"]
            vtoks = int(sum(int(c) for j, c in enumerate(counts.tolist()) if verify[int(sidx[j])]))
            self.ema_spec_ms = self._ema(self.ema_spec_ms, 1000.0 * seconds)
            self.ema_tokens_per_row = self._ema(self.ema_tokens_per_row, vtoks / nrows)
        elif nd == ns:
            self.ema_plain_ms = self._ema(self.ema_plain_ms, 1000.0 * seconds)

    def speedup_factor(self) -> Optional[float]:
        if self.ema_spec_ms is None or self.ema_plain_ms is None or not self.ema_spec_ms:
            return None
        return self.ema_tokens_per_row * self.ema_plain_ms / self.ema_spec_ms

    def stats(self) -> dict:
        sf = self.speedup_factor()
        return {"draft_tokens_proposed": self.proposed, "draft_tokens_accepted": self.accepted,
                "acceptance_rate": self.accepted / self.proposed if self.proposed else 0.0,
                "verify_steps": self.verifies,
                "mean_tokens_per_verify": (self.accepted + self.verifies) / self.verifies if self.verifies else 0.0,
                "spec_step_ms": self.ema_spec_ms, "plain_decode_step_ms": self.ema_plain_ms,
                "speedup_factor": None if sf is None else round(sf, 4),
                "active": sum(1 for d in self.seqs.values() if not d.disabled)}

    # ------------------------------------------------------------------ draft steps
    def _plan(self, rows) -> dict:
        """rows: (ds, tokens_slice, start_pos, want_logits) -> a runner plan dict
        (decodes first, as the runner expects)."""
        rows = sorted(rows, key=lambda r: len(r[1]) != 1)
        ns = len(rows)
        w = max(1, max(len(r[0].blocks) for r in rows))
        ids, pos, slot, ql, sl, qsl, li, bt = [], [], [], [], [], [0], [], np.zeros((ns, w), np.int32)
        nd = sum(1 for r in rows if len(r[1]) == 1)  # single-token rows lead (sorted above)
        for i, (ds, toks, p0, _) in enumerate(rows):
            q = len(toks)
            for t in range(q):
                p = p0 + t
                ids.append(toks[t])
                pos.append(p)
                slot.append(ds.blocks[p // self.bs] * self.bs + p % self.bs)
            ql.append(q)
            sl.append(p0 + q)
            bt[i, :len(ds.blocks)] = ds.blocks
            if rows[i][3]:
                li.append(qsl[-1] + q - 1)
            qsl.append(qsl[-1] + q)
        i32 = lambda a: np.asarray(a, np.int32)  # noqa: E731
        return {"num_seqs": ns, "num_decodes": nd, "num_tokens": len(ids), "num_sample": len(li),
                "max_q_len": max(ql), "bt_width": w, "input_ids": i32(ids), "positions": i32(pos),
                "slot_mapping": i32(slot), "q_lens": i32(ql), "seq_lens": i32(sl), "query_start_loc": i32(qsl),
                "block_tables": bt.reshape(-1), "logits_indices": i32(li), "is_embed": np.zeros(ns, np.uint8),
                "order": rows}

    def propose(self) -> None:
        """Called by the engine (under its lock) right before scheduling."""
        if not self.enabled or self.k <= 0:
            return
        eng = self.engine
        live = set(eng.by_seq)
        for sid in [s for s in self.seqs if s not in live]:
            self._release(sid)
        budget = self.runner.max_tokens
        rows, ready = [], []
        for sid, req in eng.by_seq.items():
            if req.finished or req.kind == RequestType.Embeddings or not req.output_ids:
                continue
            p = req.params
            if p.temperature > 0 or len(req.output_ids) + 1 >= p.max_tokens:
                continue
            ds = self.seqs.get(sid)
            if ds is None:
                ds = self.seqs[sid] = _DraftSeq(blocks=[])
            if ds.disabled:
                continue
            if ds.pending_L >= 0:  # last proposal was never verified: trust only the real tokens
                ds.computed = min(ds.computed, ds.pending_L)
                ds.pending_L = -1
            toks = req.prompt_ids + req.output_ids
            L = len(toks)
            if L + self.k > eng.max_model_len:
                continue
            if not self._ensure(ds, L + self.k):  # draft KV pool exhausted: plain decoding for this one
                self.free.extend(ds.blocks)
                ds.blocks = []
                ds.disabled = True
                continue
            new = toks[ds.computed:]
            if not new:  # cannot happen (the last token is never in the draft KV) -- be safe
                ds.computed = L - 1
                new = toks[-1:]
            if budget <= 0:
                break
            take = min(len(new), budget)
            budget -= take
            done = take == len(new)
            rows.append((ds, new[:take], ds.computed, done))
            ds.computed += take
            if done:
                ready.append((sid, ds, L))
        if not rows:
            return
        plan = self._plan(rows)
        toks, _, _ = self.runner.execute(plan, None)
        if not ready:
            return
        order = [r[0] for r in plan["order"] if r[3]]
        first = {id(ds): int(t) for ds, t in zip(order, toks)}
        drafts = {sid: [first[id(ds)]] for sid, ds, _ in ready}
        for step in range(1, self.k):
            drows = [(ds, [drafts[sid][-1]], L + step - 1, True) for sid, ds, L in ready]
            dplan = self._plan(drows)
            t2, _, _ = self.runner.execute(dplan, None)
            by_ds = {id(r[0]): int(t) for r, t in zip(dplan["order"], t2)}
            for sid, ds, _ in ready:
                drafts[sid].append(by_ds[id(ds)])
        for sid, ds, L in ready:
            ds.computed = L + self.k - 1
            ds.pending_L, ds.pending_k = L, self.k
            eng.sched.set_draft(sid, drafts[sid])

    # ------------------------------------------------------------------ verify
    def verify_execute(self, plan: dict, samp: Optional[SamplingRows]):
        """Run the target over a plan that may contain verify row blocks. Returns
        (accepted tokens concatenated per sampled sequence, logprobs, hidden, counts)."""
        sidx = plan["sample_seq_index"]
        q_lens, is_pre = plan["q_lens"], plan["is_prefill"]
        nrows = np.array([int(q_lens[s]) if (not is_pre[s] and q_lens[s] > 1) else 1 for s in sidx.tolist()],
                         dtype=np.int64)
        rsamp = None
        if samp is not None:
            rsamp = SamplingRows(np.repeat(samp.temps, nrows), np.repeat(samp.top_ps, nrows),
                                 np.repeat(samp.top_ks, nrows), np.repeat(samp.seeds, nrows))
        toks, lps, hidden = self.engine.runner.execute(plan, rsamp)
        if toks is None:
            return None, None, hidden, None
        out_t, out_l, counts = [], [], []
        k = 0
        qsl, ids, seq_ids = plan["query_start_loc"], plan["input_ids"], plan["seq_ids"]
        for j, s in enumerate(sidx.tolist()):
            n_r = int(nrows[j])
            if n_r == 1:
                out_t.append(int(toks[k]))
                out_l.append(float(lps[k]))
                counts.append(1)
                k += 1
                continue
            draft = ids[int(qsl[s]) + 1:int(qsl[s]) + n_r]
            t = toks[k:k + n_r]
            n = 0
            while n < n_r - 1 and int(draft[n]) == int(t[n]):
                n += 1
            out_t.extend(int(x) for x in t[:n + 1])  # accepted drafts == target tokens, + the bonus token
            out_l.extend(float(x) for x in lps[k:k + n + 1])
            counts.append(n + 1)
            k += n_r
            self._account(int(seq_ids[s]), n_r - 1, n)
        return (np.asarray(out_t, np.int32), np.asarray(out_l, np.float32), hidden, np.asarray(counts, np.int32))

    def _account(self, sid: int, proposed: int, accepted: int) -> None:
        self.proposed += proposed
        self.accepted += accepted
        self.verifies += 1
        ds = self.seqs.get(sid)
        if ds is None:
            return
        if ds.pending_L >= 0:
            ds.computed = ds.pending_L + min(accepted, ds.pending_k - 1)
            ds.pending_L = -1
        ds.proposed += proposed
        ds.accepted += accepted
        ds.verifies += 1
        if ds.verifies >= MIN_VERIFIES and ds.accepted < self.min_acceptance_rate * ds.proposed:
            log.debug("seq %d: acceptance %.2f < %.2f, speculation disabled", sid, ds.accepted / ds.proposed,
                      self.min_acceptance_rate)
            self.free.extend(ds.blocks)
            ds.blocks = []
            ds.disabled = True
