"""LLMEngine: one model replica (a TP group) with continuous batching.

Per step: the C++ StepScheduler packs decode tokens + prefill chunks under a
token budget (prefix-cache aware, preempting on KV exhaustion) -> the TP leader
broadcasts the plan to its followers -> every rank runs the forward (HIP graph
for pure decode) -> the leader samples, feeds tokens back to the scheduler and
produces RequestOutputs (incremental text, stop strings, finish reasons,
embeddings for prefill-only requests).

This realises the reference's spec'd worker interface
(`InferenceWorker::initialize/infer/shutdown/status/model_info`,
design.md:335-342) at iteration granularity: `infer(batch)` returning N results
(Property 21) is `generate()` on top of `step()`; per-request failures are
isolated (Property 22) because a failing request is aborted alone.
"""
from __future__ import annotations

import itertools
import logging
import math
import os
import threading
import time
from dataclasses import asdict, dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch

from .. import _runtime as R
from .. import tune
from ..models import build_model, get_config
from ..parallel import comm
from ..parallel.state import get_state
from .request import (FINISH_ABORT, FINISH_EMBED, FINISH_LENGTH, FINISH_NAMES, FINISH_STOP, FINISH_STOP_SEQ,
                      EngineRequest, RequestOutput, RequestType, SamplingParams)
from .runner import ModelRunner, SamplingRows
from .tokenizer import IncrementalDetokenizer, load_tokenizer

log = logging.getLogger("xgserve.engine")
# split a step's emission: rows that cannot wait (finished, first tokens) before the
# next step is planned, the rest in its overlap window (A/B in profiles/r2_async_mixed_ab.md)
EMIT_SPLIT = True
# Outputs emitted in a step's overlap window go to `output_sink` (the serving
# replica's writer) right away instead of riding the step's return value, which
# comes only after the GPU step in flight finishes (a whole step of delivery delay,
# Req 5.1). False: return them with the step (tests).
EARLY_OUTPUTS = True

_MASK63 = (1 << 63) - 1


@dataclass
class EngineConfig:
    model: str = "llama3-8b"
    checkpoint: Optional[str] = None
    tp: int = 1
    device: Optional[str] = None
    dtype: Optional[str] = None
    block_size: int = 16
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    max_model_len: Optional[int] = None
    gpu_memory_utilization: float = 0.90
    num_blocks: Optional[int] = None
    enable_prefix_cache: bool = True
    chunked_prefill: bool = True
    cache_threshold: float = 0.8
    use_graphs: bool = True
    graph_batch_sizes: Optional[List[int]] = None
    seed: int = 0
    moe_comm: str = "auto"
    max_prefill_seqs: int = 1 << 30
    # prefill tokens allowed in a step that also decodes (0: only the token budget)
    decode_prefill_cap: int = 0
    # prompts per decoding step under decode_prefill_cap: None = 1 when the runner
    # captured mixed-step graphs (their shape holds one chunk), else no limit (a burst
    # of short prompts shares a step)
    decode_prefill_seqs: Optional[int] = None
    # admission window (continuous batching): while rows decode, hold new prompts until
    # prompt_coalesce of them wait or the oldest was passed over by
    # prompt_coalesce_max_wait steps, then prefill them in one mixed step (1: off)
    prompt_coalesce: int = 1
    prompt_coalesce_max_wait: int = 4
    # speculative decoding (Req 12)
    draft_model: Optional[str] = None
    num_speculative_tokens: int = 0
    spec_min_acceptance_rate: float = 0.5
    # detokenise / build step N's outputs while step N+1 runs on the GPU (first
    # tokens are still emitted at once, so TTFT is unchanged)
    overlap_outputs: bool = True
    # asynchronous scheduling: plan + launch step N+1 (its decode ids substituted on
    # the GPU from step N's sampled tokens) before step N's tokens reach the host,
    # so the host's per-step work (commit, schedule, metadata, launch) overlaps the
    # GPU instead of sitting between steps. No speculation, graph decode steps; under
    # TP the followers get (plan, sampling rows, src) per launch and sample the same
    # tokens from the same all-gathered logits, so their substitutions agree.
    async_schedule: bool = True
    early_release: bool = True
    # "fp8": weight-only E4M3 copies for batch <= 16 decode (bf16 activations)
    weight_dtype: Optional[str] = None
    # custom xGMI all-reduce peer-wait limit while serving: a TP peer this late fails
    # the step (CustomAllReduceTimeout -> replica restart); warmup runs under 20 s
    collective_timeout_s: float = 2.0

    def resolved_device(self) -> torch.device:
        if self.device:
            return torch.device(self.device)
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


class LLMEngine:
    def __init__(self, cfg: EngineConfig, model=None):
        self.cfg = cfg
        self.mcfg = get_config(cfg.checkpoint or cfg.model) if model is None else model.cfg
        if cfg.checkpoint and model is None:
            self.mcfg.name = cfg.model if cfg.model else self.mcfg.name
        st = get_state()
        self.tp_rank = st.tp_rank
        self.is_driver = st.tp_rank == 0
        device = cfg.resolved_device()
        from ..tuning import enable_gemm_table
        self.gemm_table = enable_gemm_table(device)  # replay the shipped hipBLASLt / rocBLAS choices
        dtype = {"bfloat16": torch.bfloat16, "float32": torch.float32, "float16": torch.float16,
                 None: None}[cfg.dtype]
        t0 = time.time()
        self.model = model if model is not None else build_model(self.mcfg, device=device, dtype=dtype,
                                                                 checkpoint=cfg.checkpoint, seed=cfg.seed,
                                                                 weight_dtype=cfg.weight_dtype)
        self.model.set_moe_comm(cfg.moe_comm)
        self.load_time = time.time() - t0
        from ..parallel.custom_ar import maybe_enable
        m = self.mcfg
        ar_shapes = None
        if st.tp_size > 1 and m.arch != "gpt2":  # the row-parallel shards GG_AR serves: O, then down
            ar_shapes = [(m.hidden_size, m.num_heads * m.head_dim // st.tp_size)]
            if not m.num_experts:
                ar_shapes.append((m.hidden_size, m.intermediate_size // st.tp_size))
        # one-shot xGMI all-reduce for TP decode
        self.custom_ar = maybe_enable(st, self.model.device, ar_shapes)
        self.device = self.model.device
        self.max_model_len = min(cfg.max_model_len or self.mcfg.max_position, self.mcfg.max_position)
        self.tokenizer = load_tokenizer(self.mcfg, cfg.checkpoint)
        num_blocks = cfg.num_blocks or self._auto_num_blocks()
        self.num_blocks = num_blocks
        sc = R.SchedulerConfig()
        sc.block_size = cfg.block_size
        sc.num_blocks = num_blocks
        sc.max_num_seqs = cfg.max_num_seqs
        sc.max_num_batched_tokens = cfg.max_num_batched_tokens
        sc.max_model_len = self.max_model_len
        sc.enable_prefix_cache = cfg.enable_prefix_cache
        sc.chunked_prefill = cfg.chunked_prefill
        sc.cache_threshold = cfg.cache_threshold
        sc.max_prefill_seqs = cfg.max_prefill_seqs
        sc.decode_prefill_cap = cfg.decode_prefill_cap
        # stall-free batching: one prompt chunk per decoding step (the mixed-step graphs)
        sc.decode_prefill_seqs = 1 if cfg.decode_prefill_cap > 0 else 0
        sc.coalesce_prompts = max(1, int(cfg.prompt_coalesce))
        sc.coalesce_max_wait = max(0, int(cfg.prompt_coalesce_max_wait))
        # asynchronous scheduling over prompt steps too (r2_async_mixed_ab.md)
        sc.lookahead_mixed = 1
        # release length-finishing rows at lookahead: the next step is planned before a
        # finishing row's last token reaches the host, so the GPU never waits for the
        # host at a finish (a request arriving just then is admitted one step later).
        # Steady state 64 concurrent: +1.3 % tok/s, p50 TTFT 12.4 -> 16.6 ms
        # (profiles/r3_steady_state.md). XGS_TUNE early_release=0: synchronous finishing steps.
        sc.early_release = int(tune.get_bool("early_release", bool(cfg.early_release)))
        sc.eos_ids = list(self.mcfg.eos_token_ids)
        self.sched = R.StepScheduler(sc)
        # decode graphs capture the TP collectives: RCCL (and the IPC all-reduce) can be
        # captured into a HIP graph, gloo (CPU-staged) cannot -> eager decode there
        use_graphs = cfg.use_graphs and (st.tp_size == 1 or st.backend == "nccl")
        graph_bs = cfg.graph_batch_sizes
        if cfg.use_graphs and not use_graphs and self.custom_ar is not None and not self.mcfg.num_experts:
            # gloo CPU group but a dense model whose decode collectives (fused residual
            # all-reduce, LM-head gather) all run on the IPC kernels: capturable as long
            # as every captured batch stays on them (<= 64 tokens)
            use_graphs = True
            graph_bs = [b for b in (graph_bs or [1, 2, 4, 8, 16, 24, 32, 48, 64]) if b <= 64]
        if cfg.use_graphs and not use_graphs:
            log.info("TP over %s: decode graphs disabled (collectives not capturable)", st.backend)
        self.runner = ModelRunner(self.model, block_size=cfg.block_size, num_blocks=num_blocks,
                                  max_num_seqs=cfg.max_num_seqs, max_num_batched_tokens=cfg.max_num_batched_tokens,
                                  max_model_len=self.max_model_len, use_graphs=use_graphs,
                                  graph_batch_sizes=graph_bs, is_driver=self.is_driver,
                                  mixed_chunk=cfg.decode_prefill_cap)
        self.runner.collective_timeout_s = cfg.collective_timeout_s
        self._dp_seqs = cfg.decode_prefill_seqs if cfg.decode_prefill_seqs is not None else \
            (1 if self.runner.mixed_chunk > 0 else 0)
        self.sched.set_decode_prefill(cfg.decode_prefill_cap, self._dp_seqs if cfg.decode_prefill_cap > 0 else 0)
        self.runner.capture_graphs()
        H = self.mcfg.hidden_size
        self.embed_acc = torch.zeros(cfg.max_num_seqs, H, dtype=torch.float32, device=self.device)
        self.requests: Dict[str, EngineRequest] = {}
        self.by_seq: Dict[int, EngineRequest] = {}
        ns = cfg.max_num_seqs
        self.slot_owner = np.full(ns, -1, np.int64)
        self.slot_req: List[Optional[EngineRequest]] = [None] * ns
        self.slot_temp = np.zeros(ns, np.float32)
        self.slot_topp = np.ones(ns, np.float32)
        self.slot_topk = np.zeros(ns, np.int32)
        self.slot_seed = np.zeros(ns, np.uint64)
        self.slot_ngen = np.zeros(ns, np.int64)  # tokens generated by the slot's owner (sampling counter)
        self._deferred = None  # (plan, toks, lps, counts, fin_map) awaiting detokenisation
        # callable(List[RequestOutput]) taking overlap-window outputs immediately (a server
        # replica sets it); None: every output is returned by step()
        self.output_sink = None
        self._timing = None
        self._tprof = None  # torch.profiler state (XGS_TORCH_PROFILE)
        self._tprof_left = 0
        self._seq_counter = itertools.count(1)
        self._lock = threading.Lock()
        self._pending_aborts: List[str] = []
        self.step_count = 0
        self.stats_counters = {"prompt_tokens": 0, "generation_tokens": 0, "steps": 0, "decode_steps": 0,
                               "prefill_tokens_computed": 0, "requests_finished": 0, "preemptions": 0,
                               "lookahead_launches": 0}
        self.spec = None
        if cfg.draft_model and cfg.num_speculative_tokens > 0:
            from .spec_decode import SpeculativeDecoder
            self.spec = SpeculativeDecoder(self, cfg.draft_model, cfg.num_speculative_tokens,
                                           cfg.spec_min_acceptance_rate)
        self._inflight = None  # (plan, handle): launched by the previous step() (async scheduling)
        # Speculative decoding keeps the synchronous loop: asynchronous scheduling plans
        # step N+1 before step N's tokens reach the host, which needs every row's next
        # position and KV slot in advance -- exactly what verification leaves open (a
        # row advances by 1..k+1 tokens, known only after the acceptance test), and the
        # draft model's next proposal depends on those accepted tokens too. Planning for
        # every acceptance length (k+1 plans per row) would defeat the point, so a
        # speculating engine runs step by step.
        self._async = (cfg.async_schedule and tune.get_bool("async_sched", True)
                       and self.device.type == "cuda" and self.spec is None and bool(self.runner.graphs))
        log.info("engine ready: model=%s tp=%d blocks=%d (%.1f GiB KV) load=%.1fs", self.mcfg.name, get_state().tp_size,
                 num_blocks, self.runner.kv_bytes() / 2**30, self.load_time)

    # ------------------------------------------------------------------ sizing
    def _block_bytes(self) -> int:
        m = self.mcfg
        esz = torch.tensor([], dtype=self.model.dtype).element_size()
        return 2 * m.num_layers * self.model.num_kv_heads_local * self.cfg.block_size * m.head_dim * esz

    def _auto_num_blocks(self) -> int:
        if self.device.type != "cuda":
            return 512
        torch.cuda.synchronize()
        free, total = torch.cuda.mem_get_info()
        m = self.mcfg
        act = self.cfg.max_num_batched_tokens * (6 * m.hidden_size + 4 * m.intermediate_size // max(1, get_state().tp_size)) * 2
        act += self.cfg.max_num_seqs * m.vocab_size * 8 + (2 << 30)
        budget = free - (1.0 - self.cfg.gpu_memory_utilization) * total - act
        n = int(max(64, budget // self._block_bytes()))
        st = get_state()
        if st.tp_size > 1:
            t = torch.tensor([n], dtype=torch.int64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN, group=st.tp_cpu_group)
            n = int(t.item())
        return n

    # ------------------------------------------------------------------ requests
    def add_request(self, request_id: str, prompt_ids: Sequence[int], params: SamplingParams,
                    priority: int = 1, kind: RequestType = RequestType.Generate, user_data=None) -> EngineRequest:
        prompt_ids = [int(t) for t in prompt_ids]
        if not prompt_ids:
            raise ValueError("empty prompt")
        V = self.mcfg.vocab_size
        if min(prompt_ids) < 0 or max(prompt_ids) >= V:
            # an id outside the embedding table would be an out-of-bounds gather on the GPU
            raise ValueError(f"prompt token ids must be in [0, {V}), got [{min(prompt_ids)}, {max(prompt_ids)}]")
        max_tokens = params.max_tokens
        if kind != RequestType.Embeddings:
            max_tokens = min(max_tokens, self.max_model_len - len(prompt_ids))
        if kind != RequestType.Embeddings and len(prompt_ids) >= self.max_model_len:
            raise ValueError(f"prompt of {len(prompt_ids)} tokens exceeds max_model_len={self.max_model_len}")
        if kind == RequestType.Embeddings and len(prompt_ids) > self.max_model_len:
            raise ValueError(f"input of {len(prompt_ids)} tokens exceeds max_model_len={self.max_model_len}")
        seq_id = next(self._seq_counter)
        req = EngineRequest(request_id=request_id, seq_id=seq_id, prompt_ids=prompt_ids, params=params,
                            priority=priority, kind=kind, user_data=user_data)
        req.detok = IncrementalDetokenizer(self.tokenizer, params.stop)
        if params.seed is None:
            params.seed = (hash(request_id) ^ (seq_id * 0x9E3779B97F4A7C15)) & _MASK63
        with self._lock:
            ok = self.sched.add(seq_id, prompt_ids, max(0, max_tokens), priority, params.ignore_eos,
                                kind == RequestType.Embeddings, params.stop_token_ids, params.min_tokens)
            if not ok:
                raise ValueError("scheduler rejected the request (duplicate id or too long)")
            self.requests[request_id] = req
            self.by_seq[seq_id] = req
        self.stats_counters["prompt_tokens"] += len(prompt_ids)
        if max_tokens <= 0 and kind != RequestType.Embeddings:
            self.abort(request_id, reason=FINISH_LENGTH)
        return req

    def abort(self, request_id: str, reason: int = FINISH_ABORT) -> bool:
        with self._lock:
            req = self.requests.get(request_id)
            if req is None or req.finished:
                return False
            self.sched.abort(req.seq_id)
            self._finish(req, reason)
            self._pending_aborts.append(request_id)
        return True

    def _finish(self, req: EngineRequest, reason: int):
        req.finished = True
        req.finish_reason = FINISH_NAMES.get(reason, "stop")
        req.finish_time = time.monotonic()
        self.requests.pop(req.request_id, None)
        self.by_seq.pop(req.seq_id, None)
        self.stats_counters["requests_finished"] += 1

    def has_work(self) -> bool:
        return (self.sched.has_work() or bool(self._pending_aborts) or self._deferred is not None
                or self._inflight is not None)

    # ------------------------------------------------------------------ step
    def _bind_slots(self, plan) -> None:
        """Per-slot parameter arrays: rebind only slots whose owner changed."""
        slots, sids = plan["slots"], plan["seq_ids"]
        stale = np.nonzero(self.slot_owner[slots] != sids)[0]
        for i in stale.tolist():
            s, sid = int(slots[i]), int(sids[i])
            r = self.by_seq.get(sid)
            self.slot_owner[s] = sid
            self.slot_req[s] = r
            self.slot_ngen[s] = len(r.output_ids) if r is not None else 0
            if r is None:
                self.slot_temp[s], self.slot_topp[s], self.slot_topk[s], self.slot_seed[s] = 0.0, 1.0, 0, 0
                continue
            p = r.params
            self.slot_temp[s], self.slot_topp[s], self.slot_topk[s] = p.temperature, p.top_p, p.top_k
            self.slot_seed[s] = np.uint64(p.seed & _MASK63)

    def _sampling_rows(self, plan) -> Optional[SamplingRows]:
        if not self.is_driver:
            return None
        idx = plan["sample_seq_index"]
        if idx.shape[0] == 0:
            return None
        slots = plan["slots"][idx]
        temps = self.slot_temp[slots]
        # counter-based per-request stream: mix(seed, #tokens generated so far)
        n = self.slot_ngen[slots].astype(np.uint64) if not (temps <= 0).all() else None
        if n is None:
            seeds = self.slot_seed[slots].view(np.int64)
        else:
            with np.errstate(over="ignore"):
                x = self.slot_seed[slots] * np.uint64(6364136223846793005) + (n + np.uint64(1)) * np.uint64(
                    1442695040888963407)
                x &= np.uint64(_MASK63)
                x ^= x >> np.uint64(29)
                x = (x * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(_MASK63)
            seeds = x.view(np.int64)
        return SamplingRows(temps, self.slot_topp[slots], self.slot_topk[slots], seeds)

    def _torch_profile_tick(self) -> None:
        """XGS_TORCH_PROFILE=N: record the next N steps with torch.profiler (CPU +
        HIP activity via roctracer) and write a Chrome trace to
        $XGS_TORCH_PROFILE_DIR (default ./gpurun_out) when done."""
        prof = self._tprof
        if prof is None:
            n = int(os.environ.get("XGS_TORCH_PROFILE", "0") or 0)
            if n <= 0:
                self._tprof = False
                return
            acts = [torch.profiler.ProfilerActivity.CPU]
            if self.device.type == "cuda":
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            prof = torch.profiler.profile(activities=acts, record_shapes=False)
            prof.__enter__()
            self._tprof, self._tprof_left = prof, n
            return
        if prof is False:
            return
        self._tprof_left -= 1
        if self._tprof_left <= 0:
            prof.__exit__(None, None, None)
            out = os.environ.get("XGS_TORCH_PROFILE_DIR", "gpurun_out")
            os.makedirs(out, exist_ok=True)
            path = os.path.join(out, f"torch_trace_rank{get_state().rank}_{os.getpid()}.json")
            prof.export_chrome_trace(path)
            log.info("torch.profiler trace written to %s", path)
            self._tprof = False

    def step(self) -> List[RequestOutput]:
        if self._tprof is not False:
            self._torch_profile_tick()
        if self._timing is None:
            return self._step()
        t0 = time.perf_counter()
        out = self._step()
        self._timing["step"] += time.perf_counter() - t0
        return out

    def _tick(self, phase: str, t0: float) -> float:
        t1 = time.perf_counter()
        if self._timing is not None:
            self._timing[phase] += t1 - t0
        return t1

    @staticmethod
    def _lookahead_src(prev: dict, nxt: dict) -> Optional[np.ndarray]:
        """Per decode row of `nxt`: the index, in `prev`'s sampled-token buffer (sample
        order: a decode graph step's rows, or an eager step's sampled rows), of the
        token that is this row's placeholder input; -1 if the row has a real id. None
        if no row needs one."""
        nd = int(nxt["num_decodes"])
        ids = nxt["input_ids"][:nd]
        need = ids == -1  # StepScheduler::kPlaceholder
        if not need.any():
            return None
        pids, cids = prev["seq_ids"][prev["sample_seq_index"]], nxt["seq_ids"][:nd]
        sorter = np.argsort(pids, kind="stable")
        k = np.clip(np.searchsorted(pids, cids, sorter=sorter), 0, len(pids) - 1)
        j = sorter[k]
        hit = pids[j] == cids
        if not hit[need].all():  # an unresolved id would be an out-of-range embedding gather
            raise RuntimeError("async scheduling: placeholder without a producing row")
        return np.where(need, j, -1).astype(np.int32)

    def _launch(self, plan, samp, src=None):
        """runner.launch on every TP rank: followers receive the same launch."""
        if get_state().tp_size > 1:
            comm.tp_broadcast_object(("launch", (plan, samp, src)), src=0)
        return self.runner.launch(plan, samp, src=src)

    def _step_async(self) -> List[RequestOutput]:
        """One step of the pipelined loop: retire the step launched by the previous
        call (or launch one now), but first plan and launch its successor when it is
        a pure-decode graph step -- the GPU always has the next step queued."""
        outs: List[RequestOutput] = []
        t = time.perf_counter()
        with self._lock:
            for rid in self._pending_aborts:
                outs.append(RequestOutput(rid, [], "", True, "abort"))
            self._pending_aborts.clear()
        cur, self._inflight = self._inflight, None
        if cur is None:
            with self._lock:
                plan = self.sched.schedule()
            t = self._tick("schedule", t)
            if plan["num_tokens"] == 0:
                return outs + self._flush_deferred()
            self._bind_slots(plan)
            samp = self._sampling_rows(plan)
            t = self._tick("prepare", t)
            handle = self._launch(plan, samp)
            t = self._tick("launch", t)
        else:
            plan, handle = cur
        ahead = False
        if self.runner.launched_as_graph(handle):
            with self._lock:
                ahead = self.sched.lookahead()
                nplan = self.sched.schedule() if ahead else None
            t = self._tick("schedule", t)
            if ahead:
                # the next step's sampling seeds count the token this step produces
                np.add.at(self.slot_ngen, plan["slots"][plan["sample_seq_index"]], 1)
                if nplan["num_tokens"] > 0:
                    self._bind_slots(nplan)
                    nsamp = self._sampling_rows(nplan)
                    src = self._lookahead_src(plan, nplan)
                    self._inflight = (nplan, self._launch(nplan, nsamp, src=src))
                    self.stats_counters["lookahead_launches"] += 1
                t = self._tick("launch", t)
        outs += self._emit_early(self._flush_deferred())  # previous step's outputs, while the GPU runs
        t = self._tick("emit_overlapped", t)
        toks, lps, hidden = self.runner.wait(handle)
        plan["_t_tokens"] = time.monotonic()
        t = self._tick("wait_gpu", t)
        n_sample = int(plan["num_sample"])
        counts = np.ones(n_sample, np.int32)
        if ahead:
            with self._lock:
                finished = self.sched.commit(toks)
            self.stats_counters["generation_tokens"] += n_sample
            fin_map = {f[0]: f for f in finished}
        else:
            fin_map = None
        return outs + self._finish_step(plan, toks, lps, hidden, counts, fin_map, t)

    def _step(self) -> List[RequestOutput]:
        if self._async:
            return self._step_async()
        outs: List[RequestOutput] = []
        t = t_step0 = time.perf_counter()
        with self._lock:
            for rid in self._pending_aborts:
                outs.append(RequestOutput(rid, [], "", True, "abort"))
            self._pending_aborts.clear()
            if self.spec is not None:
                outs += self._flush_deferred()  # the draft needs every request's tokens
                self.spec.propose()
            plan = self.sched.schedule()
        t = self._tick("schedule", t)
        st = get_state()
        if st.tp_size > 1:
            comm.tp_broadcast_object(("plan", plan), src=0)
        if plan["num_tokens"] == 0:
            return outs + self._flush_deferred()
        if self.is_driver:
            self._bind_slots(plan)
        samp = self._sampling_rows(plan)
        t = self._tick("prepare", t)
        counts = None
        if self.spec is not None and self.is_driver and plan["num_seqs"] > plan["num_decodes"]:
            toks, lps, hidden, counts = self.spec.verify_execute(plan, samp)
            plan["_t_tokens"] = time.monotonic()
        else:
            handle = self.runner.launch(plan, samp)
            t = self._tick("launch", t)
            outs += self._emit_early(self._flush_deferred())  # previous step's outputs, while this one runs
            t = self._tick("emit_overlapped", t)
            toks, lps, hidden = self.runner.wait(handle)
            plan["_t_tokens"] = time.monotonic()
            t = self._tick("wait_gpu", t)
        if counts is None:
            counts = np.ones(int(plan["num_sample"]), np.int32)
        if self.spec is not None and self.is_driver:
            self.spec.record_step(time.perf_counter() - t_step0, plan, counts)
        return outs + self._finish_step(plan, toks, lps, hidden, counts, None, t)

    def _finish_step(self, plan, toks, lps, hidden, counts, fin_map, t) -> List[RequestOutput]:
        """Bookkeeping after a step's tokens are on the host: stats, embeddings, the
        scheduler update (unless an async commit already did it: fin_map given),
        and output emission (deferred to the next step when nothing finished)."""
        self.step_count += 1
        self.stats_counters["steps"] += 1
        if plan["num_decodes"] == plan["num_seqs"]:
            self.stats_counters["decode_steps"] += 1
        self.stats_counters["prefill_tokens_computed"] += int(plan["num_tokens"]) - int(plan["num_decodes"])
        if hidden is not None:
            self._accumulate_embeddings(plan, hidden)
        n_sample = int(plan["num_sample"])
        if fin_map is None:
            fin_map = self._apply(plan, toks, counts)
        t = self._tick("apply", t)
        if not self.is_driver:
            return []
        first_tokens = bool(plan["is_prefill"][plan["sample_seq_index"]].any()) if n_sample else False
        # deferral only pays where the next step runs asynchronously (a GPU): on the CPU
        # the next launch computes the whole step, so deferring would add a step of
        # token delivery delay (Req 5.1) for nothing
        overlap = self.cfg.overlap_outputs and self.device.type == "cuda" and self.spec is None
        if overlap and not first_tokens and not fin_map:
            self._deferred = (plan, toks, lps, counts, fin_map)
            return []
        if overlap and EMIT_SPLIT:
            # only the rows whose output cannot wait -- finished requests (their slots are
            # being refilled) and first tokens (TTFT) -- are emitted before the next
            # step is planned; the other rows' outputs ride the next step's overlap window
            now_ids = set(fin_map) if fin_map else set()
            if first_tokens:
                sidx = plan["sample_seq_index"]
                pre = plan["is_prefill"][sidx].astype(bool)
                now_ids.update(int(x) for x in plan["seq_ids"][sidx][pre])
            with self._lock:
                outs = self._emit(plan, toks, lps, counts, fin_map, only=now_ids)
            self._deferred = (plan, toks, lps, counts, fin_map, now_ids)
            self._tick("emit_blocking", t)
            return outs
        with self._lock:
            outs = self._emit(plan, toks, lps, counts, fin_map)
        self._tick("emit_blocking", t)
        return outs

    def enable_step_timing(self, on: bool = True) -> None:
        """Accumulate host time per step phase (bench / profiling)."""
        import collections
        self._timing = collections.defaultdict(float) if on else None

    def step_timing(self) -> dict:
        return dict(self._timing or {})

    def _emit_early(self, outs: List[RequestOutput]) -> List[RequestOutput]:
        """Hand overlap-window outputs to the sink now (returns what is left for step())."""
        if outs and EARLY_OUTPUTS and self.output_sink is not None:
            self.output_sink(outs)
            return []
        return outs

    def _flush_deferred(self) -> List[RequestOutput]:
        d, self._deferred = self._deferred, None
        if d is None:
            return []
        with self._lock:
            if len(d) == 6:  # the rest of a split emission
                return self._emit(*d[:5], skip=d[5])
            return self._emit(*d)

    def _accumulate_embeddings(self, plan, hidden):
        from .. import ops
        emb = np.nonzero(plan["is_embed"])[0]
        if emb.size == 0:
            return
        qsl = plan["query_start_loc"]
        cu = []
        rows = []
        for i in emb.tolist():
            cu.append((int(qsl[i]), int(qsl[i + 1])))
            rows.append(int(plan["slots"][i]))
        for (a, b), r in zip(cu, rows):
            cut = torch.tensor([a, b], dtype=torch.int32, device=self.device)
            rr = torch.tensor([r], dtype=torch.int32, device=self.device)
            ops.segment_sum(hidden, cut, self.embed_acc, rr)

    def _process(self, plan, toks, lps, counts=None) -> List[RequestOutput]:
        """Apply + emit in one go (tests / callers that run the runner themselves)."""
        if counts is None:
            counts = np.ones(int(plan["num_sample"]), np.int32)
        fin_map = self._apply(plan, toks, counts)
        if not self.is_driver:
            return []
        with self._lock:
            return self._emit(plan, toks, lps, counts, fin_map)

    def _apply(self, plan, toks, counts) -> dict:
        """Feed sampled tokens to the C++ scheduler (stop checks, page publishing):
        the part the next schedule() depends on. `counts[j]` tokens belong to
        sampled sequence j (1 for plain decode; accepted drafts + 1 after a verify)."""
        with self._lock:
            finished = self.sched.update(toks if toks is not None else np.zeros(int(counts.sum()), np.int32),
                                         counts)
        if self.is_driver and counts.size:
            np.add.at(self.slot_ngen, plan["slots"][plan["sample_seq_index"]], counts)
        self.stats_counters["generation_tokens"] += int(counts.sum())
        return {f[0]: f for f in finished}

    def _emit(self, plan, toks, lps, counts, fin_map, only=None, skip=None) -> List[RequestOutput]:
        """Per-request host work of a step: detokenise, stop strings, RequestOutputs.
        only / skip: sets of sequence ids to restrict the sampled rows to / to leave out
        (a step's outputs emitted in two parts)."""
        outs: List[RequestOutput] = []
        ns = int(plan["num_seqs"])
        seq_ids = plan["seq_ids"]
        n_sample = int(plan["num_sample"])
        now = time.monotonic()
        sidx = plan["sample_seq_index"]
        t_tok = plan.get("_t_tokens", now)
        k = 0
        for j in range(n_sample):
            c = int(counts[j])
            sid = int(seq_ids[sidx[j]])
            req = self.by_seq.get(sid)
            if req is None or (only is not None and sid not in only) or (skip is not None and sid in skip):
                k += c
                continue
            f = fin_map.get(sid)
            # the scheduler stops appending at the first stop condition inside an accepted run
            take = c if f is None else max(1, min(c, f[3] - len(req.output_ids)))
            new = [int(t) for t in toks[k:k + take]]
            new_lps = [float(x) for x in lps[k:k + take]] if (lps is not None and req.params.logprobs) else None
            k += c
            if req.first_token_time is None:
                req.first_token_time = now
            req.output_ids.extend(new)
            text = req.detok.add(new)
            reason = None
            if req.detok.stopped and f is None:
                self.sched.abort(sid)
                reason = FINISH_STOP_SEQ
            elif f is not None:
                reason = f[1]
                req.cached_tokens = f[4]
                if not req.detok.stopped:
                    text += req.detok.flush()
            out = RequestOutput(req.request_id, new, text, reason is not None,
                                FINISH_NAMES.get(reason) if reason else None,
                                prompt_tokens=len(req.prompt_ids), completion_tokens=len(req.output_ids),
                                logprobs=new_lps, t_tokens=t_tok)
            if reason is not None:
                out.cached_tokens = req.cached_tokens
                self._finish(req, reason)
            outs.append(out)
        # prefill-only (embedding) completions: mean-pool + L2 normalise every finished
        # request's accumulator row in ONE device launch, one D2H copy
        done = []
        for sid, f in fin_map.items():
            if f[1] != FINISH_EMBED or (only is not None and sid not in only) or (skip is not None and sid in skip):
                continue
            req = self.by_seq.get(sid)
            if req is None:
                continue
            slot = None
            for i in range(ns):
                if int(seq_ids[i]) == sid:
                    slot = int(plan["slots"][i])
            done.append((req, slot))
        if done:
            from .. import ops
            rows = torch.tensor([s_ for _, s_ in done], dtype=torch.int32, device=self.device)
            cnt = torch.tensor([len(r.prompt_ids) for r, _ in done], dtype=torch.int32, device=self.device)
            embs = ops.mean_l2norm_rows(self.embed_acc, rows, cnt).cpu().tolist()
            for (req, _), emb in zip(done, embs):
                outs.append(RequestOutput(req.request_id, [], "", True, "stop", prompt_tokens=len(req.prompt_ids),
                                          completion_tokens=0, embedding=emb))
                self._finish(req, FINISH_EMBED)
        return outs

    # ------------------------------------------------------------------ followers (TP > 1)
    def follower_loop(self):
        """Non-leader TP ranks: mirror the leader's steps until told to stop.
        "plan" (synchronous steps): run it to completion. "launch" (asynchronous
        scheduling): enqueue it, then wait for the PREVIOUS launch only, so the
        next step is already queued behind the running one, as on the leader."""
        prev = None
        while True:
            kind, payload = comm.tp_broadcast_object(None, src=0)
            if kind == "stop":
                if prev is not None:
                    self.runner.wait(prev)
                return
            if kind == "plan":
                if prev is not None:
                    self.runner.wait(prev)
                    prev = None
                plan = payload
                if plan["num_tokens"]:
                    self.runner.execute(plan, None)
            elif kind == "launch":
                plan, samp, src = payload
                if plan["num_tokens"]:
                    h = self.runner.launch(plan, samp, src=src)
                    if prev is not None:
                        self.runner.wait(prev)
                    prev = h

    def stop_followers(self):
        if get_state().tp_size > 1 and self.is_driver:
            comm.tp_broadcast_object(("stop", None), src=0)

    # ------------------------------------------------------------------ helpers
    def generate(self, prompts: List[List[int]], params: SamplingParams, max_steps: int = 1 << 30):
        """Blocking batch generation (tests / offline use). Returns output id lists."""
        import copy
        rids = []
        for i, p in enumerate(prompts):
            rid = f"gen-{time.monotonic_ns()}-{i}"
            self.add_request(rid, p, copy.deepcopy(params))
            rids.append(rid)
        results = {r: [] for r in rids}
        done = set()
        steps = 0
        while len(done) < len(rids) and steps < max_steps:
            for o in self.step():
                if o.request_id in results:
                    results[o.request_id].extend(o.new_token_ids)
                    if o.finished:
                        done.add(o.request_id)
            steps += 1
        return [results[r] for r in rids]

    def kv_usage(self) -> float:
        """Memory pressure of the KV pool: pages pinned by live sequences. Prefix-cache
        pages nobody references are evictable on demand, so they do not count (else a
        warm cache would read as ~100 % and trip the degradation ladder)."""
        pinned = self.sched.num_used_blocks() - self.sched.num_evictable_blocks()
        return max(0, pinned) / max(1, self.sched.num_blocks())

    def stats(self) -> dict:
        cs = self.sched.cache_stats()
        bb = self._block_bytes()
        return {
            "model": self.mcfg.name,
            "waiting": self.sched.num_waiting(),
            "running": self.sched.num_running(),
            "kv_blocks_total": self.sched.num_blocks(),
            "kv_blocks_used": self.sched.num_used_blocks(),
            "kv_blocks_free": self.sched.num_free_blocks(),
            "kv_usage": self.kv_usage(),
            "memory_used": self.sched.num_used_blocks() * bb,
            "memory_available": (self.sched.num_free_blocks() + self.sched.num_evictable_blocks()) * bb,
            "memory_limit": int(self.sched.num_blocks() * bb * self.cfg.cache_threshold),
            "cache": cs,
            "preemptions": self.sched.total_preemptions(),
            **self.stats_counters,
            **({"speculative": self.spec.stats()} if self.spec is not None else {}),
        }

    def clear_prefix_cache(self):
        with self._lock:
            self.sched.clear_prefix_cache()

    def export_prefix(self, tokens: Sequence[int]):
        """CacheEntry for the longest cached page-aligned prefix of `tokens` (this rank's KV shard)."""
        from .kv_io import CacheEntry
        with self._lock:
            blocks = self.sched.cached_prefix([int(t) for t in tokens])
            idx = torch.tensor(blocks, dtype=torch.long, device=self.device)
            kv = self.runner.kv.index_select(2, idx).cpu()
        n = len(blocks) * self.cfg.block_size
        return CacheEntry([int(t) for t in tokens[:n]], kv, n, self.mcfg.name, self.cfg.block_size, self.tp_rank)

    def import_prefix(self, entry) -> int:
        """Install a CacheEntry into the prefix cache; returns #pages newly written."""
        if entry.block_size != self.cfg.block_size:
            raise ValueError(f"entry block_size {entry.block_size} != engine {self.cfg.block_size}")
        want = tuple(self.runner.kv.shape[:2]) + (entry.kv.shape[2],) + tuple(self.runner.kv.shape[3:])
        if tuple(entry.kv.shape) != want:
            raise ValueError(f"entry KV shape {tuple(entry.kv.shape)} does not match this engine {want}")
        n_pages = entry.kv.shape[2]
        with self._lock:
            res = self.sched.install_prefix([int(t) for t in entry.key], n_pages)
            if not res:
                raise MemoryError("no free KV pages to import the entry")
            before, blocks = res[0], res[1:]
            if len(blocks) > before:
                idx = torch.tensor(blocks[before:], dtype=torch.long, device=self.device)
                src = entry.kv[:, :, before:len(blocks)].to(self.device, self.runner.kv.dtype)
                self.runner.kv.index_copy_(2, idx, src)
        return len(blocks) - before

    def set_decode_prefill_cap(self, cap: Optional[int] = None) -> None:
        """Stall-free batching limit of decoding steps: at most `cap` prompt tokens of
        one prompt per step that also decodes; 0 lifts it (whole prompts, as many as
        the token budget takes); None restores the configured value. The mixed-step
        graphs captured for the configured cap stay valid for any smaller one."""
        cap = self.cfg.decode_prefill_cap if cap is None else max(0, min(int(cap), self.cfg.decode_prefill_cap or 1 << 30))
        with self._lock:
            self.sched.set_decode_prefill(cap, self._dp_seqs if cap > 0 else 0)

    def set_limits(self, max_num_seqs: int, max_num_batched_tokens: int):
        """Runtime batch limits (degradation / hot reload), clamped to the sizes the
        runner's buffers and graphs were built for."""
        with self._lock:
            self.sched.set_limits(max(1, min(max_num_seqs, self.cfg.max_num_seqs)),
                                  max(1, min(max_num_batched_tokens, self.cfg.max_num_batched_tokens)))
