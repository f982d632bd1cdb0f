"""Model runner: step plan -> device metadata -> forward -> logits -> sampled tokens.

* The paged KV cache is one zero-initialised HBM tensor [L, 2, NB, Hkv, bs, D]
  (zero-init: stale pages can never inject NaN into masked lanes), sized from
  the free HBM left after the weights (gpu_memory_utilization of 288 GB).
* All per-step int32 metadata of an eager step is packed into ONE pinned host
  buffer and moved with ONE async H2D copy.
* Pure-decode steps replay a HIP graph captured per padded batch size; the
  graph covers embedding -> all layers -> LM head -> sampling, so a decode step
  is one graph launch + one small H2D + one D2H. Padding rows use slot -1
  (no KV write) and seq_len 0 (no attention work).
* Mixed steps of the stall-free schedule -- the decode rows plus ONE prompt
  chunk of at most `mixed_chunk` tokens (the scheduler's decode_prefill_cap) --
  replay a graph too, captured per (padded decode rows, chunk): the eager
  forward of such a step costs more host time than its ~5 ms of GPU work. The
  chunk's rows are padded to the chunk size (slot -1, outside every sequence);
  its last row's logits follow the decode rows', so the sampled tokens come out
  in the plan's sample order.
"""
from __future__ import annotations

import logging
import math
import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import tune
from .. import ops
from ..models.base import AttnMeta
from ..ops.attention import DecodeWorkspace
from ..parallel import comm

# eager (prompt) steps leave their sampled tokens on the device for a looked-ahead successor
ASYNC_MIXED = True
# host wait for a step's results: poll the event (default; XGS_TUNE spin_wait=0: a
# blocking synchronize) for at most 50 ms before blocking (profiles/r2_spin_wait.md)
SPIN_WAIT = tune.get_bool("spin_wait", True)
SPIN_MAX_S = 0.050

log = logging.getLogger("xgserve.runner")


@dataclass
class SamplingRows:
    """Per-row sampling parameters (host numpy arrays), aligned with logits rows."""
    temps: np.ndarray
    top_ps: np.ndarray
    top_ks: np.ndarray
    seeds: np.ndarray  # int64, already mixed with the step counter

    @property
    def all_greedy(self) -> bool:
        return bool((self.temps <= 0).all())


def _pinned(n: int, dtype) -> torch.Tensor:
    t = torch.empty(n, dtype=dtype)
    return t.pin_memory() if torch.cuda.is_available() else t


def stage_mixed_inputs(plan: dict, Nd: int, nb: int, B: int, C: int, W: int, src: Optional[np.ndarray],
                       sec: tuple, hi: np.ndarray, hl: np.ndarray) -> None:
    """Host staging of a mixed-graph step (ModelRunner._execute_mixed): the plan's Nd
    decode rows go to rows [0, Nd) and its prompt chunk's q rows to [B, B + q) of the
    static ids / positions / slot buffers (padding: id 0, position 0, slot -1); seq
    lens [0, Nd) + the chunk's at B; the chunk's query_start_loc [0, q]; block-table
    rows likewise; lidx = the logits rows in sample order (decode rows, then the
    chunk's last row). sec: the section offsets of the int32 buffer `hi`."""
    T = int(plan["num_tokens"])
    q = T - Nd
    o = sec
    for k, arr, pad in ((0, plan["input_ids"], 0), (1, plan["positions"], 0), (2, plan["slot_mapping"], -1)):
        base = o[k]
        hi[base:base + Nd] = arr[:Nd]
        hi[base + Nd:base + nb] = pad
        hi[base + B:base + B + q] = arr[Nd:T]
        hi[base + B + q:base + B + C] = pad
    sl = plan["seq_lens"]
    hi[o[3]:o[3] + Nd] = sl[:Nd]
    hi[o[3] + Nd:o[3] + nb] = 0
    hi[o[3] + B] = sl[Nd]
    hi[o[4]:o[4] + nb] = -1
    if src is not None:
        hi[o[4]:o[4] + src.shape[0]] = src
    hi[o[5]] = 0
    hi[o[5] + 1] = q
    w = int(plan["bt_width"])
    bt = hi[o[6]:o[6] + (B + 1) * W].reshape(B + 1, W)
    pbt = plan["block_tables"].reshape(Nd + 1, w)
    bt[:Nd, :w] = pbt[:Nd]
    bt[B, :w] = pbt[Nd]
    hl[:Nd] = np.arange(Nd)
    hl[Nd] = nb + q - 1
    hl[Nd + 1:nb + 1] = 0


class ModelRunner:
    def __init__(self, model, *, block_size: int, num_blocks: int, max_num_seqs: int,
                 max_num_batched_tokens: int, max_model_len: int, use_graphs: bool = True,
                 graph_batch_sizes: Optional[List[int]] = None, is_driver: bool = True,
                 mixed_chunk: int = 0):
        self.model = model
        self.cfg = model.cfg
        self.device = model.device
        self.dtype = model.dtype
        self.bs = block_size
        self.num_blocks = num_blocks
        self.max_num_seqs = max_num_seqs
        self.max_tokens = max_num_batched_tokens
        self.max_model_len = max_model_len
        self.max_blocks_per_seq = (max_model_len + block_size - 1) // block_size + 1
        self.is_driver = is_driver
        self.capture_logits = False  # tests: keep the last eager step's logits
        self.last_logits = None
        cfg = self.cfg
        self.Hkv = model.num_kv_heads_local
        self.kv = torch.zeros(cfg.num_layers, 2, num_blocks, self.Hkv, block_size, cfg.head_dim,
                              dtype=self.dtype, device=self.device)
        self.kv_caches = [(self.kv[i, 0], self.kv[i, 1]) for i in range(cfg.num_layers)]
        self.is_cuda = self.device.type == "cuda"
        Hq_local = cfg.num_heads // model.tp
        self.max_splits = tune.get_int("decode_max_splits", 16)
        self.workspace = DecodeWorkspace(max(max_num_seqs, 1), Hq_local, cfg.head_dim, self.max_splits,
                                         self.device) if self.is_cuda else None
        # pinned staging for eager steps
        cap = 8 * max_num_batched_tokens + 4 * max_num_seqs * (self.max_blocks_per_seq + 4) + 64
        # two pinned host staging buffers + device twins: a step may return
        # before its async H2D copy ran, so the next step must not overwrite the
        # same host buffer until that copy's event has completed
        self.h_stages = [_pinned(cap, torch.int32) for _ in range(2)]
        self.d_stages = [torch.empty(cap, dtype=torch.int32, device=self.device) for _ in range(2)]
        self.stage_events = [None, None]
        self.stage_idx = 0
        # sampled tokens / logprobs D2H: two pinned buffers + an event each, so a step
        # launched before the previous one was waited on never overwrites its results
        nt = max(max_num_batched_tokens, max_num_seqs)
        self.h_toks = [_pinned(nt, torch.int32) for _ in range(2)]
        self.h_lps = [_pinned(nt, torch.float32) for _ in range(2)]
        self.out_idx = 0
        self._es_pin = [None, None]   # eager-step sampling rows: pinned stagings + events
        self._es_ev = [None, None]
        self._es_idx = 0
        # XGS_TEST_SAMPLE_LOG=1 (tests): every eager sample of this rank, to check that TP
        # followers draw exactly the leader's tokens at temperature > 0
        self.sample_log = [] if os.environ.get("XGS_TEST_SAMPLE_LOG") == "1" else None
        # graphs
        self.use_graphs = use_graphs and self.is_cuda
        if graph_batch_sizes is None:
            graph_batch_sizes = [1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 256]
        self.graph_bs = sorted(b for b in graph_batch_sizes if b <= max_num_seqs)
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        # mixed-step graphs: (decode bucket, chunk) -> graph; buckets of >= 16 decode rows
        # whose step stays on the gemm_mw path (decode rows + chunk <= MW_MAX_TOKENS)
        self.mixed_chunk = int(mixed_chunk) if (self.use_graphs and comm.get_state().tp_size == 1) else 0
        self.mixed_graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        self.mixed_bs: List[int] = []
        self.mixed_replays = 0
        if self.mixed_chunk > 0:
            # decode rows + chunk run on gemm_mw when every layer has it and they fit
            # (<= MW_MAX_TOKENS rows), else on the library GEMMs (graph-capturable too): a
            # chunk of a whole prompt (e.g. 512) replays as one graph instead of an eager
            # step whose host-side launch of ~400 kernels the GPU would wait on
            from ..models.llama import MW_MAX_TOKENS
            mw = getattr(model, "_mw_ok", False) and 16 + self.mixed_chunk <= MW_MAX_TOKENS
            lim = MW_MAX_TOKENS if mw else max_num_batched_tokens
            self.mixed_bs = [b for b in self.graph_bs if b >= 16 and b + self.mixed_chunk <= lim]
            if not self.mixed_bs:
                self.mixed_chunk = 0
        self._graph_pool = None
        self._init_graph_buffers()
        # custom all-reduce peer-wait limit while serving (EngineConfig.collective_timeout_s);
        # warmup, graph capture and the first WARM_LAUNCHES steps run under the warmup limit
        self.collective_timeout_s = 2.0
        self._warm_launches = self.WARM_LAUNCHES
        from ..parallel.custom_ar import CustomAllReduce
        self._set_comm_timeout(CustomAllReduce.WARMUP_TIMEOUT_S)

    # ------------------------------------------------------------------ utils
    def kv_bytes(self) -> int:
        return self.kv.numel() * self.kv.element_size()

    DECODE_SPLIT_WGS = 512

    def decode_splits(self, bs: int) -> int:
        wgs = max(1, bs * self.Hkv)
        target = self.DECODE_SPLIT_WGS
        if 4 * wgs >= 3 * target:
            # within a quarter of the target (e.g. the 63 decode rows of a mixed step):
            # a second split would only add the combine launch
            return 1
        return int(max(1, min(self.max_splits, (target + wgs - 1) // wgs)))

    # ------------------------------------------------------------------ graph buffers
    def _init_graph_buffers(self):
        B = max(self.graph_bs) if self.graph_bs else 1
        W = self.max_blocks_per_seq
        self.g_B, self.g_W = B, W
        # int32 region: ids | pos | slots | sl | src | bt ; sampling region separate.
        # src[i] >= 0: row i's input id is the previous graph step's sampled token
        # g_out_tok[src[i]] (asynchronous scheduling), substituted inside the graph
        n = 5 * B + B * W
        self.g_int = torch.zeros(n, dtype=torch.int32, device=self.device)
        self.g_ids = self.g_int[0:B]
        self.g_pos = self.g_int[B:2 * B]
        self.g_slot = self.g_int[2 * B:3 * B]
        self.g_sl = self.g_int[3 * B:4 * B]
        self.g_src = self.g_int[4 * B:5 * B]
        self.g_bt = self.g_int[5 * B:5 * B + B * W].view(B, W)
        # sampling parameters: one row more than the widest decode graph (mixed steps)
        self.g_temp = torch.zeros(B + 1, dtype=torch.float32, device=self.device)
        self.g_topp = torch.ones(B + 1, dtype=torch.float32, device=self.device)
        self.g_topk = torch.zeros(B + 1, dtype=torch.int32, device=self.device)
        self.g_seed = torch.zeros(B + 1, dtype=torch.int64, device=self.device)
        # two sets of pinned host inputs (event-guarded): the next step's inputs can be
        # written while this step's H2D copies are still queued behind the GPU
        self.h_ints = [_pinned(n, torch.int32) for _ in range(2)]
        self.h_samp_fs = [_pinned(2 * (B + 1), torch.float32) for _ in range(2)]
        self.h_samp_is = [_pinned(B + 1, torch.int32) for _ in range(2)]
        self.h_samp_ss = [_pinned(B + 1, torch.int64) for _ in range(2)]
        self.g_stage_events = [None, None]
        self.g_stage_idx = 0
        # sampled tokens [0, OB) and their logprobs [OB, 2 OB) in one buffer: a graph step's
        # outputs leave in ONE D2H copy (g_out[:OB + n]) instead of two; OB = B + 1 (a
        # mixed step samples its decode rows + the chunk's last row)
        OB = self.g_OB = B + 1
        self.g_out = torch.zeros(2 * OB, dtype=torch.int32, device=self.device)
        self.g_out_tok = self.g_out[:OB]
        self.g_out_lp = self.g_out[OB:].view(torch.float32)
        self.h_gout = [_pinned(2 * OB, torch.int32) for _ in range(2)]
        self.g_greedy_graph: Dict[int, bool] = {}
        # mixed-step inputs: ids | pos | slot (B + C rows each) | sl (B + 1) | src (B) |
        # qsl (2) | bt ((B + 1) x W) ; lidx (int64, B + 1)
        C = self.mixed_chunk
        if C > 0:
            R = B + C
            self.m_sec = (0, R, 2 * R, 3 * R, 3 * R + B + 1, 3 * R + 2 * B + 1, 3 * R + 2 * B + 3)
            n_m = self.m_sec[-1] + (B + 1) * W
            self.m_int = torch.zeros(n_m, dtype=torch.int32, device=self.device)
            o = self.m_sec
            self.m_ids, self.m_pos, self.m_slot = self.m_int[o[0]:o[1]], self.m_int[o[1]:o[2]], self.m_int[o[2]:o[3]]
            self.m_sl, self.m_src, self.m_qsl = self.m_int[o[3]:o[4]], self.m_int[o[4]:o[5]], self.m_int[o[5]:o[6]]
            self.m_bt = self.m_int[o[6]:].view(B + 1, W)
            self.m_lidx = torch.zeros(B + 1, dtype=torch.int64, device=self.device)
            self.h_mints = [_pinned(n_m, torch.int32) for _ in range(2)]
            self.h_mlidx = [_pinned(B + 1, torch.int64) for _ in range(2)]

    def _decode_body(self, bs: int, greedy: bool):
        ops.subst_tokens(self.g_ids[:bs], self.g_src[:bs], self.g_out_tok)
        meta = AttnMeta(num_tokens=bs, num_decodes=bs, positions=self.g_pos[:bs], slot_mapping=self.g_slot[:bs],
                        dec_block_tables=self.g_bt[:bs], dec_seq_lens=self.g_sl[:bs],
                        num_splits=self.decode_splits(bs), workspace=self.workspace)
        h = self.model(self.g_ids[:bs], meta, self.kv_caches)
        logits = self.model.compute_logits(h)
        if greedy:
            ops.argmax_logprob(logits, self.g_out_tok[:bs], self.g_out_lp[:bs])
        else:
            tok, lp = ops.sample_tokens(logits, self.g_temp[:bs], self.g_topp[:bs], self.g_topk[:bs],
                                        self.g_seed[:bs], step=0)
            self.g_out_tok[:bs].copy_(tok)
            self.g_out_lp[:bs].copy_(lp)

    def _mixed_body(self, nb: int, greedy: bool):
        """nb decode rows (padded) + one prompt chunk of up to C rows (padded) -> the
        sampled tokens of the decode rows and the chunk's last row (g_out_tok[:nb + 1])."""
        B, C = self.g_B, self.mixed_chunk
        T = nb + C
        ops.subst_tokens(self.m_ids[:nb], self.m_src[:nb], self.g_out_tok)
        ids, pos, slot = self.m_ids[:B + C], self.m_pos[:B + C], self.m_slot[:B + C]
        # decode rows [0, nb) and the chunk [B, B + C) of the B + C row buffers, as one
        # contiguous [nb + C] view when nb == B, else gathered into place
        if nb == B:
            ids_t, pos_t, slot_t = ids, pos, slot
        else:
            ids_t = torch.cat([ids[:nb], ids[B:]])
            pos_t = torch.cat([pos[:nb], pos[B:]])
            slot_t = torch.cat([slot[:nb], slot[B:]])
        meta = AttnMeta(num_tokens=T, num_decodes=nb, positions=pos_t, slot_mapping=slot_t,
                        dec_block_tables=self.m_bt[:nb], dec_seq_lens=self.m_sl[:nb],
                        num_splits=self.decode_splits(nb), workspace=self.workspace,
                        pre_block_tables=self.m_bt[B:B + 1], pre_qsl=self.m_qsl, pre_seq_lens=self.m_sl[B:B + 1],
                        pre_max_q=C)
        h = self.model(ids_t, meta, self.kv_caches)
        logits = self.model.compute_logits(h.index_select(0, self.m_lidx[:nb + 1]))
        if greedy:
            ops.argmax_logprob(logits, self.g_out_tok[:nb + 1], self.g_out_lp[:nb + 1])
        else:
            tok, lp = ops.sample_tokens(logits, self.g_temp[:nb + 1], self.g_topp[:nb + 1], self.g_topk[:nb + 1],
                                        self.g_seed[:nb + 1], step=0)
            self.g_out_tok[:nb + 1].copy_(tok)
            self.g_out_lp[:nb + 1].copy_(lp)

    # the first launches run under the generous peer-wait limit too (first-call RCCL
    # communicator setup of a subgroup, first-seen library GEMM shapes)
    WARM_LAUNCHES = 32

    def _set_comm_timeout(self, seconds: float) -> None:
        from ..parallel.custom_ar import CustomAllReduce
        ar = comm.custom_allreduce()
        if ar is not None:
            ar.set_timeout(seconds if seconds >= CustomAllReduce.WARMUP_TIMEOUT_S else ar.serve_timeout(seconds))

    @torch.no_grad()
    def capture_graphs(self):
        if not self.use_graphs or not self.graph_bs:
            return
        torch.cuda.synchronize()
        # neutral inputs: padding rows (no KV writes, no attention work)
        self.g_slot.fill_(-1)
        self.g_src.fill_(-1)
        self.g_sl.fill_(0)
        self.g_ids.fill_(0)
        self.g_pos.fill_(0)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for bs in reversed(self.graph_bs):
                for greedy in (True, False):
                    for _ in range(2):
                        self._decode_body(bs, greedy)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self._graph_pool = torch.cuda.graph_pool_handle()
        for bs in reversed(self.graph_bs):
            for greedy in (True, False):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self._graph_pool):
                    self._decode_body(bs, greedy)
                self.graphs[(bs, greedy)] = g
        torch.cuda.synchronize()
        log.info("captured %d decode graphs (batch sizes %s)", len(self.graphs), self.graph_bs)
        if self.mixed_chunk > 0:
            self._capture_mixed()

    def _capture_mixed(self):
        # neutral inputs: padding decode rows, an empty chunk (q = 0: no attention rows)
        self.m_int.zero_()
        self.m_slot.fill_(-1)
        self.m_src.fill_(-1)
        self.m_lidx.zero_()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for nb in reversed(self.mixed_bs):
                for greedy in (True, False):
                    for _ in range(2):
                        self._mixed_body(nb, greedy)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        for nb in reversed(self.mixed_bs):
            for greedy in (True, False):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self._graph_pool):
                    self._mixed_body(nb, greedy)
                self.mixed_graphs[(nb, greedy)] = g
        torch.cuda.synchronize()
        log.info("captured %d mixed-step graphs (decode rows %s + a %d-token chunk)", len(self.mixed_graphs),
                 self.mixed_bs, self.mixed_chunk)

    def _mixed_bucket(self, plan, Nd: int, ns: int, T: int) -> Optional[int]:
        """Decode bucket of a mixed-graph step, or None: Nd decode rows + exactly one
        prefill chunk of <= mixed_chunk tokens (no verify rows, no embeddings)."""
        if not self.mixed_graphs or ns != Nd + 1 or T - Nd > self.mixed_chunk or T - Nd < 1:
            return None
        if not plan["is_prefill"][Nd] or plan["is_embed"][Nd]:
            return None
        for b in self.mixed_bs:
            if b >= Nd:
                return b
        return None

    def _graph_bucket(self, n: int) -> Optional[int]:
        for b in self.graph_bs:
            if b >= n:
                return b
        return None

    # ------------------------------------------------------------------ execution
    @torch.no_grad()
    def execute(self, plan: dict, samp: Optional[SamplingRows]):
        """Run one step. Returns (tokens np[int32], logprobs np[float32], hidden or None).
        On non-driver TP ranks the returned arrays are None."""
        return self.wait(self.launch(plan, samp))

    @torch.no_grad()
    def launch(self, plan: dict, samp: Optional[SamplingRows], src: Optional[np.ndarray] = None):
        """Enqueue one step (inputs H2D, forward, sampling, tokens D2H) without
        waiting for it; `wait(handle)` returns what `execute` returns. The host
        can do other work (previous step's detokenisation, planning the next step)
        while the GPU runs. `src` (asynchronous scheduling): per decode row, the
        row of the previous GRAPH step whose sampled token is this row's input
        (-1: the plan's own id)."""
        T = int(plan["num_tokens"])
        Nd = int(plan["num_decodes"])
        ns = int(plan["num_seqs"])
        if T == 0:
            return (0, None, (None, None, None), None)
        if self._warm_launches:
            self._warm_launches -= 1
            if self._warm_launches == 0:
                self._set_comm_timeout(self.collective_timeout_s)
        need_hidden = bool(plan["is_embed"].any()) if ns else False
        bucket = self._graph_bucket(Nd) if (Nd == ns and T == Nd and not need_hidden) else None
        if bucket is not None and self.graphs:
            return self._execute_graph(plan, samp, Nd, bucket, src)
        if not need_hidden and self.mixed_chunk > 0:
            mb = self._mixed_bucket(plan, Nd, ns, T)
            if mb is not None:
                return self._execute_mixed(plan, samp, Nd, mb, src)
        return self._execute_eager(plan, samp, need_hidden, src)

    def launched_as_graph(self, handle) -> bool:
        """True if the step left its sampled tokens in g_out_tok (every graph step,
        and eager steps that qualify for tokens_to_device): the next step may be
        planned and launched before this one completes."""
        return len(handle) > 4 and handle[4]

    @staticmethod
    def _poll_comm():
        """Queue the custom all-reduce's error-counter copy behind this step's work
        (TP): wait() then fails the step if a peer wait timed out."""
        ar = comm.custom_allreduce()
        if ar is not None:
            ar.poll_async()

    @staticmethod
    def _check_comm():
        ar = comm.custom_allreduce()
        if ar is not None:
            ar.check()

    def _record_out(self, n: int, tok: torch.Tensor, lp: torch.Tensor, hidden, graph: bool):
        """Tokens / logprobs D2H into the next of the two pinned buffers + an event."""
        self._poll_comm()
        i = self.out_idx
        self.out_idx ^= 1
        self.h_toks[i][:n].copy_(tok[:n], non_blocking=True)
        self.h_lps[i][:n].copy_(lp[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return (n, hidden, None, (i, ev), graph)

    @staticmethod
    def _wait_event(ev):
        """Block until `ev` completed. SPIN_WAIT: poll hipEventQuery instead of a
        blocking synchronize (whose sleeping wake-up costs ~0.1 ms per step on the host
        critical path), falling back to the blocking wait after SPIN_MAX_S."""
        if not SPIN_WAIT:
            ev.synchronize()
            return
        t_end = time.perf_counter() + SPIN_MAX_S
        while not ev.query():
            if time.perf_counter() > t_end:
                ev.synchronize()
                return

    def wait(self, handle):
        n, hidden, ready, out = handle[:4]
        if ready is not None:
            return ready
        if out is None:
            ev = handle[5] if len(handle) > 5 else None
            if ev is not None:
                self._wait_event(ev)  # this step only (TP follower with a successor queued)
            else:
                torch.cuda.current_stream().synchronize()
            self._check_comm()
            return None, None, hidden
        i, ev = out[0], out[1]
        self._wait_event(ev)  # this step only: a step queued behind it keeps running
        self._check_comm()
        if len(out) > 2:  # graph step: tokens and logprobs in one pinned buffer
            OB = out[2]
            h = self.h_gout[i]
            return h[:n].numpy().copy(), h[OB:OB + n].view(torch.float32).numpy().copy(), hidden
        return self.h_toks[i][:n].numpy().copy(), self.h_lps[i][:n].numpy().copy(), hidden

    def _execute_graph(self, plan, samp: Optional[SamplingRows], n: int, bs: int, src: Optional[np.ndarray]):
        B, W = self.g_B, self.g_W
        si = self.g_stage_idx
        self.g_stage_idx ^= 1
        if self.g_stage_events[si] is not None:
            self.g_stage_events[si].synchronize()  # the H2D copies that last read this set have run
        h_int = self.h_ints[si]
        hi = h_int.numpy()
        w = int(plan["bt_width"])
        hi[0:n] = plan["input_ids"]
        hi[n:bs] = 0
        hi[B:B + n] = plan["positions"]
        hi[B + n:B + bs] = 0
        hi[2 * B:2 * B + n] = plan["slot_mapping"]
        hi[2 * B + n:2 * B + bs] = -1
        hi[3 * B:3 * B + n] = plan["seq_lens"]
        hi[3 * B + n:3 * B + bs] = 0
        hi[4 * B:4 * B + bs] = -1
        if src is not None:
            hi[4 * B:4 * B + n] = src
        bt = hi[5 * B:5 * B + bs * W].reshape(bs, W)
        bt[:n, :w] = plan["block_tables"].reshape(n, w)
        # ids..src (5*B) and the first bs rows of bt: one contiguous H2D copy
        self.g_int[:5 * B + bs * W].copy_(h_int[:5 * B + bs * W], non_blocking=True)
        greedy = samp is None or samp.all_greedy
        if not greedy:
            self._stage_sampling(si, samp, n)
        ev = self.g_stage_events[si] or torch.cuda.Event()
        ev.record()
        self.g_stage_events[si] = ev
        self.graphs[(bs, greedy)].replay()
        self._log_samples(n)
        if not self.is_driver:
            # no D2H to wait on; wait() still drains before the pinned inputs get rewritten
            self._poll_comm()
            ev = torch.cuda.Event()
            ev.record()
            return (n, None, None, None, True, ev)
        return self._graph_out(n)

    def _stage_sampling(self, si: int, samp: SamplingRows, n: int) -> None:
        """Per-row sampling parameters of a graph step -> g_temp / g_topp / g_topk / g_seed."""
        hf, hsi, hss = self.h_samp_fs[si], self.h_samp_is[si], self.h_samp_ss[si]
        OB = self.g_OB
        f = hf.numpy()
        f[:n] = samp.temps
        f[OB:OB + n] = samp.top_ps
        hsi.numpy()[:n] = samp.top_ks
        hss.numpy()[:n] = samp.seeds
        self.g_temp[:n].copy_(hf[:n], non_blocking=True)
        self.g_topp[:n].copy_(hf[OB:OB + n], non_blocking=True)
        self.g_topk[:n].copy_(hsi[:n], non_blocking=True)
        self.g_seed[:n].copy_(hss[:n], non_blocking=True)

    def _graph_out(self, n: int):
        """Queue a graph step's D2H of its n sampled tokens + logprobs (g_out)."""
        OB = self.g_OB
        self._poll_comm()
        i = self.out_idx
        self.out_idx ^= 1
        self.h_gout[i][:OB + n].copy_(self.g_out[:OB + n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return (n, None, None, (i, ev, OB), True)

    def _execute_mixed(self, plan, samp: Optional[SamplingRows], Nd: int, nb: int, src: Optional[np.ndarray]):
        """Replay the (nb, chunk) mixed graph: Nd decode rows at [0, Nd), the prompt
        chunk's q rows at [B, B + q) of the static input buffers."""
        B, W, C = self.g_B, self.g_W, self.mixed_chunk
        n = int(plan["num_sample"])
        si = self.g_stage_idx
        self.g_stage_idx ^= 1
        if self.g_stage_events[si] is not None:
            self.g_stage_events[si].synchronize()
        stage_mixed_inputs(plan, Nd, nb, B, C, W, src, self.m_sec, self.h_mints[si].numpy(),
                           self.h_mlidx[si].numpy())
        self.m_int.copy_(self.h_mints[si], non_blocking=True)
        self.m_lidx[:nb + 1].copy_(self.h_mlidx[si][:nb + 1], non_blocking=True)
        greedy = samp is None or samp.all_greedy
        if not greedy:
            self._stage_sampling(si, samp, n)
        ev = self.g_stage_events[si] or torch.cuda.Event()
        ev.record()
        self.g_stage_events[si] = ev
        self.mixed_graphs[(nb, greedy)].replay()
        self.mixed_replays += 1
        self._log_samples(n)
        if not self.is_driver:
            self._poll_comm()
            ev = torch.cuda.Event()
            ev.record()
            return (n, None, None, None, True, ev)
        return self._graph_out(n)

    def _stage_parts(self, parts):
        """The int32 arrays of an eager step -> ONE pinned host buffer -> ONE async H2D
        copy (two buffers, event-guarded). Returns (device buffer, section offsets)."""
        sizes = [p.size for p in parts]
        total = sum(sizes)
        si = self.stage_idx
        self.stage_idx ^= 1
        ev = self.stage_events[si]
        if ev is not None:
            ev.synchronize()  # the H2D copy that last read this host buffer has run
        h_stage, d_stage = self.h_stages[si], self.d_stages[si]
        hs = h_stage.numpy()
        off = 0
        for p in parts:
            hs[off:off + p.size] = p.reshape(-1)
            off += p.size
        if self.is_cuda:
            d_stage[:total].copy_(h_stage[:total], non_blocking=True)
            if self.stage_events[si] is None:
                self.stage_events[si] = torch.cuda.Event()
            self.stage_events[si].record()
            dev = d_stage
        else:
            dev = h_stage
        return dev, np.cumsum([0] + sizes)

    def _execute_eager(self, plan, samp: Optional[SamplingRows], need_hidden: bool, src: Optional[np.ndarray]):
        T = int(plan["num_tokens"])
        Nd = int(plan["num_decodes"])
        ns = int(plan["num_seqs"])
        w = int(plan["bt_width"])
        Np = ns - Nd
        li = plan["logits_indices"]
        S = li.shape[0]
        qsl = plan["query_start_loc"]
        parts = [plan["input_ids"], plan["positions"], plan["slot_mapping"],
                 plan["block_tables"], plan["seq_lens"], (qsl[Nd:] - Nd).astype(np.int32), li]
        if src is not None:  # staged with the other inputs: no blocking copy ahead of the queued step
            parts.append(np.ascontiguousarray(src, dtype=np.int32))
        dev, o = self._stage_parts(parts)
        ids = dev[o[0]:o[1]]
        pos = dev[o[1]:o[2]]
        slots = dev[o[2]:o[3]]
        bt = dev[o[3]:o[4]].view(ns, w)
        sl = dev[o[4]:o[5]]
        pre_qsl = dev[o[5]:o[6]]
        lidx = dev[o[6]:o[7]]
        if src is not None:  # decode rows first: their ids from the previous step's sampled tokens
            ops.subst_tokens(ids[:src.shape[0]], dev[o[7]:o[8]], self.g_out_tok)
        meta = AttnMeta(num_tokens=T, num_decodes=Nd, positions=pos, slot_mapping=slots,
                        dec_block_tables=bt[:Nd], dec_seq_lens=sl[:Nd],
                        num_splits=self.decode_splits(Nd) if self.is_cuda else 1, workspace=self.workspace,
                        pre_block_tables=bt[Nd:], pre_qsl=pre_qsl, pre_seq_lens=sl[Nd:],
                        pre_max_q=int(plan["q_lens"][Nd:].max()) if Np > 0 else 0)
        h = self.model(ids, meta, self.kv_caches)
        hid = h if need_hidden else None
        if S == 0:
            return (0, hid, (np.zeros(0, np.int32), np.zeros(0, np.float32), hid), None)
        logits = self.model.compute_logits(h.index_select(0, lidx.long()))
        if self.capture_logits:
            self.last_logits = logits.float().cpu()
        if not self.is_driver:
            if self.is_cuda:
                # asynchronous prompt steps under TP: when the leader leaves this step's
                # tokens on the device, so does every follower -- the same all-gathered
                # logits and the leader's broadcast sampling rows give the same tokens, and
                # the successor's decode rows substitute their ids from this rank's
                # g_out_tok exactly as after a graph step
                on_dev = self._async_ok(S, plan)
                if on_dev:
                    tok, _ = self._sample(logits, samp)
                    self.g_out_tok[:S].copy_(tok[:S])
                    self._log_samples(S)
                # an event of THIS step: a follower that queued its successor waits
                # for this launch only (engine.follower_loop), not the whole stream
                self._poll_comm()
                ev = torch.cuda.Event()
                ev.record()
                return (S, hid, None, None, on_dev, ev)
            return (S, hid, (None, None, hid), None)
        tok, lp = self._sample(logits, samp)
        if self.is_cuda:
            on_dev = self.tokens_to_device(S, tok, plan)
            return self._record_out(S, tok, lp, hid, on_dev)
        return (S, hid, (tok.numpy().astype(np.int32), lp.numpy().astype(np.float32), hid), None)

    def _sample(self, logits: torch.Tensor, samp: Optional[SamplingRows]):
        if samp is None or samp.all_greedy:
            tok, lp = ops.argmax_logprob(logits)
        elif self.is_cuda:
            # eager-step sampling rows through two event-guarded pinned stagings (async
            # H2D; a follower samples every asynchronous eager step, so no pageable copy
            # or host sync on its step path)
            n = len(samp.temps)
            i = self._es_idx
            self._es_idx ^= 1
            if self._es_ev[i] is not None:
                self._es_ev[i].synchronize()
            if self._es_pin[i] is None or self._es_pin[i][1].numel() < n:
                m = max(n, 64)
                self._es_pin[i] = (_pinned(2 * m, torch.float32), _pinned(m, torch.int32), _pinned(m, torch.int64))
            hf, hk, hs = self._es_pin[i]
            f = hf.numpy()
            f[:n] = samp.temps
            f[n:2 * n] = samp.top_ps
            hk.numpy()[:n] = samp.top_ks
            hs.numpy()[:n] = samp.seeds
            dev_f = hf[:2 * n].to(self.device, non_blocking=True).view(2, n)
            topk = hk[:n].to(self.device, non_blocking=True)
            seeds = hs[:n].to(self.device, non_blocking=True)
            ev = self._es_ev[i] or torch.cuda.Event()
            ev.record()
            self._es_ev[i] = ev
            tok, lp = ops.sample_tokens(logits, dev_f[0], dev_f[1], topk, seeds, step=0)
        else:
            dev_f = torch.from_numpy(np.stack([samp.temps, samp.top_ps]).astype(np.float32))
            topk = torch.from_numpy(samp.top_ks.astype(np.int32))
            seeds = torch.from_numpy(samp.seeds.astype(np.int64))
            gen = torch.Generator().manual_seed(int(samp.seeds[0]) & 0x7FFFFFFF)
            tok, lp = ops.sample_tokens(logits, dev_f[0], dev_f[1], topk, seeds, step=0, generator=gen)
        return tok, lp

    def _log_samples(self, n: int) -> None:
        """(tests) the tokens of a step this rank sampled into g_out_tok -- the steps
        whose successor reads its decode ids from there on EVERY rank"""
        if self.sample_log is not None:
            self.sample_log.append(self.g_out_tok[:n].cpu().tolist())

    def _async_ok(self, S: int, plan: dict) -> bool:
        """May an eager step's successor be planned before its tokens reach the host?
        The same answer on every TP rank (it depends on the plan only)."""
        return not (not ASYNC_MIXED or not self.graphs or S > self.g_B or bool(plan["is_embed"].any())
                    or int(plan["num_sample"]) != S)

    def tokens_to_device(self, S: int, tok: torch.Tensor, plan: dict) -> bool:
        """Eager step: also leave the sampled tokens in g_out_tok, in sample order, so
        the engine can plan and launch the next step before this one ends (its decode
        rows substitute their ids from there; TP followers do the same from their own
        sampling, _execute_eager). Verify / embedding steps and batches wider than the
        graph buffers stay synchronous."""
        if not self._async_ok(S, plan):
            return False
        self.g_out_tok[:S].copy_(tok[:S])
        self._log_samples(S)
        return True
