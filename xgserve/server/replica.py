"""Model replicas: the spec's Inference Worker (Req 7, requirements.md:100-110;
design.md:310-361) as an *engine loop* that owns one LLMEngine (a TP group).

* `EngineLoop` -- the worker main loop: drains commands (add / abort /
  set_limits / clear_cache / stop), runs `engine.step()` while there is work,
  emits RequestOutputs and a heartbeat with engine stats every 0.5 s. A step
  that raises is contained: HIP OOM -> flush the prefix cache and retry once
  (Req 9.3), then fail only the requests that were in flight with
  `out_of_memory`; any other exception fails the in-flight requests with
  `inference_failed` (Property 22) and the loop keeps serving -- except a TP
  collective timeout (CustomAllReduceTimeout: a peer died or stalled, the group
  is out of step), which fails the in-flight requests and kills the replica so
  the orchestrator restarts it.
* `InProcessReplica` -- engine + loop on a thread of the server process
  (tp == 1; tests, CPU configs).
* `ProcessReplica` -- one OS process per GPU (spawned, so HIP is initialised
  fresh in each): rank 0 runs the EngineLoop and talks to the server over two
  multiprocessing queues; ranks 1..tp-1 run `engine.follower_loop()` and
  receive step plans over the TP group (design note SURVEY.md 3.3 A). Crash
  detection = process liveness + heartbeat age (Req 7.4, 9.4).
"""
from __future__ import annotations

import logging
import json
import os
import queue as pyqueue
import threading
import time
import traceback
from typing import Any, Callable, Dict, List, Optional

log = logging.getLogger("xgserve.replica")

HEARTBEAT_S = 0.5


# ---------------------------------------------------------------------------
# engine construction (runs inside the replica)
# ---------------------------------------------------------------------------
def engine_spec(worker, cache=None, spec=None, fault: Optional[dict] = None, batcher=None) -> dict:
    """Plain-dict (picklable) description of one replica's engine. `fault` holds
    MockEngine fault-injection knobs (crash_after_steps, eos_every)."""
    dt = {"bf16": "bfloat16", "fp16": "float16", "fp32": "float32", "fp8": "bfloat16", "int8": "bfloat16",
          "int4": "bfloat16"}[worker.quantization]
    wdt = worker.quantization if worker.quantization in ("fp8", "int8", "int4") else None
    return dict(mock=worker.mock, mock_latency_ms=worker.mock_latency_ms, mock_kv_seqs=worker.mock_kv_seqs, model=worker.model,
                checkpoint=worker.checkpoint, tp=worker.tp, device=worker.device, dtype=dt, weight_dtype=wdt,
                block_size=worker.block_size, max_num_seqs=worker.max_num_seqs,
                max_num_batched_tokens=worker.max_num_batched_tokens, max_model_len=worker.max_model_len,
                gpu_memory_utilization=worker.gpu_memory_utilization, num_blocks=worker.num_blocks,
                use_graphs=worker.use_graphs, seed=worker.seed, moe_comm=worker.moe_comm,
                enable_prefix_cache=True if cache is None else cache.enable_prefix_cache,
                cache_threshold=0.8 if cache is None else cache.memory_threshold,
                draft_model=None if spec is None else spec.draft_model,
                num_speculative_tokens=0 if spec is None else spec.num_speculative_tokens,
                min_acceptance_rate=0.5 if spec is None else spec.min_acceptance_rate,
                prompt_coalesce=1 if batcher is None else batcher.coalesce_prompts,
                prompt_coalesce_max_wait=4 if batcher is None else batcher.coalesce_max_wait_steps,
                fault=dict(fault or {}))


def make_engine(spec: dict):
    if spec.get("mock"):
        from ..engine.mock import MockEngine
        f = spec.get("fault") or {}
        return MockEngine(model_name=spec.get("model") or "mock", step_latency_s=spec.get("mock_latency_ms", 0) / 1000.0,
                          max_num_seqs=spec.get("max_num_seqs", 256), crash_after_steps=f.get("crash_after_steps"),
                          eos_every=f.get("eos_every"), kv_seqs=spec.get("mock_kv_seqs", 0))
    from ..engine import EngineConfig, LLMEngine
    keys = set(EngineConfig.__dataclass_fields__)
    ec = EngineConfig(**{k: v for k, v in spec.items() if k in keys})
    ec.spec_min_acceptance_rate = spec.get("min_acceptance_rate", 0.5)
    return LLMEngine(ec)


def engine_info(engine) -> dict:
    m = engine.mcfg
    info = {"model": m.name, "vocab_size": m.vocab_size, "hidden_size": m.hidden_size,
            "max_model_len": getattr(engine, "max_model_len", getattr(m, "max_position", 8192)),
            "eos_token_ids": list(m.eos_token_ids), "num_blocks": getattr(engine, "num_blocks", 0)}
    try:
        bb = engine._block_bytes()
        info["kv_bytes_per_token"] = bb // engine.cfg.block_size
    except Exception:
        info["kv_bytes_per_token"] = 1024
    return info


def _is_oom(e: BaseException) -> bool:
    try:
        import torch
        if isinstance(e, torch.cuda.OutOfMemoryError):
            return True
    except Exception:
        pass
    return "out of memory" in str(e).lower()


# ---------------------------------------------------------------------------
# the worker main loop
# ---------------------------------------------------------------------------
def encode_sse_chunk(text: str, index: int, logprob: Optional[float] = None) -> bytes:
    """One native SSE token event (byte-identical to core.wire.TokenEvent.tok(...).sse())
    framed as an HTTP/1.1 chunk, ready for the client socket."""
    body = b'data: {"type":"token","token":' + json.dumps(text).encode()
    body += b',"index":' + str(index).encode()
    if logprob is not None:
        body += b',"logprob":' + json.dumps(logprob).encode()
    body += b"}\n\n"
    return b"%x\r\n%s\r\n" % (len(body), body)


class EngineLoop:
    """Drives one engine. `emit(kind, payload)` is called from the loop thread
    with kind in {"out", "hb", "fatal"}. Outputs of requests submitted with
    sse=True carry their token event pre-encoded (RequestOutput.sse): the SSE
    bytes of a node's streams are produced by the replica processes in parallel,
    not by the one HTTP event loop (profiles/r3_frontend.md)."""

    def __init__(self, engine, emit: Callable[[str, Any], None]):
        self.engine = engine
        self.emit = emit
        self._inbox: pyqueue.SimpleQueue = pyqueue.SimpleQueue()
        self._wake = threading.Event()
        self._stop = False
        self.steps = 0
        self.last_step_s = 0.0
        self._sse: set = set()  # request ids whose outputs carry pre-encoded SSE chunks

    def _encode(self, outs: list) -> None:
        sse = self._sse
        if not sse:
            return
        for o in outs:
            rid = o.request_id
            if rid not in sse:
                continue
            if o.finished:
                sse.discard(rid)
            if o.new_token_ids and o.new_text and o.completion_tokens and not o.error:
                o.sse = encode_sse_chunk(o.new_text, o.completion_tokens - 1, o.logprobs[-1] if o.logprobs else None)

    def submit(self, cmd: tuple) -> None:
        self._inbox.put(cmd)
        self._wake.set()

    def _drain(self, outs: list) -> None:
        from ..engine.request import RequestOutput, RequestType, SamplingParams
        while True:
            try:
                cmd = self._inbox.get_nowait()
            except pyqueue.Empty:
                return
            op = cmd[0]
            if op == "add":
                _, rid, prompt_ids, params, prio, kind = cmd[:6]
                if len(cmd) > 6 and cmd[6]:
                    self._sse.add(rid)
                try:
                    self.engine.add_request(rid, prompt_ids, params, prio, RequestType(kind))
                except Exception as e:  # per-request rejection, never fatal
                    outs.append(RequestOutput(rid, [], "", True, "error", prompt_tokens=len(prompt_ids),
                                              error=f"Inference failed: {e}", error_code="inference_failed"))
            elif op == "abort":
                self.engine.abort(cmd[1])
                self._sse.discard(cmd[1])
            elif op == "limits":
                self.engine.set_limits(cmd[1], cmd[2])
            elif op == "clear_cache":
                self.engine.clear_prefix_cache()
            elif op == "hang":  # fault injection (tests)
                self.engine.hang = True
            elif op == "fail_collective":  # fault injection (tests)
                self.engine.fail_collective = True
            elif op == "stop":
                self._stop = True

    def _fail_inflight(self, code: str, msg: str) -> list:
        from ..engine.request import RequestOutput
        outs = []
        for rid in list(getattr(self.engine, "requests", {}).keys()):
            self.engine.abort(rid)
            outs.append(RequestOutput(rid, [], "", True, "error", error=msg, error_code=code))
        return outs

    def run(self) -> None:
        last_hb = 0.0
        timing = bool(os.environ.get("XGS_STEP_TIMING")) and hasattr(self.engine, "enable_step_timing")
        if timing:  # per-phase host time of the engine loop, reported with the heartbeat
            self.engine.enable_step_timing()
        loop_t = {"engine_step": 0.0, "emit": 0.0, "drain": 0.0, "idle": 0.0}
        if hasattr(self.engine, "output_sink"):
            # tokens emitted while a GPU step runs leave for the server at once (Req 5.1)
            def sink(o):
                self._encode(o)
                self.emit("out", o)
            self.engine.output_sink = sink
        while not self._stop:
            outs: list = []
            ta = time.perf_counter()
            self._drain(outs)
            loop_t["drain"] += time.perf_counter() - ta
            if self._stop:
                break
            if self.engine.has_work():
                t0 = time.perf_counter()
                try:
                    outs += self.engine.step()
                except SystemExit:
                    raise
                except Exception as e:  # contain the failure to the in-flight requests
                    from ..parallel.custom_ar import CustomAllReduceTimeout
                    if isinstance(e, CustomAllReduceTimeout):
                        # the TP group is out of step (a peer died or stalled): fail what is in
                        # flight, then let the replica die so the orchestrator restarts it
                        log.error("TP collective timed out: %s", e)
                        self.emit("out", outs + self._fail_inflight("inference_failed", f"Inference failed: {e}"))
                        raise
                    if _is_oom(e):
                        log.warning("OOM in engine step; flushing prefix cache and retrying")
                        try:
                            self.engine.clear_prefix_cache()
                            outs += self.engine.step()
                        except Exception as e2:
                            outs += self._fail_inflight("out_of_memory", f"Out of memory: {e2}")
                    else:
                        log.error("engine step failed: %s\n%s", e, traceback.format_exc())
                        outs += self._fail_inflight("inference_failed", f"Inference failed: {e}")
                self.last_step_s = time.perf_counter() - t0
                loop_t["engine_step"] += self.last_step_s
                self.steps += 1
            else:
                ti = time.perf_counter()
                self._wake.wait(0.02)
                self._wake.clear()
                loop_t["idle"] += time.perf_counter() - ti
            if outs:
                te = time.perf_counter()
                self._encode(outs)
                self.emit("out", outs)
                loop_t["emit"] += time.perf_counter() - te
            now = time.monotonic()
            if now - last_hb >= HEARTBEAT_S:
                last_hb = now
                st = self.engine.stats()
                st["last_step_ms"] = 1000 * self.last_step_s
                st["loop_steps"] = self.steps
                if timing:
                    st["loop_time_s"] = dict(loop_t)
                    st["step_timing_s"] = self.engine.step_timing()
                self.emit("hb", st)
        try:
            if hasattr(self.engine, "stop_followers"):
                self.engine.stop_followers()
        except Exception:
            pass


# ---------------------------------------------------------------------------
# replica handles (server side)
# ---------------------------------------------------------------------------
class Replica:
    """Server-side handle. Outputs are delivered through `on_event(replica_id,
    kind, payload)` on an arbitrary thread (the server hops onto its loop)."""

    kind = "base"

    def __init__(self, rid: int, spec: dict, on_event: Callable[[int, str, Any], None]):
        self.id = rid
        self.spec = spec
        self.on_event = on_event
        self.info: dict = {}
        self.stats: dict = {}
        self.last_hb = time.monotonic()
        self.ready = threading.Event()
        self.error: Optional[str] = None
        self.inflight: Dict[str, Any] = {}
        self.restarts = 0
        self.draining = False

    def _event(self, kind: str, payload: Any) -> None:
        if kind == "hb":
            self.last_hb = time.monotonic()
            self.stats = payload
        elif kind == "ready":
            self.info = payload
            self.last_hb = time.monotonic()
            self.ready.set()
            return
        elif kind == "fatal":
            self.error = payload
            self.ready.set()
        self.on_event(self.id, kind, payload)

    def wait_ready(self, timeout: float) -> bool:
        ok = self.ready.wait(timeout)
        return ok and self.error is None

    def submit(self, rid: str, prompt_ids: List[int], params, priority: int, kind: str, sse: bool = False) -> None:
        self._send(("add", rid, list(prompt_ids), params, int(priority), kind, bool(sse)))

    def abort(self, rid: str) -> None:
        self._send(("abort", rid))

    def set_limits(self, max_num_seqs: int, max_num_batched_tokens: int) -> None:
        self._send(("limits", int(max_num_seqs), int(max_num_batched_tokens)))

    def clear_cache(self) -> None:
        self._send(("clear_cache",))

    def inject_hang(self) -> None:
        self._send(("hang",))

    def inject_collective_timeout(self) -> None:
        self._send(("fail_collective",))

    def heartbeat_age(self) -> float:
        return time.monotonic() - self.last_hb

    # subclass API
    def start(self) -> None: ...
    def _send(self, cmd: tuple) -> None: ...
    def is_alive(self) -> bool: ...
    def shutdown(self, timeout: float = 10.0) -> None: ...


class InProcessReplica(Replica):
    kind = "thread"

    def __init__(self, rid, spec, on_event, engine=None):
        super().__init__(rid, spec, on_event)
        self._engine = engine
        self.loop: Optional[EngineLoop] = None
        self.thread: Optional[threading.Thread] = None

    def start(self) -> None:
        def main():
            try:
                eng = self._engine if self._engine is not None else make_engine(self.spec)
                self.engine = eng
                self.loop = EngineLoop(eng, self._event)
                self._event("ready", engine_info(eng))
                self.loop.run()
            except BaseException as e:  # noqa: BLE001 - report every death
                log.error("replica %d died: %s", self.id, e)
                self._event("fatal", f"{type(e).__name__}: {e}")

        self.thread = threading.Thread(target=main, name=f"replica-{self.id}", daemon=True)
        self.thread.start()

    def _send(self, cmd):
        if self.loop is not None:
            self.loop.submit(cmd)

    def is_alive(self) -> bool:
        return self.thread is not None and self.thread.is_alive() and self.error is None

    def shutdown(self, timeout: float = 10.0) -> None:
        if self.loop is not None:
            self.loop.submit(("stop",))
        if self.thread is not None:
            self.thread.join(timeout)


def _worker_main(spec: dict, rank: int, env: dict, cmd_q, out_q, out_w=None) -> None:
    """Entry point of a replica process (one per GPU).

    Outputs and heartbeats go over `out_w` (a one-way pipe) written synchronously by
    the engine-loop thread: an mp.Queue would pickle them on a feeder thread that
    then holds the GIL when the loop thread returns from a GPU wait, stalling the
    next launch by up to the interpreter's switch interval (measured: ~3-5 ms per
    step at 64 streams). The leader's fatal report rides the same pipe (ordered after
    its last outputs); ready and followers' fatal reports use `out_q`."""
    import pickle
    import sys
    os.environ.update(env)

    def send_fatal(msg: str) -> None:
        # the leader reports over the outputs pipe, behind the outputs it already
        # wrote (e.g. the inference_failed outputs of a collective timeout), so the
        # orchestrator sees them in order; followers have only the queue
        if out_w is not None:
            try:
                out_w.send_bytes(pickle.dumps(("fatal", msg), protocol=pickle.HIGHEST_PROTOCOL))
                return
            except (OSError, ValueError):
                pass
        out_q.put(("fatal", msg))

    sys.setswitchinterval(0.0005)  # the cmd reader thread must never hold the GIL for long
    logging.basicConfig(level=os.environ.get("XGS_LOG_LEVEL", "WARNING"),
                        format=f"[replica {env.get('XGS_REPLICA', '?')} rank {rank}] %(levelname)s %(message)s")
    try:
        eng_spec = dict(spec)
        if not spec.get("mock"):
            from ..parallel.affinity import bind_to_gpu_numa
            bind_to_gpu_numa(int(env.get("LOCAL_RANK", "0")))  # before any GPU call in this process
            from ..parallel.state import init_distributed
            import torch
            dev = None if not spec.get("device") else torch.device(spec["device"])
            init_distributed(tp_size=spec.get("tp", 1), device=dev)
        eng = make_engine(eng_spec)
        if rank != 0:
            eng.follower_loop()
            return

        def emit(kind, payload):
            if kind == "out":  # plain tuples pickle ~3x faster than dataclass instances
                kind, payload = "outp", [tuple(o.__dict__.values()) for o in payload]
            if out_w is not None and kind in ("outp", "hb"):
                out_w.send_bytes(pickle.dumps((kind, payload), protocol=pickle.HIGHEST_PROTOCOL))
            else:
                out_q.put((kind, payload))

        loop = EngineLoop(eng, emit)

        def reader():
            while True:
                cmd = cmd_q.get()
                loop.submit(cmd)
                if cmd[0] == "stop":
                    return

        threading.Thread(target=reader, daemon=True).start()
        out_q.put(("ready", engine_info(eng)))
        loop.run()
    except SystemExit as e:
        send_fatal(f"worker exited: {e}")
        raise
    except BaseException as e:  # noqa: BLE001
        send_fatal(f"{type(e).__name__}: {e}\n{traceback.format_exc()}")
        raise


class ProcessReplica(Replica):
    kind = "process"

    def __init__(self, rid, spec, on_event, gpus: Optional[List[int]] = None, master_port: int = 0, loop=None):
        super().__init__(rid, spec, on_event)
        # the serving event loop: outputs are read by a reader callback ON it (no reader
        # thread taking the GIL per step and re-hopping onto the loop); None: a thread
        self.loop = loop
        tp = spec.get("tp", 1)
        self.gpus = gpus if gpus is not None else list(range(rid * tp, rid * tp + tp))
        self.master_port = master_port or _free_port()
        self.procs: list = []
        self.cmd_q = None
        self.out_q = None
        self._reader: Optional[threading.Thread] = None

    def start(self) -> None:
        import multiprocessing as mp
        ctx = mp.get_context("spawn")
        self.cmd_q, self.out_q = ctx.Queue(), ctx.Queue()
        out_r, out_w = ctx.Pipe(duplex=False)
        tp = self.spec.get("tp", 1)
        self.procs = []
        for k in range(tp):
            env = {"RANK": str(k), "WORLD_SIZE": str(tp), "LOCAL_RANK": str(self.gpus[k]),
                   "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(self.master_port), "XGS_REPLICA": str(self.id),
                   "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
            p = ctx.Process(target=_worker_main, args=(self.spec, k, env, self.cmd_q if k == 0 else None, self.out_q,
                                                       out_w if k == 0 else None),
                            daemon=True, name=f"xgs-r{self.id}-tp{k}")
            p.start()
            self.procs.append(p)
        out_w.close()  # the child holds the write end; EOF on its death ends the pipe reader

        def reader():  # ready / fatal
            while True:
                try:
                    kind, payload = self.out_q.get()
                except (EOFError, OSError, ValueError):
                    return
                self._event(kind, payload)
                if kind == "fatal":
                    return

        def pipe_reader():  # outputs + heartbeats
            while True:
                try:
                    data = out_r.recv_bytes()
                except (EOFError, OSError):
                    return
                if self._on_pipe_msg(data):
                    return

        self._reader = threading.Thread(target=reader, daemon=True, name=f"replica-{self.id}-reader")
        self._reader.start()
        self._out_r = out_r
        loop = self.loop
        if loop is not None and not loop.is_closed():
            fd = out_r.fileno()

            def readable():
                try:
                    while out_r.poll():
                        if self._on_pipe_msg(out_r.recv_bytes()):
                            loop.remove_reader(fd)
                            return
                except (EOFError, OSError):
                    loop.remove_reader(fd)

            loop.call_soon_threadsafe(loop.add_reader, fd, readable)
        else:
            self._pipe_reader = threading.Thread(target=pipe_reader, daemon=True, name=f"replica-{self.id}-outputs")
            self._pipe_reader.start()

    def _on_pipe_msg(self, data: bytes) -> bool:
        """One outputs / heartbeat / fatal message from the leader's pipe; True at the end."""
        import pickle
        from ..engine.request import RequestOutput
        kind, payload = pickle.loads(data)
        if kind == "outp":
            kind, payload = "out", [RequestOutput(*t) for t in payload]
        self._event(kind, payload)
        return kind == "fatal"

    def _send(self, cmd):
        if self.cmd_q is not None:
            try:
                self.cmd_q.put(cmd)
            except (ValueError, OSError):
                pass

    def is_alive(self) -> bool:
        return bool(self.procs) and all(p.is_alive() for p in self.procs) and self.error is None

    def shutdown(self, timeout: float = 10.0) -> None:
        self._send(("stop",))
        t_end = time.monotonic() + timeout
        for p in self.procs:
            p.join(max(0.1, t_end - time.monotonic()))
        for p in self.procs:
            if p.is_alive():
                p.kill()
                p.join(2.0)

    def kill(self) -> None:
        """Fault injection: hard-kill the replica's processes."""
        for p in self.procs:
            if p.is_alive():
                p.kill()


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
