#!/usr/bin/env python3
"""Headline benchmark: whole-node output tokens/s (+ p50 TTFT) of Llama-3-8B
serving with continuous batching (BASELINE.json config 3: 64 concurrent
synthetic requests per replica), one DP replica per GPU by default.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--concurrency 64]
                  [--prompt-len 512] [--output-len 256] [--model llama3-8b]
                  [--tp 1]

For N > 1 launch one rank per GPU (torch.distributed.run). With --tp 1 the
ranks are independent replicas (weak scaling: per-GPU work is fixed) that only
meet at the timing barriers. With --tp T the N ranks form N/T tensor-parallel
replicas (the other BASELINE configs: Llama-3-70B TP=8, Mixtral 8x7B TP=2):
the TP leader of each replica drives its engine and the followers mirror the
leader's step plans (RCCL/xGMI collectives + the custom one-shot all-reduce).
A "step" is one engine iteration (scheduler + forward of the packed
decode/prefill batch + sampling). Weights are random-init bf16 of the full
architecture, prompts are synthetic token ids; finished requests are
immediately replaced so the concurrency stays at --concurrency. Rank 0 prints
ONE JSON line (value = whole-job output tokens/s).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree per replica")
    ap.add_argument("--concurrency", type=int, default=64, help="concurrent requests per replica")
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--max-batched-tokens", type=int, default=8192)
    ap.add_argument("--block-size", type=int, default=16, help="KV page size in tokens (multiple of 16)")
    ap.add_argument("--prefill-chunk", type=int, default=0,
                    help="stall-free batching: prompt tokens per step that also decodes (decode_prefill_cap; "
                         "mixed steps replay a graph on the gemm_mw path); 0 = whole prompts")
    ap.add_argument("--coalesce", type=int, default=1,
                    help="admission window: hold new prompts until this many wait (1: off)")
    ap.add_argument("--coalesce-max-wait", type=int, default=4, help="admission window bound, in steps")
    ap.add_argument("--moe-comm", default="auto", choices=["auto", "alltoall", "allreduce"])
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--weight-dtype", default=None, choices=["fp8", "int8", "int4"],
                    help="weight-only copies for decode batches <= 64: fp8 (E4M3), int8 (per-channel) or int4 "
                         "(per 128-k group) -- not the bf16 headline")
    ap.add_argument("--no-prefix-cache", action="store_true")
    ap.add_argument("--temperature", type=float, default=0.0,
                    help="sampling temperature of every request (0 = greedy, the headline)")
    ap.add_argument("--top-p", type=float, default=1.0)
    ap.add_argument("--top-k", type=int, default=0)
    ap.add_argument("--allow-rccl-decode", action="store_true",
                    help="with --tp > 1, report even if the custom xGMI all-reduce did not register (TP decode "
                         "all-reduces on RCCL); without it such a run exits 3")
    ap.add_argument("--tp-shard", type=int, default=1,
                    help="single-GPU simulation of ONE rank of a TP group of this degree: the rank's weight / "
                         "KV shards and kernels, collectives replaced by local reductions (not a TP measurement: "
                         "xGMI time is excluded; reported with parallelism 'tpN-shard-sim')")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`python bench.py --gpus N` without an external launcher: start N fresh rank
    processes (one per GPU, RANK/LOCAL_RANK/WORLD_SIZE set, rendezvous on
    127.0.0.1) and return the worst exit code. Runs before anything imports torch,
    so this parent never initialises the GPU; rank 0's JSON line reaches our
    stdout directly. If one rank dies the others are terminated (no hung
    collective)."""
    import signal
    import subprocess
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                for q in live:
                    q.send_signal(signal.SIGTERM)
        if live:
            time.sleep(0.05)
    return rc


def prompt_gemm(eng) -> str:
    """Which projections of the prompt-sized mixed steps run on gemm_pf (and for which
    step sizes); the rest stay on the library GEMMs."""
    layers = getattr(eng.model, "layers", None)
    if layers is None or not getattr(layers[0], "pf_ok", False):
        return "library"
    from xgserve.models import llama
    return "gemm_pf " + ", ".join(f"{k} {'+'.join(f'{lo}-{hi}' for lo, hi in ws)}"
                                  for k, ws in sorted(llama.PF_WINDOWS.items()) if ws) + " tokens"


def preflight(st, world: int, tp: int, dev, eng) -> dict:
    """First contact with a multi-GPU node, before anything is timed (every rank
    takes part): the collective backend forms the N-rank
    communicator and sums correctly, every GPU pair can reach the other (peer
    access, what the custom all-reduce's IPC mappings need), and each TP group's
    decode all-reduce is the self-tested custom kernel or, visibly, RCCL. The
    result goes into the JSON line."""
    import torch
    import torch.distributed as dist
    info = {"backend": None, "rccl_world": None, "tp_groups": None, "p2p_ok": None, "decode_ar": None,
            "decode_ar_in_gemm": None,
            "custom_ar_selftest": None, "custom_ar_selftest_passes": None}
    if world > 1:
        info["backend"] = str(dist.get_backend())
        x = torch.full((4096,), float(st.rank + 1), dtype=torch.float32, device=dev)
        dist.all_reduce(x)
        ok = bool((x == world * (world + 1) / 2).all())
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        info["rccl_world"] = dist.get_world_size() if int(flag.item()) == 1 else -1
        info["tp_groups"] = [list(range(r, r + tp)) for r in range(0, world, tp)]
    if dev.type == "cuda":
        n = torch.cuda.device_count()
        info["p2p_ok"] = all(torch.cuda.can_device_access_peer(i, j) for i in range(n) for j in range(n) if i != j) \
            if n > 1 else None
    if tp > 1:
        ar = getattr(eng, "custom_ar", None)
        lib = "rccl" if info["backend"] == "nccl" else info["backend"]  # the library collective
        info["custom_ar_selftest"] = getattr(ar, "verified", None)
        info["custom_ar_selftest_passes"] = getattr(ar, "verified_counts", None)  # launches checked vs RCCL
        # every rank must agree on the protocol (a refusal below is collective)
        mine = torch.tensor([1 if ar is not None else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(mine, op=dist.ReduceOp.MIN)
        info["decode_ar"] = ar.protocol() if (ar is not None and int(mine.item()) == 1) else lib
        # steps of <= 16 rows: the all-reduce inside the O / down GEMM launches
        info["decode_ar_in_gemm"] = bool(ar is not None and ar.gemm_ar is not None and not ar.shared_device)
    return info


def main():
    a = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        return launch_ranks(a.gpus)
    world = int(env_world or "1")
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}: refusing to report a mismatched run",
              file=sys.stderr)
        return 2
    if a.gpus % a.tp:
        print(f"bench.py: --gpus {a.gpus} is not a multiple of --tp {a.tp}", file=sys.stderr)
        return 2
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # host threads of this rank on its GPU's NUMA node, before anything touches the GPU
    from xgserve.parallel.affinity import bind_to_gpu_numa
    bind_to_gpu_numa(int(os.environ.get("LOCAL_RANK", "0")))
    import torch
    import torch.distributed as dist
    from xgserve.parallel.state import init_distributed
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams

    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if torch.cuda.is_available() and torch.cuda.device_count() < local_world:
        # two ranks sharing one device would report a fake multi-GPU number
        print(f"bench.py: {local_world} ranks on this node but only {torch.cuda.device_count()} visible GPUs",
              file=sys.stderr)
        return 2
    st = init_distributed(tp_size=a.tp)
    rank = st.rank
    dp = world // a.tp
    on_gpu = torch.cuda.is_available()
    # CPU (gloo) runs exist only to test this script's multi-rank plumbing (tests/test_bench_cli.py)
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    max_len = a.prompt_len + 2 * a.output_len + 16
    ecfg = EngineConfig(model=a.model, device=str(dev), tp=a.tp, max_num_seqs=max(64, a.concurrency),
                        max_num_batched_tokens=a.max_batched_tokens, max_model_len=max_len,
                        use_graphs=on_gpu and not a.no_graphs, enable_prefix_cache=not a.no_prefix_cache,
                        moe_comm=a.moe_comm, prompt_coalesce=a.coalesce, block_size=a.block_size,
                        prompt_coalesce_max_wait=a.coalesce_max_wait, decode_prefill_cap=a.prefill_chunk,
                        weight_dtype=a.weight_dtype, dtype=None if on_gpu else "float32",
                        graph_batch_sizes=[b for b in [1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128]
                                           if b <= max(64, a.concurrency)], seed=st.dp_rank)
    shard_model = None
    if a.tp_shard > 1:
        if world != 1 or a.tp != 1:
            print("bench.py: --tp-shard simulates one TP rank in a single process (--gpus 1 --tp 1)", file=sys.stderr)
            return 2
        from xgserve.models import build_model, get_config
        shard_model = build_model(get_config(a.model), device=dev, tp=a.tp_shard, rank=0,
                                  weight_dtype=a.weight_dtype)
    eng = LLMEngine(ecfg, model=shard_model)
    pre = preflight(st, world, a.tp, dev, eng)
    if a.tp > 1 and pre["decode_ar"] not in ("ll", "pull") and not a.allow_rccl_decode:
        if rank == 0:
            print(f"bench.py: --tp {a.tp} but the custom xGMI all-reduce did not register (TP decode all-reduces "
                  f"would run on {pre['decode_ar']}); pass --allow-rccl-decode to measure that anyway",
                  file=sys.stderr)
        dist.barrier()
        dist.destroy_process_group()
        return 3
    if world > 1 and pre["rccl_world"] != world:
        print(f"bench.py: collective check failed on the {world}-rank communicator: {pre}", file=sys.stderr)
        return 3
    leader = st.tp_rank == 0
    # timing collectives run among the TP leaders only (followers sit in follower_loop)
    leaders = [r for r in range(world) if r % a.tp == 0]
    lgroup = None
    if world > 1:
        lgroup = dist.group.WORLD if a.tp == 1 else dist.new_group(leaders)
    cpu_group = dist.new_group(leaders, backend="gloo") if world > 1 else None
    if not leader:
        eng.follower_loop()
        dist.barrier()
        dist.destroy_process_group()
        return 0

    V = eng.mcfg.vocab_size
    rng = np.random.default_rng(1234 + st.dp_rank)
    counter = [0]
    arrival = {}
    first_tok = {}

    def submit(max_tokens, extra=0):
        rid = f"r{rank}-{counter[0]}"
        counter[0] += 1
        # random token prompts: no accidental prefix sharing across requests
        prompt = rng.integers(10, V - 10, size=a.prompt_len + extra).tolist()
        eng.add_request(rid, prompt, SamplingParams(max_tokens=max_tokens, temperature=a.temperature,
                                                   top_p=a.top_p, top_k=a.top_k, seed=counter[0],
                                                   ignore_eos=True))
        arrival[rid] = time.perf_counter()

    # The initial population is drawn from the closed loop's STEADY STATE: every
    # replacement request runs exactly output_len tokens, so at any instant the live
    # requests' ages are uniform on [0, output_len). Request i starts with
    # remaining = (i + 0.5) * output_len / C tokens to generate and a context already
    # extended by its age (prompt_len + age prompt tokens), so from the first timed
    # step one request finishes every output_len / C steps and is replaced by a fresh
    # prompt_len prompt -- the same prefill share and KV-context mix as a 3,000-step run.
    initial = []
    for i in range(a.concurrency):
        remaining = max(1, int(round((i + 0.5) * a.output_len / a.concurrency)))
        submit(remaining, extra=a.output_len - remaining)
        initial.append(f"r{rank}-{counter[0] - 1}")

    step_log = [] if os.environ.get("XGS_STEP_LOG") else None

    def run_step():
        if step_log is not None:
            t0, c0 = time.perf_counter(), dict(eng.stats_counters)
            p0 = dict(eng._timing) if eng._timing is not None else None
        outs = eng.step()
        now = time.perf_counter()
        if step_log is not None:
            c1 = eng.stats_counters
            step_log.append((round(1000 * (now - t0), 3), c1["prefill_tokens_computed"] - c0["prefill_tokens_computed"],
                             c1["decode_steps"] - c0["decode_steps"], c1["generation_tokens"] - c0["generation_tokens"],
                             None if p0 is None else {k: round(1000 * (v - p0.get(k, 0.0)), 3)
                                                      for k, v in eng._timing.items()}))
        n_tok = 0
        for o in outs:
            n_tok += len(o.new_token_ids)
            if o.new_token_ids and o.request_id not in first_tok:
                first_tok[o.request_id] = now
            if o.finished:
                submit(a.output_len)
        return n_tok

    # population fill (untimed setup, before the W warmup steps): prefill the initial
    # population until every initial request has produced its first token
    # (stall-free batching is lifted while the initial population prefills: admitting
    # 64 prompts one chunk per step would leave the timed window in a transient --
    # finished requests' replacements queued behind the fill -- instead of the
    # steady state of one prompt chunk per step)
    fill_steps = 0
    eng.set_decode_prefill_cap(0)
    while any(r not in first_tok for r in initial) and fill_steps < 10_000:
        run_step()
        fill_steps += 1
    eng.set_decode_prefill_cap(None)
    for _ in range(a.warmup):
        run_step()
    sync()
    if lgroup is not None:
        dist.barrier(group=lgroup)
    sync()
    if os.environ.get("XGS_STEP_TIMING"):
        eng.enable_step_timing()
    t_start_wall = time.perf_counter()
    tokens = 0
    first_before = set(first_tok)
    c_before = dict(eng.stats_counters)
    for _ in range(a.steps):
        tokens += run_step()
    sync()
    elapsed = time.perf_counter() - t_start_wall
    c_after = dict(eng.stats_counters)
    window_steps = c_after["steps"] - c_before["steps"]
    window_mixed = window_steps - (c_after["decode_steps"] - c_before["decode_steps"])
    if lgroup is not None:
        dist.barrier(group=lgroup)
    sync()
    if step_log is not None:
        with open(os.environ["XGS_STEP_LOG"], "w") as f:
            for i, e in enumerate(step_log):
                f.write(json.dumps({"i": i, "timed": i >= a.warmup, "ms": e[0], "prefill_tokens": e[1],
                                    "decode_step": e[2], "gen_tokens": e[3], "phases_ms": e[4]}) + "\n")
    ttfts = [first_tok[r] - arrival[r] for r in first_tok if r not in first_before]
    p50_local = float(np.median(ttfts)) if ttfts else float("nan")

    t = torch.tensor([elapsed, float(tokens), p50_local], dtype=torch.float64)
    if cpu_group is not None:
        mx, sm = t.clone(), t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=cpu_group)
        dist.all_reduce(sm, op=dist.ReduceOp.SUM, group=cpu_group)
        elapsed, tokens, p50 = mx[0].item(), sm[1].item(), sm[2].item() / len(leaders)
    else:
        p50 = p50_local
    if rank == 0:
        value = tokens / elapsed
        st_ = eng.stats()
        par = f"dp{dp}" if a.tp == 1 else (f"tp{a.tp}" if dp == 1 else f"dp{dp}xtp{a.tp}")
        if a.tp_shard > 1:
            par = f"tp{a.tp_shard}-shard-sim"
        print(json.dumps({
            "metric": "output_tokens_per_sec",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * elapsed / a.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("bf16" if on_gpu else "fp32") if a.weight_dtype is None else f"bf16 activations, {a.weight_dtype} decode weights",
            "data": "synthetic (random-token prompts, random-init weights)",
            "ttft_p50_ms": round(1000 * p50, 2) if p50 == p50 else None,
            "config": {"model": a.model, "global_batch": a.concurrency * dp,
                       "seq_len": a.prompt_len + a.output_len, "prompt_len": a.prompt_len,
                       "output_len": a.output_len, "parallelism": par,
                       "concurrency_per_replica": a.concurrency,
                       "sampling": ("greedy" if a.temperature <= 0 else
                                    f"temperature {a.temperature}, top_p {a.top_p}, top_k {a.top_k}")},
            "rccl_world": pre["rccl_world"], "tp_groups": pre["tp_groups"], "p2p_ok": pre["p2p_ok"],
            "decode_ar": pre["decode_ar"], "decode_ar_in_gemm": pre["decode_ar_in_gemm"],
            "detail": {"initial_population": "steady-state (ages uniform on [0, output_len))",
                       "backend": pre["backend"], "custom_ar_selftest": pre["custom_ar_selftest"],
                       "prompt_gemm": prompt_gemm(eng),
                       "fill_steps": fill_steps, "window_engine_steps": window_steps,
                       "window_prompt_steps": window_mixed, "ttft_samples": len(ttfts),
                       "preemptions": st_["preemptions"], "kv_blocks": st_["kv_blocks_total"],
                       "decode_steps_total": st_["decode_steps"], "steps_total": st_["steps"],
                       "window_lookahead_launches": c_after["lookahead_launches"] - c_before["lookahead_launches"],
                       "gemm_table": bool(getattr(eng, "gemm_table", False)),
                       "prefill_chunk": a.prefill_chunk,
                       "mixed_graph_replays": getattr(eng.runner, "mixed_replays", 0),
                       **({"host_ms_per_step": {k: round(1000 * v / a.steps, 4)
                                                for k, v in eng.step_timing().items()}}
                          if eng._timing is not None else {})},
        }), flush=True)
    eng.stop_followers()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
