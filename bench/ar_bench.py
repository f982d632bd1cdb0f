#!/usr/bin/env python3
"""Per-call latency of the custom all-reduce protocols on ONE GPU shared by W
processes (the IPC code path of a TP group; on one device the "remote" memory is
local HBM, so this isolates the protocol's own synchronisation cost: fences, flag
round trips, the read-after-flag of the pull kernels vs the push lines).

  python bench/ar_bench.py --world 2 8 [--calls 64] [--reps 20]

Per world and protocol (pull = one-shot pull kernels, push = flag-in-payload LL):
  * fused residual all-reduce, T = 1 / 64 rows of H = 8192 (70B TP8 decode tail);
  * plain all-reduce of 16 KiB and 128 KiB.
`calls` back-to-back launches are captured into one HIP graph and replayed `reps`
times; rank 0 prints one JSON line per case with the median us per call."""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


import torch  # noqa: E402  (imported before the workers set their env, as in tests/test_custom_ar_gpu.py)


def _rank(rank, world, port, calls, reps, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0",
                       "GPU_MAX_HW_QUEUES": "1"})
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from xgserve.parallel.custom_ar import CustomAllReduce
        out = []
        for proto, ll in (("pull", 0), ("push", None)):
            ar = CustomAllReduce(rank, world, torch.device("cuda:0"), ll_max=ll)
            ar.set_timeout(ar.WARMUP_TIMEOUT_S)
            cases = []
            for T in (1, 64):
                H, S = 8192, 2
                part = torch.randn(S, T, H, device="cuda:0")
                resid = torch.zeros(T, H, dtype=torch.bfloat16, device="cuda:0")
                ss = torch.zeros(T * H // 1024, device="cuda:0")
                cases.append((f"resid T={T} H={H}", lambda p=part, r=resid, s_=ss: ar.all_reduce_resid(p, r, s_)))
            for n in (8192, 65536):
                x = torch.randn(n, device="cuda:0").bfloat16()
                y = torch.empty_like(x)
                cases.append((f"allreduce {2 * n >> 10} KiB", lambda x=x, y=y: ar.all_reduce(x, out=y)))
            for name, fn in cases:
                s = torch.cuda.Stream()
                with torch.cuda.stream(s):
                    for _ in range(3):
                        fn()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(calls):
                        fn()
                times = []
                for _ in range(reps):
                    dist.barrier()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    g.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    times.append(e0.elapsed_time(e1) * 1000.0 / calls)
                out.append({"world": world, "protocol": proto, "case": name, "us_per_call": round(statistics.median(times), 2),
                            "us_min": round(min(times), 2), "timeouts": ar.timeouts()})
            dist.barrier()
            ar.close()
        q.put((rank, out))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[2, 8])
    ap.add_argument("--calls", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    for w in a.world:
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_rank, args=(r, w, port, a.calls, a.reps, q)) for r in range(w)]
        for p in ps:
            p.start()
        res = dict(q.get(timeout=600) for _ in ps)
        for p in ps:
            p.join(60)
        if not isinstance(res[0], list):
            print(json.dumps({"world": w, "error": res[0]}), flush=True)
            return 1
        for row in res[0]:
            print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
