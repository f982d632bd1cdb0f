"""The RCCL backend itself (torch.distributed "nccl" = librccl on ROCm), at world 1
on the one GPU of a test box -- every collective pattern the TP / EP code issues
(parallel/comm.py), eagerly and inside a HIP graph capture, so the first time RCCL
runs is not on the 8-GPU node:
  * init_process_group("nccl", device_id=...)  (parallel/state.py init_distributed)
  * all_reduce                                  (tp_all_reduce, prefill all-reduces)
  * all_reduce(async_op=True) + wait() making the COMPUTE stream wait
                                                (tp_all_reduce_async, _forward_tp_overlap)
  * all_to_all_single with explicit splits      (tp_all_to_all, tp_exchange_counts)
  * all_gather_into_tensor                      (tp_all_gather_rows / lastdim)
  * the same collectives captured in a CUDA/HIP graph and replayed with new inputs
    (decode graphs capture the TP collectives under nccl, engine.py)."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _child(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    import datetime
    import torch.distributed as dist
    errs = []
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev,
                                timeout=datetime.timedelta(seconds=60))
        g = dist.new_group([0], backend="nccl")
        assert dist.get_backend(g) == "nccl"
        # all_reduce
        x = torch.randn(3, 4096, device=dev, dtype=torch.bfloat16)
        want = x.clone()
        dist.all_reduce(x, group=g)
        if not torch.equal(x, want):
            errs.append("all_reduce")
        # async all_reduce: wait() orders the compute stream, the host does not block
        big = torch.randn(1 << 22, device=dev, dtype=torch.bfloat16)
        ref = big.float() * 2
        w = dist.all_reduce(big, group=g, async_op=True)
        w.wait()
        y = big.float() * 2
        if not torch.equal(y, ref):
            errs.append("async_all_reduce")
        # all_to_all_single with explicit (uneven-capable) splits + counts exchange
        rows = torch.randn(37, 256, device=dev, dtype=torch.bfloat16)
        out = torch.empty_like(rows)
        dist.all_to_all_single(out, rows, [37], [37], group=g)
        if not torch.equal(out, rows):
            errs.append("all_to_all_single")
        cnt = torch.tensor([37], dtype=torch.int64, device=dev)
        cnt_out = torch.empty_like(cnt)
        dist.all_to_all_single(cnt_out, cnt, group=g)
        if int(cnt_out.item()) != 37:
            errs.append("exchange_counts")
        # all_gather_into_tensor
        shard = torch.randn(5, 1000, device=dev, dtype=torch.bfloat16)
        full = torch.empty(5, 1000, device=dev, dtype=torch.bfloat16)
        dist.all_gather_into_tensor(full, shard, group=g)
        if not torch.equal(full, shard):
            errs.append("all_gather_into_tensor")
        # the same collectives inside a graph capture, replayed with new inputs
        a = torch.zeros(64, 4096, device=dev, dtype=torch.bfloat16)
        b = torch.empty(64, 4096, device=dev, dtype=torch.bfloat16)
        r = torch.randn(64, 1000, device=dev, dtype=torch.bfloat16)
        r_out = torch.empty_like(r)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):  # warm up the communicator on the capture stream
            dist.all_reduce(a, group=g)
            dist.all_gather_into_tensor(r_out, r, group=g)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph):
            dist.all_reduce(a, group=g)
            torch.mul(a, 3, out=b)
            dist.all_gather_into_tensor(r_out, r, group=g)
        for it in range(4):
            a.fill_(float(it + 1))
            r.normal_()
            gph.replay()
            torch.cuda.synchronize()
            if not bool((b.float() == 3.0 * (it + 1)).all()) or not torch.equal(r_out, r):
                errs.append(("graph", it))
        dist.destroy_process_group()
        q.put(errs)
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put([f"{type(e).__name__}: {e}\n{traceback.format_exc()}"])


def test_rccl_collectives_eager_and_captured():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_port(), q))
    p.start()
    try:
        errs = q.get(timeout=180)
    finally:
        p.join(60)
        if p.is_alive():
            p.kill()
    assert errs == [], errs
