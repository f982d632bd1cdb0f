"""Custom one-shot all-reduce (csrc/comm/custom_allreduce.hip): two processes
share the single GPU of the test box through IPC handles (the same code path
as peers over xGMI), against a fp32 reference summed in rank order."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q, two_shot_min=None):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from xgserve.parallel.custom_ar import CustomAllReduce
        ar = CustomAllReduce(rank, world, torch.device("cuda:0"), two_shot_min=two_shot_min)
        errs = []
        for n in (8, 512, 4096, 8192, 24584, 65536, 1 << 20, 2 << 20, 6 << 20):  # elements (bf16)
            for it in range(3):
                g = torch.Generator().manual_seed(1000 * it + n)
                xs = [torch.randn(n, generator=g).bfloat16() for _ in range(world)]
                ref = xs[0].float()
                for r in range(1, world):
                    ref = ref + xs[r].float()
                x = xs[rank].cuda()
                y = ar.all_reduce(x.clone(), out=torch.empty_like(x))
                torch.cuda.synchronize()
                if not torch.equal(y.cpu(), ref.bfloat16()):
                    errs.append((n, it, float((y.cpu().float() - ref).abs().max())))
        # graph capture + replay with changing inputs
        x = torch.zeros(4096, dtype=torch.bfloat16, device="cuda:0")
        y = torch.empty_like(x)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            ar.all_reduce(x, out=y)
        torch.cuda.synchronize()
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph):
            ar.all_reduce(x, out=y)
        for it in range(5):
            x.fill_(float(rank + it))
            gph.replay()
            torch.cuda.synchronize()
            want = float(sum(r + it for r in range(world)))
            if not bool((y.float() == want).all()):
                errs.append(("graph", it))
        q.put((rank, errs, ar.timeouts()))
        ar.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, [repr(e)], -1))


@pytest.mark.parametrize("world,two_shot_min", [(2, None), (2, 0), (4, None), (4, 0)])
def test_custom_allreduce_one_gpu(world, two_shot_min):
    """world ranks share the GPU; two_shot_min=0 forces the two-shot kernel for
    every size, None is the production choice (one-shot small, two-shot large at 4 ranks)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, two_shot_min)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(60)
    for rank, errs, tmo in res:
        assert errs == [], (rank, errs)
        assert tmo == 0
