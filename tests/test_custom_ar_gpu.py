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


SIZES = (8, 512, 4096, 8192, 24584, 65536, 1 << 20, 2 << 20, 6 << 20)


def _worker(rank, world, port, q, two_shot_min=None, sizes=SIZES, ll_max=None):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from xgserve.parallel.custom_ar import CustomAllReduce
        ar = CustomAllReduce(rank, world, torch.device("cuda:0"), two_shot_min=two_shot_min, ll_max=ll_max)
        ar.set_timeout(ar.WARMUP_TIMEOUT_S)  # ranks share one GPU and arrive seconds apart
        errs = []
        for n in sizes:  # elements (bf16)
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


def _run(target, world, *args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(60)
    return res


@pytest.mark.parametrize("world,two_shot_min,ll_max", [(2, None, None), (2, 0, 0), (4, None, None), (4, 0, 0),
                                                       (8, None, None), (8, 0, 0), (2, None, 0), (8, None, 0)])
def test_custom_allreduce_one_gpu(world, two_shot_min, ll_max):
    """world ranks share the GPU; two_shot_min=0 forces the two-shot kernel for
    every size, None is the production choice (push protocol up to 256 KiB, one-shot
    pull above, two-shot large at 4 ranks); ll_max=0 forces the pull kernels.
    world=8 is the Llama-3-70B TP8 group's protocol (8 peers, 7 remote slots per block)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    sizes = SIZES if world < 8 else SIZES[:7]
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, two_shot_min, sizes, ll_max)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(60)
    for rank, errs, tmo in res:
        assert errs == [], (rank, errs)
        assert tmo == 0


def _resid_worker(rank, world, port, q, ll_max=None):
    """custom_allreduce_resid against an fp32 loop reference with the kernel's
    summation order: local split-K slices in order, bf16 contribution per rank,
    rank-order sum, + residual, one bf16 rounding."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0",
                       "GPU_MAX_HW_QUEUES": "1"})
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from xgserve.parallel.custom_ar import CustomAllReduce
        ar = CustomAllReduce(rank, world, torch.device("cuda:0"), ll_max=ll_max)
        # 8 ranks time-share one GPU and each builds its fp32 reference on the CPU
        # between collectives: peers arrive seconds apart, as in engine warmup
        ar.set_timeout(ar.WARMUP_TIMEOUT_S)
        errs = []
        shapes = ((4, 1, 4096), (8, 16, 8192), (2, 64, 8192), (1, 3, 1024), (3, 64, 4096))
        if world == 8:  # T x H/1024 blocks per rank, all 8 grids co-resident on the one GPU
            shapes = tuple(sh for sh in shapes if sh[1] * sh[2] // 1024 <= 128)
        for (S, T, H) in shapes:
            for it in range(2):
                g = torch.Generator().manual_seed(7 * it + 131 * T + H + S)
                parts = [torch.randn(S, T, H, generator=g) for _ in range(world)]
                resid0 = torch.randn(T, H, generator=g).bfloat16()
                contrib = []
                for r in range(world):
                    a = torch.zeros(T, H)
                    for s_ in range(S):
                        a = a + parts[r][s_]
                    contrib.append(a.bfloat16().float())
                tot = torch.zeros(T, H)
                for r in range(world):
                    tot = tot + contrib[r]
                want = (resid0.float() + tot).bfloat16()
                want_ss = want.float().view(T, H // 1024, 1024).pow(2).sum(-1).t().contiguous()  # [chunk, T]
                resid = resid0.cuda()
                ss = torch.full((H // 1024 * T,), -1.0, device="cuda:0")
                ar.all_reduce_resid(parts[rank].cuda(), resid, ss)
                torch.cuda.synchronize()
                if ar.timeouts():
                    errs.append(("timeout", S, T, H, it))
                    break
                if not torch.equal(resid.cpu(), want):
                    errs.append(("resid", S, T, H, it, float((resid.cpu().float() - want.float()).abs().max())))
                if not torch.allclose(ss.cpu().view(H // 1024, T), want_ss, rtol=1e-4, atol=1e-2):
                    errs.append(("ss", S, T, H, it))
        ar.poll_async()
        torch.cuda.synchronize()
        if not errs:
            ar.check()
        q.put((rank, errs, ar.timeouts()))
        ar.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, [repr(e)], -1))


# world 8 = 8 processes sharing ONE GPU while their kernels spin on each other (on a
# real node every rank owns a GPU). Each rank runs with one hardware queue
# (GPU_MAX_HW_QUEUES=1): 8 queues are all mapped at once, and the shapes are capped at
# 128 blocks per rank so all 8 grids are co-resident (8 x 512 blocks of the T=64,
# H=8192 shape are not: the first grids spin until the wait limit while the last
# rank's blocks cannot be placed -- an artifact of sharing one GPU).
@pytest.mark.parametrize("world,ll_max", [(2, None), (4, None), (8, None), (2, 0), (8, 0)])
def test_custom_allreduce_resid_one_gpu(world, ll_max):
    """ll_max None: the push protocol (production); 0: the pull kernel."""
    for rank, errs, tmo in _run(_resid_worker, world, ll_max):
        assert errs == [], (rank, errs)
        assert tmo == 0


def _timeout_worker(rank, world, port, q):
    """Rank 1 skips the collective: rank 0's kernel must give up, count the timeout,
    and check() must raise -- never return the stale sum silently."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from xgserve.parallel.custom_ar import CustomAllReduce, CustomAllReduceTimeout
        ar = CustomAllReduce(rank, world, torch.device("cuda:0"))
        raised = None
        if rank == 0:
            x = torch.ones(1024, dtype=torch.bfloat16, device="cuda:0")
            ar.all_reduce(x, out=torch.empty_like(x))
            ar.poll_async()
            torch.cuda.synchronize()
            try:
                ar.check()
                raised = False
            except CustomAllReduceTimeout:
                raised = True
        dist.barrier()
        q.put((rank, raised, ar.timeouts()))
        ar.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), -1))


def test_custom_allreduce_timeout_is_fatal():
    res = dict((r, (raised, n)) for r, raised, n in _run(_timeout_worker, 2))
    assert res[0][0] is True and res[0][1] >= 1, res
    assert res[1][1] == 0, res


def _slow_rank_worker(rank, world, port, q, limit_s, delay_s, n_coll):
    """Rank 1 joins `delay_s` late; rank 0 issues `n_coll` all-reduces in a row under
    a `limit_s` peer-wait limit. Returns (rank, timeouts, seconds rank 0 spent)."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    import time
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from xgserve.parallel.custom_ar import CustomAllReduce
        ar = CustomAllReduce(rank, world, torch.device("cuda:0"))
        ar.set_timeout(limit_s)
        x = torch.ones(4096, dtype=torch.bfloat16, device="cuda:0")
        outs = [torch.empty_like(x) for _ in range(n_coll)]
        torch.cuda.synchronize()
        dist.barrier()
        if rank == 1 and delay_s > 0:
            time.sleep(delay_s)
        t0 = time.perf_counter()
        if rank == 0 or delay_s >= 0:
            for o in outs:
                ar.all_reduce(x, out=o)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ok = all(bool((o.float() == world).all()) for o in outs)
        q.put((rank, ar.timeouts(), dt, ok))
        dist.barrier()
        ar.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), -1, False))


def test_slow_rank_within_limit_is_not_a_failure():
    """A peer 0.6 s late under a 5 s limit: every collective completes exactly."""
    res = {r: (n, dt, ok) for r, n, dt, ok in _run(_slow_rank_worker, 2, 5.0, 0.6, 4)}
    assert res[0][0] == 0 and res[1][0] == 0, res
    assert res[0][2] and res[1][2], res


def test_dead_peer_costs_one_limit_not_one_per_collective():
    """Rank 1 never calls (delay -1): rank 0's ten collectives give up after ~ONE
    0.5 s limit in total (the first timeout makes the later waits return at once)."""
    res = {r: (n, dt, ok) for r, n, dt, ok in _run(_slow_rank_worker, 2, 0.5, -1.0, 10)}
    n0, dt0, _ = res[0]
    assert n0 >= 1, res
    assert dt0 < 2.5, res  # ten full limits would be >= 5 s


def _selftest_worker(rank, world, port, q, ll_max):
    """maybe_enable's first-contact check on the ranks of this box: every protocol
    agrees with the reference all-reduce, so nothing is switched off. GG_AR runs on
    the 8B TP2 and 70B TP8 O / down shards (tile widths differ between the two)."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0",
                       "XGS_TUNE": "gemm_ar_shared=1"})
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from xgserve.parallel.custom_ar import CustomAllReduce
        ar = CustomAllReduce(rank, world, torch.device("cuda:0"), ll_max=ll_max)
        shapes = [(4096, 2048), (4096, 7168), (8192, 1024), (8192, 3584)]
        res = ar.self_test(dist.group.WORLD, dist.group.WORLD, shapes)
        q.put((rank, (res, ar.verified_counts), ar.protocol(), ar.timeouts()))
        dist.barrier()
        ar.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), None, -1))


@pytest.mark.parametrize("world,ll_max", [(2, None), (2, 0), (4, None)])
def test_custom_allreduce_self_test(world, ll_max):
    from xgserve.parallel.custom_ar import CustomAllReduce
    n = CustomAllReduce.SELF_TEST_ITERS
    for rank, out, proto, tmo in _run(_selftest_worker, world, ll_max):
        assert isinstance(out, tuple), out
        res, counts = out
        assert res["pull"] and res["pull_resid"], res
        assert res["gemm_ar"], res  # the all-reduce inside the row-parallel GEMM launch
        # every protocol ran its full repetition count on fresh data (GG_AR: per shape)
        assert counts["pull"] == n and counts["pull_resid"] == n, counts
        assert counts["gemm_ar"] == 4 * n, counts
        if ll_max == 0:
            assert res["ll"] is None and proto == "pull" and counts["ll"] is None
        else:
            assert res["ll"] and res["ll_resid"] and proto == "ll", res
            assert counts["ll"] == n and counts["ll_resid"] == n, counts
        assert tmo == 0
