"""Shared-memory plan channel (csrc/runtime/shm_channel.cpp): ordering, multi-reader
broadcast across processes, timeouts, and the TP plan-broadcast path that uses it."""
import multiprocessing as mp
import os
import time

import pytest

R = pytest.importorskip("xgserve._runtime")


def _name(tag):
    return f"xgs_t_{tag}_{os.getpid()}"


def _reader(name, rank, n, q):
    try:
        c = R.ShmChannel(name, 0, 2, False)
        for i in range(n):
            b = c.receive(rank, 20.0)
            if b != (b"m%d;" % i) * (i % 50 + 1):
                q.put(("bad", rank, i))
                return
        q.put(("ok", rank, n))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("err", rank, repr(e)))


def test_single_process_roundtrip():
    ch = R.ShmChannel(_name("a"), 4096, 1, True)
    rd = R.ShmChannel(ch.name, 0, 1, False)
    assert rd.capacity == 4096
    for i in range(5):
        assert ch.publish(b"x" * i + b"!", 1.0)
        assert rd.receive(0, 1.0) == b"x" * i + b"!"
    assert ch.seq == 5
    # nothing new: receive times out and returns None
    t = time.time()
    assert rd.receive(0, 0.05) is None
    assert time.time() - t < 5.0  # a 50 ms timeout must not block (slack for a loaded host)
    # the producer cannot publish twice without the reader acknowledging
    assert ch.publish(b"one", 1.0)
    assert not ch.publish(b"two", 0.05)
    assert rd.receive(0, 1.0) == b"one"
    assert ch.publish(b"two", 1.0)
    assert rd.receive(0, 1.0) == b"two"


def test_rejects_oversize_and_bad_rank():
    ch = R.ShmChannel(_name("b"), 64, 1, True)
    with pytest.raises(ValueError):
        ch.publish(b"z" * 65, 0.1)
    rd = R.ShmChannel(ch.name, 0, 1, False)
    with pytest.raises(IndexError):
        rd.receive(1, 0.01)
    with pytest.raises(RuntimeError):
        R.ShmChannel(_name("missing"), 0, 1, False)


def test_multi_process_broadcast():
    name = _name("c")
    ch = R.ShmChannel(name, 1 << 16, 2, True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    n = 500
    ps = [ctx.Process(target=_reader, args=(name, r, n, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        for i in range(n):
            assert ch.publish((b"m%d;" % i) * (i % 50 + 1), 30.0), i
        res = sorted(q.get(timeout=60) for _ in ps)
        assert res == [("ok", 0, n), ("ok", 1, n)]
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()


def _tp_worker(rank, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np

    from xgserve.parallel import comm, state
    state.PLAN_CHANNEL_BYTES = 1 << 16
    try:
        s = state.init_distributed(tp_size=2, backend="gloo")
        got = [s.plan_channel is not None]
        for i in range(20):
            big = i % 7 == 3  # > 64 KiB: announced on the channel, sent over gloo
            obj = ("plan", {"i": i, "ids": np.arange(40000 if big else 100 + i, dtype=np.int32)})
            r = comm.tp_broadcast_object(obj if rank == 0 else None, src=0)
            got.append(r[1]["i"] == i and int(r[1]["ids"].sum()) == int(obj[1]["ids"].sum()))
        q.put((rank, all(got)))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        state.destroy_distributed()


def test_tp_plan_broadcast_over_shm():
    from xgserve.server.replica import _free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_tp_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        res = sorted(q.get(timeout=120) for _ in ps)
        assert res == [(0, True), (1, True)]
        assert not any(f.startswith("xgs_plan_") for f in os.listdir("/dev/shm"))
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
