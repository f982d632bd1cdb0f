"""bench.py's driver contract (one JSON line from rank 0, whole-job aggregate,
max-over-ranks time) exercised on CPU with gloo ranks: DP=2, TP=2 (leader +
follower) and DP=2 x TP=2 with a MoE model. The GPU path is the same script with
RCCL; only the device and the graph capture differ."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    return env


SMALL = ["--steps", "4", "--warmup", "2", "--concurrency", "2", "--prompt-len", "16", "--output-len", "4"]


def _run(nproc, *args, launcher=True):
    if launcher:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py")]
    else:  # bench.py spawns its own ranks (the driver's `python bench.py --gpus N` form)
        cmd = [sys.executable, str(ROOT / "bench.py")]
    cmd += ["--gpus", str(nproc), *SMALL, *args]
    p = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("nproc,tp,model,par", [(2, 1, "llama-tiny", "dp2"), (2, 2, "llama-tiny", "tp2"),
                                                (4, 2, "mixtral-tiny", "dp2xtp2")])
def test_bench_multi_rank_json_contract(nproc, tp, model, par):
    r = _run(nproc, "--tp", str(tp), "--model", model, *(["--allow-rccl-decode"] if tp > 1 else []))
    _check_contract(r, nproc, model, par, tp)
    # pre-flight evidence: the communicator formed at world N and summed
    # correctly, the TP groups, and which library carried the TP decode all-reduce
    assert r["rccl_world"] == nproc
    assert r["tp_groups"] == [list(range(g, g + tp)) for g in range(0, nproc, tp)]
    assert r["p2p_ok"] is None  # no GPUs here
    assert r["decode_ar"] == ("gloo" if tp > 1 else None)
    assert r["detail"]["backend"] == "gloo"


def test_bench_refuses_tp_without_custom_allreduce():
    """--tp > 1 whose decode all-reduce would not be the custom xGMI kernel exits 3
    unless --allow-rccl-decode says that is what is being measured."""
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", *SMALL, "--tp", "2", "--model", "llama-tiny"]
    p = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert "allow-rccl-decode" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("nproc,tp,par", [(2, 1, "dp2"), (4, 2, "dp2xtp2")])
def test_bench_self_launches_ranks(nproc, tp, par):
    """`python bench.py --gpus N` with no external launcher starts N ranks itself."""
    r = _run(nproc, "--tp", str(tp), "--model", "llama-tiny", *(["--allow-rccl-decode"] if tp > 1 else []),
             launcher=False)
    _check_contract(r, nproc, "llama-tiny", par, tp)


def test_bench_single_gpu_default_unchanged():
    r = _run(1, "--model", "llama-tiny", launcher=False)
    _check_contract(r, 1, "llama-tiny", "dp1", 1)


def test_bench_rejects_world_mismatch():
    env = dict(_env(), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", *SMALL, "--model", "llama-tiny"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 2 and "WORLD_SIZE" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def _check_contract(r, nproc, model, par, tp):
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in r
    assert r["n_gpus"] == nproc and r["steps"] == 4 and r["warmup"] == 2
    assert r["higher_is_better"] is True and r["scaling"] == "weak"
    cfg = r["config"]
    assert cfg["model"] == model and cfg["parallelism"] == par
    assert cfg["global_batch"] == 2 * (nproc // tp)  # concurrency per replica x replicas
    # whole-job tokens / slowest rank's time. A step emits at most one token per running
    # sequence plus the immediate first token of a sequence admitted in it (outputs of
    # step N are delivered while step N+1 runs): <= 2 x concurrency per replica.
    assert 0 < r["value"] <= 2 * cfg["global_batch"] * 1000.0 / r["ms_per_step"] + 1e-6


def test_numa_cpulist_parsing_and_noop_without_gpu():
    from xgserve.parallel import affinity as A
    assert A._parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert A._parse_cpulist("") == set()
    # no KFD GPU nodes in this container: nothing to bind, affinity untouched
    import os
    before = os.sched_getaffinity(0)
    assert A.bind_to_gpu_numa(0) is None
    assert os.sched_getaffinity(0) == before
