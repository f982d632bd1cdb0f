"""All-reduce prologue of gemm_m64g (gemm_m64g_arx): reducer workgroups fold the
previous projection's split-K partials into the residual stream inside the next
GEMM's launch. Checked against the separate-launch chain (add_partials_resid, itself
checked elsewhere) -- the residual bit for bit -- and against fp32 for the GEMM."""
from dataclasses import replace

import pytest
import torch
import torch.nn.functional as F

from xgserve.ops import _native
from xgserve.ops import linear as lin
from xgserve.ops.linear import MODE_PARTIAL, MODE_SILU, PendingSum, interleave_gate_up, m64_arx_linear

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _k():
    _native.kernels()  # fail loudly: the HIP library must be the one that runs
    torch.manual_seed(0)


def rnd(*s, scale=1.0):
    return (torch.randn(*s, device=DEV) * scale).bfloat16()


def rel_err(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-6))


# (N, K, mode, plan for M <= 16, plan above): deep ring, SiLU at split 1 (2 waves),
# split-K SiLU (tile tickets), a 70B-TP8-shaped QKV at K = 8192
SHAPES = [(6144, 4096, MODE_PARTIAL, (1, 2, 9), (1, 2, 0)),
          (8192, 4096, MODE_SILU, (2, 1, 5), (2, 1, 5)),
          (8192, 4096, MODE_SILU, (2, 2, 6), (2, 2, 6)),
          (1280, 8192, MODE_PARTIAL, (1, 6, 0), (1, 6, 1))]


@pytest.mark.parametrize("M", [1, 5, 16, 40])
@pytest.mark.parametrize("shape", range(len(SHAPES)))
@pytest.mark.parametrize("ticks", [0, 2000])
def test_arx_matches_separate_fold(M, shape, ticks):
    N, K, mode, p_small, p_big = SHAPES[shape]
    if ticks and M not in (1, 16):
        pytest.skip("the simulated wait is exercised at two sizes")
    S_prev, eps = 4, 1e-5
    r0 = rnd(M, K)
    prev = torch.randn(S_prev, M, K, device=DEV) * 0.3
    if mode == MODE_SILU:
        g, u = rnd(N // 2, K, scale=0.02), rnd(N // 2, K, scale=0.02)
        w = interleave_gate_up(g, u)
    else:
        w = rnd(N, K, scale=0.02)
    # the separate-launch chain's residual and statistics
    r_ref = r0.clone()
    ss_ref = torch.zeros(K // 1024 * M, device=DEV)
    _native.kernels().add_partials_resid(prev.data_ptr(), S_prev, M, r_ref.data_ptr(), ss_ref.data_ptr(), K,
                                         torch.cuda.current_stream().cuda_stream)
    h = r_ref.float() * torch.rsqrt((r_ref.float() ** 2).sum(-1, keepdim=True) / K + eps)
    ref = F.silu(h @ g.float().t()) * (h @ u.float().t()) if mode == MODE_SILU else h @ w.float().t()
    key = (N, K, mode)
    old = lin._M64_TUNED.get(key)
    lin._M64_TUNED[key] = {16: p_small, 32: p_big, 64: p_big}
    flags = torch.zeros(3, dtype=torch.int32, device=DEV)
    try:
        runs = []
        for _ in range(3):  # the flags are re-armed by each launch
            r = r0.clone()
            ss = torch.full((K // 1024 * M,), -1.0, device=DEV)
            y = m64_arx_linear(r, PendingSum(prev, S_prev), w, mode, ss, eps, flags, ticks=ticks)
            y = y.part.sum(0) if mode == MODE_PARTIAL else y
            torch.cuda.synchronize()
            assert torch.equal(r, r_ref)
            assert rel_err(ss, ss_ref) < 1e-5
            assert rel_err(y, ref) < (2e-3 if mode == MODE_PARTIAL else 1e-2)
            assert int(flags.abs().sum()) == 0  # re-armed, and no wait timed out (word 2)
            runs.append(y.clone())
        assert all(torch.equal(runs[0], t) for t in runs)
    finally:
        if old is None:
            del lin._M64_TUNED[key]
        else:
            lin._M64_TUNED[key] = old


@pytest.fixture(scope="module")
def llama_tp4_shard():
    from xgserve.models import build_model, get_config
    cfg = replace(get_config("llama3-8b"), num_layers=2, name="llama3-8b-2l")
    return build_model(cfg, device="cuda:0", seed=7, tp=4, rank=0)


@pytest.mark.parametrize("n_seqs", [1, 3])
def test_tp_shard_decode_with_ar_prologue(llama_tp4_shard, n_seqs, monkeypatch):
    """One rank of a simulated TP-4 group: greedy decode with the residual all-reduces
    folded into the next GEMMs matches the separate-launch chain (same arithmetic up
    to the statistics' summation order)."""
    import xgserve.models.llama as ll
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
    prompts = [[128000] + list(range(900 + 7 * i, 960 + 3 * i)) for i in range(n_seqs)]
    sp = SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True)
    logits = {}
    calls = [0]
    real = ll.m64_arx_linear

    def counted(*a, **k):
        calls[0] += 1
        return real(*a, **k)

    monkeypatch.setattr(ll, "m64_arx_linear", counted)
    for on in (False, True):
        monkeypatch.setattr(ll, "AR_PROLOGUE", on)
        eng = LLMEngine(EngineConfig(model=llama_tp4_shard.cfg.name, device="cuda:0", num_blocks=256, max_num_seqs=8,
                                     max_num_batched_tokens=1024, max_model_len=512, use_graphs=False),
                        model=llama_tp4_shard)
        eng.runner.capture_logits = True
        assert llama_tp4_shard.layers[0]._ar_prologue(n_seqs) is on
        eng.generate(prompts, sp)
        logits[on] = eng.runner.last_logits[-1].float().cpu()
        assert (calls[0] > 0) is on  # the fused decode layer ran the prologue form
        assert lin.m64_arx_fault(llama_tp4_shard._fused_ws.ar_flags) == 0
    assert rel_err(logits[True], logits[False]) < 1e-2
