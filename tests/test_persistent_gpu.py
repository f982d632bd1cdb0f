"""Persistent batch-1 decode (csrc/kernels/decode_b1.hip) on the MI355X: every decode
step of a one-sequence greedy generation -- all layers in one launch, K/V appended by
the kernel -- against the dense fp32 reference forward with the same weights, for the
Llama-3-8B layer shape, a Llama-3.2-1B-sized shape (head_dim 128) and the Llama-3-70B TP8 rank shape
(8 q heads over 1 kv head, G = 8), eager and graph-captured; plus the kernel's
timeout path (a grid that cannot be co-resident must fail the step, not hang)."""
from dataclasses import replace

import pytest
import torch

from xgserve.ops import _native

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module")
def _k():
    _native.kernels()


@pytest.fixture(autouse=True)
def _on(monkeypatch):
    import xgserve.models.llama as ll
    monkeypatch.setattr(ll, "PERSISTENT_DECODE", True)


def _model(base: str, seed: int, **kw):
    from xgserve.models import build_model, get_config
    cfg = replace(get_config(base), num_layers=2, name=f"{base}-b1-{seed}", **kw)
    return build_model(cfg, device="cuda:0", seed=seed)


SHAPES = {
    "8b": ("llama3-8b", {}),
    "1b_hd128": ("llama3.2-1b", dict(head_dim=128, num_heads=16, num_kv_heads=8)),
    "70b_tp8_rank": ("llama3-8b", dict(hidden_size=8192, num_heads=8, num_kv_heads=1, intermediate_size=3584)),
}


def _generate(model, prompt, n, graphs):
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
    eng = LLMEngine(EngineConfig(model=model.cfg.name, device="cuda:0", num_blocks=512, max_num_seqs=4,
                                 max_num_batched_tokens=4096, max_model_len=4096, use_graphs=graphs,
                                 graph_batch_sizes=[1, 2, 4]), model=model)
    eng.runner.capture_logits = not graphs
    eng.add_request("r", prompt, SamplingParams(max_tokens=n, temperature=0.0, ignore_eos=True))
    toks, logits = [], []
    while eng.has_work():
        for o in eng.step():
            toks += o.new_token_ids
        if not graphs and eng.runner.last_logits is not None:
            logits.append(eng.runner.last_logits[-1].clone())
    return toks, logits, eng


@pytest.mark.parametrize("shape", list(SHAPES))
@pytest.mark.parametrize("plen", [37, 700])
def test_b1_decode_steps_match_reference(shape, plen):
    from xgserve.models.reference import reference_logits
    base, kw = SHAPES[shape]
    model = _model(base, 11, **kw)
    prompt = [128000] + [(977 * i + 13) % 120000 for i in range(plen)]
    toks, logits, eng = _generate(model, prompt, 6, graphs=False)
    assert model._b1 is not None, "the persistent kernel did not run"
    assert model._b1.timeouts() == 0
    assert len(toks) == 6 and len(logits) >= 6
    # logits[0] is the prefill step's; logits[i] (i >= 1) are persistent decode steps
    for i in range(1, 6):
        ref = reference_logits(model, prompt + toks[:i])[-1].float().cpu()
        err = float((logits[i] - ref).norm() / ref.norm())
        assert err < 2e-2, (i, err)
        gap = ref.max() - ref[toks[i]]
        assert gap <= 0.1 * ref.std(), (i, float(gap))


def test_b1_graphs_match_eager():
    """Graph-captured persistent steps (the memset node + kernel, replayed with new
    metadata) produce the eager tokens; a second engine on the same model reuses the
    decoder with its own KV caches."""
    model = _model("llama3-8b", 7)
    prompt = [128000] + list(range(4000, 4300))
    eager, _, _ = _generate(model, prompt, 24, graphs=False)
    graph, _, eng = _generate(model, prompt, 24, graphs=True)
    assert model._b1 is not None and model._b1.timeouts() == 0
    assert eager == graph


def test_b1_timeout_fails_the_step_instead_of_hanging():
    """A producer that never publishes (ctl[2]: workgroup 0 drops its QKV granules)
    must not hang the grid: the waiting workgroups give up after the wait limit, count
    the timeout, every later wait returns at once, the launch drains and check()
    raises. The same launch without the fault completes with no timeout."""
    from xgserve.ops.persistent import PersistentDecodeTimeout
    model = _model("llama3-8b", 5)
    prompt = [128000] + list(range(100, 160))
    _generate(model, prompt, 2, graphs=False)
    dec = model._b1
    assert dec is not None
    resid = torch.zeros(1, model.cfg.hidden_size, dtype=torch.bfloat16, device="cuda:0")
    kv = [(torch.zeros(8, model.layers[0].Hkv, 16, 128, dtype=torch.bfloat16, device="cuda:0"),) * 2
          for _ in model.layers]
    i32 = lambda *v: torch.tensor(v, dtype=torch.int32, device="cuda:0")  # noqa: E731
    args = (resid, i32(3), i32(3), i32(0, 1, 2, 3, 4, 5, 6, 7), i32(4), model.cos_sin, kv)
    dec.ctl[0].zero_()
    dec.ctl[2].fill_(1)
    dec.set_timeout(0.05)
    t0 = __import__("time").monotonic()
    dec(*args)
    torch.cuda.synchronize()
    dt = __import__("time").monotonic() - t0
    assert dec.timeouts() > 0 and dt < 5.0, (dec.timeouts(), dt)
    dec.poll_async()
    torch.cuda.synchronize()
    with pytest.raises(PersistentDecodeTimeout):
        dec.check()
    dec.ctl[0].zero_()
    dec.ctl[2].zero_()
    dec.set_timeout(20.0)
    dec(*args)
    torch.cuda.synchronize()
    assert dec.timeouts() == 0
