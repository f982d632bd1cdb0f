"""Speculative decoding (Req 12): exactness vs plain greedy decoding, acceptance
accounting, adaptive disable below 50 % acceptance, mixing with sampled requests."""
from __future__ import annotations

import pytest

from xgserve.engine import EngineConfig, LLMEngine, SamplingParams


def _engine(draft=None, k=0, **kw):
    return LLMEngine(EngineConfig(model="llama-tiny", device="cpu", dtype="float32", num_blocks=128, max_num_seqs=8,
                                  max_num_batched_tokens=256, use_graphs=False, seed=7, draft_model=draft,
                                  num_speculative_tokens=k, **kw))


PROMPTS = [[1] + list(range(10, 40)), [1, 5, 9, 200, 300], [1] + list(range(100, 160))]
SP = SamplingParams(max_tokens=20, temperature=0.0, ignore_eos=True)


@pytest.mark.parametrize("k", [1, 3, 5])
def test_self_draft_accepts_everything_and_matches_greedy(k):
    want = _engine().generate(PROMPTS, SP)
    eng = _engine("llama-tiny", k)  # draft == target weights -> every draft token accepted
    got = eng.generate(PROMPTS, SP)
    assert got == want
    st = eng.stats()["speculative"]
    assert st["draft_tokens_proposed"] > 0
    assert st["acceptance_rate"] == 1.0
    assert st["mean_tokens_per_verify"] == pytest.approx(k + 1, rel=0.35)
    assert eng.stats()["steps"] < _steps_plain() / (1 + 0.5 * k)


def _steps_plain():
    e = _engine()
    e.generate(PROMPTS, SP)
    return e.stats()["steps"]


def test_weak_draft_is_exact_and_gets_disabled():
    want = _engine().generate(PROMPTS, SP)
    eng = _engine("llama-tiny-draft", 4)
    got = eng.generate(PROMPTS, SP)
    assert got == want  # verification keeps greedy output exact whatever the draft says
    st = eng.stats()["speculative"]
    assert st["acceptance_rate"] < 0.5
    assert st["active"] == 0 or all(d.disabled for d in eng.spec.seqs.values())


def test_mixed_greedy_and_sampled_batch():
    eng = _engine("llama-tiny", 3)
    rids = []
    eng.add_request("g", PROMPTS[0], SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True))
    eng.add_request("s", PROMPTS[1], SamplingParams(max_tokens=12, temperature=0.8, seed=3, ignore_eos=True))
    toks = {"g": [], "s": []}
    for _ in range(200):
        if not eng.has_work():
            break
        for o in eng.step():
            toks[o.request_id] += o.new_token_ids
    assert len(toks["g"]) == 12 and len(toks["s"]) == 12
    assert toks["g"] == _engine().generate([PROMPTS[0]], SamplingParams(max_tokens=12, temperature=0.0,
                                                                        ignore_eos=True))[0]


def test_stop_inside_accepted_run():
    """EOS / max_tokens inside an accepted draft run truncates exactly like plain decoding."""
    sp = SamplingParams(max_tokens=7, temperature=0.0, ignore_eos=True)
    assert _engine("llama-tiny", 4).generate(PROMPTS, sp) == _engine().generate(PROMPTS, sp)


def test_speedup_factor_is_measured():
    """Req 12.4: the engine times speculating steps (propose + verify) and plain
    decode steps; speedup = tokens per speculated row-step x plain / spec step time."""
    eng = _engine("llama-tiny", 3)
    eng.add_request("g", PROMPTS[0], SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True))
    eng.add_request("s", PROMPTS[1], SamplingParams(max_tokens=40, temperature=0.8, seed=3, ignore_eos=True))
    for _ in range(300):
        if not eng.has_work():
            break
        eng.step()
    st = eng.stats()["speculative"]
    sp = eng.spec
    assert sp.ema_spec_ms and sp.ema_plain_ms  # both kinds of steps were seen
    assert 1.0 < sp.ema_tokens_per_row <= 4.0
    want = sp.ema_tokens_per_row * sp.ema_plain_ms / sp.ema_spec_ms
    assert st["speedup_factor"] == pytest.approx(want, rel=1e-3)
    assert st["speedup_factor"] > 0


def test_speedup_factor_exported():
    from xgserve.obs.metrics import MetricsCollector
    m = MetricsCollector()
    assert "xgs_spec_speedup_factor" not in m.prometheus()
    m.set_spec_totals(100, 80, 1.75)
    assert "xgs_spec_speedup_factor 1.75" in m.prometheus()
    assert m.snapshot()["speculative"]["speedup_factor"] == 1.75
