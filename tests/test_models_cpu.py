"""Model-level CPU checks (no GPU): RMSNorm folding is an exact reparametrisation."""
import torch

from xgserve.models import build_model, get_config
from xgserve.models.reference import reference_logits


def test_fold_norms_preserves_reference_logits():
    m = build_model(get_config("llama-tiny"), device="cpu", dtype=torch.float32, seed=1)
    g = torch.Generator().manual_seed(0)
    with torch.no_grad():
        for layer in m.layers:
            layer.input_norm.copy_(1 + 0.3 * torch.randn(layer.input_norm.shape, generator=g))
            layer.post_norm.copy_(1 + 0.3 * torch.randn(layer.post_norm.shape, generator=g))
    toks = [1, 5, 9, 13, 200, 31, 77]
    before = reference_logits(m, toks)
    m.fold_norms()
    assert m.norms_folded
    assert all(bool((layer.input_norm == 1).all()) and bool((layer.post_norm == 1).all()) for layer in m.layers)
    after = reference_logits(m, toks)
    torch.testing.assert_close(after, before, atol=1e-4, rtol=1e-4)


def test_fold_norms_keeps_moe_post_norm():
    m = build_model(get_config("mixtral-tiny"), device="cpu", dtype=torch.float32, seed=2)
    with torch.no_grad():
        for layer in m.layers:
            layer.post_norm.fill_(1.5)
            layer.input_norm.fill_(0.5)
    toks = [1, 4, 8, 15]
    before = reference_logits(m, toks)
    m.fold_norms()
    assert all(bool((layer.post_norm == 1.5).all()) for layer in m.layers)  # router + experts read it
    torch.testing.assert_close(reference_logits(m, toks), before, atol=1e-4, rtol=1e-4)


def test_engine_rejects_out_of_vocab_prompt_ids():
    """An id outside the embedding table must never reach the GPU gather."""
    import pytest
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
    eng = LLMEngine(EngineConfig(model="llama-tiny", device="cpu", dtype="float32", num_blocks=32, max_num_seqs=2,
                                 max_num_batched_tokens=64, use_graphs=False))
    V = eng.mcfg.vocab_size
    for bad in ([1, V], [-1, 2]):
        with pytest.raises(ValueError, match="token ids"):
            eng.add_request("x", bad, SamplingParams(max_tokens=2))
    eng.add_request("ok", [1, V - 1], SamplingParams(max_tokens=2))
