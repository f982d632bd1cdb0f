"""Weight-only FP8 decode (csrc/kernels/gemm_w8.hip) on the MI355X: the kernel
against a plain fp32 PyTorch product with the dequantised weights, and the
engine's fp8 decode path against the fp32 reference forward."""
from dataclasses import replace

import pytest
import torch
import torch.nn.functional as F

from xgserve.ops import _native
from xgserve.ops.linear import (MODE_PARTIAL, MODE_SILU, W8_CFGS, deinterleave_gate_up, dequantize_fp8,
                                interleave_gate_up, quantize_fp8, w8_linear)

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _k():
    _native.kernels()  # fail loudly: the HIP library must be the one that runs
    torch.manual_seed(0)


def rel_err(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-6))


def test_quantize_roundtrip_cpu_semantics():
    w = torch.randn(64, 256) * 0.02
    q, s = quantize_fp8(w)
    assert q.dtype == torch.uint8 and s.shape == (64,)
    d = dequantize_fp8(q, s)
    assert rel_err(d, w) < 0.05  # E4M3: 3 mantissa bits
    assert float(d.abs().amax(1).sub(w.abs().amax(1)).abs().max()) < 1e-6  # row max maps to 448 exactly


@pytest.mark.parametrize("M", [1, 5, 16, 17, 40, 64])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 4096), (4096, 14336), (1024, 512)])
@pytest.mark.parametrize("cfg", sorted(W8_CFGS))
@pytest.mark.parametrize("S", [1, 2, 4])
def test_w8_partial(M, N, K, cfg, S):
    cols, kc = W8_CFGS[cfg]
    if N % cols or K % (S * kc) or (M > 16 and cfg >= 3):
        pytest.skip("shape not divisible for this configuration")
    x = torch.randn(M, K, device=DEV).bfloat16()
    q, s = quantize_fp8(torch.randn(N, K, device=DEV) * 0.02)
    pend = w8_linear(x, q, s, MODE_PARTIAL, plan=(S, cfg))
    assert pend.part.shape == (S, M, N)
    ref = x.float() @ dequantize_fp8(q, s).t()
    assert rel_err(pend.part.sum(0), ref) < 2e-3


@pytest.mark.parametrize("M", [1, 7, 16, 33, 64])
@pytest.mark.parametrize("cfg", [0, 1, 3, 4])
def test_w8_silu(M, cfg):
    if M > 16 and cfg >= 3:
        pytest.skip("KC 256 is M <= 16 only")
    Fh, K = 2048, 4096
    x = torch.randn(M, K, device=DEV).bfloat16()
    g = torch.randn(Fh, K, device=DEV) * 0.02
    u = torch.randn(Fh, K, device=DEV) * 0.02
    q, s = quantize_fp8(interleave_gate_up(g, u))
    y = w8_linear(x, q, s, MODE_SILU, plan=(1, cfg))
    gd, ud = deinterleave_gate_up(dequantize_fp8(q, s))
    ref = F.silu(x.float() @ gd.t()) * (x.float() @ ud.t())
    assert rel_err(y, ref) < 1e-2


def test_fp8_engine_decode_matches_reference():
    """Weights made exactly E4M3-representable (per-channel scale), so the bf16
    prefill and the fp8 decode compute the same function: every greedy token of
    the fp8 engine (HIP graphs, batch 3) is an argmax of the fp32 reference."""
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
    from xgserve.models import build_model, get_config
    from xgserve.models.reference import reference_logits
    cfg = replace(get_config("llama3-8b"), num_layers=2, name="llama3-8b-2l-fp8")
    m = build_model(cfg, device="cuda:0", seed=5)
    with torch.no_grad():
        for layer in m.layers:
            for n in ("qkv", "o", "gate_up", "down"):
                w = getattr(layer, n)
                w.copy_(dequantize_fp8(*quantize_fp8(w)).to(w.dtype))
    assert m.quantize_fp8() and m.weight_dtype == "fp8"
    eng = LLMEngine(EngineConfig(model=cfg.name, device="cuda:0", num_blocks=512, max_num_seqs=16,
                                 max_num_batched_tokens=2048, max_model_len=1024, graph_batch_sizes=[1, 2, 4, 8]),
                    model=m)
    prompts = [[128000] + list(range(200 + 7 * i, 260 + 11 * i)) for i in range(3)]
    prompts += [[128000] + list(range(900 + 3 * i, 930 + 3 * i)) for i in range(17)]  # 20 rows: the MT=4 kernel
    outs = eng.generate(prompts, SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True))
    for p, gen in zip(prompts, outs):
        assert len(gen) == 8
        ref = reference_logits(m, p + gen[:-1]).float()
        for i, tok in enumerate(gen):
            row = ref[len(p) - 1 + i]
            assert float(row.max() - row[tok]) < 0.15, (i, tok, int(row.argmax()))
