"""Weight-only INT8 / INT4 decode (Req 10.3; csrc/kernels/gemm_w8.hip FMT = WQ_INT8 /
WQ_INT4) on the MI355X: the kernel against a plain fp32 PyTorch product with the
dequantised weights (every configuration, split and row count, both epilogues), and
the engine's quantized decode path against the fp32 reference forward."""
from dataclasses import replace

import pytest
import torch
import torch.nn.functional as F

from xgserve.ops import _native
from xgserve.ops.linear import (MODE_PARTIAL, MODE_SILU, W8_CFGS, WQ_INT4, WQ_INT8, deinterleave_gate_up,
                                dequantize_weight, interleave_gate_up, quantize_weight, w8_linear, w8_plan)

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _k():
    _native.kernels()  # fail loudly: the HIP library must be the one that runs
    torch.manual_seed(0)


def rel_err(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-6))


@pytest.mark.parametrize("fmt", [WQ_INT8, WQ_INT4])
@pytest.mark.parametrize("M", [1, 5, 16, 17, 64])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 14336), (1024, 512)])
@pytest.mark.parametrize("cfg", sorted(W8_CFGS))
@pytest.mark.parametrize("S", [1, 2, 4])
def test_wq_partial(fmt, M, N, K, cfg, S):
    cols, kc = W8_CFGS[cfg]
    if N % cols or K % (S * kc) or (M > 16 and cfg >= 3):
        pytest.skip("shape not divisible for this configuration")
    if fmt == WQ_INT4 and (K // S // 128) * cols > 4096:
        pytest.skip("int4 group scales exceed the workgroup's LDS stage (the planner raises the split)")
    x = torch.randn(M, K, device=DEV).bfloat16()
    q, s = quantize_weight(torch.randn(N, K, device=DEV) * 0.02, fmt)
    pend = w8_linear(x, q, s, MODE_PARTIAL, plan=(S, cfg), fmt=fmt)
    assert pend.part.shape == (S, M, N)
    ref = x.float() @ dequantize_weight(q, s, fmt).t()
    assert rel_err(pend.part.sum(0), ref) < 2e-3


@pytest.mark.parametrize("fmt", [WQ_INT8, WQ_INT4])
@pytest.mark.parametrize("M", [1, 7, 16, 33, 64])
@pytest.mark.parametrize("cfg", [0, 1, 3, 4])
def test_wq_silu(fmt, M, cfg):
    if M > 16 and cfg >= 3:
        pytest.skip("KC 256 is M <= 16 only")
    Fh, K = 2048, 4096
    x = torch.randn(M, K, device=DEV).bfloat16()
    g = torch.randn(Fh, K, device=DEV) * 0.02
    u = torch.randn(Fh, K, device=DEV) * 0.02
    q, s = quantize_weight(interleave_gate_up(g, u), fmt)
    y = w8_linear(x, q, s, MODE_SILU, plan=(1, cfg), fmt=fmt)
    gd, ud = deinterleave_gate_up(dequantize_weight(q, s, fmt))
    ref = F.silu(x.float() @ gd.t()) * (x.float() @ ud.t())
    assert rel_err(y, ref) < 1e-2


@pytest.mark.parametrize("fmt", [WQ_INT8, WQ_INT4])
def test_wq_planned_70b_shapes(fmt):
    """The planner's choices for the Llama-3-70B projections (int4: splits raised so
    the group scales fit), each run once against the fp32 product at M = 1 and 64."""
    for N, K, mode in ((10240, 8192, MODE_PARTIAL), (8192, 28672, MODE_PARTIAL), (57344, 8192, MODE_SILU)):
        for M in (1, 64):
            p = w8_plan(M, N, K, mode, fmt)
            assert p is not None, (N, K, mode, M)
            if mode == MODE_SILU:
                continue  # (the 57344-row gate_up: plan existence only; 3.7 GB of fp32 reference)
            x = torch.randn(M, K, device=DEV).bfloat16()
            q, s = quantize_weight(torch.randn(N, K, device=DEV) * 0.02, fmt)
            pend = w8_linear(x, q, s, mode, fmt=fmt)
            ref = x.float() @ dequantize_weight(q, s, fmt).t()
            assert rel_err(pend.part.sum(0), ref) < 2e-3


@pytest.mark.parametrize("kind", ["int8", "int4"])
def test_wq_engine_decode_matches_reference(kind):
    """Weights replaced by their dequantised values (so the bf16 prefill and the
    quantized decode compute nearly the same function): every greedy token of the
    quantized engine (HIP graphs, 3 and 20 rows) is an argmax of the fp32 reference."""
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
    from xgserve.models import build_model, get_config
    from xgserve.models.reference import reference_logits
    from xgserve.ops.linear import WQ_FORMATS
    fmt = WQ_FORMATS[kind]
    cfg = replace(get_config("llama3-8b"), num_layers=2, name=f"llama3-8b-2l-{kind}")
    m = build_model(cfg, device="cuda:0", seed=5)
    with torch.no_grad():
        for layer in m.layers:
            for n in ("qkv", "o", "gate_up", "down"):
                w = getattr(layer, n)
                w.copy_(dequantize_weight(*quantize_weight(w, fmt), fmt).to(w.dtype))
    assert m.quantize_weights(kind) and m.weight_dtype == kind
    assert all(q[2] == fmt for q in m.layers[0].w8.values())
    eng = LLMEngine(EngineConfig(model=cfg.name, device="cuda:0", num_blocks=512, max_num_seqs=32,
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
