"""CPU checks of the decode / prefill GEMM plan logic in xgserve/ops/linear.py: plan
validity rules, the XGS_M64_PLANS override parser, the split-K prefill gate, and the
host-side shape checks of gemm_m64g's split-K SiLU and cooperative-residual modes
(rejected before any launch, so they run without a GPU)."""
import pytest
import torch

from xgserve.ops import linear as L
from xgserve.ops._native import kernels


def test_every_tuned_plan_is_valid():
    for (N, K, mode), buckets in L._M64_TUNED.items():
        for bucket, (nw, S, cfg) in buckets.items():
            assert cfg in L.M64G_CFGS
            assert L._m64_valid(N, K, mode, nw, S, cfg), (N, K, mode, bucket)
            assert L.m64_plan(min(bucket, 64), N, K, mode) is not None


def test_split_silu_plans_are_valid_only_for_pair_tiles():
    assert L._m64_valid(7168, 8192, L.MODE_SILU, 2, 2, 6)
    assert not L._m64_valid(7168, 8192, L.MODE_SILU, 1, 2, 6)   # gate / up pairs need nw = 2
    assert not L._m64_valid(4096, 4096, L.MODE_BF16, 2, 2, 0)   # bf16 output has no split form
    assert L._m64_valid(57344, 8192, L.MODE_SILU, 2, 1, 7)      # 8-wave 256-column tile
    assert not L._m64_valid(4096 + 128, 4096, L.MODE_SILU, 2, 1, 7)


def test_plan_override_parser(monkeypatch):
    table = {k: dict(v) for k, v in L._M64_TUNED.items()}
    monkeypatch.setattr(L, "_M64_TUNED", table)
    L._apply_plan_overrides("28672x4096x2@64=2,2,7; 1234x4096x1@16=1,4,0")
    assert table[(28672, 4096, L.MODE_SILU)][64] == (2, 2, 7)
    assert table[(28672, 4096, L.MODE_SILU)][16] == L._M64_TUNED[(28672, 4096, L.MODE_SILU)][16]
    assert table[(1234, 4096, L.MODE_PARTIAL)] == {16: (1, 4, 0)}
    L._apply_plan_overrides("")  # no-op


def test_splitk_prefill_gate_cpu():
    x = torch.zeros(575, 14336, dtype=torch.bfloat16)
    w = torch.zeros(4096, 14336, dtype=torch.bfloat16)
    assert not L.splitk_prefill_ok(x, w)  # CPU tensors never take the batched-GEMM path


def _check(mode, M=64, N=28672, K=4096, S=2, nw=2, cfg=1, part=1, counters=0, resid=0, ss=0):
    k = kernels()
    return k.gemm_m64g_ex(1, M, K, 1, N, part, 1, S, mode, nw, cfg, 0, 0, 0, 1e-5, resid, ss, counters, 0)


def test_split_silu_needs_slabs_and_tickets():
    with pytest.raises(Exception):
        _check(L.MODE_SILU, counters=0)          # S > 1 without ticket words
    with pytest.raises(Exception):
        _check(L.MODE_SILU, part=0, counters=1)  # S > 1 without fp32 slabs
    with pytest.raises(Exception):
        _check(L.MODE_SILU, nw=1, counters=1)


