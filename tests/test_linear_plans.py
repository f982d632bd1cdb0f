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


def test_arx_gate_follows_the_plans():
    assert L.m64_arx_ok(1, 7168, 4096, L.MODE_SILU)         # gate_up8t4: (2, 4, 1), 4 waves
    assert L.m64_arx_ok(1, 1536, 4096, L.MODE_PARTIAL)      # qkv8t4: (1, 8, 4), 2 waves
    assert not L.m64_arx_ok(1, 14336, 4096, L.MODE_SILU)    # gate_up8t2 at 16 rows: 8-wave cfg 7
    assert not L.m64_arx_ok(1, 6144, 3072, L.MODE_PARTIAL)  # K not a multiple of 1024


def _arx(mode=L.MODE_PARTIAL, M=1, K=4096, N=6144, S=2, nw=1, cfg=0, ar_part=1, ar_S=4, wgs=4, flags=1):
    return kernels().gemm_m64g_arx(1, M, K, 1, N, 1, 1, S, mode, nw, cfg, 1, 1e-5, 1, ar_part, ar_S, wgs, flags, 0, 0)


@pytest.mark.parametrize("bad", [dict(mode=3), dict(mode=0, S=1), dict(K=4096 + 256), dict(K=16384, N=1024),
                                 dict(wgs=0), dict(wgs=65), dict(flags=0), dict(ar_part=0), dict(ar_S=0),
                                 dict(cfg=7, nw=2, N=8192)])
def test_arx_host_checks_reject_before_launch(bad):
    with pytest.raises(Exception):
        _arx(**bad)
