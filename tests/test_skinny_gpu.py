"""Decode skinny GEMM + its split-K consumers vs fp32 PyTorch references."""
import pytest
import torch

from xgserve import ops
from xgserve.ops import _native
from xgserve.ops.linear import (MODE_BF16, MODE_PARTIAL, MODE_SILU, interleave_gate_up, pick_split,
                                skinny_linear)

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _k():
    _native.kernels()
    torch.manual_seed(0)


def rnd(*s, scale=1.0):
    return (torch.randn(*s, device=DEV) * scale).bfloat16()


def rel_err(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-6))


@pytest.mark.parametrize("M", [1, 7, 16, 33, 64, 100, 128])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 14336), (512, 256), (1024, 512)])
def test_skinny_partial(M, N, K):
    x, w = rnd(M, K), rnd(N, K, scale=0.02)
    S = pick_split(N, K)
    pend = skinny_linear(x, w, S, MODE_PARTIAL)
    got = pend.part.sum(0)
    ref = x.float() @ w.float().t()
    assert rel_err(got, ref) < 5e-3
    assert rel_err(pend.materialize(), ref) < 1e-2


@pytest.mark.parametrize("M", [17, 33, 48, 64])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 4096), (4096, 14336)])
def test_skinny_slab_auto_split(M, N, K):
    from xgserve.ops.linear import choose_split
    x, w = rnd(M, K), rnd(N, K, scale=0.02)
    S = choose_split(M, N, K)
    pend = skinny_linear(x, w, S, MODE_PARTIAL)
    ref = x.float() @ w.float().t()
    assert rel_err(pend.part.sum(0), ref) < 5e-3, (S,)


@pytest.mark.parametrize("M", [1, 64, 128])
def test_skinny_bf16(M):
    x, w = rnd(M, 4096), rnd(2048, 4096, scale=0.02)
    y = skinny_linear(x, w, mode=MODE_BF16)
    assert rel_err(y, x.float() @ w.float().t()) < 1e-2


@pytest.mark.parametrize("M", [1, 64, 97])
def test_skinny_silu_interleaved(M):
    F, H = 1792, 4096
    g, u = rnd(F, H, scale=0.02), rnd(F, H, scale=0.02)
    w = interleave_gate_up(g, u).contiguous()
    x = rnd(M, H)
    y = skinny_linear(x, w, mode=MODE_SILU)
    ref = torch.nn.functional.silu(x.float() @ g.float().t()) * (x.float() @ u.float().t())
    assert y.shape == (M, F)
    assert rel_err(y, ref) < 1e-2
    # the hipBLASLt-path activation on the same interleaved layout
    gu = x @ w.t()
    assert rel_err(ops.silu_and_mul(gu, interleave16=True), ref) < 1e-2


def test_add_partials_rmsnorm():
    T, H, S = 37, 4096, 4
    part = torch.randn(S, T, H, device=DEV)
    res = rnd(T, H)
    w = rnd(H)
    res0 = res.clone()
    pend = ops.linear.PendingSum(part, S)
    y, r = ops.fused_add_rmsnorm(pend, res, w, 1e-5)
    rr = (res0.float() + part.sum(0)).bfloat16()
    torch.testing.assert_close(r.float(), rr.float(), atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(y.float(), ops.rmsnorm_ref(rr, w, 1e-5).float(), atol=3e-2, rtol=3e-2)


def test_rope_cache_partials_matches_bf16_path():
    Hq, Hkv, D, T, bs, NB = 32, 8, 128, 19, 16, 8
    S = 4
    W = (Hq + 2 * Hkv) * D
    part = torch.randn(S, T, W, device=DEV)
    qkv = part.sum(0).bfloat16()
    pos = torch.arange(T, device=DEV, dtype=torch.int32) * 7
    cs = ops.build_cos_sin(D, 4096, 500000.0, device=DEV)
    slots = torch.randperm(NB * bs, device=DEV)[:T].int()
    kc1 = torch.zeros(NB, Hkv, bs, D, dtype=torch.bfloat16, device=DEV)
    vc1, kc2, vc2 = kc1.clone(), kc1.clone(), kc1.clone()
    q = torch.empty(T, Hq * D, dtype=torch.bfloat16, device=DEV)
    ops.rope_cache_partials(ops.linear.PendingSum(part, S), q, pos, cs, kc1, vc1, slots, Hq, Hkv, D)
    ops.rope_cache(qkv, pos, cs, kc2, vc2, slots, Hq, Hkv, D)
    torch.testing.assert_close(q.float(), qkv[:, :Hq * D].float(), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(kc1.float(), kc2.float(), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(vc1.float(), vc2.float(), atol=3e-2, rtol=2e-2)


# ---------------------------------------------------------------- gemm_m64 (16 < M <= 64)
@pytest.mark.parametrize("M", [17, 24, 32, 33, 48, 63, 64])
@pytest.mark.parametrize("N,K,nw,S", [(6144, 4096, 1, 4), (4096, 4096, 1, 4), (4096, 14336, 1, 4),
                                      (4096, 14336, 2, 1), (1024, 512, 1, 2), (768, 256, 1, 1)])
def test_gemm_m64_partial(M, N, K, nw, S):
    from xgserve.ops.linear import m64_linear
    if N % (64 * nw) or K % (S * 256):
        pytest.skip("shape not tileable")
    x, w = rnd(M, K), rnd(N, K, scale=0.02)
    pend = m64_linear(x, w, MODE_PARTIAL, split_k=S, nw=nw)
    ref = x.float() @ w.float().t()
    assert pend.part.shape == (S, M, N)
    assert rel_err(pend.part.sum(0), ref) < 1e-5
    assert rel_err(pend.materialize(), ref) < 1e-2


@pytest.mark.parametrize("M", [17, 40, 64])
def test_gemm_m64_modes(M):
    from xgserve.ops.linear import m64_linear
    F_, H = 1024, 512
    x = rnd(M, H)
    g, u = rnd(F_, H, scale=0.05), rnd(F_, H, scale=0.05)
    w = interleave_gate_up(g, u)
    got = m64_linear(x, w, MODE_SILU)
    ref = torch.nn.functional.silu(x.float() @ g.float().t()) * (x.float() @ u.float().t())
    assert got.shape == (M, F_)
    assert rel_err(got, ref) < 1e-2
    w2 = rnd(2048, H, scale=0.02)
    got2 = m64_linear(x, w2, MODE_BF16)
    assert rel_err(got2, x.float() @ w2.float().t()) < 1e-2


@pytest.mark.parametrize("M", [17, 33, 64])
@pytest.mark.parametrize("N,K,nw,S", [(6144, 4096, 1, 4), (4096, 14336, 1, 4), (28672, 4096, 2, 1), (1024, 768, 1, 2),
                                      (512, 1280, 2, 1), (2048, 1792, 1, 1), (512, 512, 2, 2)])
def test_gemm_m64g_partial(M, N, K, nw, S):
    """Every chunk/slot phase of the LDS-DMA ring, incl. odd chunk counts."""
    from xgserve.ops.linear import m64_linear
    x, w = rnd(M, K), rnd(N, K, scale=0.02)
    pend = m64_linear(x, w, MODE_PARTIAL, split_k=S, nw=nw)
    ref = x.float() @ w.float().t()
    assert rel_err(pend.part.sum(0), ref) < 1e-5


def test_gemm_m64_rejects_bad_shapes():
    from xgserve.ops.linear import m64_linear
    with pytest.raises(ValueError):
        m64_linear(rnd(8, 256), rnd(256, 256), MODE_PARTIAL)   # M <= 16: not this kernel
    with pytest.raises(ValueError):
        m64_linear(rnd(32, 200), rnd(256, 200), MODE_PARTIAL)  # K % 256


# ---------------------------------------------------------------- gemm_mw (64 < M <= 320)
@pytest.mark.parametrize("M", [65, 100, 128, 192, 257, 320])
@pytest.mark.parametrize("cfg", list(range(7)))
def test_gemm_mw_partial_every_cfg(M, cfg):
    """Every ring depth / tile width, incl. uneven split-K chunk ranges (K / 64 = 22
    chunks over S = 3 and 5) and short splits (1-2 chunks per split)."""
    from xgserve.ops.linear import MW_CFGS, mw_linear
    cols = MW_CFGS[cfg][0]
    N, K = 2 * cols, 1408
    x, w = rnd(M, K), rnd(N, K, scale=0.02)
    ref = x.float() @ w.float().t()
    for S in (1, 3, 5, 16):
        try:
            pend = mw_linear(x, w, MODE_PARTIAL, plan=(S, cfg))
        except ValueError:
            # x tiles beyond the cfg's LDS budget: 320 rows fit cfg 2 only
            limit = {2: 320}.get(cfg, 256)
            assert M > limit, (M, cfg)
            return
        assert pend.part.shape == (S, M, N)
        assert rel_err(pend.part.sum(0), ref) < 1e-5, (S,)


@pytest.mark.parametrize("M", [65, 128, 192, 256, 257, 320])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 4096), (4096, 14336)])
def test_gemm_mw_llama_shapes(M, N, K):
    from xgserve.ops.linear import mw_linear
    x, w = rnd(M, K), rnd(N, K, scale=0.02)
    pend = mw_linear(x, w, MODE_PARTIAL)
    ref = x.float() @ w.float().t()
    assert rel_err(pend.part.sum(0), ref) < 1e-5
    assert rel_err(pend.materialize(), ref) < 1e-2


@pytest.mark.parametrize("M", [65, 128, 192, 257, 320])
@pytest.mark.parametrize("cfg", [0, 1, 2, 5, 6])
def test_gemm_mw_silu_and_bf16(M, cfg):
    from xgserve.ops.linear import MW_CFGS, mw_linear
    if M > {2: 320}.get(cfg, 256):
        pytest.skip("x tile beyond this configuration's LDS budget")
    F_, H = 2 * MW_CFGS[cfg][0], 1024
    x = rnd(M, H)
    g, u = rnd(F_, H, scale=0.05), rnd(F_, H, scale=0.05)
    w = interleave_gate_up(g, u).contiguous()
    got = mw_linear(x, w, MODE_SILU, plan=(1, cfg))
    ref = torch.nn.functional.silu(x.float() @ g.float().t()) * (x.float() @ u.float().t())
    assert got.shape == (M, F_)
    assert rel_err(got, ref) < 1e-2
    w2 = rnd(2 * MW_CFGS[cfg][0], H, scale=0.02)
    got2 = mw_linear(x, w2, MODE_BF16, plan=(1, cfg))
    assert rel_err(got2, x.float() @ w2.float().t()) < 1e-2


def test_gemm_mw_gate_up_8b():
    from xgserve.ops.linear import mw_linear
    M, F_, H = 191, 14336, 4096
    x = rnd(M, H)
    g, u = rnd(F_, H, scale=0.02), rnd(F_, H, scale=0.02)
    w = interleave_gate_up(g, u).contiguous()
    got = mw_linear(x, w, MODE_SILU)
    ref = torch.nn.functional.silu(x.float() @ g.float().t()) * (x.float() @ u.float().t())
    assert rel_err(got, ref) < 1e-2


def test_gemm_mw_rejects_bad_shapes():
    from xgserve.ops.linear import mw_linear
    with pytest.raises(ValueError):
        mw_linear(rnd(321, 256), rnd(256, 256), MODE_PARTIAL)   # M > 320
    with pytest.raises(ValueError):
        mw_linear(rnd(100, 200), rnd(256, 200), MODE_PARTIAL)   # K % 64
    with pytest.raises(ValueError):
        mw_linear(rnd(100, 256), rnd(256, 256), MODE_SILU, plan=(2, 1))  # SiLU needs split 1


@pytest.mark.parametrize("M", [1, 5, 16])
@pytest.mark.parametrize("cfg", [8, 9, 10])
@pytest.mark.parametrize("N,K,S", [(4096, 14336, 4), (6144, 4096, 8), (4096, 4096, 4), (512, 1280, 1),
                                   (1024, 768, 3)])
def test_gemm_m64g_deep_ring(M, cfg, N, K, S):
    """The 4- / 5- / 6-slot LDS rings of the one-x-tile kernel (M <= 16), every
    chunk count phase (incl. fewer chunks than slots), partial and SiLU epilogues."""
    from xgserve.ops.linear import M64G_CFGS, m64_linear
    wv, kc, _ = M64G_CFGS[cfg]
    nw = 2 if N % (32 * wv) == 0 else 1
    if N % (16 * nw * wv) or K % (S * kc):
        pytest.skip("shape not tileable")
    x, w = rnd(M, K), rnd(N, K, scale=0.02)
    pend = m64_linear(x, w, MODE_PARTIAL, split_k=S, nw=nw, cfg=cfg)
    assert rel_err(pend.part.sum(0), x.float() @ w.float().t()) < 1e-5
    if nw == 2:
        g, u = rnd(N // 2, K, scale=0.02), rnd(N // 2, K, scale=0.02)
        wi = interleave_gate_up(g, u).contiguous()
        got = m64_linear(x, wi, MODE_SILU, split_k=1, nw=2, cfg=cfg)
        ref = torch.nn.functional.silu(x.float() @ g.float().t()) * (x.float() @ u.float().t())
        assert rel_err(got, ref) < 1e-2


def test_gemm_m64g_deep_ring_rejects_m_above_16():
    from xgserve.ops._native import stream_ptr
    x, w = rnd(17, 4096), rnd(4096, 4096, scale=0.02)
    part = torch.empty(4, 17, 4096, device=DEV)
    with pytest.raises(ValueError):
        _native.kernels().gemm_m64g(x.data_ptr(), 17, 4096, w.data_ptr(), 4096, part.data_ptr(), 0, 4, MODE_PARTIAL,
                                    1, 8, stream_ptr())


@pytest.mark.parametrize("M", [1, 16, 40, 64])
@pytest.mark.parametrize("N,K,nw,S,cfg", [(6144, 4096, 2, 5, 3), (6144, 4096, 1, 3, 0), (4096, 14336, 2, 3, 1),
                                          (4096, 14336, 2, 7, 3), (1024, 768, 1, 5, 4)])
def test_gemm_m64g_uneven_splits(M, N, K, nw, S, cfg):
    """Split-K ranges of unequal chunk counts (K / KC not a multiple of S)."""
    from xgserve.ops.linear import m64_linear
    x, w = rnd(M, K), rnd(N, K, scale=0.02)
    pend = m64_linear(x, w, MODE_PARTIAL, split_k=S, nw=nw, cfg=cfg)
    assert pend.part.shape == (S, M, N)
    assert rel_err(pend.part.sum(0), x.float() @ w.float().t()) < 1e-5


@pytest.mark.parametrize("M", [1, 17, 64, 65, 128, 192, 256])
def test_lm_head_linear_matches_fp32(M):
    """The LM head (Llama-3 vocab 128,256 x 4,096): gemm_mw where a measured plan exists
    (M >= LM_HEAD_MW_MIN_M), hipBLASLt otherwise -- bf16 logits vs fp32."""
    from xgserve.ops.linear import lm_head_linear
    h, w = rnd(M, 4096), rnd(128256, 4096, scale=0.02)
    got = lm_head_linear(h, w)
    assert got.shape == (M, 128256) and got.dtype == torch.bfloat16
    assert rel_err(got, h.float() @ w.float().t()) < 1e-2
