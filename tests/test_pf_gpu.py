"""gemm_pf (csrc/kernels/gemm_pf.hip, the prompt-sized MFMA GEMM) vs fp32 PyTorch.

Every epilogue (bf16, fp32 split-K partials, fused SiLU-gate) at the mixed-step
and prefill row counts, each tile height, even and uneven K splits."""
import pytest
import torch

from xgserve.ops import _native
from xgserve.ops import linear as L

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


def ref(x, w, mode):
    if mode == L.MODE_SILU:
        g, u = L.deinterleave_gate_up(w)
        return torch.nn.functional.silu(x.float() @ g.float().t()) * (x.float() @ u.float().t())
    return x.float() @ w.float().t()


def run(x, w, mode, plan):
    r = L.pf_linear(x, w, mode, plan=plan)
    return r.part.sum(0) if mode == L.MODE_PARTIAL else r


MS = [65, 257, 512, 575, 1024, 2048]


@pytest.mark.parametrize("M", MS)
@pytest.mark.parametrize("mode", [L.MODE_BF16, L.MODE_PARTIAL, L.MODE_SILU])
def test_pf_default_plan(M, mode):
    """The plan the model uses, at the 8B gate_up (SiLU) / QKV shapes."""
    N, K = (28672, 4096) if mode == L.MODE_SILU else (6144, 4096)
    x, w = rnd(M, K), rnd(N, K, scale=0.02)
    got = run(x, w, mode, None)
    assert rel_err(got, ref(x, w, mode)) < 1e-2


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("M", [1, 100, 575, 600])
def test_pf_cfgs_bf16(cfg, M):
    x, w = rnd(M, 1024), rnd(1024, 1024, scale=0.05)
    got = run(x, w, L.MODE_BF16, (1, cfg))
    assert rel_err(got, ref(x, w, L.MODE_BF16)) < 1e-2


@pytest.mark.parametrize("S", [2, 3, 5, 7])
@pytest.mark.parametrize("M", [65, 575, 1024])
def test_pf_splitk_uneven(S, M):
    """Uneven K ranges per split (K / 64 not a multiple of S), down-projection K."""
    x, w = rnd(M, 14336), rnd(4096, 14336, scale=0.02)
    got = run(x, w, L.MODE_PARTIAL, (S, L.pf_plan(M, 4096, 14336, L.MODE_PARTIAL)[1]))
    assert rel_err(got, ref(x, w, L.MODE_PARTIAL)) < 1e-2


def test_pf_rows_past_m_untouched():
    """Rows >= M of the last tile are computed from clamped rows and never stored."""
    M, N, K = 70, 512, 512
    x, w = rnd(M, K), rnd(N, K, scale=0.05)
    out = torch.full((M + 8, N), 7.0, device=DEV, dtype=torch.bfloat16)
    L.pf_linear(x, w, L.MODE_BF16, plan=(1, 0), out=out[:M])
    assert bool((out[M:] == 7.0).all())
    assert rel_err(out[:M], ref(x, w, L.MODE_BF16)) < 1e-2
