"""gemm_pf (csrc/kernels/gemm_pf.hip, the prompt-sized MFMA GEMM) vs fp32 PyTorch.

Every epilogue (bf16, fp32 split-K partials, fused SiLU-gate) at the mixed-step
and prefill row counts, each tile height, data-parallel and stream-K grids; the
stream-K tickets must be re-armed after every launch."""
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
    got = run(x, w, L.MODE_BF16, (1, cfg, 0))
    assert rel_err(got, ref(x, w, L.MODE_BF16)) < 1e-2


@pytest.mark.parametrize("S", [2, 3, 5, 7])
@pytest.mark.parametrize("M", [65, 575, 1024])
def test_pf_splitk_uneven(S, M):
    """Uneven K ranges per split (K / 64 not a multiple of S), down-projection K."""
    x, w = rnd(M, 14336), rnd(4096, 14336, scale=0.02)
    got = run(x, w, L.MODE_PARTIAL, (S, L.pf_plan(M, 4096, 14336, L.MODE_PARTIAL)[1], 0))
    assert rel_err(got, ref(x, w, L.MODE_PARTIAL)) < 1e-2


@pytest.mark.parametrize("cfg", [1, 3, 4, 7])
@pytest.mark.parametrize("M", [257, 575, 1024])
@pytest.mark.parametrize("grid", [7, 100, 256])
def test_pf_streamk(cfg, M, grid):
    """Stream-K: tiles shared by 1..many workgroups (grid 7 puts whole tiles plus a
    fraction in each range, grid 256 splits most tiles), SiLU epilogue after the
    last arriver's combine; twice, so the self re-arming tickets are exercised."""
    x, w = rnd(M, 4096), rnd(28672 if grid != 7 else 2048, 4096, scale=0.02)
    r = ref(x, w, L.MODE_SILU)
    for _ in range(2):
        got = run(x, w, L.MODE_SILU, (1, cfg, grid))
        assert rel_err(got, r) < 1e-2
    ws, tickets = L._PF_SK.get(x.device, grid, cfg, 1)
    torch.cuda.synchronize()
    assert int(tickets.abs().sum()) == 0


def test_pf_streamk_bf16_small_k():
    """nk = 1 and 2 K tiles per tile: ranges shorter than a tile."""
    for K in (64, 128):
        x, w = rnd(300, K), rnd(512, K, scale=0.1)
        got = run(x, w, L.MODE_BF16, (1, 1, 64))
        assert rel_err(got, ref(x, w, L.MODE_BF16)) < 1e-2


def test_pf_rows_past_m_untouched():
    """Rows >= M of the last tile are computed from clamped rows and never stored."""
    M, N, K = 70, 512, 512
    x, w = rnd(M, K), rnd(N, K, scale=0.05)
    out = torch.full((M + 8, N), 7.0, device=DEV, dtype=torch.bfloat16)
    L.pf_linear(x, w, L.MODE_BF16, plan=(1, 0, 0), out=out[:M])
    assert bool((out[M:] == 7.0).all())
    assert rel_err(out[:M], ref(x, w, L.MODE_BF16)) < 1e-2
