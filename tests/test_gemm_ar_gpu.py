"""gemm_m64g GG_AR (csrc/kernels/gemm_m64g.hip): the TP decode all-reduce inside the
row-parallel O / down GEMM launch, in its one-process loopback form (the form the
`--tp-shard` simulation runs): pushes and polls of a `world`-rank group through this
process's own region, numerics of one rank. Against fp32 PyTorch: resid += x . w^T
(bf16 contribution, one rounding of the sum), per-tile / per-tile-pair statistics,
tickets and generations advancing over repeated launches. The multi-rank form is
checked against RCCL by CustomAllReduce.self_test (tests/test_custom_ar_gpu.py) and
end to end by the TP engine tests (tests/test_tp_gpu.py)."""
import pytest
import torch

from xgserve.ops import _native
from xgserve.ops.linear import ResidWorkspace, m64_ar_resid_linear
from xgserve.parallel import comm

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _k():
    _native.kernels()
    torch.manual_seed(0)


def rnd(*s, scale=1.0):
    return (torch.randn(*s, device=DEV) * scale).bfloat16()


# (N, K): 70B TP8 O / down shards (128 column tiles: one statistic per tile at M <= 16,
# pair statistics above), 8B TP2 O / down
SHAPES = [(8192, 1024), (8192, 3584), (4096, 2048), (4096, 7168)]


@pytest.mark.parametrize("M", [1, 7, 16, 64])
@pytest.mark.parametrize("N,K", SHAPES)
@pytest.mark.parametrize("world", [2, 8])
def test_gemm_ar_loopback_matches_fp32(M, N, K, world):
    ar = comm._loopback_args(world, torch.device(DEV))
    ws = ResidWorkspace(2, 64, N, DEV)
    x, w = rnd(M, K), rnd(N, K, scale=0.03)
    base = rnd(M, N)
    want = base.float() + (x.float() @ w.float().t()).bfloat16().float()
    for rep in range(3):
        r = base.clone()
        st = m64_ar_resid_linear(x, w, r, ws, 1, ar)
        torch.cuda.synchronize()
        err = float((r.float() - want).norm() / want.norm())
        assert err < 1e-2, (rep, err)
        n = st.n
        assert n <= ws.max_tiles(M)
        ss_ref = (r.float().view(M, n, N // n) ** 2).sum(-1).t().reshape(-1)
        torch.testing.assert_close(st.ss[: n * M], ss_ref, rtol=1e-4, atol=1e-2)
    assert int(ar.err[0]) == 0
    assert int(ws.counters.abs().sum()) == 0 and int(ws.ar_pair.abs().sum()) == 0
