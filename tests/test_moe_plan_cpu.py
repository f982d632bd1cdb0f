"""Host-side planning of the prompt-sized expert GEMMs (xgserve/ops/moe.py): the
gemm_pf tile that covers an expert's 64-padded segment, the shapes the grouped form
takes, and the grid bound of gemm_pf_grouped (csrc/kernels/gemm_pf.hip), which must
cover every (expert, row tile) whatever the routing."""
import itertools
import random

from xgserve.ops import moe as MOE
from xgserve.ops.linear import PF_CFG_BM


def test_tile_covers_the_average_segment():
    # Mixtral mixed step: 575 tokens x top-2 over 8 experts -> ~144 rows -> 192-row tile
    assert MOE._moe_pf_cfg(1150, 8) == 8 and PF_CFG_BM[8] == 192
    assert MOE._moe_pf_cfg(2048, 8) == 7 and PF_CFG_BM[7] == 256  # 256 rows per expert
    assert MOE._moe_pf_cfg(16000, 8) == 6 and PF_CFG_BM[6] == 288  # long prompts: the widest tile
    # an EP shard sizes by its expected share of the pairs (4 of 8 experts)
    share = 1150 * 4 // 8
    assert MOE._moe_pf_cfg(share, 4) == 8


def test_grouped_shapes():
    assert MOE._moe_pf_ok(4096, 14336)      # Mixtral 8x7B
    assert MOE._moe_pf_ok(4096, 7168)       # its TP2 expert shards
    assert not MOE._moe_pf_ok(4000, 14336)  # H must be a multiple of the 256-column tile
    assert not MOE._moe_pf_ok(4096, 100)


def test_grid_bound_covers_any_routing():
    """sum over experts of ceil(64-padded segment / BM) <= (pairs + 63 E) // BM + E
    (the slot count gemm_pf_grouped launches per column tile)."""
    rnd = random.Random(0)
    for E, pairs, bm in itertools.product((1, 2, 4, 8), (257, 575, 1150, 4096), (192, 256, 288)):
        bound = (pairs + 63 * E) // bm + E
        for _ in range(50):
            cuts = sorted(rnd.randint(0, pairs) for _ in range(E - 1))
            counts = [b - a for a, b in zip([0] + cuts, cuts + [pairs])]
            segs = [-(-c // 64) * 64 for c in counts]
            need = sum(-(-s // bm) for s in segs)
            assert need <= bound, (E, pairs, bm, counts)
