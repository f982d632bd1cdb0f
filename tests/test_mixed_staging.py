"""Host staging of the mixed-step graphs (engine/runner.py stage_mixed_inputs) on a
real StepScheduler plan: decode rows + ONE prompt chunk laid out in the static
graph buffers exactly as the captured graph reads them (CPU; the graphs themselves
are covered by tests/test_engine_gpu.py::test_stall_free_*)."""
import numpy as np

from xgserve import _runtime as R
from xgserve.engine.runner import stage_mixed_inputs


def _plan():
    c = R.SchedulerConfig()
    c.block_size, c.num_blocks, c.max_num_seqs = 16, 256, 16
    c.max_num_batched_tokens, c.max_model_len, c.enable_prefix_cache = 4096, 1024, False
    c.decode_prefill_cap, c.decode_prefill_seqs = 48, 1
    s = R.StepScheduler(c)
    for i in range(3):
        assert s.add(i + 1, list(range(10 + i, 30 + i)), 20, 1, True, False, [], 0)
    p = s.schedule()
    s.update(np.full(3, 7, np.int32), np.ones(3, np.int32))
    assert s.add(9, list(range(100, 200)), 5, 1, True, False, [], 0)
    p = s.schedule()
    s.update(np.full(int(p["num_sample"]), 7, np.int32), np.ones(int(p["num_sample"]), np.int32))
    return s.schedule()  # second chunk: 3 decode rows + prompt tokens [48, 96) of seq 9


def test_stage_mixed_inputs_layout():
    plan = _plan()
    Nd, T = int(plan["num_decodes"]), int(plan["num_tokens"])
    q = T - Nd
    assert Nd == 3 and int(plan["num_seqs"]) == 4 and q == 48
    B, C, W, nb = 8, 64, 70, 4
    R_ = B + C
    sec = (0, R_, 2 * R_, 3 * R_, 3 * R_ + B + 1, 3 * R_ + 2 * B + 1, 3 * R_ + 2 * B + 3)
    hi = np.full(sec[-1] + (B + 1) * W, 12345, np.int32)
    hl = np.full(B + 1, 999, np.int64)
    src = np.array([0, -1, 2], np.int32)
    stage_mixed_inputs(plan, Nd, nb, B, C, W, src, sec, hi, hl)
    ids, pos, slot = hi[sec[0]:sec[1]], hi[sec[1]:sec[2]], hi[sec[2]:sec[3]]
    # decode rows, decode padding up to nb, chunk at B, chunk padding to B + C
    for buf, key, pad in ((ids, "input_ids", 0), (pos, "positions", 0), (slot, "slot_mapping", -1)):
        np.testing.assert_array_equal(buf[:Nd], plan[key][:Nd])
        assert (buf[Nd:nb] == pad).all()
        np.testing.assert_array_equal(buf[B:B + q], plan[key][Nd:T])
        assert (buf[B + q:B + C] == pad).all()
    assert pos[B] == 48 and pos[B + q - 1] == 95  # the second 48-token chunk
    sl = hi[sec[3]:sec[4]]
    np.testing.assert_array_equal(sl[:Nd], plan["seq_lens"][:Nd])
    assert (sl[Nd:nb] == 0).all() and sl[B] == 96
    np.testing.assert_array_equal(hi[sec[4]:sec[4] + 3], src)
    assert (hi[sec[4] + 3:sec[4] + nb] == -1).all()
    assert list(hi[sec[5]:sec[5] + 2]) == [0, q]
    w = int(plan["bt_width"])
    bt = hi[sec[6]:].reshape(B + 1, W)
    pbt = plan["block_tables"].reshape(Nd + 1, w)
    np.testing.assert_array_equal(bt[:Nd, :w], pbt[:Nd])
    np.testing.assert_array_equal(bt[B, :w], pbt[Nd])
    # logits rows in sample order: decode rows, then the chunk's last row, then padding
    assert list(hl[:Nd]) == [0, 1, 2] and hl[Nd] == nb + q - 1 and (hl[Nd + 1:nb + 1] == 0).all()
