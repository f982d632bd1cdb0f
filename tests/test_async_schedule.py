"""Asynchronous scheduling in the C++ step scheduler (StepScheduler.lookahead /
commit): step N+1 is planned while step N's tokens are still on the GPU. The
placeholder bookkeeping must give the same token streams, stop decisions and
page accounting as the synchronous update() loop."""
import numpy as np
import pytest

from xgserve import _runtime as R

PH = -1


def _sched(num_blocks=64, eos=(), max_seqs=8, early=False):
    c = R.SchedulerConfig()
    c.early_release = 1 if early else 0
    c.block_size = 4
    c.num_blocks = num_blocks
    c.max_num_seqs = max_seqs
    c.max_num_batched_tokens = 64
    c.max_model_len = 256
    c.enable_prefix_cache = True
    c.eos_ids = list(eos)
    return R.StepScheduler(c)


def _oracle(seq_id, step):  # the "model": a deterministic token per (sequence, position)
    return 1000 + 7 * seq_id + step


def _run(sync: bool, prompts, max_tokens, eos=(), abort_at=None, num_blocks=64, across=True, early=False):
    s = _sched(eos=eos, num_blocks=num_blocks, early=early)
    for i, (p, m) in enumerate(zip(prompts, max_tokens)):
        assert s.add(i + 1, p, m, 1, not eos, False, [], 0)
    out = {i + 1: [] for i in range(len(prompts))}
    finished = {}
    pos = {i + 1: len(p) for i, p in enumerate(prompts)}

    def tok_for(plan):
        ts = []
        for j in plan["sample_seq_index"]:
            sid = int(plan["seq_ids"][j])
            ts.append(_oracle(sid, pos[sid]))
        return np.array(ts, np.int32)

    def record(plan, toks, fins):
        for j, t in zip(plan["sample_seq_index"], toks):
            sid = int(plan["seq_ids"][j])
            if sid in finished:
                continue
            out[sid].append(int(t))
            pos[sid] += 1
        for f in fins:
            finished[f[0]] = f[1]

    plan = s.schedule()
    steps = 0
    while plan["num_tokens"] > 0 and steps < 500:
        steps += 1
        if abort_at is not None and steps == abort_at[0]:
            s.abort(abort_at[1])
            finished[abort_at[1]] = "abort"
        ahead = (not sync) and s.lookahead(across)
        toks = tok_for(plan)
        if ahead:
            nxt = s.schedule()
            # every placeholder input belongs to a row of the step in flight
            nd = nxt["num_decodes"]
            for i in range(nd):
                if nxt["input_ids"][i] == PH:
                    assert int(nxt["seq_ids"][i]) in set(int(x) for x in plan["seq_ids"])
            fins = s.commit(toks)
            record(plan, toks, fins)
            plan = nxt
        else:
            fins = s.update(toks, np.ones(len(toks), np.int32))
            record(plan, toks, fins)
            plan = s.schedule()
    assert s.num_inflight() == 0
    return out, finished, s


@pytest.mark.parametrize("early", [False, True])
@pytest.mark.parametrize("across", [True, False])
@pytest.mark.parametrize("eos", [(), (1000 + 7 * 2 + 9,)])
def test_lookahead_matches_sync(eos, across, early):
    prompts = [[1, 2, 3], [4, 5, 6, 7, 8], [9] * 11]
    mt = [5, 12, 3]
    a, fa, sa = _run(True, prompts, mt, eos)
    b, fb, sb = _run(False, prompts, mt, eos, across=across, early=early)
    assert a == b
    assert fa == fb
    assert sa.num_used_blocks() == sb.num_used_blocks()
    assert sb.num_running() == 0 and sb.num_waiting() == 0


def test_lookahead_with_abort():
    prompts = [[1, 2, 3], [4, 5, 6]]
    b, fb, sb = _run(False, prompts, [20, 20], abort_at=(6, 1))
    assert fb[1] == "abort" and len(b[2]) == 20
    assert sb.num_running() == 0 and sb.num_free_blocks() + sb.num_evictable_blocks() == 64 - 0


def test_lookahead_over_prefill_plans_and_update_guard():
    """A prompt step can be looked ahead too (its completing rows get placeholders,
    partial chunks advance); update() is refused while a lookahead is in flight and
    commit() resolves exactly one record."""
    s = _sched()
    assert s.add(1, [1, 2, 3], 4, 1, True, False, [], 0)
    s.schedule()  # prefill of the whole prompt: samples the first token
    assert s.lookahead()
    nxt = s.schedule()
    assert nxt["num_decodes"] == 1 and nxt["input_ids"][0] == PH  # substituted on the device
    with pytest.raises(Exception):
        s.update(np.array([6], np.int32), np.ones(1, np.int32))
    s.commit(np.array([6], np.int32))
    with pytest.raises(Exception):
        s.commit(np.array([7], np.int32))
    assert s.lookahead()
    s.commit(np.array([7], np.int32))


def test_lookahead_over_partial_prompt_chunk():
    """A chunked prompt (budget smaller than the prompt): the non-completing chunk
    advances at lookahead, the next plan carries the following chunk."""
    c = R.SchedulerConfig()
    c.block_size = 4
    c.num_blocks = 64
    c.max_num_seqs = 4
    c.max_num_batched_tokens = 8
    c.max_model_len = 256
    s = R.StepScheduler(c)
    assert s.add(1, list(range(1, 21)), 3, 1, True, False, [], 0)  # 20-token prompt, 8-token budget
    p0 = s.schedule()
    assert p0["num_tokens"] == 8 and p0["num_sample"] == 0
    assert not s.lookahead()  # nothing sampled: nothing to look ahead over
    s.update(np.zeros(0, np.int32), np.zeros(0, np.int32))
    p1 = s.schedule()
    assert int(p1["ctx_lens"][0]) == 8 and p1["num_sample"] == 0


def test_length_finish_released_at_lookahead_and_slot_reused():
    """A row that reaches max_tokens with the token in flight is released at
    lookahead(): the next plan admits the waiting request into its slot at once,
    and commit() still reports the finished sequence (reason length)."""
    s = _sched(max_seqs=1, early=True)
    assert s.add(1, [1, 2, 3], 2, 1, True, False, [], 0)
    assert s.add(2, [4, 5, 6, 7], 3, 1, True, False, [], 0)
    s.schedule()  # prompt 1 (only one slot)
    s.update(np.array([10], np.int32), np.ones(1, np.int32))  # token 1 of 2
    p = s.schedule()
    assert p["num_decodes"] == 1 and int(p["seq_ids"][0]) == 1
    assert s.lookahead()  # row 1 ends with this token: released now
    nxt = s.schedule()
    assert [int(x) for x in nxt["seq_ids"]] == [2] and nxt["num_decodes"] == 0  # admitted at once
    fins = s.commit(np.array([11], np.int32))
    assert [(f[0], f[1], f[3]) for f in fins] == [(1, 2, 2)]  # id 1, reason Length, 2 tokens generated
    assert s.num_running() == 1


def test_lookahead_under_preemption():
    """A pool too small for all sequences: the lookahead schedule() preempts
    sequences holding an unresolved placeholder; they are re-admitted only after
    commit() and still produce the synchronous token streams."""
    prompts = [[i + 1] * 8 for i in range(3)]
    a, fa, _ = _run(True, prompts, [20, 20, 20], num_blocks=12)
    b, fb, sb = _run(False, prompts, [20, 20, 20], num_blocks=12)
    assert a == b and fa == fb
    assert all(len(v) == 20 for v in b.values())
    assert sb.total_preemptions() > 0 if hasattr(sb, "total_preemptions") else True


def test_shrink_then_grow_keeps_slots_distinct():
    """set_limits(max//2) then set_limits(max) (degradation ladder, hot reload) must
    not duplicate slot ids: two running sequences sharing a slot would share the
    engine's per-slot sampling state."""
    s = _sched(num_blocks=256, max_seqs=8)
    for _ in range(3):
        s.set_limits(4, 64)
        s.set_limits(8, 64)
    for i in range(8):
        assert s.add(i + 1, [5 + i, 6, 7], 4, 1, True, False, [], 0)
    plan = s.schedule()
    assert plan["num_seqs"] == 8
    slots = [int(x) for x in plan["slots"]]
    assert sorted(slots) == list(range(8)), slots
    # growing beyond the original size creates exactly the new ids
    s.set_limits(4, 64)
    s.set_limits(10, 64)
    for i in range(2):
        assert s.add(100 + i, [9, 9, 9, 9], 4, 1, True, False, [], 0)
    s.update(np.ones(int(plan["num_sample"]), np.int32), np.ones(int(plan["num_sample"]), np.int32))
    plan2 = s.schedule()
    new = [int(x) for x, sid in zip(plan2["slots"], plan2["seq_ids"]) if int(sid) >= 100]
    assert sorted(new) == [8, 9]
    assert len(set(int(x) for x in plan2["slots"])) == plan2["num_seqs"]


def test_prefix_lookup_counted_once_per_admission():
    """A request whose admission fails for lack of pages is retried every step: its
    prefix-cache lookup must be counted once (when admitted), not per retry."""
    s = _sched(num_blocks=8, max_seqs=4)
    assert s.add(1, list(range(10, 26)), 8, 1, True, False, [], 0)   # 4 pages + decode page
    plan = s.schedule()
    assert s.add(2, list(range(40, 64)), 4, 1, True, False, [], 0)   # needs 6+ pages: must wait
    before = s.cache_stats()
    for _ in range(3):
        s.update(np.ones(int(plan["num_sample"]), np.int32), np.ones(int(plan["num_sample"]), np.int32))
        plan = s.schedule()
        if 2 in [int(x) for x in plan["seq_ids"]]:
            break
    mid = s.cache_stats()
    waiting_lookups = (mid["hit_count"] + mid["miss_count"]) - (before["hit_count"] + before["miss_count"])
    admitted = 2 in [int(x) for x in plan["seq_ids"]]
    assert waiting_lookups == (1 if admitted else 0)


def test_kv_usage_excludes_evictable_prefix_pages():
    """A warm prefix cache is not memory pressure: after every request finished, the
    cached pages stay allocated but kv_usage (the degradation ladder's input) is 0."""
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
    eng = LLMEngine(EngineConfig(model="llama-tiny", device="cpu", dtype="float32", num_blocks=64, max_num_seqs=4,
                                 max_num_batched_tokens=256, use_graphs=False))
    eng.generate([[1] + list(range(10, 80)), [1] + list(range(100, 170))],
                 SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
    st = eng.stats()
    assert st["kv_blocks_used"] > 0 and st["running"] == 0
    assert st["kv_usage"] == 0.0


def _coalesce_sched(k, wait):
    c = R.SchedulerConfig()
    c.block_size = 16
    c.num_blocks = 1024
    c.max_num_seqs = 64
    c.max_num_batched_tokens = 8192
    c.max_model_len = 2048
    c.enable_prefix_cache = False
    c.coalesce_prompts = k
    c.coalesce_max_wait = wait
    return R.StepScheduler(c)


def _step(s, plan):
    n = int(plan["num_sample"])
    s.update(np.full(n, 5, np.int32), np.ones(n, np.int32))
    return s.schedule()


def test_admission_window_coalesces_prompts():
    """coalesce_prompts = 2: with decode rows running, a lone new prompt waits until a
    second arrives, then both prefill in ONE mixed step; without decode rows running
    (idle GPU) a prompt is admitted at once."""
    s = _coalesce_sched(2, 100)
    assert s.add(1, list(range(10, 30)), 50, 1, True, False, [], 0)
    plan = s.schedule()
    assert [int(x) for x in plan["seq_ids"]] == [1]          # nothing decoding: no hold
    plan = _step(s, plan)
    assert s.add(2, list(range(40, 60)), 50, 1, True, False, [], 0)
    for _ in range(3):                                      # decode-only while 2 waits alone
        plan = _step(s, plan)
        assert int(plan["num_tokens"]) == 1 and s.num_waiting() == 1
    assert s.add(3, list(range(70, 90)), 50, 1, True, False, [], 0)
    plan = _step(s, plan)
    ids = [int(x) for x in plan["seq_ids"]]
    assert ids == [1, 2, 3] and int(plan["num_tokens"]) == 1 + 20 + 20 and s.num_waiting() == 0


def test_admission_window_wait_bound():
    """A lone prompt is admitted after coalesce_max_wait plans passed it over."""
    s = _coalesce_sched(4, 3)
    assert s.add(1, list(range(10, 30)), 50, 1, True, False, [], 0)
    plan = _step(s, s.schedule())
    assert s.add(2, list(range(40, 60)), 50, 1, True, False, [], 0)
    waited = 0
    while 2 not in [int(x) for x in plan["seq_ids"]]:
        plan = _step(s, plan)
        waited += 1
        assert waited <= 4
    assert waited == 4  # passed over by 3 plans, admitted by the 4th


def test_admission_window_off_admits_at_once():
    s = _coalesce_sched(1, 4)
    assert s.add(1, list(range(10, 30)), 50, 1, True, False, [], 0)
    plan = _step(s, s.schedule())
    assert s.add(2, list(range(40, 60)), 50, 1, True, False, [], 0)
    plan = _step(s, plan)
    assert 2 in [int(x) for x in plan["seq_ids"]]

def test_overlap_outputs_go_to_the_sink_immediately(monkeypatch):
    """A serving replica sets LLMEngine.output_sink: outputs detokenised in a step's
    overlap window are handed over before the GPU wait instead of being returned
    with step() (Req 5.1 delivery); without a sink (bench.py) they stay in step()'s
    return value, and XGS_EARLY_OUTPUTS=0 restores that for a replica too."""
    from types import SimpleNamespace

    from xgserve.engine import engine as E
    from xgserve.engine.request import RequestOutput

    outs = [RequestOutput("a", [1], "x", False), RequestOutput("b", [2], "y", False)]
    got = []
    eng = SimpleNamespace(output_sink=got.extend)
    monkeypatch.setattr(E, "EARLY_OUTPUTS", True)
    assert E.LLMEngine._emit_early(eng, list(outs)) == [] and got == outs
    assert E.LLMEngine._emit_early(eng, []) == []
    eng.output_sink = None
    assert E.LLMEngine._emit_early(eng, list(outs)) == outs
    monkeypatch.setattr(E, "EARLY_OUTPUTS", False)
    eng.output_sink = got.append
    assert E.LLMEngine._emit_early(eng, list(outs)) == outs and len(got) == 2


def test_stall_free_one_chunk_per_decode_step():
    """decode_prefill_cap = 128, decode_prefill_seqs = 1 (stall-free batching): while
    rows decode, every step carries at most ONE prompt chunk of <= 128 tokens, so a
    200-token prompt and a 60-token prompt take 2 + 1 steps -- never two prompts in
    one step (the runner's mixed-step graphs take exactly that shape)."""
    c = R.SchedulerConfig()
    c.block_size, c.num_blocks, c.max_num_seqs = 16, 1024, 64
    c.max_num_batched_tokens, c.max_model_len, c.enable_prefix_cache = 8192, 2048, False
    c.decode_prefill_cap, c.decode_prefill_seqs = 128, 1
    s = R.StepScheduler(c)
    assert s.add(1, list(range(10, 30)), 50, 1, True, False, [], 0)
    plan = s.schedule()
    assert int(plan["num_tokens"]) == 20          # nothing decoding: the whole prompt at once
    plan = _step(s, plan)
    assert s.add(2, list(range(100, 300)), 50, 1, True, False, [], 0)
    assert s.add(3, list(range(400, 460)), 50, 1, True, False, [], 0)
    shapes = []
    for _ in range(4):
        plan = _step(s, plan)
        nd, ns = int(plan["num_decodes"]), int(plan["num_seqs"])
        shapes.append((nd, ns - nd, int(plan["num_tokens"]) - nd))
    assert shapes == [(1, 1, 128), (1, 1, 72), (2, 1, 60), (3, 0, 0)], shapes


def test_decode_prefill_cap_can_be_lifted():
    """set_decode_prefill(0, 0) lifts the stall-free limits at run time (bench.py's
    untimed population fill); restoring them chunks the next prompt again."""
    c = R.SchedulerConfig()
    c.block_size, c.num_blocks, c.max_num_seqs = 16, 1024, 64
    c.max_num_batched_tokens, c.max_model_len, c.enable_prefix_cache = 8192, 2048, False
    c.decode_prefill_cap, c.decode_prefill_seqs = 128, 1
    s = R.StepScheduler(c)
    assert s.add(1, list(range(10, 30)), 50, 1, True, False, [], 0)
    plan = _step(s, s.schedule())
    s.set_decode_prefill(0, 0)
    assert s.add(2, list(range(100, 300)), 50, 1, True, False, [], 0)
    assert s.add(3, list(range(400, 460)), 50, 1, True, False, [], 0)
    plan = _step(s, plan)
    assert (int(plan["num_decodes"]), int(plan["num_tokens"])) == (1, 1 + 200 + 60)
    s.set_decode_prefill(128, 1)
    assert s.add(4, list(range(500, 800)), 50, 1, True, False, [], 0)
    plan = _step(s, plan)
    plan = _step(s, plan)
    assert int(plan["num_tokens"]) - int(plan["num_decodes"]) <= 128


@pytest.mark.parametrize("seqs,expect_steps", [(None, 1), (1, 3)])
def test_decode_prefill_burst_without_mixed_graphs(seqs, expect_steps):
    """with decode_prefill_cap set but no mixed-step graphs captured (here:
    CPU, no graphs), a burst of short prompts arriving while a request decodes is
    admitted in ONE step (the one-prompt limit exists only for the graphs' shape);
    decode_prefill_seqs=1 restores one prompt per step."""
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
    eng = LLMEngine(EngineConfig(model="llama-tiny", device="cpu", dtype="float32", num_blocks=64, max_num_seqs=8,
                                 max_num_batched_tokens=256, max_model_len=128, use_graphs=False,
                                 decode_prefill_cap=64, decode_prefill_seqs=seqs))
    sp = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
    eng.add_request("long", list(range(5, 21)), sp)
    for _ in range(3):
        eng.step()
    first_step = {}
    for i in range(3):
        eng.add_request(f"b{i}", list(range(30 + i, 38 + i)), SamplingParams(max_tokens=2, ignore_eos=True))
    for k in range(8):
        for o in eng.step():
            if o.new_token_ids and o.request_id.startswith("b") and o.request_id not in first_step:
                first_step[o.request_id] = k
    assert sorted(first_step) == ["b0", "b1", "b2"]
    assert len(set(first_step.values())) == expect_steps, first_step
