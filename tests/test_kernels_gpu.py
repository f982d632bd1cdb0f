"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op.

All tests here run on a real MI355X (pytest -m gpu). Shapes sweep the model
configs (Llama-3 8B/70B-TP8 GQA, Mixtral, GPT-2 D=64), ragged lengths, page
boundaries and split-K factors.
"""
import math

import pytest
import torch

from xgserve import ops
from xgserve.ops import _native

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _native_loaded():
    # Fail loudly: the GPU path must run the native library.
    _native.kernels()
    torch.manual_seed(0)


def rnd(*shape, scale=1.0, dtype=torch.bfloat16):
    return (torch.randn(*shape, device=DEV) * scale).to(dtype)


@pytest.mark.parametrize("T,H", [(1, 4096), (7, 4096), (64, 8192), (3, 768), (5, 1024)])
def test_rmsnorm(T, H):
    x, w = rnd(T, H), rnd(H)
    y = ops.rmsnorm(x, w, 1e-5)
    ref = ops.rmsnorm_ref(x.cpu(), w.cpu(), 1e-5)
    torch.testing.assert_close(y.cpu().float(), ref.float(), atol=2e-2, rtol=2e-2)


def test_rmsnorm_strided_rows():
    big = rnd(9, 6144)
    x = big[:, :4096]
    w = rnd(4096)
    y = ops.rmsnorm(x, w, 1e-5)
    torch.testing.assert_close(y.cpu().float(), ops.rmsnorm_ref(x.cpu(), w.cpu(), 1e-5).float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("T,H", [(1, 4096), (33, 4096), (16, 8192)])
def test_fused_add_rmsnorm(T, H):
    x, r, w = rnd(T, H), rnd(T, H), rnd(H)
    r0 = r.clone()
    y, r2 = ops.fused_add_rmsnorm(x, r, w, 1e-5)
    yr, rr = ops.fused_add_rmsnorm_ref(x.cpu(), r0.cpu(), w.cpu(), 1e-5)
    torch.testing.assert_close(r2.cpu().float(), rr.float(), atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(y.cpu().float(), yr.float(), atol=3e-2, rtol=3e-2)


def test_layernorm():
    x, w, b = rnd(5, 768), rnd(768), rnd(768)
    y = ops.layernorm(x, w, b, 1e-5)
    torch.testing.assert_close(y.cpu().float(), ops.layernorm_ref(x.cpu(), w.cpu(), b.cpu(), 1e-5).float(),
                               atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("T,F", [(1, 14336), (17, 14336), (64, 3584)])
def test_silu_and_mul(T, F):
    x = rnd(T, 2 * F)
    torch.testing.assert_close(ops.silu_and_mul(x).cpu().float(), ops.silu_and_mul_ref(x.cpu()).float(),
                               atol=2e-2, rtol=2e-2)


def test_gelu_tanh():
    x = rnd(4, 3072)
    torch.testing.assert_close(ops.gelu_tanh(x).cpu().float(), ops.gelu_tanh_ref(x.cpu()).float(), atol=2e-2,
                               rtol=2e-2)


@pytest.mark.parametrize("Hq,Hkv,D,rope", [(32, 8, 128, True), (8, 1, 128, True), (12, 12, 64, False)])
def test_rope_cache(Hq, Hkv, D, rope):
    T, bs, NB = 37, 16, 32
    qkv = rnd(T, (Hq + 2 * Hkv) * D)
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    cs = ops.build_cos_sin(D, 4096, 500000.0, device=DEV)
    slots = torch.randperm(NB * bs, device=DEV)[:T].to(torch.int32)
    slots[3] = -1
    kc = torch.zeros(NB, Hkv, bs, D, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    qkv_r, kc_r, vc_r = qkv.cpu().clone(), kc.cpu().clone(), vc.cpu().clone()
    ops.rope_cache(qkv, pos, cs, kc, vc, slots, Hq, Hkv, D, rope)
    ops.rope_cache_ref(qkv_r, pos.cpu(), cs.cpu(), kc_r, vc_r, slots.cpu(), Hq, Hkv, D, rope)
    torch.testing.assert_close(qkv.cpu().float(), qkv_r.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(kc.cpu().float(), kc_r.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(vc.cpu().float(), vc_r.float(), atol=0, rtol=0)


def _paged(lens, Hkv, D, bs, extra_pages=8):
    pages_per = [(L + bs - 1) // bs for L in lens]
    NB = sum(pages_per) + extra_pages
    kc = rnd(NB, Hkv, bs, D)
    vc = rnd(NB, Hkv, bs, D)
    perm = torch.randperm(NB).tolist()
    W = max(pages_per)
    bt = torch.zeros(len(lens), W, dtype=torch.int32)
    i = 0
    for s, n in enumerate(pages_per):
        bt[s, :n] = torch.tensor(perm[i:i + n])
        i += n
    return kc, vc, bt.to(DEV)


@pytest.mark.parametrize("Hq,Hkv,D", [(32, 8, 128), (8, 1, 128), (16, 4, 128), (12, 12, 64), (64, 8, 128)])
@pytest.mark.parametrize("splits", [1, 3, 8])
def test_decode_attention(Hq, Hkv, D, splits):
    bs = 16
    lens = [1, 17, 300, 1024, 5, 129]
    kc, vc, bt = _paged(lens, Hkv, D, bs)
    B = len(lens)
    # q as a strided view into a wider "qkv" row, like the engine passes it
    qkv = rnd(B, (Hq + 2 * Hkv) * D)
    q = qkv[:, :Hq * D].view(B, Hq, D)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    scale = 1.0 / math.sqrt(D)
    out = ops.decode_attention(q, kc, vc, bt, sl, scale, num_splits=splits)
    ref = ops.decode_attention_ref(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), sl.cpu(), scale)
    torch.testing.assert_close(out.cpu().float(), ref.float(), atol=2e-2, rtol=2e-2)


def test_decode_attention_zero_len_rows():
    Hq, Hkv, D, bs = 32, 8, 128, 16
    lens = [0, 40, 0]
    kc, vc, bt = _paged([max(1, x) for x in lens], Hkv, D, bs)
    q = rnd(3, Hq, D)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    out = ops.decode_attention(q, kc, vc, bt, sl, 0.088, num_splits=2)
    assert torch.isfinite(out.float()).all()
    assert out[0].float().abs().max().item() == 0.0


@pytest.mark.parametrize("Hq,Hkv,D,gh", [(32, 8, 128, 0), (32, 8, 128, 1), (32, 8, 128, 4), (8, 1, 128, 2),
                                         (8, 1, 128, 4), (12, 12, 64, 0), (16, 4, 64, 2)])
@pytest.mark.parametrize("qlens,ctxs", [([100], [0]), ([64, 1, 130, 7], [0, 5, 40, 300]), ([5, 5], [1000, 17])])
def test_prefill_attention(Hq, Hkv, D, gh, qlens, ctxs):
    """gh = query heads of one GQA group per workgroup (0: the kernel's default)."""
    bs = 16
    lens = [q + c for q, c in zip(qlens, ctxs)]
    kc, vc, bt = _paged(lens, Hkv, D, bs)
    T = sum(qlens)
    qkv = rnd(T, (Hq + 2 * Hkv) * D)
    q = qkv[:, :Hq * D].view(T, Hq, D)
    qsl = torch.tensor([0] + list(torch.cumsum(torch.tensor(qlens), 0)), dtype=torch.int32, device=DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    scale = 1.0 / math.sqrt(D)
    out = ops.prefill_attention(q, kc, vc, bt, qsl, sl, max(qlens), scale, gh=gh)
    ref = ops.prefill_attention_ref(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), qsl.cpu(), sl.cpu(), scale)
    torch.testing.assert_close(out.cpu().float(), ref.float(), atol=2e-2, rtol=2e-2)


# gh < 0: prefill_attn2_kernel forced to -gh = 10 * waves + heads per workgroup (D = 128)
@pytest.mark.parametrize("Hq,Hkv,gh", [(32, 8, -44), (32, 8, -84), (32, 8, -82), (32, 8, -81), (32, 8, -42),
                                       (32, 8, -41), (32, 8, -244), (32, 8, -1284), (32, 8, -1282), (32, 8, -1281), (8, 1, -1284), (8, 1, -88), (8, 1, -84), (64, 8, 0)])
@pytest.mark.parametrize("qlens,ctxs,bs", [([100], [0], 16), ([64, 1, 130, 7], [0, 5, 40, 300], 16),
                                           ([5, 5], [1000, 17], 16), ([700, 33], [300, 0], 32),
                                           ([513], [0], 64)])
def test_prefill_attention_mfma32(Hq, Hkv, gh, qlens, ctxs, bs):
    D = 128
    lens = [q + c for q, c in zip(qlens, ctxs)]
    kc, vc, bt = _paged(lens, Hkv, D, bs)
    T = sum(qlens)
    qkv = rnd(T, (Hq + 2 * Hkv) * D)
    q = qkv[:, :Hq * D].view(T, Hq, D)
    qsl = torch.tensor([0] + list(torch.cumsum(torch.tensor(qlens), 0)), dtype=torch.int32, device=DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    scale = 1.0 / math.sqrt(D)
    out = ops.prefill_attention(q, kc, vc, bt, qsl, sl, max(qlens), scale, gh=gh)
    ref = ops.prefill_attention_ref(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), qsl.cpu(), sl.cpu(), scale)
    torch.testing.assert_close(out.cpu().float(), ref.float(), atol=2e-2, rtol=2e-2)


def test_prefill_attention_nan_past_end():
    """Cache rows past a sequence's end hold NaN: the clamped DMA rows must never reach the output."""
    Hq, Hkv, D, bs = 32, 8, 128, 16
    lens = [37]
    kc, vc, bt = _paged(lens, Hkv, D, bs, extra_pages=0)
    pg = int(bt[0, 2])  # last page: rows 5.. lie past the end (37 = 2 * 16 + 5)
    kc[pg, :, 5:] = float("nan")
    vc[pg, :, 5:] = float("nan")
    q = rnd(37, Hq, D)
    qsl = torch.tensor([0, 37], dtype=torch.int32, device=DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    for gh in (0, -44, -84, -1284):
        out = ops.prefill_attention(q, kc, vc, bt, qsl, sl, 37, 0.088, gh=gh)
        ref = ops.prefill_attention_ref(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), qsl.cpu(), sl.cpu(), 0.088)
        torch.testing.assert_close(out.cpu().float(), ref.float(), atol=2e-2, rtol=2e-2)


def test_prefill_attention_spike_forces_rescale():
    # one large key early then a larger one late: the online max must rescale
    Hq, Hkv, D, bs = 8, 8, 128, 16
    lens = [256]
    kc, vc, bt = _paged(lens, Hkv, D, bs)
    q = rnd(256, Hq, D)
    p0 = int(bt[0, 0])
    p9 = int(bt[0, 9])
    kc[p0, :, 3] = q[200] * 4
    kc[p9, :, 5] = q[200] * 8
    qsl = torch.tensor([0, 256], dtype=torch.int32, device=DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    out = ops.prefill_attention(q, kc, vc, bt, qsl, sl, 256, 0.088)
    ref = ops.prefill_attention_ref(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), qsl.cpu(), sl.cpu(), 0.088)
    torch.testing.assert_close(out.cpu().float(), ref.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("V", [128256, 50257, 32000, 1000, 16387])
def test_argmax_logprob(dtype, V):
    """V >= 16K: the split-row kernel (8 slices, last arriver merges); three launches in
    a row (the per-row tickets must re-arm); ties go to the lowest index."""
    from xgserve.ops import sampling as SP
    for it in range(3):
        logits = rnd(9, V, scale=3.0, dtype=dtype)
        if it == 2:  # a tie across two slices: the lower index wins
            logits[3, V // 3] = logits[3, V - 2] = logits[3].max() + 1
        tok, lp = ops.argmax_logprob(logits)
        rt, rl = ops.argmax_logprob_ref(logits.cpu())
        assert torch.equal(tok.cpu(), rt)
        torch.testing.assert_close(lp.cpu(), rl, atol=1e-3, rtol=1e-3)
    if V >= SP.ARGMAX_SPLIT_MIN_V:
        torch.cuda.synchronize()
        assert int(SP._argmax_ws(logits.device, 9)[1].abs().sum()) == 0


def test_sample_tokens_greedy_and_distribution():
    V = 1000
    logits = rnd(4, V, scale=2.0, dtype=torch.float32)
    temps = torch.tensor([0.0, 1.0, 0.7, 1.0], device=DEV)
    top_ps = torch.tensor([1.0, 1.0, 0.9, 0.5], device=DEV)
    top_ks = torch.tensor([0, 0, 50, 0], dtype=torch.int32, device=DEV)
    tok, lp = ops.sample_tokens(logits, temps, top_ps, top_ks, step=1)
    assert int(tok[0]) == int(logits[0].argmax())
    # empirical check of row 1 (pure temperature 1): frequencies ~ softmax
    rows = logits[1:2].repeat(4096, 1)
    t = torch.ones(4096, device=DEV)
    seeds = torch.arange(4096, device=DEV, dtype=torch.int64)
    samp, _ = ops.sample_tokens(rows, t, None, None, seeds.view(torch.int64), step=7)
    freq = torch.bincount(samp.long().cpu(), minlength=V).float() / 4096
    p = torch.softmax(logits[1].float().cpu(), -1)
    top = p.argsort(descending=True)[:5]
    assert (freq[top] - p[top]).abs().max() < 0.03
    # top-p 0.5 on row 3: every sampled token lies inside the nucleus
    rows3 = logits[3:4].repeat(2048, 1)
    s3, _ = ops.sample_tokens(rows3, torch.ones(2048, device=DEV), torch.full((2048,), 0.5, device=DEV), None,
                              torch.arange(2048, device=DEV, dtype=torch.int64), step=3)
    p3 = torch.softmax(logits[3].float().cpu(), -1)
    sp, si = p3.sort(descending=True)
    n = int((sp.cumsum(0) < 0.5).sum()) + 1
    allowed = set(si[:n + 1].tolist())
    assert set(s3.cpu().tolist()) <= allowed


def _sample_v1(logits, temps, top_ps, top_ks, seeds, step):
    """The one-workgroup-per-row kernel (bisection thresholds), for cross-checks."""
    from xgserve.ops._native import kernels, stream_ptr, ptr
    B, V = logits.shape
    tok = torch.empty(B, dtype=torch.int32, device=DEV)
    lp = torch.empty(B, dtype=torch.float32, device=DEV)
    kernels().sample_tokens(logits.data_ptr(), 1 if logits.dtype == torch.float32 else 0, logits.stride(0), B, V,
                            temps.data_ptr(), ptr(top_ps), ptr(top_ks), ptr(seeds), step, tok.data_ptr(),
                            lp.data_ptr(), stream_ptr(), 0, 0)
    return tok, lp


def _nucleus(prow, top_p):
    sp, si = prow.sort(descending=True)
    n = int((sp.cumsum(0) < top_p).sum()) + 1
    return set(si[:n].tolist())


@pytest.mark.parametrize("dtype,V", [(torch.bfloat16, 128256), (torch.float32, 50257), (torch.bfloat16, 1000)])
def test_sample_split_matches_single_row_kernel(dtype, V):
    """The split-row sampler draws exactly what the single-workgroup kernel draws
    whenever the kept sets agree (same counter hash): always for temperature-only and
    greedy rows; top-p / top-k rows agree up to threshold-resolution ties."""
    assert ops.sampling.SAMPLE_SPLIT
    B = 48
    logits = rnd(B, V, scale=3.0, dtype=dtype)
    temps = torch.tensor([0.0, 1.0, 0.7, 1.3] * (B // 4), device=DEV)
    top_ps = torch.tensor([1.0, 1.0, 0.9, 0.5, 1.0, 0.95] * (B // 6), device=DEV)
    top_ks = torch.tensor([0, 0, 0, 50, 1, 7, 0, 200] * (B // 8), dtype=torch.int32, device=DEV)
    seeds = torch.arange(B, device=DEV, dtype=torch.int64) * 7919
    t2, l2 = ops.sample_tokens(logits, temps, top_ps, top_ks, seeds, step=11)
    t1, l1 = _sample_v1(logits, temps, top_ps, top_ks, seeds, 11)
    assert (t2 == t1).float().mean().item() >= 0.95
    plain = (top_ps >= 1.0) & (top_ks == 0)
    assert torch.equal(t2[plain], t1[plain])
    torch.testing.assert_close(l2, l1, atol=2e-3, rtol=1e-3)
    greedy = temps <= 0
    assert torch.equal(t2[greedy].long(), logits[greedy].float().argmax(-1))
    # reproducible: same seed / step -> same draw (the histogram workspace is re-zeroed)
    t3, _ = ops.sample_tokens(logits, temps, top_ps, top_ks, seeds, step=11)
    assert torch.equal(t3, t2)
    t4, _ = ops.sample_tokens(logits, temps, top_ps, top_ks, seeds, step=12)
    assert not torch.equal(t4[~greedy], t2[~greedy])


def test_sample_split_top_p_top_k_sets():
    V, N = 4000, 4096
    base = rnd(1, V, scale=2.0, dtype=torch.float32)
    rows = base.repeat(N, 1)
    seeds = torch.arange(N, device=DEV, dtype=torch.int64)
    ones = torch.ones(N, device=DEV)
    p = torch.softmax(base[0].cpu(), -1)
    # top-p 0.6: every draw inside the nucleus; the nucleus' head tokens all drawn
    s, _ = ops.sample_tokens(rows, ones, torch.full((N,), 0.6, device=DEV), None, seeds, step=5)
    nuc = _nucleus(p, 0.6)
    got = set(s.cpu().tolist())
    assert got <= nuc
    # frequencies follow the renormalised nucleus
    keep = torch.tensor(sorted(nuc))
    q = torch.zeros(V)
    q[keep] = p[keep] / p[keep].sum()
    freq = torch.bincount(s.long().cpu(), minlength=V).float() / N
    top = q.argsort(descending=True)[:5]
    assert (freq[top] - q[top]).abs().max() < 0.03
    # top-k 20: exactly the 20 most likely tokens are reachable
    s, _ = ops.sample_tokens(rows, ones, None, torch.full((N,), 20, dtype=torch.int32, device=DEV), seeds, step=5)
    top20 = set(p.argsort(descending=True)[:20].tolist())
    got = set(s.cpu().tolist())
    assert got <= top20 and len(got) >= 15
    # top-k 1 is greedy
    s, _ = ops.sample_tokens(rows[:64], ones[:64], None, torch.ones(64, dtype=torch.int32, device=DEV), seeds[:64])
    assert (s.long().cpu() == int(p.argmax())).all()


def test_segment_sum():
    h = rnd(20, 4096)
    cu = torch.tensor([0, 3, 3, 20], dtype=torch.int32, device=DEV)
    out = torch.zeros(3, 4096, device=DEV)
    ops.segment_sum(h, cu, out)
    ref = torch.stack([h[0:3].float().sum(0), torch.zeros(4096, device=DEV), h[3:20].float().sum(0)])
    torch.testing.assert_close(out, ref, atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("T,V,H", [(1, 1000, 4096), (37, 128256, 4096), (5, 512, 8192), (3, 300, 256)])
def test_embed_gather(T, V, H):
    table = rnd(V, H)
    ids = torch.randint(0, V, (T,), dtype=torch.int32, device=DEV)
    ids[0] = V - 1
    if T > 2:
        ids[2] = -1  # invalid ids give zero rows, never an out-of-bounds read
    ss = torch.full((T,), -1.0, device=DEV)
    out = ops.embed_gather(ids, table, ss)
    ref = table.cpu().float()[ids.cpu().long().clamp(0, V - 1)]
    ref[ids.cpu() < 0] = 0
    assert torch.equal(out.cpu().float(), ref)
    torch.testing.assert_close(ss.cpu(), ref.pow(2).sum(-1), rtol=1e-4, atol=1e-3)
    out2 = ops.embed_gather(ids, table)  # without the statistic
    assert torch.equal(out2, out)


def test_mean_l2norm_rows():
    acc = torch.randn(8, 4096, device=DEV)
    rows = torch.tensor([5, 1, 6], dtype=torch.int32, device=DEV)
    cnt = torch.tensor([3, 1, 100], dtype=torch.int32, device=DEV)
    ref_in = acc.cpu().clone()
    out = ops.mean_l2norm_rows(acc, rows, cnt).cpu()
    for i, (r, n) in enumerate(zip(rows.tolist(), cnt.tolist())):
        v = ref_in[r] / n
        torch.testing.assert_close(out[i], v / v.norm(), rtol=1e-4, atol=1e-6)
        assert bool((acc[r] == 0).all())
    assert torch.equal(acc[0].cpu(), ref_in[0])  # other rows untouched


def _w13(E, F, H):
    """per-expert block-16 interleaved gate|up rows (the serving layout)."""
    from xgserve.ops.linear import interleave_gate_up
    return torch.stack([interleave_gate_up(rnd(F, H, scale=0.05), rnd(F, H, scale=0.05)) for _ in range(E)])


@pytest.mark.parametrize("T,E,k,H,F", [(1, 8, 2, 512, 256), (2, 8, 2, 1024, 512), (37, 8, 2, 1024, 512),
                                       (64, 8, 2, 4096, 1792), (200, 8, 2, 4096, 1792),
                                       # prefill-sized: experts with > 64 rows -> 128-row tile pairs
                                       # (odd tile counts, a partial second tile, one-tile experts)
                                       (300, 4, 2, 1024, 512), (575, 8, 2, 4096, 1792), (97, 2, 2, 512, 256)])
def test_fused_moe(T, E, k, H, F):
    x = rnd(T, H)
    w13 = _w13(E, F, H)
    w2 = rnd(E, H, F, scale=0.05)
    logits = rnd(T, E, dtype=torch.float32)
    w, ids = ops.moe_topk_softmax(logits, k)
    rw, rids = ops.moe_topk_softmax(logits.cpu(), k)
    assert torch.equal(ids.cpu().sort(-1).values, rids.sort(-1).values)
    out = ops.fused_moe(x, w13, w2, w, ids)
    ref = ops.moe_forward_ref(x.cpu(), w13.cpu(), w2.cpu(), w.cpu(), ids.cpu()).float()
    # bf16 intermediates: compare relative to the output scale (1-2 bf16 ulps)
    tol = 2e-2 * ref.std().item()
    torch.testing.assert_close(out.cpu().float(), ref, atol=tol, rtol=2e-2)


def test_fused_moe_expert_parallel_shard():
    T, E, k, H, F = 50, 8, 2, 512, 256
    x = rnd(T, H)
    w13 = _w13(E, F, H)
    w2 = rnd(E, H, F, scale=0.05)
    w, ids = ops.moe_topk_softmax(rnd(T, E, dtype=torch.float32), k)
    full = ops.moe_forward_ref(x.cpu(), w13.cpu(), w2.cpu(), w.cpu(), ids.cpu()).float()
    half0 = ops.fused_moe(x, w13[:4].contiguous(), w2[:4].contiguous(), w, ids, expert_offset=0).cpu().float()
    half1 = ops.fused_moe(x, w13[4:].contiguous(), w2[4:].contiguous(), w, ids, expert_offset=4).cpu().float()
    torch.testing.assert_close(half0 + half1, full, atol=4e-2, rtol=4e-2)


@pytest.mark.parametrize("T,E,k,H", [(1, 8, 2, 4096), (64, 8, 2, 4096), (5, 16, 4, 512), (3, 64, 6, 1024),
                                     (2, 4, 1, 8192), (7, 8, 2, 14336), (1, 6, 2, 1000)])
def test_moe_route_matches_fp32(T, E, k, H):
    h = rnd(T, H)
    router = rnd(E, H, scale=0.05)
    w, ids = ops.moe_route(h, router, k)
    logits = h.float() @ router.float().t()
    rw, rids = ops.moe_topk_softmax(logits.cpu(), k)
    assert torch.equal(ids.cpu().long().sort(-1).values, rids.long().sort(-1).values)
    torch.testing.assert_close(w.cpu().sort(-1).values, rw.sort(-1).values, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("T", [1, 3, 64, 150, 300])
def test_fused_moe_grouped(T):
    E, k, H, F = 8, 2, 1024, 512
    x = rnd(T, H)
    w13 = _w13(E, F, H)
    w2 = rnd(E, H, F, scale=0.05)
    w, ids = ops.moe_topk_softmax(rnd(T, E, dtype=torch.float32), k)
    out = ops.fused_moe(x, w13, w2, w, ids)
    ref = ops.moe_forward_ref(x.cpu(), w13.cpu(), w2.cpu(), w.cpu(), ids.cpu()).float()
    torch.testing.assert_close(out.cpu().float(), ref, atol=2e-2 * ref.std().item(), rtol=2e-2)


@pytest.mark.parametrize("T,E,skew,eoff", [(300, 8, 0.0, 0), (575, 8, 6.0, 0), (700, 4, 3.0, 0), (575, 8, 0.0, 4)])
def test_fused_moe_prefill_on_gemm_pf(T, E, skew, eoff, monkeypatch):
    """Prefill-sized expert GEMMs on gemm_pf's grouped form (> 256 pairs): balanced and
    skewed routing (an expert with several 192-288-row tiles), an EP shard (pairs of
    another rank's experts are not placed), against fp32 and against the m64g path."""
    from xgserve.ops import moe as MOE
    k, H, F = 2, 1024, 512
    x = rnd(T, H)
    w13 = _w13(E, F, H)
    w2 = rnd(E, H, F, scale=0.05)
    logits = rnd(T, E, dtype=torch.float32)
    logits[:, 0] += skew  # skew > 0: expert 0 takes most tokens
    w, ids = ops.moe_topk_softmax(logits, k)
    El = E // 2 if eoff else E
    w13l, w2l = w13[eoff:eoff + El].contiguous(), w2[eoff:eoff + El].contiguous()
    assert MOE.MOE_PF and MOE._moe_pf_ok(H, F)
    out = ops.fused_moe(x, w13l, w2l, w, ids, expert_offset=eoff)
    monkeypatch.setattr(MOE, "MOE_PF", False)
    base = ops.fused_moe(x, w13l, w2l, w, ids, expert_offset=eoff)
    ref = ops.moe_forward_ref(x.cpu(), w13l.cpu(), w2l.cpu(), w.cpu(), ids.cpu(), expert_offset=eoff).float()
    tol = 2e-2 * ref.std().item()
    torch.testing.assert_close(out.cpu().float(), ref, atol=tol, rtol=2e-2)
    torch.testing.assert_close(out.cpu().float(), base.cpu().float(), atol=tol, rtol=2e-2)


def test_decode_attention_split_combine_repeats():
    """Repeated split-K launches on one workspace (as graph replays do) with varying
    split counts stay correct."""
    from xgserve.ops import attention as A
    Hq, Hkv, D, bs = 32, 8, 128, 16
    lens = [700, 33, 1, 256]
    kc, vc, bt = _paged(lens, Hkv, D, bs)
    B = len(lens)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    ws = A.DecodeWorkspace(B, Hq, D, 16, DEV)
    for it, splits in enumerate((16, 16, 5, 16)):
        q = rnd(B, Hq, D)
        out = ops.decode_attention(q, kc, vc, bt, sl, 0.088, num_splits=splits, workspace=ws)
        ref = ops.decode_attention_ref(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), sl.cpu(), 0.088)
        torch.testing.assert_close(out.cpu().float(), ref.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("Ts,k,E_local,tp", [(1, 2, 4, 2), (37, 2, 4, 2), (64, 2, 2, 4), (700, 2, 1, 8), (5, 4, 2, 8)])
def test_ep_dispatch_kernels_match_torch(Ts, k, E_local, tp, packed):
    """ep_plan / ep_scatter / ep_combine (HIP) against their torch fallbacks: identical
    slots, local expert ids and counts (the plan is deterministic), identical rows,
    and the weighted combine against an fp32 loop."""
    H = 512
    ids = torch.randint(0, E_local * tp, (Ts, k), dtype=torch.int32)
    cap = Ts * k
    s_ref, e_ref, c_ref = ops.ep_plan(ids, E_local, tp, cap, packed)
    s, e, c = ops.ep_plan(ids.to(DEV), E_local, tp, cap, packed)
    assert torch.equal(s.cpu(), s_ref) and torch.equal(c.cpu(), c_ref) and torch.equal(e.cpu(), e_ref)
    x = rnd(Ts, H)
    rows = Ts * k if packed else tp * cap
    send = ops.ep_scatter(x, k, s, rows)
    src = torch.arange(Ts * k) // k
    assert torch.equal(send[s.long()].cpu(), x.cpu()[src])
    w = torch.rand(Ts, k, device=DEV)
    back = rnd(rows, H)
    out = torch.zeros(Ts + 3, H, dtype=torch.bfloat16, device=DEV)
    ops.ep_combine(back, s, w, out)
    want = (back.cpu().float()[s.long().cpu()] * w.cpu().reshape(-1, 1)).view(Ts, k, H).sum(1)
    torch.testing.assert_close(out[:Ts].cpu().float(), want, atol=2e-2, rtol=1e-2)
    assert bool((out[Ts:] == 0).all())


@pytest.mark.parametrize("T,E,k,H", [(1, 8, 2, 4096), (33, 8, 2, 4096), (2, 4, 1, 8192), (3, 8, 2, 14336)])
def test_moe_route_norm_matches_fp32(T, E, k, H):
    """Router with the RMSNorm prologue (one-round-trip route2 kernel, 1 / 2 / 4 chunks
    per thread): normalised rows vs fp32 up to one bf16 rounding, routing on them."""
    h = rnd(T, H)
    g = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16()
    router = rnd(E, H, scale=0.05)
    hn, w, ids = ops.moe_route_norm(h, g, 1e-5, router, k)
    hf = h.float()
    want = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5) * g.float()
    torch.testing.assert_close(hn.float(), want, atol=2e-2, rtol=1e-2)
    rw, rids = ops.moe_topk_softmax((hn.float() @ router.float().t()).cpu(), k)
    assert torch.equal(ids.cpu().long().sort(-1).values, rids.long().sort(-1).values)
    torch.testing.assert_close(w.cpu().sort(-1).values, rw.sort(-1).values, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("T,E_local,eoff", [(1, 8, 0), (1, 4, 4), (1, 4, 0), (1, 2, 6), (5, 8, 0)])
def test_moe_route_norm_align_matches_moe_align(T, E_local, eoff):
    """moe_route_norm(align=...): for one token the router launch writes moe_align's
    layout itself (sorted_rows, offsets, dest), bit-identical to the align kernel's;
    more tokens fall back to moe_align."""
    H, E, k = 4096, 8, 2
    h = rnd(T, H)
    g = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16()
    router = rnd(E, H, scale=0.05)
    hn, w, ids, (rows, offs, dest) = ops.moe_route_norm(h, g, 1e-5, router, k, align=(E_local, eoff))
    rows2, offs2, dest2 = ops.moe_align(ids, E_local, eoff)
    assert torch.equal(offs.cpu(), offs2.cpu())
    assert torch.equal(dest.cpu(), dest2.cpu())
    assert torch.equal(rows.cpu(), rows2.cpu())
