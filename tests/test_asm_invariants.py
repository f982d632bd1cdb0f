"""Pinned code-generation invariants of the LDS-DMA kernels (CPU: hipcc -S, gfx950).

The weight-streaming GEMMs issue global_load_lds_dwordx4 from inline asm and retire
them with hand-counted `s_waitcnt vmcnt(N)` (csrc/kernels/glds.h): hipcc's waitcnt
pass cannot see those loads, so a compiler update that re-schedules or re-waits the
loop would silently de-pipeline (an extra vmcnt(0)) or break (a count that no longer
matches the issue order) the kernels. This test compiles them and checks:
  * no "reserved registers on the clobber list" warning (M0 goes in as a "{m0}"
    operand, not a clobber);
  * every vmcnt wait in each instantiation is one the pipeline's issue order allows
    (gemm_mw: the ring formula of gemm_mw.hip; gemm_m64g: G = x + W instructions per
    chunk, or 0);
  * no VGPR / SGPR spills.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, "csrc", "kernels")
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)

pytestmark = pytest.mark.skipif(HIPCC is None, reason="hipcc not available")


def _compile(name: str, tmp_path):
    out = tmp_path / f"{name}.s"
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", f"-I{KDIR}", "-S", "--cuda-device-only",
                        os.path.join(KDIR, f"{name}.hip"), "-o", str(out)],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    return out.read_text(), r.stdout


def _kernels(asm: str, prefix: str):
    """{template args string: body} for every kernel symbol starting with prefix."""
    parts = re.split(r"\n(_ZN3xgk\w+):[^\n]*\n", asm)
    out = {}
    for i in range(1, len(parts), 2):
        name, body = parts[i], parts[i + 1].split(".Lfunc_end")[0]
        if name.startswith(prefix):
            out[name] = body
    return out


def _targs(name: str):
    """Template arguments of a mangled xgk kernel: Li<int>E / Lb<0|1>E in order."""
    inner = name[name.index("I") + 1:]
    return [int(v) for v in re.findall(r"L[ib](\d+)E", inner)]


def _vmcnts(body: str):
    return {int(v) for v in re.findall(r"s_waitcnt[^\n]*vmcnt\((\d+)\)", body)}


_EPILOGUE_OPS = re.compile(r"\b(global_load_dword|global_load_dwordx[234]|global_store|global_atomic|flat_)")


def _without_epilogue_blocks(body: str) -> str:
    """The body minus every basic block holding an ordinary (compiler-counted) global
    load / store / atomic: the split-K tails and the statistics loads, whose waits
    are the compiler's own. The LDS-DMA pipeline blocks hold none of these."""
    blocks = re.split(r"\n(?=\.LBB\d+_\d+:)", body)
    return "\n".join(b for b in blocks if not _EPILOGUE_OPS.search(b))


def _pipeline(body: str, through_barrier: bool = False) -> str:
    """The weight-streaming span: first LDS-DMA issue .. last MFMA (the prologue's
    statistics loads and the epilogue's hand-offs carry compiler-counted waits of
    their own, outside this span); through_barrier: .. the later of the last MFMA
    and the last s_barrier (a rotated loop keeps its wait + barrier below the MFMAs)."""
    a = body.index("global_load_lds_dwordx4")
    b = body.rindex("v_mfma")
    if through_barrier and "s_barrier" in body:
        b = max(b, body.rindex("s_barrier"))
    return body[a:b]


def _no_spills(asm: str):
    v = [int(x) for x in re.findall(r"\.vgpr_spill_count:\s*(\d+)", asm)]
    s = [int(x) for x in re.findall(r"\.sgpr_spill_count:\s*(\d+)", asm)]
    assert v and s, "no spill metadata in the assembly"
    assert max(v) == 0 and max(s) == 0, (max(v), max(s))


def test_gemm_mw_waits_follow_the_ring(tmp_path):
    asm, log = _compile("gemm_mw", tmp_path)
    assert "reserved registers on the clobber list" not in log
    ks = _kernels(asm, "_ZN3xgk14gemm_mw_kernel")
    assert len(ks) >= 20, len(ks)
    for name, body in ks.items():
        targs = _targs(name)
        if len(targs) > 5 and targs[5] != 0:
            continue  # anatomy probes (PR != 0): parts of the pipeline removed on purpose
        WN, NWT, MTW, D, _nt = targs[:5]
        WI = WN * 16 * NWT // 64
        XI = (8 // WN) * 16 * MTW // 64
        allowed = {0, WI + (XI if D >= 3 else 0)}
        if D >= 3:
            allowed.add(2 * WI + min(D - 2, 2) * XI)
        if D >= 4:
            allowed.add(3 * WI + 2 * XI)
        got = _vmcnts(_pipeline(body, through_barrier=True))
        assert got <= allowed, (name, sorted(got), sorted(allowed))
        assert WI + (XI if D >= 3 else 0) in got, (name, sorted(got))  # the steady-state counted wait exists
        n_glds = len(re.findall(r"global_load_lds_dwordx4", body))
        assert n_glds >= WI + XI, name
        assert len(re.findall(r"v_mfma_f32_16x16x32_bf16", body)) >= 2 * NWT * MTW, name
    _no_spills(asm)


def _pf_wait_counts(P: int, NA: int, L: int = 1):
    """Python twin of pf::wait_count (csrc/kernels/gemm_pf.hip): the steady-state
    vmcnt before phase p = every DMA issued after the last piece phase p reads.
    A piece q of tile u is issued in global phase (u - 2)P + q + L, W piece i in
    (u - 2)P + L + i % P (global phase of (tile t, phase p) = tP + p)."""
    NBW = 4
    b_phase = lambda i: (L + i % P) % P  # noqa: E731
    n_issue = [NA + sum(1 for i in range(NBW) if b_phase(i) == ph) for ph in range(P)]
    T = sum(n_issue)

    def pos(tau, ph, j):
        return tau * T + sum(n_issue[:ph]) + j

    def pos_a(u, q):
        g = (u - 2) * P + q + L
        return pos(g // P, g % P, NA - 1)

    def pos_b(u, i):
        g = (u - 2) * P + L + i % P
        ph = g % P
        j = NA + sum(1 for i2 in range(i) if b_phase(i2) == ph)
        return pos(g // P, ph, j)

    t = 8
    out = []
    for p in range(P):
        latest = pos_a(t, p)
        if p == 0:
            latest = max([latest] + [pos_b(t, i) for i in range(NBW)])
        out.append(pos(t, p, 0) - 1 - latest)
    return out


def test_gemm_pf_waits_and_fragments(tmp_path):
    """gemm_pf: every vmcnt is a count of its DMA issue order (or 0 at a range's
    tail), the MFMA operands come straight from ds_read_b128 (no VALU shuffles of the
    fragments between the reads and the MFMAs), and nothing spills."""
    asm, log = _compile("gemm_pf", tmp_path)
    assert "reserved registers" not in log
    assert _pf_wait_counts(4, 1) == [6, 13, 13, 13] and _pf_wait_counts(2, 2) == [4, 10]
    ks = _kernels(asm, "_ZN3xgk14gemm_pf_kernel")
    assert len(ks) >= 8
    for name, body in ks.items():
        ta = _targs(name)
        bm, mtp, _nt, pr = ta[:4]
        lag = ta[4] if len(ta) > 4 else 1  # <BM, MTP, NT, PR, LAG, GRP>
        if pr:  # anatomy-probe builds (no DMA / no MFMA)
            continue
        P = bm // (32 * mtp)
        na0, na1 = (4 * mtp + 7) // 8, (4 * mtp) // 8  # per-wave A pieces of the two wave groups
        allowed = {0} | set(_pf_wait_counts(P, na0, lag)) | set(_pf_wait_counts(P, na1, lag))
        got = _vmcnts(_without_epilogue_blocks(_pipeline(body)))
        assert got <= allowed, (name, sorted(got), sorted(allowed))
        assert "v_pk_mov_b32" not in _pipeline(body), name
    meta = asm[asm.index("amdhsa.kernels"):]
    assert ".vgpr_spill_count: 0" in meta and not re.search(r"\.vgpr_spill_count:\s+[1-9]", meta)


def test_gemm_m64g_waits_are_counted(tmp_path):
    asm, log = _compile("gemm_m64g", tmp_path)
    assert "reserved registers on the clobber list" not in log
    ks = _kernels(asm, "_ZN3xgk16gemm_m64g_kernel")
    assert len(ks) >= 8, len(ks)
    for name, body in ks.items():
        NW, WV, KC, _nt, MT, *rest = _targs(name)
        NS = rest[0] if rest else 3
        RPI = 1024 // (KC * 2)
        XI = 16 * MT // RPI // WV
        G = XI + 16 * NW // RPI
        counted = {k * G for k in range(1, NS - 1)}  # 1 .. NS - 2 chunks left in flight
        if NS == 3:
            # blocks with ordinary loads (the all-reduce prologue's reducer path, the
            # statistics loads) carry the compiler's own waits and are skipped
            got = _vmcnts(_without_epilogue_blocks(_pipeline(body)))
            # XI: the all-reduce prologue leaves chunk 1's x DMAs in flight
            assert got <= {0, XI, G}, (name, sorted(got), G)
        else:
            # deep rings: the rotated loop may be laid out ahead of the prologue, so every
            # block without ordinary global memory ops is checked -- the counted waits are
            # all there and no other wait between G and the ring's depth (smaller ones and,
            # with four x tiles, the prologue's waits for its statistics loads issued ahead
            # of the ring -- above (NS - 2) G, never draining it -- are the compiler's own)
            got = _vmcnts(_without_epilogue_blocks(body if MT == 1 else _pipeline(body)))
            assert not {v for v in got if G <= v <= (NS - 2) * G} - counted, (name, sorted(got), sorted(counted))
        assert counted <= got, (name, sorted(got), sorted(counted))
    _no_spills(asm)


def test_prefill_attention_has_no_clobber_warning(tmp_path):
    _, log = _compile("prefill_attention", tmp_path)
    assert "reserved registers on the clobber list" not in log


def test_gemm_w8_waits_are_counted(tmp_path):
    """gemm_w8 (fp8 / int8 / int4 weights): inside the LDS-DMA pipeline every vmcnt wait
    is the steady count G = x + weight DMAs per chunk (chunk c + 1 stays in flight) or the
    drain; the int4 form's group-scale staging (ordinary loads, before the first DMA) keeps
    its own compiler waits outside that span. No spills."""
    asm, log = _compile("gemm_w8", tmp_path)
    assert "reserved registers on the clobber list" not in log
    ks = _kernels(asm, "_ZN3xgk14gemm_w8_kernel")
    assert len(ks) >= 24, len(ks)  # 8 geometries x 3 weight formats
    for name, body in ks.items():
        NW, WV, KC, MT, FMT = _targs(name)
        wrb = KC // 2 if FMT == 2 else KC
        XI = 16 * MT // (1024 // (2 * KC)) // WV
        WI = 16 * NW // (1024 // wrb)
        G = XI + WI
        got = _vmcnts(_without_epilogue_blocks(_pipeline(body)))
        assert got <= {0, G}, (name, sorted(got), G)
        assert G in got, (name, sorted(got), G)
    _no_spills(asm)
