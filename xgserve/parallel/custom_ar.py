"""Custom one-shot / two-shot all-reduce over xGMI peer memory (csrc/comm/custom_allreduce.hip).

Each TP rank allocates one uncached HBM buffer (2 slots x max_bytes) and one
signal array, exports both with hipIpcGetMemHandle, and exchanges the handles
over the CPU (gloo) group; every rank then maps all peers' buffers. The kernel
is graph capturable, so TP decode graphs contain the all-reduce.

Path choice, bf16 messages of 16-byte multiples:
  * one-shot (each rank reads every peer's whole message; lowest latency) up to
    `two_shot_min` bytes, or up to `max_bytes` when TP < 4 (at 2 ranks the
    two-shot moves the same bytes per link plus a second synchronisation);
  * two-shot (reduce-scatter + all-gather through peer memory, ~2n/W bytes per
    xGMI link) from `two_shot_min` to `two_shot_max` bytes at TP >= 4;
  * RCCL above that (comm.tp_all_reduce falls back automatically).

Fused decode layer under TP: `all_reduce_resid` takes a row-parallel GEMM's
fp32 split-K partials and, in one launch, reduces them locally, exchanges the
bf16 contributions over IPC, adds the sum to the replicated residual stream and
writes the new residual's RMSNorm statistics (custom_allreduce_resid). It has
its own slots, signals and generation counters.

Push protocol ("LL", the default for decode-sized messages): instead of staging
the message locally, fencing, raising flags and then READING every peer's copy
over xGMI (the pull kernels), each rank writes its contribution straight into
every peer's receive region as 16-byte lines {data, gen, data, gen}; the receiver
polls its own memory until the generations match -- no fence, no flag word, no
remote read round trip after the synchronisation. It serves the fused residual
all-reduce and plain all-reduces up to `ll_max` bytes (XGS_TUNE ar_ll_max, 0 = pull
kernels everywhere).

First contact (`self_test`, run by `maybe_enable` on every start): before the
instance is registered, every protocol it would use -- push (LL) and pull plain
all-reduces at decode sizes, the fused residual all-reduce in both forms, the
two-shot form when TP >= 4 -- runs on the real links against an RCCL all-reduce
of the same data. A protocol whose result differs is switched off on every rank
(the group agrees through a MIN all-reduce), and if the pull kernels themselves
fail the custom path is not registered at all (RCCL serves). The outcome is
kept in `self.verified` ({"ll": bool, "pull": bool, ...}) and reported by
bench.py. This is the gate for the push protocol on multi-GPU nodes: it has
only been measured with every rank on one GPU (profiles/r4_ar_protocols.md),
and its correctness depends on each peer's 8-byte {data, gen} halves landing
intact over xGMI.

Failure semantics: a peer that does not arrive within the wait limit makes the
kernels bump a device error counter and give up (the GPU never hangs); once the
counter is non-zero every later wait returns at once, so a dead peer costs one
limit per step, not one per collective. The limit is a device word read by every
launch (graph replays included): `set_timeout` makes it generous around warmup
and graph capture (first-call RCCL setup, first-seen GEMM shapes) and sets the
configured collective timeout for serving. After every step the runner copies
the counter to pinned host memory behind the step's work (`poll_async`) and
`check()` raises CustomAllReduceTimeout, so the step fails (and the replica
restarts) instead of returning a stale sum.
"""
from __future__ import annotations

import logging
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops._native import kernels, stream_ptr

log = logging.getLogger("xgserve.comm")


class CustomAllReduceTimeout(RuntimeError):
    """A TP peer did not reach a custom all-reduce within the kernel's wait limit."""


class CustomAllReduce:
    # fused residual path: T * H bf16 per rank (decode: T <= 64, H <= 8192 -> 1 MiB)
    RESID_SLOT = 1 << 20
    # last-dim all-gather (vocab-parallel LM head of decode steps): T * V/W bf16 per rank
    GATHER_SLOT = 16 << 20
    # push-protocol receive regions: [2 parities][8 sources][2 x payload] per rank
    RESID_LL_REGION = 32 << 20   # fused residual: T * H bf16 <= 1 MiB of payload
    LL_REGION = 8 << 20          # plain all-reduce: <= 256 KiB of payload
    GEMM_LL_REGION = 32 << 20    # all-reduce inside the row-parallel GEMM (gemm_m64g GG_AR)
    # peer-wait limits: while serving, and around warmup / graph capture
    SERVE_TIMEOUT_S = 2.0
    WARMUP_TIMEOUT_S = 20.0  # (the 32-bit tick word caps the limit at ~21 s at 100 MHz)

    def __init__(self, rank: int, world: int, device: torch.device, cpu_group=None, max_bytes: int = 8 << 20,
                 two_shot_min: Optional[int] = None, two_shot_max: int = 32 << 20, ll_max: Optional[int] = None):
        k = kernels()
        max_ranks, self.max_blocks, chunk = k.car_limits()
        if not (2 <= world <= max_ranks):
            raise ValueError(f"custom all-reduce supports 2..{max_ranks} ranks, got {world}")
        self.rank, self.world, self.device = rank, world, device
        self.slot = min(max_bytes, self.max_blocks * chunk) // chunk * chunk
        if two_shot_min is None:
            two_shot_min = (512 << 10) if world >= 4 else self.slot + 1
        # a two-shot shard of n/W bytes must fit max_blocks chunks
        self.slot2 = min(two_shot_max, self.max_blocks * chunk * world) // chunk * chunk
        self.two_shot_min = two_shot_min
        nsig = max_ranks * self.max_blocks * 4  # bytes per phase
        self._k = k
        self.data = self.sig = 0
        self._opened: List[int] = []
        # phase 1 (local): allocate + export; every rank reports success so a
        # failure anywhere disables the path everywhere instead of hanging peers
        mine = None
        props = torch.cuda.get_device_properties(device)
        self.device_id = (props.pci_domain_id, props.pci_bus_id, props.pci_device_id, str(props.uuid))
        try:
            # [one-shot 2 x slot | two-shot 2 x slot2 | resid 2 x RESID_SLOT | gather 2 x GATHER_SLOT
            #  | resid LL region | LL region] and [one-shot | two-shot phase 0 | phase 1 | resid |
            # gather] signals
            self.data = k.car_alloc_uncached(2 * self.slot + 2 * self.slot2 + 2 * self.RESID_SLOT
                                             + 2 * self.GATHER_SLOT + self.RESID_LL_REGION + self.LL_REGION
                                             + self.GEMM_LL_REGION)
            self.sig = k.car_alloc_uncached(5 * nsig)
            mine = (k.car_ipc_handle(self.data), k.car_ipc_handle(self.sig))
        except RuntimeError as e:
            log.warning("custom all-reduce: local setup failed: %s", e)
        handles: List = [None] * world
        dist.all_gather_object(handles, (mine, self.device_id), group=cpu_group)
        # ranks sharing one GPU (the single-GPU test boxes): kernels that spin on peers
        # must stay small enough to be co-resident with every peer's (the GEMM-fused
        # all-reduce is not: comm.gemm_ar_args keeps the separate launches there)
        self.shared_device = len({h[1] for h in handles}) < world
        handles = [h[0] for h in handles]
        if any(h is None for h in handles):
            self.close()
            raise RuntimeError("custom all-reduce setup failed on some rank")
        # phase 2: map the peers
        ok = 1
        self.data_ptrs, self.sig_ptrs = [], []
        try:
            for r in range(world):
                if r == rank:
                    self.data_ptrs.append(self.data)
                    self.sig_ptrs.append(self.sig)
                    continue
                d = k.car_ipc_open(handles[r][0])
                self._opened.append(d)
                s_ = k.car_ipc_open(handles[r][1])
                self._opened.append(s_)
                self.data_ptrs.append(d)
                self.sig_ptrs.append(s_)
        except RuntimeError as e:
            log.warning("custom all-reduce: mapping peers failed: %s", e)
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=cpu_group)
        if int(flag.item()) == 0:
            self.close()
            raise RuntimeError("custom all-reduce: peer mapping failed on some rank")
        self.data_ptrs2 = [d + 2 * self.slot for d in self.data_ptrs]
        self.sig_ptrs2 = [s_ + nsig for s_ in self.sig_ptrs]
        self.data_ptrs3 = [d + 2 * self.slot + 2 * self.slot2 for d in self.data_ptrs]
        self.sig_ptrs3 = [s_ + 3 * nsig for s_ in self.sig_ptrs]
        self.data_ptrs4 = [d + 2 * self.slot + 2 * self.slot2 + 2 * self.RESID_SLOT for d in self.data_ptrs]
        self.sig_ptrs4 = [s_ + 4 * nsig for s_ in self.sig_ptrs]
        ll0 = 2 * self.slot + 2 * self.slot2 + 2 * self.RESID_SLOT + 2 * self.GATHER_SLOT
        self.data_ptrs_rll = [d + ll0 for d in self.data_ptrs]
        self.data_ptrs_ll = [d + ll0 + self.RESID_LL_REGION for d in self.data_ptrs]
        self.data_ptrs_gll = [d + ll0 + self.RESID_LL_REGION + self.LL_REGION for d in self.data_ptrs]
        self.gens_gll = torch.zeros(4096, dtype=torch.int32, device=device)
        self.gens_rll = torch.zeros(self.max_blocks + 1, dtype=torch.int32, device=device)
        self.gens_ll = torch.zeros(self.max_blocks + 1, dtype=torch.int32, device=device)
        import os
        if ll_max is None:
            from .. import tune
            ll_max = tune.get_int("ar_ll_max", 256 << 10)
        self.ll_max = min(ll_max, k.car_ll_max_bytes(self.LL_REGION))
        self.resid_ll = self.ll_max > 0
        self.chunk = chunk
        self.gens = torch.zeros(self.max_blocks + 1, dtype=torch.int32, device=device)
        self.gens2 = torch.zeros(self.max_blocks + 1, dtype=torch.int32, device=device)
        self.gens3 = torch.zeros(self.max_blocks + 1, dtype=torch.int32, device=device)
        self.gens4 = torch.zeros(self.max_blocks + 1, dtype=torch.int32, device=device)
        # ctl[0]: peer-wait timeouts of every path (device), mirrored to pinned host
        # memory; ctl[1]: the wait limit in wall-clock ticks (set_timeout)
        self.ctl = torch.zeros(2, dtype=torch.int32, device=device)
        self.err = self.ctl[:1]
        self.h_err = torch.zeros(1, dtype=torch.int32).pin_memory()
        self._khz = max(1, int(k.car_wallclock_khz()) or 100_000)
        self.timeout_s = 0.0
        self.set_timeout(self.serve_timeout())
        self.verified = None  # self_test() outcome
        self.verified_counts = None  # launches that passed per protocol
        # operands of the all-reduce inside the row-parallel GEMMs (comm.gemm_ar_args);
        # None until self_test() has verified it against RCCL
        from .comm import GemmArArgs
        self._gemm_ar = GemmArArgs(self.data_ptrs_gll, self.GEMM_LL_REGION, rank, world, 0, self.gens_gll,
                                   self.ctl)
        self.gemm_ar = None
        log.info("custom all-reduce ready: rank %d/%d, one-shot <= %d KiB, two-shot <= %d MiB", rank, world,
                 min(self.slot, self.two_shot_min) >> 10, self.slot2 >> 20)

    def _two_shot(self, n: int) -> bool:
        if not self.two_shot_min <= n <= self.slot2:
            return False
        # slot layout [block][rank shard][chunk]: the padded shards must fit the slot
        shard = (-(-n // self.world) + 15) // 16 * 16
        blocks = -(-shard // self.chunk)
        return blocks <= self.max_blocks and blocks * self.world * self.chunk <= self.slot2

    def can_run(self, x: torch.Tensor) -> bool:
        n = x.numel() * x.element_size()
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and n > 0 and n % 16 == 0
                and (n <= self.slot or self._two_shot(n)))

    def all_reduce(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        out = x if out is None else out
        n = x.numel() * x.element_size()
        if n <= self.ll_max:
            self._k.custom_allreduce_ll(x.data_ptr(), out.data_ptr(), n, self.LL_REGION, self.data_ptrs_ll,
                                        self.rank, self.gens_ll.data_ptr(), self.err.data_ptr(), stream_ptr())
        elif self._two_shot(n):
            self._k.custom_allreduce_2shot(x.data_ptr(), out.data_ptr(), n, self.slot2, self.data_ptrs2,
                                           self.sig_ptrs2, self.rank, self.gens2.data_ptr(), self.err.data_ptr(),
                                           stream_ptr())
        else:
            self._k.custom_allreduce(x.data_ptr(), out.data_ptr(), n, self.slot, self.data_ptrs, self.sig_ptrs,
                                     self.rank, self.gens.data_ptr(), self.err.data_ptr(), stream_ptr())
        return out

    def can_resid(self, T: int, H: int) -> bool:
        return 1 <= T and H % 1024 == 0 and T * (H // 1024) <= self.max_blocks and T * H * 2 <= self.RESID_SLOT

    def all_reduce_resid(self, part: torch.Tensor, resid: torch.Tensor, ss: torch.Tensor) -> None:
        """resid (bf16 [T, H], replicated) += sum over ranks of sum_s part[s] (this
        rank's fp32 split-K partials [S, T, H]); ss[chunk * T + t] <- the new
        residual's sum of squares per 1024-column chunk. One launch."""
        S, T, H = part.shape
        if not (part.is_contiguous() and part.dtype == torch.float32 and resid.is_contiguous()
                and tuple(resid.shape) == (T, H) and resid.dtype == torch.bfloat16 and ss.numel() >= T * (H // 1024)):
            raise ValueError(f"all_reduce_resid: bad operands part={tuple(part.shape)} resid={tuple(resid.shape)}")
        if self.resid_ll:
            self._k.custom_allreduce_resid_ll(part.data_ptr(), S, T, resid.data_ptr(), ss.data_ptr(), H,
                                              self.RESID_LL_REGION, self.data_ptrs_rll, self.rank,
                                              self.gens_rll.data_ptr(), self.err.data_ptr(), stream_ptr())
            return
        self._k.custom_allreduce_resid(part.data_ptr(), S, T, resid.data_ptr(), ss.data_ptr(), H, self.RESID_SLOT,
                                       self.data_ptrs3, self.sig_ptrs3, self.rank, self.gens3.data_ptr(),
                                       self.err.data_ptr(), stream_ptr())

    def can_gather(self, x: torch.Tensor) -> bool:
        cb = x.shape[-1] * x.element_size()
        return (x.is_cuda and x.dim() == 2 and x.is_contiguous() and cb % 16 == 0 and 0 < x.numel()
                and x.numel() * x.element_size() <= self.GATHER_SLOT)

    def all_gather_lastdim(self, x: torch.Tensor) -> torch.Tensor:
        """[T, n] per rank -> [T, world * n] (rank-major columns), one launch."""
        T, n = x.shape
        out = torch.empty(T, self.world * n, dtype=x.dtype, device=x.device)
        self._k.custom_allgather_lastdim(x.data_ptr(), out.data_ptr(), T, n * x.element_size(), self.GATHER_SLOT,
                                         self.data_ptrs4, self.sig_ptrs4, self.rank, self.gens4.data_ptr(),
                                         self.err.data_ptr(), stream_ptr())
        return out

    # first-contact repetitions: each protocol runs this many times on fresh data (an
    # intermittent fault -- a torn 16-byte line over xGMI -- would not show in one trial)
    SELF_TEST_ITERS = 50
    LL_SIZES = (16 << 10, 32 << 10, 64 << 10, 128 << 10, 256 << 10)

    def gemm_ar_allowed(self) -> bool:
        """GG_AR (the all-reduce inside the row-parallel GEMM) spins on its peers from
        a GEMM-sized grid: on separate GPUs always; on ranks sharing one GPU only
        under the test-only XGS_TUNE gemm_ar_shared=1, for <= 4 ranks (whose grids are
        co-resident there), so the engine path can be exercised on one-GPU boxes."""
        from .. import tune
        if not self.shared_device:
            return True
        return self.world <= 4 and tune.get_bool("gemm_ar_shared", False)

    def self_test(self, group, cpu_group, ar_shapes=None) -> dict:
        """Run every protocol this instance would use against RCCL on the real links
        (module docstring, "First contact"), SELF_TEST_ITERS times each on fresh data;
        switch off the ones that disagree on any rank. ar_shapes: the model's
        row-parallel (N, K) shapes in layer order (O, down), replayed for GG_AR at
        T = 1..4 rows -- the serving sequence, whose tile widths may differ between the
        two launches. Returns {"ll", "ll_resid", "pull", "pull_resid", "two_shot",
        "gemm_ar"} -> bool (None: protocol not in use); the passing launch counts are
        kept in self.verified_counts."""
        from .comm import GEMM_AR_MAX_T
        dev = self.device
        g = torch.Generator(device=dev).manual_seed(4321 + self.rank)
        res = {"ll": None, "ll_resid": None, "pull": None, "pull_resid": None, "two_shot": None, "gemm_ar": None}
        counts = {k: 0 for k in res}
        iters = self.SELF_TEST_ITERS

        def close_enough(got: torch.Tensor, ref: torch.Tensor) -> bool:
            return bool(torch.isfinite(got).all()) and float((got.float() - ref).abs().max()) <= \
                2e-2 * max(1e-3, float(ref.abs().max()))

        def plain(name: str, sizes, ll: bool) -> bool:
            keep = self.ll_max
            for i in range(iters):
                nbytes = sizes[i % len(sizes)]
                x = (torch.randn(nbytes // 2, generator=g, device=dev) * 0.5).bfloat16()
                ref = x.float()
                dist.all_reduce(ref, group=group)
                if not ll:
                    self.ll_max = 0
                try:
                    y = self.all_reduce(x.clone())
                finally:
                    self.ll_max = keep
                torch.cuda.synchronize(dev)
                if not close_enough(y, ref):
                    return False
                counts[name] += 1
            return True

        def resid(name: str, ll: bool) -> bool:
            H = 4096
            keep = self.resid_ll
            for i in range(iters):
                T, S = (1, 2, 3, 4, 8, 16, 64)[i % 7], 1 + i % 4
                part = torch.randn(S, T, H, generator=g, device=dev) * 0.25
                base = torch.randn(T, H, generator=torch.Generator(device=dev).manual_seed(99 + i),
                                   device=dev).bfloat16()
                ref = part.sum(0)
                dist.all_reduce(ref, group=group)
                ref = base.float() + ref
                r = base.clone()
                ss = torch.zeros(T * (H // 1024), dtype=torch.float32, device=dev)
                self.resid_ll = ll
                try:
                    self.all_reduce_resid(part, r, ss)
                finally:
                    self.resid_ll = keep
                torch.cuda.synchronize(dev)
                ss_ref = (r.float().view(T, H // 1024, 1024) ** 2).sum(-1).t().reshape(-1)
                if not (close_enough(r, ref) and bool(torch.allclose(ss, ss_ref, rtol=2e-2, atol=1e-2))):
                    return False
                counts[name] += 1
            return True

        def gemm_ar() -> bool:
            from ..ops.linear import ResidWorkspace, m64_ar_resid_linear, m64_plan
            # default: the Llama-3-8B TP2 O / down shards (64- and 32-column tiles)
            shapes = [(n, k) for n, k in (ar_shapes or [(4096, 2048), (4096, 7168)])
                      if m64_plan(1, n, k) is not None]
            if not shapes:
                return True
            ws = ResidWorkspace(len(shapes), 64, max(n for n, _ in shapes), dev)
            wts = [(torch.randn(n, k, generator=g, device=dev) * (0.5 / k ** 0.5)).bfloat16() for n, k in shapes]
            for i in range(iters):
                T = 1 + i % GEMM_AR_MAX_T
                outs = []
                for site, ((n, k), w) in enumerate(zip(shapes, wts)):  # one layer's O then down
                    x = (torch.randn(T, k, generator=g, device=dev) * 0.5).bfloat16()
                    base = (torch.randn(T, n, generator=g, device=dev)).bfloat16()
                    r = base.clone()
                    st = m64_ar_resid_linear(x, w, r, ws, site, self._gemm_ar)
                    outs.append((x, w, base, r, st))
                torch.cuda.synchronize(dev)
                for x, w, base, r, st in outs:
                    ref = (x.float() @ w.float().t()).bfloat16().float()
                    dist.all_reduce(ref, group=group)
                    ref = base.float() + ref
                    n = st.n
                    N = w.shape[0]
                    ss_ref = (r.float().view(T, n, N // n) ** 2).sum(-1).t().reshape(-1)
                    if not (close_enough(r, ref) and bool(torch.allclose(st.ss[: n * T], ss_ref, rtol=2e-2,
                                                                         atol=1e-2))):
                        return False
                    counts["gemm_ar"] += 1
            return True

        checks = {"pull": lambda: plain("pull", (16 << 10, min(self.slot, 256 << 10)), False),
                  "pull_resid": lambda: resid("pull_resid", False)}
        if self.gemm_ar_allowed():
            checks["gemm_ar"] = gemm_ar
        if self.ll_max > 0:
            checks["ll"] = lambda: plain("ll", [n for n in self.LL_SIZES if n <= self.ll_max] or [self.ll_max], True)
        if self.resid_ll:
            checks["ll_resid"] = lambda: resid("ll_resid", True)
        if self.world >= 4 and self._two_shot(1 << 20):
            checks["two_shot"] = lambda: plain("two_shot", (1 << 20,), False)
        self.set_timeout(self.WARMUP_TIMEOUT_S)
        for name, fn in checks.items():
            try:
                ok = int(fn() and self.timeouts() == 0)
            except Exception as e:  # noqa: BLE001 - a protocol that raises is a failed protocol
                log.warning("custom all-reduce self-test %s raised: %s", name, e)
                ok = 0
            self.reset_errors()
            flag = torch.tensor([ok], dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=cpu_group)
            res[name] = bool(flag.item())
        self.set_timeout(self.serve_timeout())
        if res["ll"] is False or res["ll_resid"] is False:
            log.warning("custom all-reduce: push (LL) protocol disagreed with RCCL on this node (%s); "
                        "using the pull kernels", res)
            self.ll_max = 0
            self.resid_ll = False
        if res["two_shot"] is False:
            self.two_shot_min = self.slot2 + 1  # one-shot up to its slot, RCCL above
        # the all-reduce inside the row-parallel GEMMs only once it agreed with RCCL
        self.gemm_ar = self._gemm_ar if res["gemm_ar"] else None
        if res["gemm_ar"] is False:
            log.warning("custom all-reduce: the GEMM-fused all-reduce disagreed with RCCL; separate launches")
        self.verified = res
        self.verified_counts = {k: (counts[k] if res[k] is not None else None) for k in res}
        return res

    def protocol(self) -> str:
        """The decode all-reduce protocol in use: "ll" (push) or "pull"."""
        return "ll" if self.resid_ll else "pull"

    def serve_timeout(self, seconds: Optional[float] = None) -> float:
        """The peer-wait limit while serving: `seconds` (the configured collective
        timeout, default SERVE_TIMEOUT_S), at least 10 s when the ranks share one GPU
        (test boxes: up to 8 processes time-share its queues, so a live peer can be
        descheduled that long)."""
        s = self.SERVE_TIMEOUT_S if seconds is None else seconds
        return max(s, 10.0) if getattr(self, "shared_device", False) else s

    def set_timeout(self, seconds: float) -> None:
        """Peer-wait limit of every later launch (stream-ordered; captured graphs read
        the word at replay). Clamped to the 32-bit tick range."""
        ticks = int(min(max(seconds, 1e-3) * self._khz * 1000, 0x7FFFFFFF))
        self.ctl[1].fill_(ticks)
        self.timeout_s = float(seconds)

    def reset_errors(self) -> None:
        self.err.zero_()

    def timeouts(self) -> int:
        """Peer-wait timeouts recorded by the kernels (0 when healthy). Synchronises."""
        return int(self.err.item())

    def poll_async(self) -> None:
        """Queue a copy of the error counter behind the current stream's work."""
        self.h_err.copy_(self.err, non_blocking=True)

    def check(self) -> None:
        """Raise if any wait timed out up to the last poll_async whose stream work has
        completed (call after synchronising on the step)."""
        n = int(self.h_err[0])
        if n:
            raise CustomAllReduceTimeout(f"custom all-reduce: {n} peer wait(s) timed out on TP rank {self.rank} "
                                         "(a peer is dead or stalled); failing the step")

    def close(self) -> None:
        for p in self._opened:
            self._k.car_ipc_close(p)
        self._opened = []
        for p in (self.data, self.sig):
            if p:
                self._k.car_free(p)
        self.data = self.sig = 0


def maybe_enable(state, device: torch.device, ar_shapes=None) -> Optional[CustomAllReduce]:
    """Register the custom all-reduce for this TP group (GPU, 2..8 ranks), unless
    XGS_CUSTOM_AR=0. Falls back to RCCL on any setup failure. ar_shapes: the model's
    row-parallel (N, K) projection shards (self_test replays them)."""
    import os
    from . import comm
    if state.tp_size < 2 or device.type != "cuda" or os.environ.get("XGS_CUSTOM_AR", "1") == "0":
        return None
    try:
        ar = CustomAllReduce(state.tp_rank, state.tp_size, device, cpu_group=state.tp_cpu_group)
    except Exception as e:  # noqa: BLE001 - RCCL remains correct
        log.warning("custom all-reduce unavailable (%s); using RCCL", e)
        return None
    res = ar.self_test(state.tp_group, state.tp_cpu_group, ar_shapes)
    if not (res["pull"] and res["pull_resid"]):
        log.warning("custom all-reduce: pull kernels disagreed with RCCL (%s); using RCCL", res)
        ar.close()
        return None
    comm.register_custom_allreduce(ar)
    return ar
