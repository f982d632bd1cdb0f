"""Infinity-Cache warm-up of a weight range (csrc/kernels/prefetch.hip)."""
from __future__ import annotations

import torch

from ._native import kernels, stream_ptr

PREFETCH_BLOCKS = 128  # half the CUs: the attention it runs beside holds the rest


def mall_prefetch(w: torch.Tensor, nbytes: int, sink: torch.Tensor, blocks: int = PREFETCH_BLOCKS) -> None:
    """Read the first nbytes of w once (16-B non-temporal loads, results discarded)."""
    nbytes = min(int(nbytes), w.numel() * w.element_size()) // 16 * 16
    if nbytes > 0:
        kernels().mall_prefetch(w.data_ptr(), nbytes, blocks, sink.data_ptr(), stream_ptr())
