"""K7 token-embedding gather and K11 embeddings-output normalisation on the device
(csrc/kernels/norm.hip embed_gather, csrc/kernels/sampling.hip mean_l2norm_rows)."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from ._native import kernels, stream_ptr, use_native


def embed_gather(ids: torch.Tensor, table: torch.Tensor, ss: Optional[torch.Tensor] = None) -> torch.Tensor:
    """table[ids] ([T, H] bf16); with `ss` (fp32, >= T) also ss[t] = sum of squares of
    row t -- the first RMSNorm statistic of the fused decode layer, same launch.
    Ids outside [0, V) give zero rows."""
    T = ids.shape[0]
    V, H = table.shape
    if not use_native(table) or table.dtype != torch.bfloat16:
        out = F.embedding(ids.long().clamp(0, V - 1), table)
        out[(ids < 0) | (ids >= V)] = 0
        if ss is not None:
            ss.view(-1)[:T] = out.float().pow(2).sum(-1)
        return out
    assert ids.dtype == torch.int32 and ids.is_contiguous() and table.is_contiguous()
    out = torch.empty(T, H, dtype=table.dtype, device=table.device)
    kernels().embed_gather(ids.data_ptr(), T, table.data_ptr(), V, H, out.data_ptr(),
                           0 if ss is None else ss.data_ptr(), stream_ptr())
    return out


def mean_l2norm_rows(acc: torch.Tensor, rows: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    """Embeddings output (mean pooling + L2): out[i] = normalize(acc[rows[i]] / counts[i]);
    the accumulator rows are re-zeroed. acc fp32 [R, H]; rows / counts int32 [n]."""
    n, H = rows.shape[0], acc.shape[1]
    if not use_native(acc):
        v = acc[rows.long()] / counts.clamp_min(1).to(acc.dtype)[:, None]
        out = v / v.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        acc[rows.long()] = 0
        return out
    assert acc.dtype == torch.float32 and acc.is_contiguous()
    out = torch.empty(n, H, dtype=torch.float32, device=acc.device)
    kernels().mean_l2norm_rows(acc.data_ptr(), rows.data_ptr(), counts.data_ptr(), out.data_ptr(), n, H,
                               stream_ptr())
    return out
