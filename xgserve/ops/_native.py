"""Loader for the native kernel library (xgserve._kernels, built for gfx950).

Policy (fail loudly): a GPU tensor is only ever processed by the HIP kernels.
If the extension is missing or fails to import while a GPU op is requested we
raise -- there is no silent fall-back to PyTorch ops on the device. CPU tensors
use the PyTorch reference implementations (CPU tests, GPT-2 CPU plumbing
config). Set XGS_ALLOW_TORCH_FALLBACK=1 only for debugging.
"""
from __future__ import annotations

import os

import torch

_K = None
_ERR = None


def kernels():
    """Return the loaded xgserve._kernels module (raises if unavailable)."""
    global _K, _ERR
    if _K is not None:
        return _K
    if _ERR is not None:
        raise RuntimeError(f"xgserve._kernels unavailable: {_ERR}")
    try:
        from .. import _kernels as k  # noqa: WPS433
        # weight-streaming GEMMs: K-chunk rotation policy (csrc/kernels/gemm_m64g.hip
        # k_rotation; XGS_TUNE krot: 0 never, 1 grids of split <= 2 (default), 2 always)
        from .. import tune
        k.set_k_rotation(tune.get_int("krot", 1))
        _K = k
        return k
    except Exception as e:  # pragma: no cover - depends on build
        _ERR = repr(e)
        raise RuntimeError(
            "xgserve._kernels (HIP/gfx950) is not built or failed to load: "
            f"{e!r}. Run `python -m xgserve._build`.") from e


def available() -> bool:
    try:
        kernels()
        return True
    except RuntimeError:
        return False


def use_native(t: torch.Tensor) -> bool:
    """True when `t` lives on the GPU (native path mandatory)."""
    if t.device.type != "cuda":
        return False
    if os.environ.get("XGS_ALLOW_TORCH_FALLBACK") == "1" and not available():
        return False
    return True


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()
