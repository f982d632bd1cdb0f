"""Shipped GEMM selection table for the library GEMMs (hipBLASLt / rocBLAS).

The prefill / mixed-step projections and the LM head go through torch.matmul ->
hipBLASLt, whose default heuristic picks one solution per shape. PyTorch's
TunableOp times every hipBLASLt and rocBLAS solution for a shape (rotating
buffers, i.e. cold operands as in a real step) and keeps the fastest; the table
`mi355x_gemm.csv` holds those choices for the shapes our benchmark configs issue
(`bash bench/gpu.sh tune` builds it on an MI355X; its validator rows pin the
PyTorch / HIP / hipBLASLt / rocBLAS versions and gfx950, and TunableOp ignores the
file on any mismatch). The engine only REPLAYS it (no tuning at serve time);
shapes not in the table keep the default heuristic. XGS_GEMM_TUNING=0 disables it
(A/B: profiles/r2_gemm_tuning_ab.md).
"""
from __future__ import annotations

import logging
import os
from pathlib import Path

import torch

TABLE = Path(__file__).with_name("mi355x_gemm.csv")
_log = logging.getLogger(__name__)
_state = {"loaded": None}


def enable_gemm_table(device: torch.device) -> bool:
    """Replay the shipped GEMM table for GEMMs on `device` (idempotent). Returns
    whether the table is active."""
    if _state["loaded"] is not None:
        return _state["loaded"]
    ok = False
    if (device.type == "cuda" and os.environ.get("XGS_GEMM_TUNING", "1") != "0" and TABLE.exists()
            and not os.environ.get("PYTORCH_TUNABLEOP_TUNING") == "1"):
        try:
            arch = torch.cuda.get_device_properties(device).gcnArchName
        except Exception:  # noqa: BLE001
            arch = ""
        if arch.startswith("gfx950"):
            import torch.cuda.tunable as tunable
            tunable.enable(True)
            tunable.tuning_enable(False)
            ok = bool(tunable.read_file(str(TABLE)))
            if not ok:
                tunable.enable(False)
                _log.warning("GEMM table %s rejected (version / arch mismatch); default heuristics", TABLE)
    _state["loaded"] = ok
    return ok
