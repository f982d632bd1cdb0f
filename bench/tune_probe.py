#!/usr/bin/env python3
"""TunableOp re-tune of the continuous-batching mixed-step projections (M = 575) under
the current environment (e.g. HIPBLASLT_WORKSPACE_SIZE): prints the tuned solution and
time per shape from the CSV TunableOp writes (PYTORCH_TUNABLEOP_FILENAME)."""
import os
import sys

import torch
import torch.nn.functional as F


def main():
    out = os.environ["PYTORCH_TUNABLEOP_FILENAME"]
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_filename(out)
    torch.cuda.tunable.set_max_tuning_duration(60)
    dev = "cuda"
    for N, K in ((28672, 4096), (6144, 4096), (4096, 4096)):
        x = torch.randn(575, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
        F.linear(x, w)
        torch.cuda.synchronize()
    torch.cuda.tunable.write_file()
    for line in open(torch.cuda.tunable.get_filename()):
        if "_575_" in line:
            print(line.strip(), flush=True)


if __name__ == "__main__":
    sys.exit(main())
