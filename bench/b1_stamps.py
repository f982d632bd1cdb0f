#!/usr/bin/env python3
"""Where a persistent batch-1 decode step spends its time (csrc/kernels/decode_b1.hip
with in-kernel phase clocks): Llama-3-8B (random init, full depth), one sequence,
prompt --prompt-len, eager steps; prints one JSON line with, per phase, the mean / max
over the 256 workgroups of its time summed over layers, plus the loader's ring-full
stall and the consumers' ring-line waits."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--steps", type=int, default=8)
    a = ap.parse_args()
    import xgserve.models.llama as ll
    ll.PERSISTENT_DECODE = True
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
    from xgserve.models import build_model, get_config
    model = build_model(get_config(a.model), device="cuda:0", seed=1)
    eng = LLMEngine(EngineConfig(model=a.model, device="cuda:0", num_blocks=1024, max_num_seqs=4,
                                 max_num_batched_tokens=8192, max_model_len=a.prompt_len + 64, use_graphs=False),
                    model=model)
    prompt = [128000] + [(31 * i + 7) % 120000 for i in range(a.prompt_len - 1)]
    eng.add_request("r", prompt, SamplingParams(max_tokens=32, temperature=0.0, ignore_eos=True))
    reports = {}
    modes = {0: "full", 1: "loader alone (consumers ignore the ring)", 2: "consumers alone (no weight loads)",
             5: "loader alone, no projection work", 9: "loader alone, consumers exit"}
    for _ in range(3):
        eng.step()
    dec = model._b1
    dec.enable_stamps()
    for m in (0, 1, 2, 5, 9):
        torch.cuda.synchronize()
        dec.ctl[3].fill_(m)
        for _ in range(3):  # async scheduling: the mode is live from the second step on
            eng.step()
        torch.cuda.synchronize()
        reports[modes[m]] = dec.stamp_report()
    dec = model._b1
    dec.ctl[3].zero_()
    for name, rep in reports.items():
        print(json.dumps({"model": a.model, "prompt_len": a.prompt_len, "L": dec.L, "ring_lines": dec.plan[2],
                          "mode": name, "phases_us": {k: [round(v[0], 1), round(v[1], 1)] for k, v in rep.items()},
                          "timeouts": dec.timeouts()}))


if __name__ == "__main__":
    main()
