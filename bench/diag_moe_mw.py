"""Diagnostic: decode-step logits of a 2-layer Mixtral / Llama vs the fp32 reference,
with the 64 < T <= 320 prompt step on gemm_mw or on the library GEMMs, fused and
unfused decode chains. Prints one line per case (relative L2 error, argmax match).

    python bench/diag_moe_mw.py
"""
import os
import sys
from dataclasses import replace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import xgserve.models.llama as ll  # noqa: E402
from xgserve.engine import EngineConfig, LLMEngine, SamplingParams  # noqa: E402
from xgserve.models import build_model, get_config  # noqa: E402
from xgserve.models.reference import reference_logits  # noqa: E402


def run(model, prompt, mw: int, fused: bool):
    ll.MW_MAX_TOKENS, ll.FUSED_DECODE = mw, fused
    eng = LLMEngine(EngineConfig(model=model.cfg.name, device="cuda:0", num_blocks=256, max_num_seqs=8,
                                 max_num_batched_tokens=1024, max_model_len=512, use_graphs=False), model=model)
    eng.runner.capture_logits = True
    eng.add_request("d", prompt, SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True))
    toks, logits = [], []
    while eng.has_work():
        for o in eng.step():
            toks += o.new_token_ids
        logits.append(eng.runner.last_logits[-1].clone())
    ref = reference_logits(model, prompt + toks[:1]).float().cpu()
    out = []
    for name, got, r in (("prefill", logits[0], ref[len(prompt) - 1]), ("decode", logits[-1], ref[-1])):
        out.append(f"{name} rel={float((got - r).norm() / r.norm()):.4f} argmax_ok={int(got.argmax()) == int(r.argmax())}")
    return " ".join(out)


def main():
    mw0 = ll.MW_MAX_TOKENS
    mix = replace(get_config("mixtral-8x7b"), num_layers=2, intermediate_size=1792, name="mixtral-2l")
    cases = [("mixtral", mix, 5, [1] + list(range(300, 380))),
             ("mixtral", mix, 5, [1] + list(range(1000, 1100, 2))[:90]),
             ("mixtral", mix, 5, [1] + list(range(5000, 5120))),
             ("llama", replace(get_config("llama3-8b"), num_layers=2, name="llama3-8b-2l"), 3,
              [128000] + list(range(700, 790)))]
    for name, cfg, seed, prompt in cases:
        model = build_model(cfg, device="cuda:0", seed=seed)
        for mw in (mw0, 0):
            for fused in ((True, False) if name == "llama" else (True,)):
                print(f"{name} T={len(prompt)} mw_max={mw} fused={fused}: {run(model, prompt, mw, fused)}",
                      flush=True)
        del model
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
