"""Command line: `python -m xgserve <command>`.

  serve             start the HTTP server (config: file < XGS_* env < CLI, Req 10.1)
  generate          offline generation with one engine (no HTTP)
  check-config      load + validate a configuration and print it (exit 2 on error)
  models            list the built-in model configurations

Invalid configuration prints every error and exits with status 2 (Req 10.4);
a replica that fails to load exits with status 3.
"""
from __future__ import annotations

import argparse
import json
import logging
import sys
from typing import List, Optional

from .core.errors import ApiError, ConfigError


def _common(p: argparse.ArgumentParser) -> None:
    p.add_argument("--config", help="TOML / JSON / YAML configuration file")
    p.add_argument("--set", action="append", default=[], metavar="SECTION.KEY=VALUE",
                   help="override any config key (repeatable)")
    p.add_argument("--host")
    p.add_argument("--port", type=int)
    p.add_argument("--model")
    p.add_argument("--checkpoint", help="safetensors checkpoint directory (HF layout)")
    p.add_argument("--tp", type=int, help="tensor-parallel degree per replica")
    p.add_argument("--replicas", type=int, help="data-parallel replicas")
    p.add_argument("--gpus", help="comma-separated GPU ids, e.g. 0,1,2,3")
    p.add_argument("--device", help="force a device, e.g. cpu")
    p.add_argument("--quantization", choices=["bf16", "fp16", "fp32", "fp8", "int8", "int4"],
                   help="fp8: E4M3 weights (per-channel scales) for batch <= 16 decode, bf16 activations")
    p.add_argument("--strategy", choices=["round_robin", "least_loaded", "memory_aware"])
    p.add_argument("--batch-mode", choices=["continuous", "static"])
    p.add_argument("--max-num-seqs", type=int)
    p.add_argument("--max-model-len", type=int)
    p.add_argument("--mock", action="store_true", default=None, help="deterministic mock engine")
    p.add_argument("--in-process", action="store_true", default=None, help="engine thread in the server process")
    p.add_argument("--no-graphs", action="store_true", default=None)
    p.add_argument("--draft-model", help="speculative decoding draft model")
    p.add_argument("--num-speculative-tokens", type=int)
    p.add_argument("--log-level")
    p.add_argument("--frontends", type=int, help="HTTP front-end processes over one orchestrator")


def _overrides(a) -> dict:
    return {
        "api": {"host": a.host, "port": a.port, "frontends": getattr(a, "frontends", None)},
        "worker": {"model": a.model, "checkpoint": a.checkpoint, "tp": a.tp, "replicas": a.replicas, "gpus": a.gpus,
                   "device": a.device, "quantization": a.quantization, "max_num_seqs": a.max_num_seqs,
                   "max_model_len": a.max_model_len, "mock": a.mock, "in_process": a.in_process,
                   "use_graphs": (False if a.no_graphs else None),
                   "random_init": (False if a.checkpoint else None)},
        "scheduler": {"strategy": a.strategy},
        "batcher": {"mode": a.batch_mode},
        "spec": {"draft_model": a.draft_model, "num_speculative_tokens": a.num_speculative_tokens},
        "observability": {"log_level": a.log_level},
    }


def load(a):
    from .server.config import load_config
    return load_config(a.config, cli=a.set, overrides=_overrides(a))


def cmd_serve(a) -> int:
    cfg = load(a)
    logging.basicConfig(level=cfg.observability.log_level.upper(),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    from .server.app import serve
    from .server.orchestrator import InferenceServer
    try:
        nfe = cfg.api.resolved_frontends(cfg.worker)
        if nfe > 1:
            import asyncio
            from .server.frontend import run_hub
            asyncio.run(run_hub(InferenceServer(cfg), nfe))
        else:
            serve(InferenceServer(cfg))
    except ApiError as e:
        print(f"startup failed: {e.message}", file=sys.stderr)
        return 3
    return 0


def cmd_generate(a) -> int:
    cfg = load(a)
    logging.basicConfig(level=cfg.observability.log_level.upper())
    from .engine import SamplingParams
    from .server.replica import engine_spec, make_engine
    spec = engine_spec(cfg.worker, cfg.cache, cfg.spec)
    eng = make_engine(spec)
    ids = eng.tokenizer.encode(a.prompt)
    out = eng.generate([ids], SamplingParams(max_tokens=a.max_tokens, temperature=a.temperature))[0]
    print(json.dumps({"prompt_tokens": len(ids), "output_ids": out, "text": eng.tokenizer.decode(out)}))
    return 0


def cmd_check_config(a) -> int:
    cfg = load(a)
    print(json.dumps(cfg.to_dict(), indent=2))
    return 0


def cmd_models(a) -> int:
    from .models import get_config, list_models
    for n in list_models():
        c = get_config(n)
        print(f"{n:20s} layers={c.num_layers} hidden={c.hidden_size} heads={c.num_heads}/{c.num_kv_heads} "
              f"vocab={c.vocab_size} experts={c.num_experts}")
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="xgserve", description="MI355X-native distributed LLM inference server")
    sub = ap.add_subparsers(dest="cmd")
    ps = sub.add_parser("serve", help="run the HTTP server")
    _common(ps)
    pg = sub.add_parser("generate", help="offline generation")
    _common(pg)
    pg.add_argument("--prompt", required=True)
    pg.add_argument("--max-tokens", type=int, default=32)
    pg.add_argument("--temperature", type=float, default=0.0)
    pc = sub.add_parser("check-config", help="validate configuration")
    _common(pc)
    sub.add_parser("models", help="list model configurations")
    a = ap.parse_args(argv)
    if a.cmd is None:
        ap.print_help()
        return 1
    try:
        return {"serve": cmd_serve, "generate": cmd_generate, "check-config": cmd_check_config,
                "models": cmd_models}[a.cmd](a)
    except ConfigError as e:
        print(str(e), file=sys.stderr)
        return 2


if __name__ == "__main__":
    sys.exit(main())
