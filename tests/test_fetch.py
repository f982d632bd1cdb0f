"""Remote checkpoints (Req 10.2): an http:// checkpoint directory served by a
local http.server (no external network) is fetched into the cache by
load_config and loads to the same weights as the local directory; an unreachable
URL is a configuration error naming the URL, and `check-config` exits 2 on it."""
import functools
import http.server
import os
import subprocess
import sys
import threading
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture()
def served_checkpoint(tmp_path):
    from xgserve.models import build_model, get_config, save_checkpoint
    ck = tmp_path / "ck"
    model = build_model(get_config("llama-tiny"), "cpu", torch.float32, seed=7)
    save_checkpoint(model, str(ck))
    handler = functools.partial(http.server.SimpleHTTPRequestHandler, directory=str(tmp_path))
    handler.log_message = lambda *a, **k: None
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), handler)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    try:
        yield f"http://127.0.0.1:{srv.server_address[1]}/ck", ck, model
    finally:
        srv.shutdown()


def test_url_checkpoint_fetched_and_loaded(served_checkpoint, tmp_path, monkeypatch):
    url, local, model = served_checkpoint
    monkeypatch.setenv("XGS_CHECKPOINT_CACHE", str(tmp_path / "cache"))
    from xgserve.server.config import load_config
    cfg = load_config(env={}, overrides={"worker": {"checkpoint": url, "random_init": False, "device": "cpu"}})
    d = cfg.worker.checkpoint
    assert d.startswith(str(tmp_path / "cache")) and os.path.exists(os.path.join(d, ".complete"))
    for name in os.listdir(local):
        assert (Path(d) / name).read_bytes() == (local / name).read_bytes(), name
    from xgserve.models import build_model, get_config
    m2 = build_model(get_config(d), "cpu", torch.float32, checkpoint=d)
    sd1, sd2 = model.state_dict(), m2.state_dict()
    assert sd1.keys() == sd2.keys()
    for k in sd1:
        assert torch.equal(sd1[k], sd2[k]), k
    # a second start reuses the cache (no server needed)
    from xgserve.models.fetch import fetch_checkpoint
    assert fetch_checkpoint(url) == d


def test_unreachable_url_is_a_config_error(tmp_path, monkeypatch):
    monkeypatch.setenv("XGS_CHECKPOINT_CACHE", str(tmp_path / "cache"))
    from xgserve.core.errors import ConfigError
    from xgserve.server.config import load_config
    with pytest.raises(ConfigError, match="cannot fetch http://127.0.0.1:9/nope"):
        load_config(env={}, overrides={"worker": {"checkpoint": "http://127.0.0.1:9/nope", "random_init": False}})


def test_missing_file_on_server_is_a_config_error(served_checkpoint, tmp_path, monkeypatch):
    url, _, _ = served_checkpoint
    monkeypatch.setenv("XGS_CHECKPOINT_CACHE", str(tmp_path / "cache"))
    from xgserve.core.errors import ConfigError
    from xgserve.server.config import load_config
    with pytest.raises(ConfigError, match="HTTP 404"):
        load_config(env={}, overrides={"worker": {"checkpoint": url + "-missing", "random_init": False}})


def test_cli_exit_code_on_bad_url(tmp_path):
    env = dict(os.environ, XGS_CHECKPOINT_CACHE=str(tmp_path / "cache"))
    p = subprocess.run([sys.executable, "-m", "xgserve", "check-config", "--checkpoint", "http://127.0.0.1:9/x"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "cannot fetch" in p.stderr


def test_index_server_error_is_not_read_as_unsharded(tmp_path, monkeypatch):
    """Only a 404 on model.safetensors.index.json means "one file": a 5xx on the index
    of a sharded checkpoint is reported as itself, and no .part file stays behind."""
    import json as _json
    d = tmp_path / "srv"
    d.mkdir()
    (d / "config.json").write_text(_json.dumps({"model_type": "llama"}))

    class H(http.server.SimpleHTTPRequestHandler):
        def __init__(self, *a, **k):
            super().__init__(*a, directory=str(d), **k)

        def log_message(self, *a, **k):
            pass

        def do_GET(self):  # noqa: N802
            if self.path.endswith("model.safetensors.index.json"):
                self.send_response(503)
                self.send_header("Content-Length", "0")
                self.end_headers()
                return
            super().do_GET()

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    from xgserve.models.fetch import FetchError, fetch_checkpoint
    cache = tmp_path / "cache"
    try:
        with pytest.raises(FetchError, match="HTTP 503") as ei:
            fetch_checkpoint(f"http://127.0.0.1:{srv.server_address[1]}/", root=str(cache))
        assert ei.value.status == 503
    finally:
        srv.shutdown()
    assert not list(cache.rglob("*.part"))
