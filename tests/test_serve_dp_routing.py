"""The serving path bench/scale.sh measures on an 8-GPU node (serve_dp$n), rehearsed on
the CPU: `xgserve serve --mock --replicas 8 --frontends 2` -- eight PROCESS replicas
behind the C++ least-loaded router and two HTTP front-end processes -- driven by
bench/serve_bench.py's closed-loop SSE clients (64 streams). Checks the JSON line
contract the scaling sheet reads and that the router spreads the requests evenly:
every replica within +-10 % of the mean (Req 6.1 / 7.1, BASELINE north star
"per-request routing across the 8 GPUs of one node")."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_eight_process_replicas_through_router_and_front_ends():
    launch = ("--mock --replicas 8 --frontends 2 --log-level WARNING --set worker.in_process=false "
              "--set worker.mock_latency_ms=4")
    cmd = [sys.executable, "bench/serve_bench.py", "--launch", launch, "--concurrency", "64", "--prompt-len", "32",
           "--output-len", "8", "--warmup", "3", "--duration", "8", "--procs", "2", "--ready-timeout", "240",
           "--label", "serve_dp8_mock"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=420)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, (p.returncode, p.stdout[-2000:], p.stderr[-3000:])
    r = json.loads(lines[0])
    # the contract bench/scale.sh's summary reads
    for key in ("metric", "value", "unit", "ttft_p50_ms", "ttft_p99_ms", "requests_completed", "errors",
                "replica_requests", "label"):
        assert key in r, key
    assert r["metric"] == "serve_output_tokens_per_sec" and r["label"] == "serve_dp8_mock"
    assert r["errors"] == 0 and r["value"] > 0 and r["requests_completed"] > 100, r
    split = r["replica_requests"]["per_replica"]
    assert sorted(split) == [str(i) for i in range(8)], split
    mean = sum(split.values()) / 8
    assert all(abs(v - mean) <= 0.1 * mean for v in split.values()), split
    assert r["replica_requests"]["imbalance"] <= 0.1
