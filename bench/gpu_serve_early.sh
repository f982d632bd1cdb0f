# serve path: overlap-window outputs sent to the server before the GPU step in flight finishes (XGS_EARLY_OUTPUTS): A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/serve_early; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_server_process.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || { tail -n 20 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
for v in 1 0; do
XGS_EARLY_OUTPUTS=$v timeout -k 10 400 python -u bench/serve_bench.py --launch "--model llama3-8b --max-num-seqs 64" --concurrency 64 --prompt-len 512 --output-len 256 --warmup 30 --duration 40 --out $o/serve_e$v.jsonl > $o/serve_e$v.log 2>&1 || exit 1
python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["value"], d["ttft_p50_ms"], d["ttft_p99_ms"], d["client_itl_p50_ms"], d["client_itl_p99_ms"], d["token_delivery_ms"])' $o/serve_e$v.jsonl early=$v
done
