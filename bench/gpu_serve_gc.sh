# serve path with / without the server GC tuning (XGS_SERVER_GC): delivery delay (Req 5.1) A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/serve_gc; mkdir -p $o
for v in 1 0; do
XGS_SERVER_GC=$v timeout -k 10 400 python -u bench/serve_bench.py --launch "--model llama3-8b --max-num-seqs 64" --concurrency 64 --prompt-len 512 --output-len 256 --warmup 30 --duration 40 --out $o/serve_gc$v.jsonl > $o/serve_gc$v.log 2>&1 || exit 1
python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["value"], d["ttft_p50_ms"], d["token_delivery_ms"], d["event_loop_lag_ms"]["p99"], d["event_loop_lag_ms"]["max"])' $o/serve_gc$v.jsonl gc=$v
done
