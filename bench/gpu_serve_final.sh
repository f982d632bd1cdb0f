# end-of-round serve path (HTTP/SSE, 64 concurrent) and the long steady-state in-process reference
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/serve_final; mkdir -p $o
timeout -k 10 300 python -u bench.py --steps 3000 --warmup 100 > $o/bench_long.log 2>&1 && \
tail -n 1 $o/bench_long.log | cut -c1-220 && \
timeout -k 10 400 python -u bench/serve_bench.py --launch "--model llama3-8b --max-num-seqs 64" --concurrency 64 --prompt-len 512 --output-len 256 --warmup 40 --duration 40 --out $o/serve_8b_c64.jsonl > $o/serve.log 2>&1
rc=$?
tail -n 3 $o/serve.log
exit $rc
