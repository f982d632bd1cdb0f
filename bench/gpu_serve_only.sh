set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
XGS_STEP_TIMING=1 timeout -k 10 400 python -u bench/serve_bench.py --launch "--model llama3-8b --max-num-seqs 64 ${SERVE_EXTRA:-}" --concurrency 64 --prompt-len 512 --output-len 256 --warmup 40 --duration 40 --out gpurun_out/r2_serve_8b_c64.jsonl > gpurun_out/r2_serve_8b_c64.log 2>&1
rc=$?
tail -n 3 gpurun_out/r2_serve_8b_c64.log
exit $rc
