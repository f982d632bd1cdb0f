# new kernel tests, default bench (regression check), HTTP serve path at 64 concurrent on one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_decode_gpu.py tests/test_engine_gpu.py > gpurun_out/r2_kern_tests.log 2>&1 && \
timeout -k 10 240 python -u bench.py > gpurun_out/r2_bench_default2.log 2>&1 && \
timeout -k 10 400 python -u bench/serve_bench.py --launch "--model llama3-8b --max-num-seqs 64" --concurrency 64 --prompt-len 512 --output-len 256 --warmup 40 --duration 40 --out gpurun_out/r2_serve_8b_c64.jsonl > gpurun_out/r2_serve_8b_c64.log 2>&1
rc=$?
tail -n 3 gpurun_out/r2_kern_tests.log; tail -n 1 gpurun_out/r2_bench_default2.log; tail -n 2 gpurun_out/r2_serve_8b_c64.log
exit $rc
