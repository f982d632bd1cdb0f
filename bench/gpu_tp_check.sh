# TP fused decode path: custom all-reduce / resid / gather kernels, TP engine tests, one-rank TP8 shard sim bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_custom_ar_gpu.py tests/test_tp_gpu.py > gpurun_out/r2_tp_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20 > gpurun_out/r2_tp8sim_c1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model llama3-70b --tp-shard 8 --steps 60 --warmup 20 > gpurun_out/r2_tp8sim_c64.log 2>&1
rc=$?
tail -n 25 gpurun_out/r2_tp_tests.log
tail -n 1 gpurun_out/r2_tp8sim_c1.log gpurun_out/r2_tp8sim_c64.log
exit $rc
