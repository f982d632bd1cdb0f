set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/r2_bench_default.log 2>&1 && \
timeout -k 10 200 python -u bench.py --concurrency 1 --steps 200 --warmup 20 > gpurun_out/r2_bench_c1.log 2>&1
echo rc=$?
tail -n 3 gpurun_out/r2_gputests.log; tail -n 2 gpurun_out/r2_bench_default.log gpurun_out/r2_bench_c1.log
