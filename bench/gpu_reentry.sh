set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s5_gputests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2s5_smoke.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2s5_bench_driver.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > gpurun_out/r2s5_bench_200.log 2>&1 && \
timeout -k 10 200 python -u bench.py --concurrency 1 --steps 200 --warmup 20 > gpurun_out/r2s5_bench_c1.log 2>&1 && \
export TMPDIR=/tmp && \
bash bench/profile.sh gpurun_out/prof_r2s5_c64 && \
bash bench/profile.sh gpurun_out/prof_r2s5_c1 --concurrency 1
rc=$?
echo rc=$rc
tail -n 3 gpurun_out/r2s5_gputests.log; tail -n 2 gpurun_out/r2s5_smoke.log gpurun_out/r2s5_bench_*.log
exit $rc
