set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
XGS_STEP_TIMING=1 timeout -k 10 300 python -u bench.py --steps 3000 --warmup 100 > gpurun_out/r2_bench_long_timing.log 2>&1
rc=$?
tail -n 1 gpurun_out/r2_bench_long_timing.log
exit $rc
