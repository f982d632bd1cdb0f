# host step wait: event polling (XGS_SPIN_WAIT=1) vs blocking synchronize -- A/B c64 / c1 + tests
set -o pipefail
cd $GRAFT_REPO_ROOT
XGS_SPIN_WAIT=1 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_spin_tests.log 2>&1 || exit 1
tail -n 1 gpurun_out/r2_spin_tests.log
for rep in 1 2; do
for v in 0 1; do
XGS_SPIN_WAIT=$v XGS_STEP_TIMING=1 timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > gpurun_out/r2_spin_c64_$v.log 2>&1 || exit 1
echo "c64 spin=$v $(tail -n 1 gpurun_out/r2_spin_c64_$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ttft_p50_ms"], d["detail"].get("host_ms_per_step"))')"
XGS_SPIN_WAIT=$v timeout -k 10 200 python -u bench.py --concurrency 1 --steps 200 --warmup 20 > gpurun_out/r2_spin_c1_$v.log 2>&1 || exit 1
echo "c1 spin=$v $(tail -n 1 gpurun_out/r2_spin_c1_$v.log | cut -c1-80)"
XGS_SPIN_WAIT=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_spin_drv_$v.log 2>&1 || exit 1
echo "drv spin=$v $(tail -n 1 gpurun_out/r2_spin_drv_$v.log | cut -c1-80)"
done
done
