# in-launch residual reduce at 16 < M <= 64 (tall per-tile statistics): tests + c64 A/B on the threshold
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_fused_decode_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_resid64_tests.log 2>&1 && \
for b in 32768 65536 262144 32768; do
XGS_RESID_INLAUNCH_MAX_BYTES=$b timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > gpurun_out/r2_resid64_b$b.log 2>&1 || exit 1
tail -n 1 gpurun_out/r2_resid64_b$b.log | cut -c1-140
done
echo rc=$?
tail -n 2 gpurun_out/r2_resid64_tests.log
