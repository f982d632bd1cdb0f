# grouped MoE GEMM tile groups for prefill-sized steps: tests + Mixtral c64 A/B (pairs vs triples vs off)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "moe" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_mt8_tests.log 2>&1 && \
for v in 3 2; do
XGS_M64G_GROUP=$v XGS_STEP_LOG=gpurun_out/r2_grp_steps_$v.jsonl timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > gpurun_out/r2_grp_$v.log 2>&1 || exit 1
echo "group=$v $(tail -n 1 gpurun_out/r2_grp_$v.log | cut -c1-150)"
done
XGS_M64G_GROUP=3 timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > gpurun_out/r2_grp_3b.log 2>&1 && \
echo "group=3 again $(tail -n 1 gpurun_out/r2_grp_3b.log | cut -c1-150)"
rc=$?
tail -n 2 gpurun_out/r2_mt8_tests.log
exit $rc
