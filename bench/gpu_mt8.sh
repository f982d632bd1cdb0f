# grouped MoE GEMM 128-row tile pairs for prefill-sized steps: tests + Mixtral c64 A/B (XGS_M64G_MT8) + w2 cfg
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "moe" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_mt8_tests.log 2>&1 && \
for v in 1 0; do
XGS_M64G_MT8=$v XGS_STEP_LOG=gpurun_out/r2_mt8_steps_$v.jsonl timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > gpurun_out/r2_mt8_$v.log 2>&1 || exit 1
echo "mt8=$v $(tail -n 1 gpurun_out/r2_mt8_$v.log | cut -c1-150)"
done
XGS_MOE_CFG_W2_PREFILL=3 timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > gpurun_out/r2_mt8_w2c3.log 2>&1 && \
echo "mt8=1 w2cfg3 $(tail -n 1 gpurun_out/r2_mt8_w2c3.log | cut -c1-150)"
rc=$?
tail -n 2 gpurun_out/r2_mt8_tests.log
exit $rc
