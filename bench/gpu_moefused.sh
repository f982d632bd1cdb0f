# fused MoE decode layer: tests + Mixtral A/B (XGS_FUSED_MOE_DECODE) at c64 / c1 + TP2 shard sim
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_fused_decode_gpu.py tests/test_tp_gpu.py tests/test_kernels_gpu.py -k "moe or mixtral or tp2" -x -q --timeout 240 --timeout-method thread > gpurun_out/r2_moefused_tests.log 2>&1 || { tail -n 30 gpurun_out/r2_moefused_tests.log; exit 1; }
for v in 1 0; do
XGS_FUSED_MOE_DECODE=$v XGS_STEP_LOG=gpurun_out/r2_moefused_steps_$v.jsonl timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > gpurun_out/r2_moefused_c64_$v.log 2>&1 || exit 1
echo "c64 fused=$v $(tail -n 1 gpurun_out/r2_moefused_c64_$v.log | cut -c100-140)"
XGS_FUSED_MOE_DECODE=$v timeout -k 10 300 python -u bench.py --model mixtral-8x7b --concurrency 1 --steps 100 --warmup 10 > gpurun_out/r2_moefused_c1_$v.log 2>&1 || exit 1
echo "c1 fused=$v $(tail -n 1 gpurun_out/r2_moefused_c1_$v.log | cut -c100-140)"
done
XGS_FUSED_MOE_DECODE=1 timeout -k 10 300 python -u bench.py --model mixtral-8x7b --tp-shard 2 --steps 60 --warmup 20 > gpurun_out/r2_moefused_tp2sim.log 2>&1 && \
echo "tp2sim c64 fused $(tail -n 1 gpurun_out/r2_moefused_tp2sim.log | cut -c100-140)"
tail -n 2 gpurun_out/r2_moefused_tests.log
