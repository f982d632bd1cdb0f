set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_tp_gpu.py tests/test_fused_decode_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r2_fq_tests.log 2>&1 && \
XGS_STEP_LOG=gpurun_out/r2_fq_steps.jsonl timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > gpurun_out/r2_fq_mixtral.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model mixtral-8x7b --concurrency 1 --steps 100 --warmup 10 > gpurun_out/r2_fq_mixtral_c1.log 2>&1
rc=$?
tail -n 2 gpurun_out/r2_fq_tests.log
tail -n 1 gpurun_out/r2_fq_mixtral.log | cut -c1-200; tail -n 1 gpurun_out/r2_fq_mixtral_c1.log | cut -c1-200
exit $rc
