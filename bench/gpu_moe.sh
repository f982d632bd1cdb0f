set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "moe" > gpurun_out/r2_moe_tests.log 2>&1 && \
timeout -k 10 300 python -u bench/gemm_bench.py --moe-sweep --M 1 8 32 64 > gpurun_out/r2_moe_sweep.jsonl 2> gpurun_out/r2_moe_sweep.err && \
timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > gpurun_out/r2_mixtral_c64.log 2>&1 && \
XGS_MOE_ROW_DISPATCH=0 timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > gpurun_out/r2_mixtral_c64_norow.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model mixtral-8x7b --concurrency 1 --steps 100 --warmup 10 > gpurun_out/r2_mixtral_c1.log 2>&1
rc=$?
tail -n 2 gpurun_out/r2_moe_tests.log; tail -n 1 gpurun_out/r2_mixtral_c64.log gpurun_out/r2_mixtral_c64_norow.log gpurun_out/r2_mixtral_c1.log
exit $rc
