# batched-load argmax + optional gemm_m64g LM head (XGS_LMHEAD_M64) -- tests + A/B (c64, c1)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u bench/kernel_bench.py --what sampling > gpurun_out/r2_sampling_kb.jsonl 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "argmax or sample" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_lmh_tests.log 2>&1 || exit 1
tail -n 1 gpurun_out/r2_lmh_tests.log
XGS_LMHEAD_M64=1 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_lmh_tests2.log 2>&1 || exit 1
tail -n 1 gpurun_out/r2_lmh_tests2.log
for rep in 1 2; do
for v in 0 1; do
XGS_LMHEAD_M64=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > gpurun_out/r2_lmh_c64_$v.log 2>&1 || exit 1
echo "c64 lmhead_m64=$v $(tail -n 1 gpurun_out/r2_lmh_c64_$v.log | cut -c60-200)"
XGS_LMHEAD_M64=$v timeout -k 10 200 python -u bench.py --concurrency 1 --steps 200 --warmup 20 > gpurun_out/r2_lmh_c1_$v.log 2>&1 || exit 1
echo "c1 lmhead_m64=$v $(tail -n 1 gpurun_out/r2_lmh_c1_$v.log | cut -c60-200)"
done
done
