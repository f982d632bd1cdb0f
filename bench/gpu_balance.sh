# decode attention: length-balanced workgroup order (XGS_DECODE_BALANCE 0/1/2) -- tests + kernel bench + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 1 2; do
XGS_DECODE_BALANCE=$v timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_decode_gpu.py tests/test_engine_gpu.py -k "decode or attention or greedy" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_bal_tests_$v.log 2>&1 || exit 1
tail -n 1 gpurun_out/r2_bal_tests_$v.log
done
for v in 0 1 2; do
XGS_DECODE_BALANCE=$v timeout -k 10 200 python -u bench/kernel_bench.py --what decode > gpurun_out/r2_bal_kb_$v.jsonl 2>&1 || exit 1
done
for rep in 1 2; do
for v in 0 2 1; do
XGS_DECODE_BALANCE=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > gpurun_out/r2_bal_c64_$v.log 2>&1 || exit 1
echo "c64 balance=$v $(tail -n 1 gpurun_out/r2_bal_c64_$v.log | cut -c60-160)"
done
done
