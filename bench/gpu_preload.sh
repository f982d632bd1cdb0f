# decode attention: first K/V tiles requested before the fused prologue -- tests + A/B (c1, c64)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_decode_gpu.py -k "decode or attention or o_projection" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_preload_tests.log 2>&1 || exit 1
for r in 1 2; do
for v in 1 0; do
XGS_DECODE_PRELOAD=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > gpurun_out/r2_preload_c64_$v.log 2>&1 || exit 1
echo "c64 preload=$v $(tail -n 1 gpurun_out/r2_preload_c64_$v.log | cut -c100-140)"
XGS_DECODE_PRELOAD=$v timeout -k 10 200 python -u bench.py --concurrency 1 --steps 200 --warmup 20 > gpurun_out/r2_preload_c1_$v.log 2>&1 || exit 1
echo "c1 preload=$v $(tail -n 1 gpurun_out/r2_preload_c1_$v.log | cut -c100-140)"
done
done
tail -n 2 gpurun_out/r2_preload_tests.log
