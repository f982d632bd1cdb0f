# XA (attention split combine folded into the O GEMM prologue): tests + batch-1/8 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_fused_decode_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_xa_tests.log 2>&1 && \
for c in 1 8; do
for xa in 16 0; do
XGS_XA_MAX_M=$xa timeout -k 10 200 python -u bench.py --concurrency $c --steps 200 --warmup 20 > gpurun_out/r2_xa_c${c}_xa${xa}.log 2>&1 || exit 1
done
done
echo rc=$?
tail -n 2 gpurun_out/r2_xa_tests.log
for f in gpurun_out/r2_xa_c*.log; do echo $f; tail -n 1 $f | cut -c1-160; done
