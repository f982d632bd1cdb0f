set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill" > gpurun_out/r2_prefill_tests.log 2>&1 && \
timeout -k 10 300 python -u bench/prefill_bench.py > gpurun_out/r2_prefill_bench.jsonl 2> gpurun_out/r2_prefill_bench.err
rc=$?
tail -n 2 gpurun_out/r2_prefill_tests.log; cat gpurun_out/r2_prefill_bench.jsonl
exit $rc
