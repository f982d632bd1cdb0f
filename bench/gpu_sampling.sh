# split-row sampler: tests + kernel bench (v2 vs single-workgroup v1) + engine tests
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "sample or argmax" -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_samp_tests.log 2>&1 || { tail -n 40 gpurun_out/r2_samp_tests.log; exit 1; }
tail -n 1 gpurun_out/r2_samp_tests.log
timeout -k 10 200 python -u bench/kernel_bench.py --what sampling > gpurun_out/r2_samp_kb_v2.jsonl 2>&1 || exit 1
XGS_SAMPLE_SPLIT=0 timeout -k 10 200 python -u bench/kernel_bench.py --what sampling > gpurun_out/r2_samp_kb_v1.jsonl 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_samp_tests2.log 2>&1 || { tail -n 40 gpurun_out/r2_samp_tests2.log; exit 1; }
tail -n 1 gpurun_out/r2_samp_tests2.log
