# EP: TP/EP GPU tests (custom AR + HIP dispatch kernels) and one-rank Mixtral TP2 shard sims (config 5 per-rank compute)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_tp_gpu.py tests/test_kernels_gpu.py -k "tp2 or ep_dispatch" -x -q --timeout 240 --timeout-method thread > gpurun_out/r2_ep_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model mixtral-8x7b --tp-shard 2 --steps 60 --warmup 20 > gpurun_out/r2_mixtral_tp2sim_c64.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model mixtral-8x7b --tp-shard 2 --concurrency 1 --steps 100 --warmup 10 > gpurun_out/r2_mixtral_tp2sim_c1.log 2>&1
rc=$?
tail -n 2 gpurun_out/r2_ep_tests.log
tail -n 1 gpurun_out/r2_mixtral_tp2sim_c64.log | cut -c1-220; tail -n 1 gpurun_out/r2_mixtral_tp2sim_c1.log | cut -c1-220
exit $rc
