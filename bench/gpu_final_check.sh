# round-end gate: full GPU suite, smoke, driver-form bench, batch 1
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/final_check; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $o/bench_driver.log 2>&1 && \
timeout -k 10 200 python -u bench.py --concurrency 1 --steps 200 --warmup 20 > $o/bench_c1.log 2>&1
rc=$?
tail -n 1 $o/gputests.log; tail -n 1 $o/smoke.log; tail -n 1 $o/bench_driver.log | cut -c1-200; tail -n 1 $o/bench_c1.log | cut -c1-200
exit $rc
