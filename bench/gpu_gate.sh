# Round gate on one MI355X: the full GPU test suite, smoke(), the driver-form bench and
# a long steady-state bench, batch 1.   bash bench/gpu_gate.sh [tag]   (through gpurun)
set -o pipefail
cd "$(dirname "$0")/.."
tag=${1:-gate}
o=${GRAFT_REPO_ROOT:-.}/gpurun_out/$tag; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    > $o/gputests.log 2>&1; rc=$?
tail -n 3 $o/gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $o/bench_driver.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3000 --warmup 100 > $o/bench_long.log 2>&1 && \
timeout -k 10 200 python -u bench.py --concurrency 1 --steps 200 --warmup 20 > $o/bench_c1.log 2>&1
rc=$?
tail -n 1 $o/smoke.log; for f in bench_driver bench_long bench_c1; do tail -n 1 $o/$f.log | cut -c1-330; done
exit $rc
