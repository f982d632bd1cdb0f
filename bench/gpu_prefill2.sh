# prefill attention with two register tiles in flight: tests, kernel bench (512 / 2K / 8K, TTFT 8K), c64 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/prefill2; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "prefill" > $o/tests.log 2>&1 || { tail -n 30 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_spec_decode.py -x -q --timeout 120 --timeout-method thread > $o/tests2.log 2>&1 || { tail -n 30 $o/tests2.log; exit 1; }
tail -n 1 $o/tests2.log
timeout -k 10 300 python -u bench/prefill_bench.py > $o/prefill.jsonl 2>&1 || { tail -n 20 $o/prefill.jsonl; exit 1; }
grep '^{' $o/prefill.jsonl
j() { python3 -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["ttft_p50_ms"])'; }
for r in 1 2; do
timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > $o/c64_$r.log 2>&1 || exit 1
echo "c64 r$r $(j < $o/c64_$r.log)"
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $o/s20.log 2>&1 || exit 1
echo "c64 20/5 $(j < $o/s20.log)"
