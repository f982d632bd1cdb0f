# O projection of prefill-sized steps as a K-split batched GEMM (XGS_SPLITK_O): A/B at 64 concurrent
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/splitk_o; mkdir -p $o
XGS_SPLITK_O=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -n 30 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
j() { python3 -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["ttft_p50_ms"])'; }
for r in 1 2 3; do
for v in 1 0; do
XGS_SPLITK_O=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > $o/c64_${v}_$r.log 2>&1 || exit 1
echo "c64 splitk_o=$v r$r $(j < $o/c64_${v}_$r.log)"
done
done
