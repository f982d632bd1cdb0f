# prefill-sized down projection as a K-split batched GEMM (fp32 partials into add+rmsnorm): tests + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/splitk; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_fused_decode_gpu.py -x -q --timeout 120 --timeout-method thread -k "splitk" > $o/tests.log 2>&1 || { tail -n 30 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_async_schedule.py tests/test_spec_decode.py -x -q --timeout 120 --timeout-method thread > $o/tests2.log 2>&1 || { tail -n 30 $o/tests2.log; exit 1; }
tail -n 1 $o/tests2.log
j() { python3 -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["ttft_p50_ms"])'; }
for r in 1 2; do
for v in 1536 0; do
XGS_SPLITK_PREFILL_MAX_M=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > $o/c64_${v}_$r.log 2>&1 || exit 1
echo "c64 splitk_max=$v r$r $(j < $o/c64_${v}_$r.log)"
done
done
for v in 1536 0; do
XGS_SPLITK_PREFILL_MAX_M=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $o/s20_${v}.log 2>&1 || exit 1
echo "c64 20/5 splitk_max=$v $(j < $o/s20_${v}.log)"
XGS_SPLITK_PREFILL_MAX_M=$v timeout -k 10 300 python -u bench.py --model llama3-70b --steps 40 --warmup 10 > $o/l70_${v}.log 2>&1 || exit 1
echo "70b c64 splitk_max=$v $(j < $o/l70_${v}.log)"
done
