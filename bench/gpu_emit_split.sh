# split emission (urgent rows before the next plan, the rest in its overlap window): tests + c64 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/emit_split; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_fused_decode_gpu.py tests/test_async_schedule.py tests/test_tp_gpu.py -x -q --timeout 240 --timeout-method thread > $o/tests.log 2>&1 || { tail -n 30 $o/tests.log; exit 1; }
tail -n 2 $o/tests.log
j() { python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ttft_p50_ms"])'; }
for r in 1 2; do
for v in 1 0; do
XGS_EMIT_SPLIT=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > $o/c64_${v}_$r.log 2>&1 || exit 1
echo "c64 split=$v r$r $(tail -n 1 $o/c64_${v}_$r.log | j)"
done
done
for v in 1 0; do
XGS_EMIT_SPLIT=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $o/s20_${v}.log 2>&1 || exit 1
echo "c64 20/5 split=$v $(tail -n 1 $o/s20_${v}.log | j)"
done
