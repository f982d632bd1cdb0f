# decode attention: K tile through LDS (coalesced full-row loads) vs MFMA-shaped K loads from HBM: tests + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/klds; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_decode_gpu.py -x -q --timeout 120 --timeout-method thread -k "decode or attention or step" > $o/tests.log 2>&1 || { tail -n 30 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_tp_gpu.py -x -q --timeout 120 --timeout-method thread > $o/tests2.log 2>&1 || { tail -n 30 $o/tests2.log; exit 1; }
tail -n 1 $o/tests2.log
j() { python3 -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["ttft_p50_ms"])'; }
for r in 1 2; do
for v in 1 0; do
XGS_DECODE_K_LDS=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > $o/c64_${v}_$r.log 2>&1 || exit 1
echo "c64 klds=$v r$r $(j < $o/c64_${v}_$r.log)"
done
done
for v in 1 0; do
XGS_DECODE_K_LDS=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $o/s20_${v}.log 2>&1 || exit 1
echo "c64 20/5 klds=$v $(j < $o/s20_${v}.log)"
XGS_DECODE_K_LDS=$v timeout -k 10 200 python -u bench.py --concurrency 1 --steps 200 --warmup 20 > $o/c1_${v}.log 2>&1 || exit 1
echo "c1 klds=$v $(j < $o/c1_${v}.log)"
done
