# asynchronous scheduling over prompt steps (XGS_ASYNC_MIXED) and early release of length-finishing rows
# (XGS_EARLY_RELEASE): tests + A/B of the three policies on throughput and p50 TTFT
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/async_mixed; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_async_schedule.py -x -q --timeout 240 --timeout-method thread > $o/tests.log 2>&1 || { tail -n 30 $o/tests.log; exit 1; }
tail -n 2 $o/tests.log
XGS_EARLY_RELEASE=1 timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 240 --timeout-method thread > $o/tests_early.log 2>&1 || { tail -n 30 $o/tests_early.log; exit 1; }
tail -n 1 $o/tests_early.log
j() { python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ttft_p50_ms"])'; }
for r in 1 2; do
for cfg in "1 0" "1 1" "0 0"; do
set -- $cfg
XGS_ASYNC_MIXED=$1 XGS_EARLY_RELEASE=$2 timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > $o/c64_$1$2_$r.log 2>&1 || exit 1
echo "c64 mixed=$1 early=$2 r$r $(tail -n 1 $o/c64_$1$2_$r.log | j)"
done
done
for cfg in "1 0" "0 0"; do
set -- $cfg
XGS_ASYNC_MIXED=$1 XGS_EARLY_RELEASE=$2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $o/s20_$1$2.log 2>&1 || exit 1
echo "c64 20/5 mixed=$1 early=$2 $(tail -n 1 $o/s20_$1$2.log | j)"
XGS_ASYNC_MIXED=$1 XGS_EARLY_RELEASE=$2 timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > $o/mix_$1$2.log 2>&1 || exit 1
echo "mixtral mixed=$1 early=$2 $(tail -n 1 $o/mix_$1$2.log | j)"
done
