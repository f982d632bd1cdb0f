# shipped GEMM table (xgserve/tuning/mi355x_gemm.csv, TunableOp replay) vs the default hipBLASLt heuristic
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/tuning_ab; mkdir -p $o
for r in 1 2; do
for v in 1 0; do
XGS_GEMM_TUNING=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > $o/c64_${v}_$r.log 2>&1 || exit 1
echo "c64 table=$v r$r $(tail -n 1 $o/c64_${v}_$r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ttft_p50_ms"], d["detail"]["gemm_table"])')"
done
done
for v in 1 0; do
XGS_GEMM_TUNING=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $o/s20_${v}.log 2>&1 || exit 1
echo "c64 20/5 table=$v $(tail -n 1 $o/s20_${v}.log | cut -c80-150)"
XGS_GEMM_TUNING=$v timeout -k 10 200 python -u bench.py --concurrency 1 --steps 200 --warmup 20 > $o/c1_${v}.log 2>&1 || exit 1
echo "c1 table=$v $(tail -n 1 $o/c1_${v}.log | cut -c80-150)"
XGS_GEMM_TUNING=$v timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > $o/mix_${v}.log 2>&1 || exit 1
echo "mixtral table=$v $(tail -n 1 $o/mix_${v}.log | cut -c80-150)"
done
XGS_GEMM_TUNING=1 timeout -k 10 300 python -u bench/prefill_bench.py --lens 512 --gh 4 > $o/prefill_1.log 2>&1 && \
XGS_GEMM_TUNING=0 timeout -k 10 300 python -u bench/prefill_bench.py --lens 512 --gh 4 > $o/prefill_0.log 2>&1 && \
grep -h ttft $o/prefill_1.log $o/prefill_0.log
