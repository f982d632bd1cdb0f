# mixed-step attention overlap (decode attention on a side stream under the prefill attention): tests + c64 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/mixed_overlap; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_async_schedule.py -x -q --timeout 240 --timeout-method thread > $o/tests.log 2>&1 || { tail -n 30 $o/tests.log; exit 1; }
tail -n 2 $o/tests.log
j() { python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ttft_p50_ms"])'; }
mixed() { python3 -c 'import sys,json; r=[json.loads(l) for l in open(sys.argv[1])]; m=[x for x in r if x.get("prefill_tokens",0)>0]; d=[x for x in r if x.get("prefill_tokens",0)==0]; k=[k for k in r[0] if "ms" in k][0]; print("mixed", len(m), round(sum(x[k] for x in m)/max(1,len(m)),3), "decode", len(d), round(sum(x[k] for x in d)/max(1,len(d)),3))' $1; }
for r in 1 2; do
for v in 1 0; do
XGS_STEP_LOG=$o/steps_${v}_$r.jsonl XGS_MIXED_ATTN_OVERLAP=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > $o/c64_${v}_$r.log 2>&1 || exit 1
echo "c64 overlap=$v r$r $(tail -n 1 $o/c64_${v}_$r.log | j) $(mixed $o/steps_${v}_$r.jsonl)"
done
done
for v in 1 0; do
XGS_MIXED_ATTN_OVERLAP=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $o/s20_${v}.log 2>&1 || exit 1
echo "c64 20/5 overlap=$v $(tail -n 1 $o/s20_${v}.log | j)"
done
