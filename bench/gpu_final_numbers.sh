# end-of-round numbers for the non-headline configs (Mixtral TP1 / TP2 shard, 70B TP8 shard, 8K TTFT)
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/final_numbers; mkdir -p $o
j() { python3 -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["ttft_p50_ms"])'; }
timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > $o/mx_c64.log 2>&1 || exit 1
echo "mixtral c64 $(j < $o/mx_c64.log)"
timeout -k 10 300 python -u bench.py --model mixtral-8x7b --concurrency 1 --steps 100 --warmup 10 > $o/mx_c1.log 2>&1 || exit 1
echo "mixtral c1 $(j < $o/mx_c1.log)"
timeout -k 10 300 python -u bench.py --model mixtral-8x7b --tp-shard 2 --steps 60 --warmup 20 > $o/mx2_c64.log 2>&1 || exit 1
echo "mixtral tp2-shard c64 $(j < $o/mx2_c64.log)"
timeout -k 10 300 python -u bench.py --model mixtral-8x7b --tp-shard 2 --concurrency 1 --steps 100 --warmup 10 > $o/mx2_c1.log 2>&1 || exit 1
echo "mixtral tp2-shard c1 $(j < $o/mx2_c1.log)"
timeout -k 10 300 python -u bench.py --model llama3-70b --tp-shard 8 --steps 40 --warmup 10 > $o/t8_c64.log 2>&1 || exit 1
echo "70b tp8-shard c64 $(j < $o/t8_c64.log)"
timeout -k 10 300 python -u bench.py --model llama3-70b --tp-shard 8 --concurrency 1 --steps 60 --warmup 10 > $o/t8_c1.log 2>&1 || exit 1
echo "70b tp8-shard c1 $(j < $o/t8_c1.log)"
timeout -k 10 300 python -u bench/prefill_bench.py --lens 512 --gh 0 > $o/prefill.jsonl 2>&1 || exit 1
grep ttft $o/prefill.jsonl
