# K-via-LDS decode attention at G = 8 (70B TP8 shard: one kv head per rank) and Mixtral: A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/klds_g8; mkdir -p $o
j() { python3 -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["ttft_p50_ms"])'; }
for r in 1 2; do
for v in 1 0; do
XGS_DECODE_K_LDS=$v timeout -k 10 300 python -u bench.py --model llama3-70b --tp-shard 8 --steps 100 --warmup 20 > $o/t8_${v}_$r.log 2>&1 || exit 1
echo "70b tp8-shard c64 klds=$v r$r $(j < $o/t8_${v}_$r.log)"
done
done
for v in 1 0; do
XGS_DECODE_K_LDS=$v timeout -k 10 300 python -u bench.py --model llama3-70b --tp-shard 8 --concurrency 1 --steps 60 --warmup 10 > $o/t8c1_${v}.log 2>&1 || exit 1
echo "70b tp8-shard c1 klds=$v $(j < $o/t8c1_${v}.log)"
XGS_DECODE_K_LDS=$v timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > $o/mx_${v}.log 2>&1 || exit 1
echo "mixtral c64 klds=$v $(j < $o/mx_${v}.log)"
done
