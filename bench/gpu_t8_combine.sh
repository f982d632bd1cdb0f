# one rank of 70B TP8, batch 1: in-launch split combine vs the combine launch (A/B, 2 pairs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/t8_combine; mkdir -p $o
j() { python3 -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
for r in 1 2; do
for v in 1 0; do
XGS_DECODE_INLAUNCH_COMBINE=$v timeout -k 10 300 python -u bench.py --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 10 > $o/c1_${v}_$r.log 2>&1 || exit 1
echo "t8 c1 inlaunch=$v r$r $(j < $o/c1_${v}_$r.log)"
done
done
XGS_DECODE_INLAUNCH_COMBINE=1 timeout -k 10 300 python -u bench.py --model llama3-70b --tp-shard 8 --steps 100 --warmup 20 > $o/c64_1.log 2>&1 || exit 1
echo "t8 c64 inlaunch=1 $(j < $o/c64_1.log)"
timeout -k 10 300 python -u bench.py --model llama3-70b --tp-shard 8 --steps 100 --warmup 20 > $o/c64_0.log 2>&1 || exit 1
echo "t8 c64 inlaunch=0 $(j < $o/c64_0.log)"
