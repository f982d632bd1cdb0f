# mixed-step down projection: split 4 vs split 2 (A/B, 3 pairs)
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/splitk_s; mkdir -p $o
j() { python3 -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["ttft_p50_ms"])'; }
for r in 1 2 3; do
for v in 4 2; do
XGS_SPLITK_PREFILL_S=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > $o/s${v}_$r.log 2>&1 || exit 1
echo "c64 split=$v r$r $(j < $o/s${v}_$r.log)"
done
done
