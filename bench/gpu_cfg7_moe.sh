# 8-wave tile (cfg 7) on the grouped MoE GEMM and the 8B gate_up at batch 1-16 (split SiLU): tests + sweeps
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/cfg7_moe; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "moe" > $o/tests.log 2>&1 || { tail -n 30 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
timeout -k 10 300 python -u bench/gemm_bench.py --m64g-sweep --M 1 16 --shapes gate_up > $o/sweep_gu.jsonl 2>&1 || exit 1
grep '^{' $o/sweep_gu.jsonl | head -6
timeout -k 10 400 python -u bench/gemm_bench.py --moe-sweep --M 1 16 64 > $o/sweep_moe.jsonl 2>&1 || exit 1
grep '^{' $o/sweep_moe.jsonl | python3 -c '
import sys, json
rows = [json.loads(l) for l in sys.stdin]
seen = {}
for r in rows:
    k = (r["moe"], r["T"])
    seen.setdefault(k, []).append(r)
for k, rs in seen.items():
    print(k, [(r["nw"], r["S"], r["cfg"], r["us"]) for r in rs[:4]])
'
