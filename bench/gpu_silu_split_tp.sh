# split-K SiLU gate_up at the TP shard shapes (small N, few column tiles): sweep at M = 1 / 16 / 32 / 64
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/silu_split_tp; mkdir -p $o
timeout -k 10 500 python -u bench/gemm_bench.py --m64g-sweep --M 1 16 32 64 --shapes gate_up70t8 gate_up70t4 gate_up70t2 gate_up8t2 gate_up8t4 gate_up8t8 gate_up70 > $o/sweep.jsonl 2>&1 || { tail -n 20 $o/sweep.jsonl; exit 1; }
python3 - $o/sweep.jsonl <<'PY'
import json, sys
best = {}
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    r = json.loads(l)
    best.setdefault((r["shape"], r["M"]), []).append(r)
for k, rs in best.items():
    s1 = [r for r in rs if "S=1," in r["op"]][:1]
    print(k, [(r["op"], r["us"]) for r in rs[:3]], "best S=1:", [(r["op"], r["us"]) for r in s1])
PY
