# 8-wave 256-column gemm_m64g tile (cfg 7) + split-K SiLU: GPU tests, then the decode-shape sweep at M = 64 / 32
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/wide_tile; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_fused_decode_gpu.py -x -q --timeout 120 --timeout-method thread -k "split_silu or wide_tile or norm_linear" > $o/tests.log 2>&1 || { tail -n 30 $o/tests.log; exit 1; }
tail -n 2 $o/tests.log
timeout -k 10 400 python -u bench/gemm_bench.py --m64g-sweep --M 64 32 --shapes gate_up qkv down o > $o/sweep.jsonl 2>&1 || { tail -n 20 $o/sweep.jsonl; exit 1; }
python3 - $o/sweep.jsonl <<'PY'
import json, sys
best = {}
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    r = json.loads(l)
    k = (r["shape"], r["M"])
    best.setdefault(k, []).append(r)
for k, rs in best.items():
    print(k, [(r["op"], r["us"]) for r in rs[:4]])
PY
