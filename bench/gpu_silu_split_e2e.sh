# split-K SiLU / 8-wave gate_up plans end to end: GPU tests, 70B TP1 and TP-shard benches (new plans vs
# the previous ones through XGS_M64_PLANS), then the partial-shape sweep with cfg 7
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/silu_e2e; mkdir -p $o
j() { python3 -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 400 python -u -m pytest tests/test_fused_decode_gpu.py tests/test_tp_gpu.py tests/test_engine_gpu.py -x -q --timeout 240 --timeout-method thread > $o/tests.log 2>&1 || { tail -n 30 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
OLD70="57344x8192x2@64=2,1,3;57344x8192x2@32=2,1,3;57344x8192x2@16=2,1,5"
OLDT8="7168x8192x2@64=2,1,6;7168x8192x2@32=2,1,6;7168x8192x2@16=2,1,6"
for c in 1 64; do
  st=$([ $c = 1 ] && echo 60 || echo 40)
  timeout -k 10 300 python -u bench.py --model llama3-70b --tp-shard 8 --concurrency $c --steps $st --warmup 10 > $o/t8_new_c$c.log 2>&1 || exit 1
  echo "70b tp8-shard c$c new $(j < $o/t8_new_c$c.log)"
  XGS_M64_PLANS="$OLDT8" timeout -k 10 300 python -u bench.py --model llama3-70b --tp-shard 8 --concurrency $c --steps $st --warmup 10 > $o/t8_old_c$c.log 2>&1 || exit 1
  echo "70b tp8-shard c$c old $(j < $o/t8_old_c$c.log)"
done
for c in 1 64; do
  st=$([ $c = 1 ] && echo 40 || echo 40)
  timeout -k 10 400 python -u bench.py --model llama3-70b --concurrency $c --steps $st --warmup 10 > $o/t1_new_c$c.log 2>&1 || exit 1
  echo "70b tp1 c$c new $(j < $o/t1_new_c$c.log)"
  XGS_M64_PLANS="$OLD70" timeout -k 10 400 python -u bench.py --model llama3-70b --concurrency $c --steps $st --warmup 10 > $o/t1_old_c$c.log 2>&1 || exit 1
  echo "70b tp1 c$c old $(j < $o/t1_old_c$c.log)"
done
timeout -k 10 500 python -u bench/gemm_bench.py --m64g-sweep --M 1 16 64 --shapes qkv70 o70 down70 qkv70t8 o70t8 down70t8 qkv70t2 o70t2 down70t2 qkv8t2 o8t2 down8t2 qkv down o > $o/sweep_partial.jsonl 2>&1 || exit 1
echo sweep done
