# O projection at M 33-64 with split 2 (its 32 KB slab reduced in-launch, no add_partials_resid launch): A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/o_s2; mkdir -p $o
j() { python3 -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["ttft_p50_ms"])'; }
P="4096x4096x1@64=1,2,0"
XGS_M64_PLANS="$P" timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused or graph or reference" > $o/tests.log 2>&1 || { tail -n 30 $o/tests.log; exit 1; }
tail -n 1 $o/tests.log
for r in 1 2 3; do
XGS_M64_PLANS="$P" timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > $o/new_$r.log 2>&1 || exit 1
echo "c64 O split2 r$r $(j < $o/new_$r.log)"
timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > $o/old_$r.log 2>&1 || exit 1
echo "c64 O split4 r$r $(j < $o/old_$r.log)"
done
