# prefill-sized MoE step: w13 / w2 grouped-GEMM configuration sweep on Mixtral c64 (mixed-step time)
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in "5 3" "3 3" "4 3" "2 3" "3 2" "5 5"; do
set -- $c
XGS_MOE_CFG_W13_PREFILL=$1 XGS_MOE_CFG_W2_PREFILL=$2 XGS_STEP_LOG=gpurun_out/r2_moecfg_$1_$2.jsonl timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > gpurun_out/r2_moecfg_$1_$2.log 2>&1 || exit 1
echo "w13=$1 w2=$2 $(tail -n 1 gpurun_out/r2_moecfg_$1_$2.log | cut -c100-140)"
done
