# MoE prefill-sized steps: grouped m64g (tile pairs) vs per-expert hipBLASLt (XGS_MOE_DENSE_MIN_PAIRS)
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 1073741824 256; do
XGS_MOE_DENSE_MIN_PAIRS=$v XGS_STEP_LOG=gpurun_out/r2_moedense_$v.jsonl timeout -k 10 300 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > gpurun_out/r2_moedense_$v.log 2>&1 || exit 1
echo "dense_min=$v $(tail -n 1 gpurun_out/r2_moedense_$v.log | cut -c100-140)"
done
