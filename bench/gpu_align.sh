# mixed-step GEMM tile alignment (scheduler align_tokens/align_slack): c64 A/B, 200-step and driver-form windows
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for a in 256 0; do
XGS_ALIGN_TOKENS=$a timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > gpurun_out/r2_align_a${a}_r$r.log 2>&1 || exit 1
echo "align=$a run=$r $(tail -n 1 gpurun_out/r2_align_a${a}_r$r.log | cut -c1-150)"
done
done
for a in 256 0; do
XGS_ALIGN_TOKENS=$a timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_align_a${a}_s20.log 2>&1 || exit 1
echo "align=$a steps20 $(tail -n 1 gpurun_out/r2_align_a${a}_s20.log | cut -c1-150)"
done
XGS_ALIGN_TOKENS=256 timeout -k 10 200 python -u bench.py --model mixtral-8x7b --steps 60 --warmup 20 > gpurun_out/r2_align_mixtral.log 2>&1 || exit 1
echo "mixtral align=256 $(tail -n 1 gpurun_out/r2_align_mixtral.log | cut -c1-150)"
