# end-to-end c64 / c1 with temperature + top-p sampling: split-row sampler vs the single-workgroup kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 1 0; do
XGS_SAMPLE_SPLIT=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 --temperature 0.8 --top-p 0.9 > gpurun_out/r2_samp_e2e_c64_$v.log 2>&1 || exit 1
echo "c64 top-p split=$v $(tail -n 1 gpurun_out/r2_samp_e2e_c64_$v.log | cut -c1-60,160-260)"
XGS_SAMPLE_SPLIT=$v timeout -k 10 200 python -u bench.py --concurrency 1 --steps 200 --warmup 20 --temperature 0.8 --top-p 0.9 > gpurun_out/r2_samp_e2e_c1_$v.log 2>&1 || exit 1
echo "c1 top-p split=$v $(tail -n 1 gpurun_out/r2_samp_e2e_c1_$v.log | cut -c1-60,160-260)"
done
