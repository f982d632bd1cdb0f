# final-state kernel tables (rocprofv3 kernel + HIP API trace) for the headline and batch-1 configs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash bench/profile.sh gpurun_out/prof_r2_c64 && \
bash bench/profile.sh gpurun_out/prof_r2_c1 --concurrency 1 && \
bash bench/profile.sh gpurun_out/prof_r2_mixtral --model mixtral-8x7b
