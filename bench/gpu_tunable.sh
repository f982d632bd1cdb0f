# PyTorch TunableOp (every hipBLASLt/rocBLAS solution timed per GEMM shape with rotating buffers) for the
# prefill-sized projection GEMMs: tune during one run, replay the table in another, vs the default heuristic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tunable
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunable/tunableop_results%d.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=100 \
  timeout -k 10 500 python -u bench.py --steps 120 --warmup 40 > gpurun_out/tunable/tune_run.log 2>&1 || exit 1
echo "tune run $(tail -n 1 gpurun_out/tunable/tune_run.log | cut -c100-150)"
ls -la gpurun_out/tunable/
for r in 1 2; do
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > gpurun_out/tunable/replay_$r.log 2>&1 || exit 1
echo "replay $r $(tail -n 1 gpurun_out/tunable/replay_$r.log | cut -c100-150)"
timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 > gpurun_out/tunable/default_$r.log 2>&1 || exit 1
echo "default $r $(tail -n 1 gpurun_out/tunable/default_$r.log | cut -c100-150)"
done
