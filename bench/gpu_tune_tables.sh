# Build the shipped TunableOp GEMM table (xgserve/tuning/): tune the hipBLASLt / rocBLAS GEMMs each benchmark
# configuration issues (prefill / mixed-step projections, LM heads), one CSV per run, merged afterwards.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tunable
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=100
export XGS_GEMM_TUNING=0   # tune from scratch (do not replay the shipped table)
run() { name=$1; shift; PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunable/t_$name.csv timeout -k 10 600 python -u "$@" > gpurun_out/tunable/t_$name.log 2>&1 || { echo "FAIL $name"; tail -n 5 gpurun_out/tunable/t_$name.log; exit 1; }; echo "ok $name"; }
run c64 bench.py --steps 120 --warmup 40
run c1 bench.py --concurrency 1 --steps 40 --warmup 10
run c8 bench.py --concurrency 8 --steps 60 --warmup 20
run mixtral_c64 bench.py --model mixtral-8x7b --steps 40 --warmup 20
run mixtral_c1 bench.py --model mixtral-8x7b --concurrency 1 --steps 30 --warmup 10
run prefill bench/prefill_bench.py
ls -la gpurun_out/tunable/
