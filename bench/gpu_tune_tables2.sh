# extend the shipped GEMM table: TP-shard simulations (configs 4 / 5 per-rank shapes) and Llama-3-70B TP1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tunable
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=100
export XGS_GEMM_TUNING=0
run() { name=$1; shift; PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunable/t2_$name.csv timeout -k 10 600 python -u "$@" > gpurun_out/tunable/t2_$name.log 2>&1 || { echo "FAIL $name"; tail -n 5 gpurun_out/tunable/t2_$name.log; exit 1; }; echo "ok $name"; }
run tp8_70b_c64 bench.py --model llama3-70b --tp-shard 8 --steps 60 --warmup 20
run tp8_70b_c1 bench.py --model llama3-70b --tp-shard 8 --concurrency 1 --steps 30 --warmup 10
run tp2_mix_c64 bench.py --model mixtral-8x7b --tp-shard 2 --steps 40 --warmup 20
run l70_c64 bench.py --model llama3-70b --steps 30 --warmup 20
ls gpurun_out/tunable/
