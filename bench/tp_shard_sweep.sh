# gemm_m64g configuration sweep at the TP shard shapes (one GPU; per-shard GEMMs do not need peers)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u bench/gemm_bench.py --m64g-sweep --M 1 16 32 64 --shapes \
  qkv70t8 o70t8 gate_up70t8 down70t8 qkv8t2 o8t2 gate_up8t2 down8t2 qkv8t4 o8t4 gate_up8t4 down8t4 \
  qkv8t8 o8t8 gate_up8t8 down8t8 qkv70t2 o70t2 gate_up70t2 down70t2 qkv70t4 o70t4 gate_up70t4 down70t4 \
  > gpurun_out/r2_tp_shard_sweep.jsonl 2> gpurun_out/r2_tp_shard_sweep.err
