#!/usr/bin/env bash
# Every GPU measurement this repo takes, as named suites (run through gpurun, from the
# repo or from the .snap/ copy made by bench/snap.sh):
#   bash bench/gpu.sh <suite> [tag] [extra bench.py args...]
# Suites:
#   gate     full GPU test suite, smoke(), driver-form bench, 3000-step bench, batch 1
#   steady   headline at steady state: driver form twice, long window, step log, profile
#   ab       same bench under each XGS_AB setting (XGS_AB="A=1;A=0"), driver form + 400 steps
#   tp       custom all-reduce + TP tests, Llama-3-70B TP8 shard (one rank) c1 / c64
#   moe      Mixtral: MoE tests, c64 / c1, TP2 shard c64
#   prefill  prefill kernels: tests, 512 / 2K / 8K kernel bench + TTFT, c64 bench
#   serve    HTTP/SSE serve bench (64 streams) next to the in-process long bench
#   tune     rebuild the shipped TunableOp GEMM tables (xgserve/tuning/)
#   sweep    gemm_m64g configuration sweep at the TP shard shapes
#   arsim    one rank of 70B TP8 at batch 1 under a simulated 0 / 4 / 8 us all-reduce
#   coalesce admission-window A/B: driver form + 1000 steps at --coalesce 1 / 2 / 3
#   profile  rocprofv3 kernel + gap profile of the headline (bench/profile.sh)
#   mw       gemm_mw numerics + sweep, stall-free mixed-step tests, headline with prompt chunks
#   m64      LM head on gemm_mw, deep-ring / uneven-split gemm_m64g tests + sweeps
#   ar       custom all-reduce push vs pull: tests + per-call latency (bench/ar_bench.py)
#   r4b/r4c  round-4 passes: AR + TP + prefetch A/B; Mixtral + profiles
#   r4d      in-launch residual reduce + decode-attention depth A/Bs at 64 rows (step logs)
#   r5a      gemm_pf: tests, per-projection A/B at the mixed-step rows, headline on / off + profile
#   r6q      int8 / int4 / fp8 weight-only decode: kernel + engine tests, batch 1 and 64 concurrent
#   r6a      GG_AR per-launch generations: custom all-reduce + TP engine tests, headline, 70B TP8 rank c1
# Each GPU step has its own time limit; the first failure ends the suite.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
suite=${1:?suite}; tag=${2:-$1}; shift; shift || true
o=${GRAFT_REPO_ROOT:-.}/gpurun_out/$tag; mkdir -p "$o"

run() {  # name seconds cmd...   -> $o/name.log, prints its last line
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$o/$name.log" 2>&1
  local rc=$?
  echo "[$name rc=$rc] $(tail -n 1 "$o/$name.log" | cut -c1-400)"
  [ $rc -eq 0 ] || { tail -n 30 "$o/$name.log"; exit $rc; }
}
pyt() {  # name seconds pytest-args...
  local name=$1 secs=$2; shift 2
  run "$name" "$secs" python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider "$@"
}
pyt_soft() {  # like pyt, but ordinary test failures (rc 1) do not end the suite; faults / timeouts do
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" python -u -m pytest -q --timeout 240 --timeout-method thread -p no:cacheprovider "$@" \
      > "$o/$name.log" 2>&1
  local rc=$?
  echo "[$name rc=$rc] $(tail -n 1 "$o/$name.log" | cut -c1-400)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -n 30 "$o/$name.log"; exit $rc; }
}
B="python -u bench.py"

case $suite in
gate)
  pyt gputests 900 tests -m gpu
  run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
  run bench_driver 200 $B --steps 20 --warmup 5 "$@"
  run bench_long 300 $B --steps 3000 --warmup 100 "$@"
  run bench_c1 200 $B --concurrency 1 --steps 200 --warmup 20 "$@" ;;
steady)
  run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
  run driver_a 200 $B --steps 20 --warmup 5 "$@"
  run driver_b 200 $B --steps 20 --warmup 5 "$@"
  run long 300 $B --steps 3000 --warmup 100 "$@"
  run steplog 200 env XGS_STEP_LOG="$o/steps.jsonl" $B --steps 400 --warmup 20 "$@"
  bash bench/profile.sh "$o/prof" "$@" ;;
ab)
  IFS=';' read -ra settings <<< "${XGS_AB:?set XGS_AB='VAR=a;VAR=b'}"
  for s in "${settings[@]}"; do
    n=$(echo "$s" | tr -c 'A-Za-z0-9_=\n' '_')
    run "driver_$n" 200 env $s $B --steps 20 --warmup 5 "$@"
    run "w400_$n" 250 env $s $B --steps 400 --warmup 40 "$@"
  done ;;
r6g1)  # closing gate, part 1: every GPU test + smoke()
  pyt gputests 1100 tests -m gpu
  run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
r6g2)  # closing gate, part 2: the driver-form headline twice, 3000 steps, batch 1, the serving path at DP 1
  run driver_a 200 $B --steps 20 --warmup 5
  run driver_b 200 $B --steps 20 --warmup 5
  run long 300 $B --steps 3000 --warmup 100
  run c1 200 $B --concurrency 1 --steps 300 --warmup 30
  run serve_dp1 400 python -u bench/serve_bench.py --launch "--model llama3-8b --max-num-seqs 64 --replicas 1 --frontends 2" \
      --concurrency 64 --prompt-len 512 --output-len 256 --warmup 40 --duration 40 --procs 4 --label serve_dp1 ;;
r6f)  # closing kernel profiles: 8B c64 / c1, Mixtral c1, one 70B TP8 rank c1
  bash bench/profile.sh "$o/c64"
  bash bench/profile.sh "$o/c1" --concurrency 1
  bash bench/profile.sh "$o/mix_c1" --model mixtral-8x7b --concurrency 1
  bash bench/profile.sh "$o/tp8_c1" --model llama3-70b --tp-shard 8 --concurrency 1 ;;
r6fg)  # fused decode-GEMM forms vs plain forms, graph-timed, cold weights (70B TP8 / TP1 shard, 8B)
  run fg_70t8 200 python -u bench/fused_gemm_bench.py --model llama3-70b --tp 8 --M 1 4
  run fg_8b 200 python -u bench/fused_gemm_bench.py --model llama3-8b --tp 1 --M 1 64 ;;
r6fs)  # fused-form plan sweeps (norm128 / GG_RESID), graph-timed, cold weights
  run fs_70t8 400 python -u bench/fused_gemm_bench.py --model llama3-70b --tp 8 --M 1 --sweep
  run fs_8b 400 python -u bench/fused_gemm_bench.py --model llama3-8b --tp 1 --M 1 64 --sweep ;;
r6fp)  # fused-form plans from the r6fs sweep: same-box end-to-end A/B
  for r in 1 2; do
    run "tp8_base_$r" 300 $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20
    run "tp8_new_$r" 300 env "XGS_TUNE=m64_plans=1280x8192x1@16=1,8,0;8192x1024x1@16=1,1,0" $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20
    run "c1_base_$r" 200 $B --concurrency 1 --steps 300 --warmup 30
    run "c1_gu3_$r" 200 env "XGS_TUNE=m64_plans=28672x4096x2@16=2,1,3" $B --concurrency 1 --steps 300 --warmup 30
    run "c64_base_$r" 250 $B --steps 300 --warmup 30
    run "c64_dn141_$r" 250 env "XGS_TUNE=m64_plans=4096x14336x1@64=1,4,1" $B --steps 300 --warmup 30
  done ;;
r6rt)  # tests after the S=1 GG_RESID LDS tail + fused-form plans
  pyt rt_tests 1100 tests/test_fused_decode_gpu.py tests/test_gemm_ar_gpu.py tests/test_tp_gpu.py tests/test_custom_ar_gpu.py tests/test_engine_gpu.py tests/test_skinny_gpu.py ;;
r6fs2)  # fused-form plan sweeps, 70B TP8 at M 16 / 64, 8B at M 16
  run fs2_70t8 600 python -u bench/fused_gemm_bench.py --model llama3-70b --tp 8 --M 16 64 --sweep
  run fs2_8b 400 python -u bench/fused_gemm_bench.py --model llama3-8b --tp 1 --M 16 --sweep ;;
r6fp2)  # 70B TP8 rank: down plans from the r6fs2 sweep, same-box end-to-end A/B (c1 and c64)
  for r in 1 2; do
    run "tp8c1_base_$r" 300 $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20
    run "tp8c1_dn129_$r" 300 env "XGS_TUNE=m64_plans=8192x3584x1@16=1,2,9" $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20
    run "tp8c64_base_$r" 400 $B --model llama3-70b --tp-shard 8 --steps 60 --warmup 20
    run "tp8c64_dn120_$r" 400 env "XGS_TUNE=m64_plans=8192x3584x1@64=1,2,0" $B --model llama3-70b --tp-shard 8 --steps 60 --warmup 20
  done ;;
r6g64)  # 70B TP8 rank, 64 concurrent: per-kernel (by grid) times
  raw=$(mktemp -d "${TMPDIR:-/tmp}/xgs_g64.XXXXXX")
  timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "$raw" -o run -- \
      python3 bench.py --steps 40 --warmup 20 --model llama3-70b --tp-shard 8 > "$o/bench.log" 2>&1
  tr=$(find "$raw" -name '*kernel_trace.csv' | sort | tail -n 1)
  python3 bench/prof_summary.py "$tr" --window-ms 300 --by-grid --top 30 > "$o/grid.md"
  rm -rf "$raw" ;;
r6ri)  # in-launch residual reduce bound at 64 rows (8B o / down): fused microbench + end to end
  for kb in 32 64 256; do
    run "ri_fg_$kb" 200 env XGS_TUNE=resid_inlaunch_kb=$kb python -u bench/fused_gemm_bench.py --model llama3-8b --tp 1 --M 64
  done
  for r in 1 2; do
    for kb in 32 64 256; do
      run "ri_c64_${kb}_$r" 250 env XGS_TUNE=resid_inlaunch_kb=$kb $B --steps 300 --warmup 30
    done
  done ;;
r6c1)  # 8B batch 1: runner-up fused-form plans (r6fs) end to end, same box
  for r in 1 2; do
    run "c1_base_$r" 200 $B --concurrency 1 --steps 300 --warmup 30
    run "c1_dn246_$r" 200 env "XGS_TUNE=m64_plans=4096x14336x1@16=2,4,6" $B --concurrency 1 --steps 300 --warmup 30
    run "c1_o141_$r" 200 env "XGS_TUNE=m64_plans=4096x4096x1@16=1,4,1" $B --concurrency 1 --steps 300 --warmup 30
    run "c1_qkv241_$r" 200 env "XGS_TUNE=m64_plans=6144x4096x1@16=2,4,1" $B --concurrency 1 --steps 300 --warmup 30
    run "c1_gu219_$r" 200 env "XGS_TUNE=m64_plans=28672x4096x2@16=2,1,9" $B --concurrency 1 --steps 300 --warmup 30
  done ;;
r6mo)  # Mixtral decode expert GEMMs in the fused forms (w13 SiLU, w2 + combine into the residual): sweep
  run mo_sweep 600 python -u bench/moe_fused_bench.py --T ${MO_T:-1 4 16} ;;
r6mw)  # Mixtral: decode-sized w2 on 64-column tiles (moe_w2_small) -- tests + same-box end-to-end A/B
  pyt mw_tests 600 tests/test_fused_decode_gpu.py tests/test_kernels_gpu.py -k "moe or mixtral or expert"
  for r in 1 2; do
    run "mix_c1_new_$r" 250 $B --model mixtral-8x7b --concurrency 1 --steps 100 --warmup 20
    run "mix_c1_old_$r" 250 env XGS_TUNE=moe_w2_small=0 $B --model mixtral-8x7b --concurrency 1 --steps 100 --warmup 20
  done
  run "mix_c8_new" 250 $B --model mixtral-8x7b --concurrency 8 --steps 100 --warmup 20
  run "mix_c8_old" 250 env XGS_TUNE=moe_w2_small=0 $B --model mixtral-8x7b --concurrency 8 --steps 100 --warmup 20 ;;
r6fs3)  # fused-form plan sweeps: 70B TP1 at M 1, 8B TP2 (Mixtral TP2 attention) at M 1 / 64
  run fs3_70t1 900 python -u bench/fused_gemm_bench.py --model llama3-70b --tp 1 --M 1 --sweep
  run fs3_8t2 500 python -u bench/fused_gemm_bench.py --model llama3-8b --tp 2 --M 1 64 --sweep ;;
r6fp3)  # fused-form plans from r6fs3: 70B TP1 batch 1 and Mixtral TP2 rank batch 1, same box
  P70="10240x8192x1@16=1,1,9;8192x8192x1@16=1,1,9;8192x28672x1@16=1,2,1"
  P8T2="3072x4096x1@16=1,4,0;4096x2048x1@16=1,1,0"
  for r in 1 2; do
    run "t1_base_$r" 300 $B --model llama3-70b --concurrency 1 --steps 40 --warmup 10
    run "t1_new_$r" 300 env "XGS_TUNE=m64_plans=$P70" $B --model llama3-70b --concurrency 1 --steps 40 --warmup 10
    run "mx2_base_$r" 300 $B --model mixtral-8x7b --tp-shard 2 --concurrency 1 --steps 100 --warmup 20
    run "mx2_new_$r" 300 env "XGS_TUNE=m64_plans=$P8T2" $B --model mixtral-8x7b --tp-shard 2 --concurrency 1 --steps 100 --warmup 20
  done ;;
r6sp)  # decode attention split cap at batch 1 (8B and one 70B TP8 rank), same box (SPLITS="16 8 4 2 1")
  SPLITS=${SPLITS:-16 8 4 2 1}
  for r in 1 2; do
    for m in $SPLITS; do
      run "c1_s${m}_$r" 200 env XGS_TUNE=decode_max_splits=$m $B --concurrency 1 --steps 300 --warmup 30
      run "tp8_s${m}_$r" 300 env XGS_TUNE=decode_max_splits=$m $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20
    done
  done ;;
r6am)  # split-row greedy argmax: tests + end to end at batch 1 and 64 (before/after on one box is the next suite)
  pyt am_tests 600 tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "argmax or greedy or async or sample"
  for r in 1 2; do
    run "c1_$r" 200 $B --concurrency 1 --steps 300 --warmup 30
    run "c1_old_$r" 200 env XGS_TUNE=argmax_split=0 $B --concurrency 1 --steps 300 --warmup 30
    run "c64_$r" 250 $B --steps 300 --warmup 30
    run "c64_old_$r" 250 env XGS_TUNE=argmax_split=0 $B --steps 300 --warmup 30
  done ;;
r6lm)  # LM head at batch 1 / 64: hipBLASLt vs gemm_m64g (bf16 logits), cold weights
  run lm 200 python -u bench/gemm_bench.py --shapes lm_head --M 1 16 64 ;;
r6qo)  # mixed steps: QKV / O on gemm_pf at 513-576 rows (fp32 partials into their consumers), same box
  W0="gate_up:448-576/down:513-576"
  for r in 1 2; do
    run "base_$r" 250 $B --steps 300 --warmup 30
    run "o_$r" 250 env "XGS_TUNE=pf_windows=$W0/o:513-576" $B --steps 300 --warmup 30
    run "qkv_$r" 250 env "XGS_TUNE=pf_windows=$W0/qkv:513-576" $B --steps 300 --warmup 30
    run "qkvo_$r" 250 env "XGS_TUNE=pf_windows=$W0/qkv:513-576/o:513-576" $B --steps 300 --warmup 30
  done ;;
r6mx2)  # MoE decode plans as adopted: tests + Mixtral TP1 c64 / c1 and one Mixtral TP2/EP2 rank c64, same box
  pyt mx_tests 900 tests/test_fused_decode_gpu.py tests/test_kernels_gpu.py tests/test_tp_gpu.py -k "moe or mixtral or expert or ep"
  for r in 1 2; do
    run "c64_new_$r" 300 $B --model mixtral-8x7b --steps 60 --warmup 20
    run "c64_old_$r" 300 env XGS_TUNE=moe_w2_small=0 $B --model mixtral-8x7b --steps 60 --warmup 20
    run "ep2_new_$r" 300 $B --model mixtral-8x7b --tp-shard 2 --steps 60 --warmup 20
    run "ep2_old_$r" 300 env XGS_TUNE=moe_w2_small=0 $B --model mixtral-8x7b --tp-shard 2 --steps 60 --warmup 20
  done ;;
r6p512)  # prefill attention at 512 / 576-token prompts: every configuration (8B heads)
  run p512 300 python -u bench/prefill_bench.py --lens 512 576 1024 --no-ttft --gh 0 -1282 -1284 -1281 -242 -241 -244 -82 -81 -84 -42 -41 -44 ;;
r6t1c64)  # 70B TP1, 64 concurrent: bucket-64 plans from the fused-form sweep (r6fs4), same box
  P="10240x8192x1@64=1,3,7;8192x8192x1@64=1,2,1;8192x28672x1@64=2,4,1"
  for r in 1 2; do
    run "base_$r" 400 $B --model llama3-70b --steps 40 --warmup 10
    run "new_$r" 400 env "XGS_TUNE=m64_plans=$P" $B --model llama3-70b --steps 40 --warmup 10
  done ;;
r6g8)  # 70B TP8 rank, batch 1: per-GEMM (by grid) kernel times under the fused decode layer (and A/B knobs)
  for v in base "fused_decode=0" "krot=0" "krot=2"; do
    n=$(echo "$v" | tr -c 'A-Za-z0-9_\n' '_')
    raw=$(mktemp -d "${TMPDIR:-/tmp}/xgs_g8.XXXXXX")
    if [ "$v" = base ]; then e="XGS_TUNE="; else e="XGS_TUNE=$v"; fi
    env $e timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$raw" -o run -- \
        python3 bench.py --steps 60 --warmup 20 --model llama3-70b --tp-shard 8 --concurrency 1 > "$o/bench_$n.log" 2>&1
    tr=$(find "$raw" -name '*kernel_trace.csv' | sort | tail -n 1)
    python3 bench/prof_summary.py "$tr" --window-ms 200 --by-grid > "$o/grid_$n.md"
    rm -rf "$raw"
    tail -n 1 "$o/bench_$n.log" | cut -c1-200
  done ;;
r6e)  # split QKV prologue in decode attention (partials issued ahead of the K/V preloads): tests + same-box A/B vs depth 4 (classic)
  pyt e_tests 600 tests/test_fused_decode_gpu.py
  run e_cold 200 python -u bench/decode_cold.py --graph --depth 2 4 3 --splits 1 2 4
  run e_cold_b1 200 python -u bench/decode_cold.py --graph --B 1 --L 768 --depth 2 4 --splits 4 8 16
  for r in 1 2; do
    run "c64_split_$r" 250 $B --steps 300 --warmup 30
    run "c64_classic_$r" 250 env XGS_TUNE=decode_depth=4 $B --steps 300 --warmup 30
    run "c1_split_$r" 200 $B --concurrency 1 --steps 300 --warmup 30
    run "c1_classic_$r" 200 env XGS_TUNE=decode_depth=4 $B --concurrency 1 --steps 300 --warmup 30
  done ;;
r6w)  # gate_up on gemm_pf at 448-512-row mixed steps: same-box A/B at --prompt-len 416 (479-row steps)
  for r in 1 2; do
    run "p416_new_$r" 250 $B --steps 400 --warmup 40 --prompt-len 416
    run "p416_old_$r" 250 env XGS_TUNE=pf_windows=gate_up:513-576/down:513-576 $B --steps 400 --warmup 40 --prompt-len 416
  done ;;
r6d)  # 70B TP8 rank, batch 1: down-projection plans under GG_AR (same box)
  for pl in base "8192x3584x1@16=1,1,9" "8192x3584x1@16=1,2,9" "8192x3584x1@16=2,2,6" "8192x3584x1@16=1,2,5"; do
    n=$(echo "$pl" | tr -c 'A-Za-z0-9_\n' '_')
    if [ "$pl" = base ]; then e="XGS_TUNE=krot=1"; else e="XGS_TUNE=m64_plans=$pl"; fi
    run "tp8_$n" 300 env $e $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20
  done ;;
r6t)  # same-box A/B: 128-tile statistics at M <= 16 vs the pair combine (70B TP8 rank, 8B batch 1)
  for r in 1 2; do
    for v in 64 128; do
      run "tp8_c1_t${v}_$r" 300 env XGS_TUNE=small_m_tiles=$v $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20
    done
  done
  for v in 64 128; do
    run "c1_t$v" 200 env XGS_TUNE=small_m_tiles=$v $B --concurrency 1 --steps 300 --warmup 30
  done ;;
r6b)  # 128-tile statistics (no GG_AR pair combine at TP8), measured pf windows: tests + A/Bs
  pyt b_tests 900 tests/test_fused_decode_gpu.py tests/test_custom_ar_gpu.py tests/test_pf_gpu.py tests/test_engine_gpu.py
  pyt moe_tests 400 tests/test_kernels_gpu.py -k "moe or mixtral or expert"
  run mix_c1 300 $B --model mixtral-8x7b --concurrency 1 --steps 100 --warmup 10
  run tp8_c1 300 $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20
  run driver 200 $B --steps 20 --warmup 5
  run p384_new 250 $B --steps 400 --warmup 40 --prompt-len 384
  run p384_old 250 env XGS_TUNE=pf_windows=gate_up:513-576 $B --steps 400 --warmup 40 --prompt-len 384 ;;
r6p)  # gemm_pf vs the tuned library GEMMs over the prompt-sized step range (the pf decision table)
  run pfsweep 900 python -u bench/pf_gemm_bench.py --no-check --rounds 3 --iters 10 --cfgs 2 4 8 3 7 6 \
      --shapes gate_up down_p qkv_p o_p --M 320 384 448 512 575 640 768 896 1024 1280 1536 2048 3072 4096 8192 ;;
r6s)  # m64g sweeps: deep four-x-tile rings at the 8B decode shapes (M 64), deep splits at M 1
  pyt pf_tests 300 tests/test_pf_gpu.py
  run sweep64 500 python -u bench/gemm_bench.py --m64g-sweep --M 64 --shapes qkv o down gate_up
  run sweep1 600 python -u bench/gemm_bench.py --m64g-sweep --M 1 --shapes qkv70t8 o70t8 down70t8 gate_up70t8 qkv o down \
      --splits 1 2 3 4 6 8 10 12 16 20 24 32 ;;
r6q)
  pyt wq_tests 600 tests/test_wq_gpu.py tests/test_fp8_gpu.py
  for q in int4 int8 fp8; do
    run "c1_$q" 200 $B --concurrency 1 --steps 200 --warmup 20 --weight-dtype $q "$@"
    run "c64_$q" 200 $B --steps 20 --warmup 5 --weight-dtype $q "$@"
  done ;;
r6a)
  pyt tp_tests 900 tests/test_custom_ar_gpu.py tests/test_tp_gpu.py
  run bench_driver 200 $B --steps 20 --warmup 5 "$@"
  run tp8_c1 300 $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20 "$@" ;;
tp)
  pyt tp_tests 600 tests/test_custom_ar_gpu.py tests/test_rccl_gpu.py tests/test_tp_gpu.py
  run tp8_c1 300 $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20 "$@"
  run tp8_c64 300 $B --model llama3-70b --tp-shard 8 --steps 60 --warmup 20 "$@" ;;
moe)
  pyt moe_tests 400 tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "moe or mixtral or expert"
  run mixtral_c64 300 $B --model mixtral-8x7b --steps 60 --warmup 20 "$@"
  run mixtral_c1 300 $B --model mixtral-8x7b --concurrency 1 --steps 60 --warmup 10 "$@"
  run mixtral_tp2_c64 300 $B --model mixtral-8x7b --tp-shard 2 --steps 60 --warmup 20 "$@" ;;
prefill)
  pyt prefill_tests 300 tests/test_kernels_gpu.py -k prefill
  run prefill 300 python -u bench/prefill_bench.py
  run c64 200 $B --steps 200 --warmup 40 "$@" ;;
serve)
  run bench_long 300 $B --steps 3000 --warmup 100
  run serve 400 python -u bench/serve_bench.py --launch "--model llama3-8b --max-num-seqs 64" --concurrency 64 \
      --prompt-len 512 --output-len 256 --warmup 40 --duration 40 --out "$o/serve_8b_c64.jsonl" "$@"
  run serve_fe2 400 python -u bench/serve_bench.py --launch "--model llama3-8b --max-num-seqs 64 --frontends 2" \
      --concurrency 64 --prompt-len 512 --output-len 256 --warmup 40 --duration 40 --out "$o/serve_8b_c64.jsonl" "$@" ;;
tune)
  export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=100
  export XGS_GEMM_TUNING=0   # tune from scratch (do not replay the shipped table)
  for spec in "c64:--steps 120 --warmup 40" "c1:--concurrency 1 --steps 40 --warmup 10" \
              "c8:--concurrency 8 --steps 60 --warmup 20" "mixtral_c64:--model mixtral-8x7b --steps 40 --warmup 20" \
              "mixtral_c1:--model mixtral-8x7b --concurrency 1 --steps 30 --warmup 10"; do
    n=${spec%%:*}
    run "t_$n" 600 env PYTORCH_TUNABLEOP_FILENAME="$o/t_$n.csv" $B ${spec#*:}
  done
  run t_prefill 600 env PYTORCH_TUNABLEOP_FILENAME="$o/t_prefill.csv" python -u bench/prefill_bench.py ;;
sweep)
  run sweep 500 python -u bench/gemm_bench.py --m64g-sweep --M 1 16 32 64 --shapes \
      qkv70t8 o70t8 gate_up70t8 down70t8 qkv8t2 o8t2 gate_up8t2 down8t2 qkv8t4 o8t4 gate_up8t4 down8t4 \
      qkv8t8 o8t8 gate_up8t8 down8t8 qkv70t2 o70t2 gate_up70t2 down70t2 qkv70t4 o70t4 gate_up70t4 down70t4 ;;
arsim)  # simulated xGMI all-reduce latency on one rank of 70B TP8 (XGS_SIM_AR_US), with / without prefetch
  for cfgv in "XGS_TUNE=sim_ar_us=0" "XGS_TUNE=sim_ar_us=4" "XGS_TUNE=sim_ar_us=8"; do
    n=$(echo "$cfgv" | tr -c 'A-Za-z0-9_=\n' '_')
    run "c1_$n" 300 env $cfgv $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20 "$@"
  done ;;
coalesce)  # admission window A/B (EngineConfig.prompt_coalesce)
  for k in ${XGS_COALESCE_LIST:-1 2 3}; do
    run "driver_k$k" 200 $B --steps 20 --warmup 5 --coalesce $k "$@"
    run "long_k$k" 300 $B --steps 1000 --warmup 100 --coalesce $k "$@"
  done ;;
profile)
  bash bench/profile.sh "$o" "$@" ;;
mw)  # gemm_mw: numerics, shape sweep, stall-free mixed-step engine tests, headline with / without chunks
  pyt mw_tests 300 tests/test_skinny_gpu.py -k mw
  run mw_sweep 700 python -u bench/gemm_bench.py --mw-sweep --M 64 128 192 256 320 --shapes qkv o gate_up down
  pyt stall_free 300 tests/test_engine_gpu.py -k "stall_free or graph_decode or chunked or async"
  run c64_chunk128 200 $B --steps 20 --warmup 5 --prefill-chunk 128 "$@"
  run c64_chunk128_long 240 env XGS_STEP_LOG="$o/steps_chunk128.jsonl" $B --steps 600 --warmup 60 --prefill-chunk 128 "$@"
  run c64_chunk128_lib 240 env XGS_TUNE=mw_max_tokens=0 $B --steps 600 --warmup 60 --prefill-chunk 128 "$@"
  run c64_base_long 240 $B --steps 600 --warmup 60 "$@" ;;
m64)  # decode GEMM plans: LM head on gemm_mw, deep-ring / uneven-split gemm_m64g tests and sweeps
  run mw_sweep_lm 200 python -u bench/gemm_bench.py --mw-sweep --M 64 65 --shapes lm_head --top 3
  pyt deep_ring 200 tests/test_skinny_gpu.py -k "deep_ring or uneven"
  run m64g_sweep 700 python -u bench/gemm_bench.py --m64g-sweep --M 1 64 --shapes qkv o gate_up down ;;
r4b)  # round 4: all-reduce protocols, TP tests (async mixed steps), batch-1 Infinity-Cache prefetch A/B
  pyt ar_tests 600 tests/test_custom_ar_gpu.py
  run ar_bench 240 python -u bench/ar_bench.py --world 2 4 8
  pyt tp_tests 500 tests/test_tp_gpu.py
 ;;
r4c)  # round 4: Mixtral with / without prompt chunks, profiles of the chunked headline and Mixtral batch 1
  run mixtral_c1 300 $B --model mixtral-8x7b --concurrency 1 --steps 60 --warmup 10
  run mixtral_c64_chunk 300 $B --model mixtral-8x7b --steps 120 --warmup 20 --prefill-chunk 128
  run mixtral_c64 300 $B --model mixtral-8x7b --steps 120 --warmup 20
  bash bench/profile.sh "$o/prof_chunk128" --prefill-chunk 128
  bash bench/profile.sh "$o/prof_mixtral_c1" --model mixtral-8x7b --concurrency 1 ;;
r4d)  # round 4: batched in-launch residual reduce at M = 64 (GG_RESID) vs add_partials_resid;
      # decode attention with 2 / 3 register tiles in flight per wave (cold cache)
  pyt fused_tests 400 tests/test_fused_decode_gpu.py
  run attn_cold 200 python -u bench/decode_cold.py --L 768 --splits 1 --depth 2 3
  run attn_cold_2k 200 python -u bench/decode_cold.py --L 2048 --caches 3 --splits 1 --depth 2 3
  for v in "XGS_TUNE=resid_inlaunch_kb=32" "XGS_TUNE=resid_inlaunch_kb=1024" "XGS_TUNE=decode_depth=3"; do
    n=$(echo "$v" | tr -c 'A-Za-z0-9_=\n' '_')
    run "steplog_$n" 240 env $v XGS_STEP_LOG="$o/steps_$n.jsonl" $B --steps 400 --warmup 40 "$@"
  done ;;
r4e)  # round 4 re-entry: MoE/mw numerics diagnostic, GPU tests, headline, mw2 sweep, chunked headline
  run diag 200 python -u bench/diag_moe_mw.py
  pyt_soft gputests 900 tests -m gpu --maxfail=10 --deselect "tests/test_fused_decode_gpu.py::test_mixtral_decode_step_logits_match_reference"
  run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
  run bench_driver 200 $B --steps 20 --warmup 5 "$@"
  run mw_sweep 500 python -u bench/gemm_bench.py --mw-sweep --M 64 128 192 256 --shapes qkv o gate_up down --top 8
  run c64_chunk128 240 env XGS_STEP_LOG="$o/steps_chunk128.jsonl" $B --steps 600 --warmup 60 --prefill-chunk 128 "$@"
  run c64_base 240 env XGS_STEP_LOG="$o/steps_base.jsonl" $B --steps 600 --warmup 60 "$@" ;;
r4f)  # round 4: decode / prompt GEMM overlap probe, then the r4d and r4b A/Bs
  run overlap 200 python -u bench/overlap_probe.py --prompt 256 512 1024
  run overlap_prio 200 python -u bench/overlap_probe.py --prompt 512 --prio
  bash "$0" r4d r4f_d "$@" || exit $?
  bash "$0" r4b r4f_b "$@" || exit $? ;;
r4g)  # round 4: gemm_mw anatomy probes, AR latency at world 4 / 8, batch-1 prefetch A/B, c64 profile
  run mw_probe 300 python -u bench/gemm_bench.py --mw-probe --M 64 128 192 256 --shapes gate_up down qkv o
  bash bench/profile.sh "$o/prof_c64" "$@" ;;
r4h)  # round 4: K-chunk rotation -- kernel tests, m64g / mw / LM-head sweeps, engine A/B (XGS_KROT)
  run m64g_sweep 300 python -u bench/gemm_bench.py --m64g-sweep --M 64 --shapes gate_up qkv o down
  run m64g_sweep_off 300 env XGS_TUNE=krot=0 python -u bench/gemm_bench.py --m64g-sweep --M 64 --shapes gate_up
  pyt mw3_tests 300 tests/test_skinny_gpu.py -k "mw"
  run mw_sweep 500 python -u bench/gemm_bench.py --mw-sweep --M 64 128 192 256 --shapes gate_up down qkv o lm_head --top 5
  for v in "XGS_TUNE=krot=1" "XGS_TUNE=krot=0" "XGS_TUNE=krot=2"; do
    n=$(echo "$v" | tr -c 'A-Za-z0-9_=\n' '_')
    run "c64_$n" 240 env $v XGS_STEP_LOG="$o/steps_$n.jsonl" $B --steps 600 --warmup 60 "$@"
  done
  run c1 150 $B --concurrency 1 --steps 200 --warmup 20 "$@"
  run c1_off 150 env XGS_TUNE=krot=0 $B --concurrency 1 --steps 200 --warmup 20 "$@" ;;
r4i)  # round 4: full GPU tests + smoke + headline with rotation and the LM head on gemm_mw; MoE rotation A/B
  pyt_soft gputests 900 tests -m gpu --maxfail=10
  run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
  run bench_driver 200 $B --steps 20 --warmup 5 "$@"
  run c64_long 240 env XGS_STEP_LOG="$o/steps_c64.jsonl" $B --steps 600 --warmup 60 "$@"
  run c1 150 $B --concurrency 1 --steps 200 --warmup 20 "$@"
  for v in "XGS_TUNE=krot=1" "XGS_TUNE=krot=0"; do
    n=$(echo "$v" | tr -c 'A-Za-z0-9_=\n' '_')
    run "mixtral_c1_$n" 200 env $v $B --model mixtral-8x7b --concurrency 1 --steps 60 --warmup 10
    run "mixtral_c64_$n" 240 env $v $B --model mixtral-8x7b --steps 120 --warmup 20
  done
  bash bench/profile.sh "$o/prof_c64" "$@" ;;
r4j)  # round 4: whole-prompt mixed graphs (library GEMMs) A/B, decode-attention anatomy
  pyt mixed_tests 300 tests/test_engine_gpu.py -k "whole_prompt or stall_free"
  run attn_probe 200 python -u bench/decode_cold.py --L 768 --splits 1 --probe
  run c64_chunk512 240 env XGS_STEP_LOG="$o/steps_chunk512.jsonl" $B --steps 600 --warmup 60 --prefill-chunk 512 "$@"
  run c64_chunk512_driver 200 $B --steps 20 --warmup 5 --prefill-chunk 512 "$@"
  run c64_base 240 env XGS_STEP_LOG="$o/steps_base.jsonl" $B --steps 600 --warmup 60 "$@" ;;
r4k)  # round 4: Mixtral profiles (batch 1, 64 concurrent, TP2 shard), AR latency at world 4 / 8
  bash bench/profile.sh "$o/prof_mixtral_c1" --model mixtral-8x7b --concurrency 1
  bash bench/profile.sh "$o/prof_mixtral_c64" --model mixtral-8x7b
  run mixtral_tp2_c64 300 $B --model mixtral-8x7b --tp-shard 2 --steps 60 --warmup 20
  run ar_w4 200 python -u bench/ar_bench.py --world 4
  run ar_w8 240 python -u bench/ar_bench.py --world 8 ;;
r4l)  # round 4: one-round-trip MoE router -- MoE tests, Mixtral batch 1 / 64 concurrent / TP2 shard
  pyt moe_tests 400 tests/test_kernels_gpu.py tests/test_fused_decode_gpu.py tests/test_engine_gpu.py -k "moe or mixtral or expert or route"
  run mixtral_c1 200 $B --model mixtral-8x7b --concurrency 1 --steps 100 --warmup 10
  run mixtral_c64 240 $B --model mixtral-8x7b --steps 120 --warmup 20
  run mixtral_tp2_c64 300 $B --model mixtral-8x7b --tp-shard 2 --steps 60 --warmup 20
  run mixtral_tp2_c1 200 $B --model mixtral-8x7b --tp-shard 2 --concurrency 1 --steps 100 --warmup 10 ;;
r4m)  # round 4: re-sweep the batch-1 / 32-row gemm_m64g plans with K rotation, then the headline and batch 1
  run m64g_sweep_1 400 python -u bench/gemm_bench.py --m64g-sweep --M 1 32 --shapes qkv o gate_up down
  run c64 240 $B --steps 600 --warmup 60 "$@"
  run c1 150 $B --concurrency 1 --steps 200 --warmup 20 "$@" ;;
r4n)  # round 4: re-swept batch-1 / 32-row plans vs the round-3 ones, decode splits at batch 1, QKV S=4 vs 5 at 64 rows
  pyt plan_tests 300 tests/test_skinny_gpu.py tests/test_fused_decode_gpu.py -k "m64 or deep_ring or uneven or logits"
  OLD16="6144x4096x1@16=2,8,5;4096x4096x1@16=2,4,4;28672x4096x2@16=2,1,6;4096x14336x1@16=2,4,6"
  run c1_new 150 $B --concurrency 1 --steps 300 --warmup 20
  run c1_old 150 env XGS_TUNE=m64_plans="$OLD16" $B --concurrency 1 --steps 300 --warmup 20
  for sp in 1 4; do
    run c1_splits$sp 150 env XGS_TUNE=decode_max_splits=$sp $B --concurrency 1 --steps 300 --warmup 20
  done
  run c8 150 $B --concurrency 8 --steps 200 --warmup 20
  run c64_qkv5 240 $B --steps 600 --warmup 60
  run c64_qkv4 240 env XGS_TUNE=m64_plans="6144x4096x1@64=2,4,3" $B --steps 600 --warmup 60
  run mixtral_c1 200 $B --model mixtral-8x7b --concurrency 1 --steps 100 --warmup 10 ;;
r4o)  # round 4: kernel profiles of batch 1 and 64 concurrent on the final plans; TP-shard plan re-sweep (K rotation)
  bash bench/profile.sh "$o/prof_c1" --concurrency 1
  bash bench/profile.sh "$o/prof_c64"
  run sweep_tp 600 python -u bench/gemm_bench.py --m64g-sweep --M 1 64 --shapes \
      qkv70t8 o70t8 gate_up70t8 down70t8 qkv70t2 o70t2 gate_up70t2 down70t2 qkv70t4 o70t4 gate_up70t4 down70t4 ;;
final)  # round-end gate: every GPU test, smoke, the driver form twice, a 3000-step window, batch 1, the c64 profile
  pyt_soft gputests 900 tests -m gpu --maxfail=10
  run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
  run driver_a 200 $B --steps 20 --warmup 5 "$@"
  run driver_b 200 $B --steps 20 --warmup 5 "$@"
  run long 300 $B --steps 3000 --warmup 100 "$@"
  run c1 150 $B --concurrency 1 --steps 300 --warmup 20 "$@"
  bash bench/profile.sh "$o/prof_c64" "$@" ;;
r4p)  # round 4: one rank of the Llama-3-70B TP8 group (config 4 proxy), 70B TP1, batch 1 and 64 concurrent
  run tp8_c1 300 $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20
  run tp8_c64 300 $B --model llama3-70b --tp-shard 8 --steps 60 --warmup 20
  run tp1_c1 300 $B --model llama3-70b --concurrency 1 --steps 40 --warmup 10
  run tp1_c64 300 $B --model llama3-70b --steps 40 --warmup 10 ;;
r4q)  # round 4: two-stream overlap with the decode GEMMs on 72-KB-LDS (KC 64) configurations
  run overlap_kc64 200 env XGS_TUNE=m64_plans="4096x4096x1@64=1,4,2;28672x4096x2@64=2,1,3" \
      python -u bench/overlap_probe.py --prompt 512 1024
  run overlap_base 200 python -u bench/overlap_probe.py --prompt 512 1024 ;;
r4r)  # round 4: decode attention with non-temporal K/V loads (depth 14 = PR 4), kernel + engine A/B
  run dnt_768 200 python -u bench/decode_cold.py --depth 2 14 --splits 1 2
  run dnt_2k 200 python -u bench/decode_cold.py --L 2048 --depth 2 14 --splits 1
  run eng_base 300 python -u bench.py --steps 600 --warmup 50
  run eng_nt 300 env XGS_TUNE=decode_depth=14 python -u bench.py --steps 600 --warmup 50
  run eng_base2 300 python -u bench.py --steps 600 --warmup 50 ;;
r4s)  # round 4: non-temporal K/V loads as the default -- numerics, then batch 1 / 64 / 70B A/Bs (14 = cached loads)
  pyt attn_tests 400 tests/test_fused_decode_gpu.py tests/test_kernels_gpu.py -k "decode or attention"
  run c1_nt 300 $B --concurrency 1 --steps 300 --warmup 30
  run c1_cached 300 env XGS_TUNE=decode_depth=14 $B --concurrency 1 --steps 300 --warmup 30
  run c1_nt2 300 $B --concurrency 1 --steps 300 --warmup 30
  run c64_nt 300 $B --steps 1000 --warmup 100
  run c64_cached 300 env XGS_TUNE=decode_depth=14 $B --steps 1000 --warmup 100
  run tp8_c1 300 $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20
  run tp8_c64 300 $B --model llama3-70b --tp-shard 8 --steps 60 --warmup 20 ;;
r4t)  # round 4: all-reduce prologue in the next GEMM (gemm_m64g_arx): tests, then simulated-TP8 70B batch 1 A/B
  pyt arx_tests 400 tests/test_ar_prologue_gpu.py
  pyt fused_tests 400 tests/test_fused_decode_gpu.py
  run tp8_ar0_base 300 env XGS_TUNE=sim_ar_us=0 $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20
  run tp8_ar8_base 300 env XGS_TUNE=sim_ar_us=8 $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 20
  run c64_default 300 $B --steps 600 --warmup 50 ;;
r4u)  # round 4: decode-attention depth / page size with the non-temporal K/V loads
  run dnt_depth 200 python -u bench/decode_cold.py --depth 2 3 --splits 1
  run dnt_depth_2k 200 python -u bench/decode_cold.py --L 2048 --depth 2 3 --splits 1
  run dnt_bs32 200 python -u bench/decode_cold.py --bs 32 --depth 2 3 --splits 1 ;;
r4v)  # round 4: K rotation for every split (XGS_TUNE=krot=2) and non-temporal O-projection plans, c64 / c1 A/B
  run c64_base 300 $B --steps 600 --warmup 50
  run c64_krot2 300 env XGS_TUNE=krot=2 $B --steps 600 --warmup 50
  run c64_ont 300 env XGS_TUNE=m64_plans="4096x4096x1@64=1,4,1;4096x4096x1@32=1,4,1" $B --steps 600 --warmup 50
  run c64_base2 300 $B --steps 600 --warmup 50
  run c1_base 300 $B --concurrency 1 --steps 300 --warmup 30
  run c1_krot2 300 env XGS_TUNE=krot=2 $B --concurrency 1 --steps 300 --warmup 30
  run c1_ont 300 env XGS_TUNE=m64_plans="4096x4096x1@16=1,3,1" $B --concurrency 1 --steps 300 --warmup 30 ;;
r4w)  # round 4: split attention combine inside the O GEMM (gemm_m64g_xl): tests, batch-1 / batch-8 A/B
  pyt xl_tests 400 tests/test_fused_decode_gpu.py -k "xl or combines or logits"
  run c1_base 300 $B --concurrency 1 --steps 300 --warmup 30
  run c1_xl 300 env XGS_XL_COMBINE=1 $B --concurrency 1 --steps 300 --warmup 30
  run c1_base2 300 $B --concurrency 1 --steps 300 --warmup 30
  run c1_xl2 300 env XGS_XL_COMBINE=1 $B --concurrency 1 --steps 300 --warmup 30
  run c8_base 300 $B --concurrency 8 --steps 200 --warmup 30
  run c8_xl 300 env XGS_XL_COMBINE=1 $B --concurrency 8 --steps 200 --warmup 30 ;;
r4x)  # round 4: decode-attention split target at batch 1 / 8 (16 / 8 / 4 splits at batch 1; needed a temporary XGS_DECODE_SPLIT_WGS override of ModelRunner.DECODE_SPLIT_WGS)
  run c1_512 300 $B --concurrency 1 --steps 300 --warmup 30
  run c1_64 300 env XGS_DECODE_SPLIT_WGS=64 $B --concurrency 1 --steps 300 --warmup 30
  run c1_32 300 env XGS_DECODE_SPLIT_WGS=32 $B --concurrency 1 --steps 300 --warmup 30
  run c1_512b 300 $B --concurrency 1 --steps 300 --warmup 30
  run c8_512 300 $B --concurrency 8 --steps 200 --warmup 30
  run c8_128 300 env XGS_DECODE_SPLIT_WGS=128 $B --concurrency 8 --steps 200 --warmup 30 ;;
r4y)  # round 4: re-tune the config-3 library GEMMs with a 5x longer TunableOp budget per shape
  export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=500
  export XGS_GEMM_TUNING=0
  run t_c64_long 900 env PYTORCH_TUNABLEOP_FILENAME="$o/t_c64_long.csv" $B --steps 120 --warmup 40 ;;
r4z)  # round 4: the re-tuned mixed-step QKV entry in the shipped TunableOp table
  run c64_a 300 $B --steps 600 --warmup 50
  run driver 200 $B --steps 20 --warmup 5
  run c64_b 300 $B --steps 600 --warmup 50 ;;
r5a)  # round 5: gemm_pf (prompt-sized MFMA GEMM) -- numerics, per-projection A/B vs the library at the
      # mixed-step rows, then the headline with gemm_pf on / off and its kernel profile
  pyt pf_tests 300 tests/test_pf_gpu.py
  pyt moe_resid 200 tests/test_fused_decode_gpu.py -k "combine_resid or mixtral"
  run pf_gate_up 300 python -u bench/pf_gemm_bench.py --shapes gate_up --M 575 1024 --cfgs 1 3 4 --sk 0 256 --rounds 3 --iters 10
  run pf_gate_up288 300 python -u bench/pf_gemm_bench.py --shapes gate_up --M 575 1024 --cfgs 5 --sk 0 --rounds 3 --iters 10
  run pf_proj 300 python -u bench/pf_gemm_bench.py --shapes qkv_p o_p down_p --M 575 --cfgs 4 5 --splits 1 2 3 5 8 --rounds 3 --iters 10
  run pf_proj_sk 300 python -u bench/pf_gemm_bench.py --shapes qkv o down --M 575 --cfgs 2 4 --sk 0 256 --rounds 3 --iters 10
  run c64_pf 300 $B --steps 400 --warmup 40 "$@"
  run c64_lib 300 env XGS_TUNE=pf=0 $B --steps 400 --warmup 40 "$@"
  run c64_pf_driver 200 $B --steps 20 --warmup 5 "$@"
  bash bench/profile.sh "$o/prof_c64" "$@" ;;
r5b)  # r5a after the gate_up sweep
  run pf_gate_up288 300 python -u bench/pf_gemm_bench.py --shapes gate_up --M 575 1024 --cfgs 5 --sk 0 --rounds 3 --iters 10
  run pf_proj 300 python -u bench/pf_gemm_bench.py --shapes qkv_p o_p down_p --M 575 --cfgs 4 5 --splits 1 2 3 5 8 --rounds 3 --iters 10
  run pf_proj_sk 300 python -u bench/pf_gemm_bench.py --shapes qkv o down --M 575 --cfgs 2 4 --sk 0 256 --rounds 3 --iters 10
  run c64_pf 300 $B --steps 400 --warmup 40 "$@"
  run c64_lib 300 env XGS_TUNE=pf=0 $B --steps 400 --warmup 40 "$@"
  bash bench/profile.sh "$o/prof_c64" "$@" ;;
r5c)  # gemm_pf anatomy at the mixed-step shapes (tuned library baselines)
  run pf_probe 300 python -u bench/pf_gemm_bench.py --shapes gate_up --M 575 --cfgs 5 --sk 0 --probe --rounds 3 --iters 10
  run pf_probe2 300 python -u bench/pf_gemm_bench.py --shapes qkv_p o_p down_p --M 575 --cfgs 4 5 --splits 3 5 8 --probe --rounds 3 --iters 10
  run pf_sq 300 python -u bench/pf_gemm_bench.py --shapes sq8k --M 8192 --cfgs 3 --sk 0 --probe --rounds 2 --iters 5 ;;
r5d)  # gemm_pf DMA lag 2 (template-form fragment waits) vs lag 1
  pyt pf_tests 300 tests/test_pf_gpu.py -k "cfgs or streamk"
  run pf_lag 300 python -u bench/pf_gemm_bench.py --shapes gate_up --M 575 --cfgs 5 6 3 7 0 --sk 0 --probe --rounds 3 --iters 10
  run pf_lag_sq 300 python -u bench/pf_gemm_bench.py --shapes sq8k --M 8192 --cfgs 3 7 0 --sk 0 --rounds 2 --iters 5 ;;
r5e)  # gemm_pf cfg sweep for the planner fit (lag-2 configs), then the headline on / off
  pyt pf_tests 300 tests/test_pf_gpu.py
  run pf_gu 300 python -u bench/pf_gemm_bench.py --shapes gate_up --M 512 575 1024 --cfgs 3 4 6 8 --sk 0 256 --rounds 3 --iters 10 --no-check
  run pf_pr 300 python -u bench/pf_gemm_bench.py --shapes qkv_p o_p down_p --M 575 1024 --cfgs 2 4 6 8 --splits 2 3 4 5 8 --rounds 3 --iters 10 --no-check
  run c64_pf 300 $B --steps 400 --warmup 40 "$@"
  run c64_lib 300 env XGS_TUNE=pf=0 $B --steps 400 --warmup 40 "$@" ;;
r5f)  # gemm_pf per-projection A/B in the headline (400 steps each, then the driver form)
  run c64_gu 300 env XGS_TUNE=pf=gate_up $B --steps 400 --warmup 40 "$@"
  run c64_gud 300 env XGS_TUNE=pf=gate_up,down $B --steps 400 --warmup 40 "$@"
  run c64_all 300 env XGS_TUNE=pf=qkv,o,gate_up,down $B --steps 400 --warmup 40 "$@"
  run c64_lib 300 env XGS_TUNE=pf=0 $B --steps 400 --warmup 40 "$@"
  run c64_gud2 300 env XGS_TUNE=pf=gate_up,down $B --steps 400 --warmup 40 "$@"
  run c64_gu2 300 env XGS_TUNE=pf=gate_up $B --steps 400 --warmup 40 "$@" ;;
r5m)  # MoE with the combine in the w2 launch: tests, Mixtral c1 / c64 / TP2-EP2 rank, c1 profile; 8K prefill
  pyt moe_tests 400 tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_fused_decode_gpu.py -k "moe or mixtral or expert"
  run mixtral_c1 300 $B --model mixtral-8x7b --concurrency 1 --steps 100 --warmup 10 "$@"
  run mixtral_c64 300 $B --model mixtral-8x7b --steps 100 --warmup 20 "$@"
  run mixtral_tp2_c64 300 $B --model mixtral-8x7b --tp-shard 2 --steps 100 --warmup 20 "$@"
  bash bench/profile.sh "$o/prof_mixtral_c1" --model mixtral-8x7b --concurrency 1 "$@"
  run prefill 300 python -u bench/prefill_bench.py ;;
r5t)  # TP decode: all-reduce inside the row-parallel GEMMs (GG_AR) -- loopback + self-test + TP engine
      # tests, then one simulated 70B TP8 rank at batch 1 / 64 with it on / off, simulated links 0 / 8 us
  pyt gar_tests 300 tests/test_gemm_ar_gpu.py
  pyt ar_selftest 400 tests/test_custom_ar_gpu.py -k self_test
  [ -n "$R5T_SKIP_TP" ] || pyt tp_tests 600 tests/test_tp_gpu.py
  run tp8_c1 300 $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 10 "$@"
  run tp8_c1_off 300 env XGS_TUNE=gemm_ar=0 $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 10 "$@"
  run tp8_c1_ar8 300 env XGS_TUNE=sim_ar_us=8 $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 10 "$@"
  run tp8_c1_ar8_off 300 env "XGS_TUNE=sim_ar_us=8|gemm_ar=0" $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 10 "$@"
  run tp8_c4 300 $B --model llama3-70b --tp-shard 8 --concurrency 4 --steps 100 --warmup 20 "$@"
  run tp8_c4_off 300 env XGS_TUNE=gemm_ar=0 $B --model llama3-70b --tp-shard 8 --concurrency 4 --steps 100 --warmup 20 "$@"
  run tp8_c64 300 $B --model llama3-70b --tp-shard 8 --steps 100 --warmup 20 "$@"
  run c64 300 $B --steps 400 --warmup 40 ;;
r5p)  # round-5 kernel tables of the defaults: 8B c64 / c1, 70B TP8 shard c1
  bash bench/profile.sh "$o/prof_c64" "$@" &&
  bash bench/profile.sh "$o/prof_c1" --concurrency 1 "$@" &&
  bash bench/profile.sh "$o/prof_tp8_c1" --model llama3-70b --tp-shard 8 --concurrency 1 "$@" ;;
r5s)  # host side of the headline: per-phase host timing and per-step wall log
  run c64_t 300 env XGS_STEP_TIMING=1 XGS_STEP_LOG=$o/steps.jsonl $B --steps 400 --warmup 40 "$@"
  run c64 300 $B --steps 400 --warmup 40 "$@" ;;
r5q)  # gemm_pf projection sets again after the planner refit (interleaved, two passes)
  for pass in 1 2; do
    run c64_def_$pass 300 $B --steps 400 --warmup 40 "$@"
    run c64_qkv_$pass 300 env XGS_TUNE=pf=qkv,gate_up,down $B --steps 400 --warmup 40 "$@"
    run c64_o_$pass 300 env XGS_TUNE=pf=o,gate_up,down $B --steps 400 --warmup 40 "$@"
    run c64_all_$pass 300 env XGS_TUNE=pf=qkv,o,gate_up,down $B --steps 400 --warmup 40 "$@"
  done ;;
r5z)  # round-5 closing gate: every GPU test, smoke, the headline (driver form x2, 3000 steps), batch 1,
      # Mixtral c64 / c1 / TP2 shard, 70B TP8 shard c1, the 8K TTFT, a c64 kernel profile
  pyt_soft gputests 900 tests -m gpu --maxfail=10
  run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
  run driver_a 200 $B --steps 20 --warmup 5
  run driver_b 200 $B --steps 20 --warmup 5
  run long 300 $B --steps 3000 --warmup 100
  run c1 150 $B --concurrency 1 --steps 300 --warmup 30
  run mx_c64 300 $B --model mixtral-8x7b --steps 100 --warmup 20
  run mx_c1 300 $B --model mixtral-8x7b --concurrency 1 --steps 150 --warmup 20
  run mx_tp2 300 $B --model mixtral-8x7b --tp-shard 2 --steps 100 --warmup 20
  run tp8_c1 300 $B --model llama3-70b --tp-shard 8 --concurrency 1 --steps 100 --warmup 10
  run ttft8k 300 python -u bench/prefill_bench.py --lens
  bash bench/profile.sh "$o/prof_c64" ;;
r5k)  # where the c64 step idles: kernel-trace-only profile (no HIP API trace), gaps by neighbouring kernels
  run c64_plain 300 $B --steps 400 --warmup 40 "$@"
  raw=$(mktemp -d "$TMPDIR/xgs_k.XXXXXX")
  run c64_ktrace 400 rocprofv3 --kernel-trace --output-format csv -d "$raw" -o run -- \
      python3 bench.py --steps 400 --warmup 40 "$@"
  trace=$(find "$raw" -name '*kernel_trace.csv' | sort | tail -n 1)
  python3 bench/prof_summary.py "$trace" --window-ms 600 --gap-us 8 --top 30 > "$o/c64_kernels_gaps.md"
  run c1_plain 200 $B --concurrency 1 --steps 300 --warmup 30 "$@"
  run c1_ktrace 300 rocprofv3 --kernel-trace --output-format csv -d "$raw/c1" -o run -- \
      python3 bench.py --concurrency 1 --steps 300 --warmup 30 "$@"
  trace=$(find "$raw/c1" -name '*kernel_trace.csv' | sort | tail -n 1)
  python3 bench/prof_summary.py "$trace" --window-ms 300 --gap-us 4 --top 30 > "$o/c1_kernels_gaps.md"
  rm -rf "$raw" ;;
r5l)  # step-boundary gaps: kernel + HIP API trace, each gap's kernel matched to its enqueue call
  raw=$(mktemp -d "$TMPDIR/xgs_l.XXXXXX")
  run c64_htrace 400 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d "$raw" -o run -- \
      python3 bench.py --steps 300 --warmup 40 "$@"
  python3 bench/gap_corr.py "$raw" --window-ms 400 --min-us 8 --dump 3 > "$o/c64_gap_corr.md"
  rm -rf "$raw" ;;
ar)  # custom all-reduce: push (LL) vs pull protocols, correctness + latency
  pyt ar_tests 600 tests/test_custom_ar_gpu.py
  run ar_bench 300 python -u bench/ar_bench.py --world 2 4 8 ;;
dmaprobe)
  run dma_probe 120 ./bench/dma_probe.bin ;;
*)
  echo "unknown suite $suite"; exit 2 ;;
esac
