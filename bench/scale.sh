#!/usr/bin/env bash
# Multi-GPU scaling sheet for an 8-GPU MI355X node (NOT for the 1-GPU gpurun box):
#   * config 3 weak scaling: Llama-3-8B, 64 concurrent per replica, DP 1/2/4/8;
#   * config 4: Llama-3-70B TP8 (one replica over all 8 GPUs, custom xGMI all-reduce);
#   * config 5: Mixtral 8x7B TP2 / EP2 (expert all-to-all over xGMI);
#   * the serving path with per-request routing (BASELINE north star): `xgserve serve
#     --replicas N` (one process replica per GPU behind the C++ router and two HTTP
#     front ends), 64 x N SSE streams from bench/serve_bench.py: tok/s, TTFT p50 / p99
#     and the router's per-replica request split (replica_requests) per N.
# Every line is bench.py's JSON (rccl_world / tp_groups / p2p_ok / decode_ar record
# what the pre-flight saw); a TP run whose custom all-reduce did not register exits 3
# instead of reporting an RCCL-decode number.
#   bash bench/scale.sh [steps] [warmup]   ->  gpurun_out/scale.jsonl
set -u -o pipefail
cd "$(dirname "$0")/.."
STEPS=${1:-200}
WARM=${2:-40}
OUT=gpurun_out/scale.jsonl
mkdir -p gpurun_out
: > "$OUT"
NGPU=$(python -c 'import torch; print(torch.cuda.device_count())')
run() {  # label, timeout, args...
  local label=$1 tmo=$2
  shift 2
  echo "== $label" >&2
  timeout -k 10 "$tmo" python -u bench.py "$@" --steps "$STEPS" --warmup "$WARM" 2> "gpurun_out/scale_${label}.err" \
    | grep '^{' | python -c "import json,sys; [print(json.dumps(dict(json.loads(l), label='$label'))) for l in sys.stdin]" \
    | tee -a "$OUT"
}
for n in 1 2 4 8; do
  [ "$n" -le "$NGPU" ] || break
  run "dp$n" 900 --gpus "$n" || exit $?
done
serve() {  # n: DP replicas behind the router, 64 streams each
  local n=$1
  echo "== serve_dp$n" >&2
  timeout -k 10 1200 python -u bench/serve_bench.py --launch "--model llama3-8b --max-num-seqs 64 --replicas $n --frontends 2" \
    --concurrency $((64 * n)) --prompt-len 512 --output-len 256 --warmup 40 --duration 40 --procs $((4 * n)) \
    --label "serve_dp$n" 2> "gpurun_out/scale_serve_dp$n.err" | grep '^{' | tee -a "$OUT"
}
for n in 1 2 4 8; do
  [ "$n" -le "$NGPU" ] || break
  serve "$n" || exit $?
done
if [ "$NGPU" -ge 8 ]; then
  run "llama3-70b_tp8" 1200 --gpus 8 --tp 8 --model llama3-70b || exit $?
  run "llama3-70b_tp8_c1" 1200 --gpus 8 --tp 8 --model llama3-70b --concurrency 1 || exit $?
fi
if [ "$NGPU" -ge 2 ]; then
  run "mixtral_tp2" 1200 --gpus 2 --tp 2 --model mixtral-8x7b || exit $?
fi
python - "$OUT" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
base = next((r for r in rows if r["label"] == "dp1"), None)
print(f"{'label':22s} {'gpus':>4s} {'tok/s':>10s} {'ms/step':>8s} {'ttft p50':>8s} {'eff':>6s} {'decode_ar':>9s}")
for r in rows:
    if r["label"].startswith("serve_dp"):
        n = int(r["label"][len("serve_dp"):])
        sb = next((x for x in rows if x["label"] == "serve_dp1"), None)
        eff = r["value"] / (sb["value"] * n) if sb else None
        print(f"{r['label']:22s} {n:4d} {r['value']:10.1f} {'':>8s} {(r.get('ttft_p50_ms') or 0):8.1f} "
              f"{('%.3f' % eff) if eff else '':>6s} split={r.get('replica_requests')} ttft_p99={r.get('ttft_p99_ms')}")
        continue
    eff = (r["value"] / (base["value"] * r["n_gpus"])) if (base and r["label"].startswith("dp")) else None
    print(f"{r['label']:22s} {r['n_gpus']:4d} {r['value']:10.1f} {r['ms_per_step']:8.2f} "
          f"{(r.get('ttft_p50_ms') or 0):8.1f} {('%.3f' % eff) if eff else '':>6s} {str(r.get('decode_ar')):>9s}")
PY
