#!/usr/bin/env bash
# Multi-GPU scaling sheet for an 8-GPU MI355X node (NOT for the 1-GPU gpurun box):
#   * config 3 weak scaling: Llama-3-8B, 64 concurrent per replica, DP 1/2/4/8;
#   * config 4: Llama-3-70B TP8 (one replica over all 8 GPUs, custom xGMI all-reduce);
#   * config 5: Mixtral 8x7B TP2 / EP2 (expert all-to-all over xGMI).
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
    eff = (r["value"] / (base["value"] * r["n_gpus"])) if (base and r["label"].startswith("dp")) else None
    print(f"{r['label']:22s} {r['n_gpus']:4d} {r['value']:10.1f} {r['ms_per_step']:8.2f} "
          f"{(r.get('ttft_p50_ms') or 0):8.1f} {('%.3f' % eff) if eff else '':>6s} {str(r.get('decode_ar')):>9s}")
PY
