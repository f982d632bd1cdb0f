#!/usr/bin/env bash
# Kernel-level profile of the headline benchmark on one MI355X (run through gpurun):
#   bash bench/profile.sh [out_dir] [bench.py args...]
# Writes <out>/kernels.md (per-kernel time, GPU busy share) and <out>/gaps.md
# (host gaps between engine steps) from a rocprofv3 kernel + HIP API trace; the
# raw CSVs stay in $TMPDIR so gpurun_out/ stays small.
set -euo pipefail
out=${1:-gpurun_out/profile}
shift || true
export TMPDIR=${TMPDIR:-/tmp}
raw=$(mktemp -d "$TMPDIR/xgs_prof.XXXXXX")
mkdir -p "$out"
timeout -k 10 600 rocprofv3 --kernel-trace --hip-trace --output-format csv -d "$raw" -o run -- \
    python3 bench.py --steps 80 --warmup 30 "$@" > "$out/bench.log" 2>&1
trace=$(find "$raw" -name '*kernel_trace.csv' | sort | tail -n 1)
python3 bench/prof_summary.py "$trace" --window-ms 300 > "$out/kernels.md"
python3 bench/gap_analysis.py "$raw" --window-ms 300 > "$out/gaps.md"
rm -rf "$raw"
echo "wrote $out/kernels.md $out/gaps.md"
