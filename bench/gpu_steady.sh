# Headline (config 3) at steady state: driver form vs a long window, the early-release
# policy, and a kernel/gap profile of the steady-state mix.
#   bash bench/gpu_steady.sh [tag]        (run through gpurun, from the repo or .snap/)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=${1:-steady}
o=${GRAFT_REPO_ROOT:-.}/gpurun_out/$tag; mkdir -p $o
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > $o/$name.log 2>&1
  local rc=$?
  tail -n 1 $o/$name.log | cut -c1-400
  return $rc
}
run smoke python -u -c "import __graft_entry__ as g; g.smoke()" && \
run driver_a python -u bench.py --steps 20 --warmup 5 && \
run driver_b python -u bench.py --steps 20 --warmup 5 && \
run long python -u bench.py --steps 3000 --warmup 100 && \
run driver_er XGS_EARLY_RELEASE=1 python -u bench.py --steps 20 --warmup 5 && \
run long_er XGS_EARLY_RELEASE=1 python -u bench.py --steps 3000 --warmup 100 && \
run steplog XGS_STEP_LOG=$o/steps.jsonl python -u bench.py --steps 400 --warmup 20 && \
bash bench/profile.sh $o/prof
