#!/usr/bin/env bash
# Host-side helper: submit one gpurun call, re-submitting ONLY when gpurun reports
# that no box / slot was available (exit 3: nothing ran, nothing charged).
#   bash bench/gpurun_retry.sh <timeout_s> '<command>' [log]
t=$1; cmd=$2; log=${3:-/tmp/gpurun_last.log}
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "backing off\|status=transient" "$log"; then break; fi
  sleep 45
done
echo "exit $rc"; tail -n 15 "$log"
exit $rc
