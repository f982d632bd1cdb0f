#!/usr/bin/env bash
# Host-side helper: submit one gpurun call, re-submitting ONLY when gpurun reports
# that no box / slot was available (exit 3, or a transient provisioning status:
# nothing ran, nothing charged). Honours gpurun's "retry in Ns" back-off hint.
#   bash bench/gpurun_retry.sh <timeout_s> '<command>' [log]
t=$1; cmd=$2; log=${3:-/tmp/gpurun_last.log}
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "backing off\|status=transient" "$log"; then break; fi
  wait_s=$(grep -o "retry in [0-9]*s" "$log" | grep -o "[0-9]*" | tail -n 1)
  [ -n "$wait_s" ] && [ "$wait_s" -gt 45 ] || wait_s=45
  sleep $((wait_s + 5))
done
echo "exit $rc"; tail -n 15 "$log"
exit $rc
