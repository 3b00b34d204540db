#!/usr/bin/env bash
# gpurun with waits while no GPU slot / box is free (nothing ran, nothing charged); any other outcome returns at once.
# usage: tools/gpurun_retry.sh <timeout-seconds> <log> '<command>'
t="$1"; log="$2"; cmd="$3"
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient\|backing off" "$log" && ! grep -q "status=ok" "$log"; then
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
