#!/usr/bin/env bash
# Run GPU steps in order on the gpurun box. Each step has its own time limit. A step that exits 0 or 1
# (pass / ordinary test failure) lets the next step run; any other status (GPU fault, abort 134, segfault
# 139, timeout 124/137, ...) ends the job there, so nothing else touches the GPU after trouble.
# usage: tools/gpu_job.sh "<seconds>|<logname>|<command>" ...
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; log="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$(date +%T)] step ${log}: ${cmd} (limit ${secs}s)"
  timeout -k 10 "${secs}" bash -c "${cmd}" > "gpurun_out/${log}.log" 2>&1
  rc=$?
  echo "=== [$(date +%T)] step ${log} exit ${rc}"
  tail -n 25 "gpurun_out/${log}.log"
  if [ "${rc}" -ne 0 ] && [ "${rc}" -ne 1 ]; then
    echo "=== stopping: step ${log} ended with status ${rc}"
    exit "${rc}"
  fi
done
exit 0
