#!/bin/bash
# Run GPU steps in order; each under its own time limit.  A step that exits 0
# or 1 (e.g. failing tests) lets the next one run; anything else (timeout,
# abort, segfault, GPU fault) ends the script.
#   usage: tools/gpu_steps.sh NAME:SECONDS:'command' ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${secs}s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc after $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)"; exit $rc
  fi
done
