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
  # a GPU fault inside a step that still exits 1 (a failed test, a rank that
  # caught it): nothing more runs on the GPU in this call
  if grep -q -E "illegal memory access|MEMORY_APERTURE|Memory access fault|HSA_STATUS_ERROR|page fault" \
       "gpurun_out/$name.log"; then
    echo "stopping after $name: GPU fault in its output"; exit 86
  fi
done
