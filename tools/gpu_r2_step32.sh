#!/bin/bash
# round-end rehearsal: smoke() and the driver's default N = 1 bench
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "smoke:240:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:400:python3 -u bench.py > gpurun_out/r2_bench_default.json"
