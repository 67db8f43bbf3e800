#!/bin/bash
# round-end rehearsal: the whole -m gpu suite
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "suite:1100:python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/ > gpurun_out/r2_gpu_suite.txt"
