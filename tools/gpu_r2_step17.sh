#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "ops:900:python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu.py -k 'logic or bits or bitwise or loc or complex or reference_goldens or reduce_local or reduce_tree'"
