#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "gold:900:python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu.py -k 'reference_goldens'"
