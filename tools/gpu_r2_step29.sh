#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "fuzz:600:python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py"
