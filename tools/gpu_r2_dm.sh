#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1 BINE_DIRECT_TIMEOUT_S=5
bash tools/gpu_steps.sh \
  "dm4r:200:python3 -u tools/direct_probe.py 4 4194304 relay" \
  "dm8r:200:python3 -u tools/direct_probe.py 8 4194304 relay" \
  "t_large:500:python3 -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_gpu_rccl.py -k large"
