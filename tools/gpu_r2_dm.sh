#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1 BINE_DIRECT_TIMEOUT_S=5 BINE_TRACE=1
bash tools/gpu_steps.sh \
  "dm2:200:python3 -u tools/direct_probe.py 2 67108864 direct"
grep "bine dm" gpurun_out/dm2.log | head -30
