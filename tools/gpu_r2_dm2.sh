#!/bin/bash
# direct transport: separate push / pull launches (BINE_DIRECT_MERGE=0) vs
# merged (default), P = 4 and 8 processes on the one GPU
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1 BINE_DIRECT_TIMEOUT_S=5 PROBE_DM_ONLY=1
bash tools/gpu_steps.sh \
  "m0p4:200:BINE_DIRECT_MERGE=0 python3 -u tools/direct_probe.py 4 67108864 direct,flatrs+flat,relay+flat" \
  "m1p4:200:BINE_DIRECT_MERGE=1 python3 -u tools/direct_probe.py 4 67108864 direct,flatrs+flat,relay+flat" \
  "m0p8:300:BINE_DIRECT_MERGE=0 python3 -u tools/direct_probe.py 8 67108864 direct,flatrs+flat" \
  "m1p8:300:BINE_DIRECT_MERGE=1 python3 -u tools/direct_probe.py 8 67108864 direct,flatrs+flat" \
  "t_large:500:python3 -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_gpu_rccl.py"
for f in m0p4 m1p4 m0p8 m1p8; do echo "$f: $(grep '^{' gpurun_out/$f.log | tail -1)"; done
