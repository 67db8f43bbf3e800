#!/bin/bash
# the direct transport under other workgroups-per-message settings (bench.py
# trials 16 / 32 / 64 on the node): 64 MiB/rank, every transport, 4 processes
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "wgs16:400:BINE_DIRECT_WGS=16 python3 -u tools/rccl_large.py 4 > gpurun_out/r2_rccl_large_wgs16.txt" \
  "wgs64:400:BINE_DIRECT_WGS=64 python3 -u tools/rccl_large.py 4 > gpurun_out/r2_rccl_large_wgs64.txt"
