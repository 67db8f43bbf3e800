#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "suite:1100:python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r2_gpu_suite.txt" \
  "rehearsal8:500:BINE_FAKE_HOSTS=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 8 --steps 5 --warmup 1 > gpurun_out/r2_rehearsal8.json"
