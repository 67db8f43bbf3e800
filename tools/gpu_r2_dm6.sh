#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1 BINE_DIRECT_TIMEOUT_S=5
bash tools/gpu_steps.sh \
  "large:240:python3 -u tools/rccl_large.py 4" \
  "large8:400:python3 -u tools/rccl_large.py 8" \
  "rehearsal4:300:BINE_FAKE_HOSTS=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 10 --warmup 2 > gpurun_out/r2_rehearsal4.json"
grep -h RESULT gpurun_out/large.log gpurun_out/large8.log
