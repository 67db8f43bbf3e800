#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "large:300:python3 -u tools/rccl_large.py 4" \
  "rehearsal4:300:BINE_FAKE_HOSTS=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 10 --warmup 2 > gpurun_out/r2_rehearsal4.json" \
  "t_rccl:500:python3 -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_gpu_rccl.py"
grep -E "RESULT|MISMATCH|failed" gpurun_out/large.log
