#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "benchmr:450:python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_bench_multirank.py" \
  "rehearsal4:450:BINE_FAKE_HOSTS=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 20 --warmup 5 > gpurun_out/r2_rehearsal4.json" \
  "bench_n1:300:python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench_n1_driver_args.json"
