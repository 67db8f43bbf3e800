#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "smoke:240:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_n1:300:python3 -u bench.py > gpurun_out/r2_bench_n1.json" \
  "prof_n1:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_n1 -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5" \
  "rehearsal4:450:BINE_FAKE_HOSTS=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 10 --warmup 2 > gpurun_out/r2_rehearsal4.json"
