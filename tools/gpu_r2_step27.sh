#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "bench_n1:300:python3 -u bench.py > gpurun_out/r2_bench_n1.json" \
  "prof_n1:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_n1b -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5"
