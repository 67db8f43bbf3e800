#!/bin/bash
# round-2 measurement pass: bench N=1, its kernel-trace stats, PMC passes, and
# a 4-rank rehearsal of the N>1 bench on one GPU (socket transport)
cd "$(dirname "$0")/.." && rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
bash tools/gpu_steps.sh \
  "bench_n1:300:python3 -u bench.py --no-cpu-baseline > gpurun_out/r2_bench_n1_nocpu.json" \
  "prof:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -- python3 bench.py --no-cpu-baseline" \
  "pmc_fetch:120:BENCH_NO_SMALL_WINDOWS=1 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2" \
  "pmc_write:120:BENCH_NO_SMALL_WINDOWS=1 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2" \
  "rehearsal4:600:BINE_FAKE_HOSTS=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 10 --warmup 2 > gpurun_out/r2_rehearsal4.json"
