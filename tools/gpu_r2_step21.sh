#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "e2e:200:bash integration/run_pico_core.sh 1 ALLREDUCE 67108864 10 bine_bdw_remap_over float > gpurun_out/r2_pico_core_e2e.txt" \
  "e2e2:300:BINE_FAKE_HOSTS=1 BINE_FLAT_RS=1 BINE_FLAT_AG=1 bash integration/run_pico_core.sh 2 ALLREDUCE 16777216 10 bine_bdw_remap_over float > gpurun_out/r2_pico_core_e2e_p2.txt"
