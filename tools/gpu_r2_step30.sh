#!/bin/bash
cd "$(dirname "$0")/.."
bash tools/gpu_steps.sh \
  "opcheck1:240:bash integration/run_op_check.sh 1 > gpurun_out/r2_op_check_p1.txt 2>&1" \
  "opcheck2:300:BINE_FAKE_HOSTS=1 bash integration/run_op_check.sh 2 > gpurun_out/r2_op_check_p2.txt 2>&1" \
  "opcheck4:400:BINE_FAKE_HOSTS=1 bash integration/run_op_check.sh 4 > gpurun_out/r2_op_check_p4.txt 2>&1"
