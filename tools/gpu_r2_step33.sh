#!/bin/bash
# bcast latency trees: reference goldens through the device path (loopback
# ranks, direct and relay), then op_check (incl. bcast vs PMPI_Bcast) at P = 1, 2, 4
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "bcast_goldens:400:python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py -k 'goldens and bcast' > gpurun_out/r2_gpu_bcast_goldens.txt" \
  "opcheck1:240:bash integration/run_op_check.sh 1 > gpurun_out/r2_op_check_p1.txt 2>&1" \
  "opcheck2:300:BINE_FAKE_HOSTS=1 bash integration/run_op_check.sh 2 > gpurun_out/r2_op_check_p2.txt 2>&1" \
  "opcheck4:400:BINE_FAKE_HOSTS=1 bash integration/run_op_check.sh 4 > gpurun_out/r2_op_check_p4.txt 2>&1"
