#!/bin/bash
# direct transport launches per round: 2 (pushes + pulls of the round in one
# launch, default), 1 (round k-1's pulls with round k's pushes), 0 (separate);
# C3 (256 MiB/rank) and C1 (1 MiB/rank), P = 2, 4, 8 processes on the one GPU
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1 BINE_DIRECT_TIMEOUT_S=5 PROBE_DM_ONLY=1
steps=()
for P in 2 4 8; do
  for M in 2 1 0; do
    steps+=("c3m${M}p${P}:150:BINE_DIRECT_MERGE=$M python3 -u tools/direct_probe.py $P 67108864 direct,flatrs+flat")
    steps+=("c1m${M}p${P}:150:BINE_DIRECT_MERGE=$M python3 -u tools/direct_probe.py $P 262144 direct,flatrs+flat")
  done
done
steps+=("large:240:python3 -u tools/rccl_large.py 4")
bash tools/gpu_steps.sh "${steps[@]}"
for f in gpurun_out/c[13]m*p*.log; do echo "$(basename $f .log): $(grep '^{' $f | tail -1)"; done
grep RESULT gpurun_out/large.log
