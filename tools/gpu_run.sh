# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
F="python -u tools/fused8_probe.py"
bash tools/gpu_steps.sh \
 "r6e_fusedck:200:GPU_MAX_HW_QUEUES=2 python -u tools/dm_fused_check.py 2 && GPU_MAX_HW_QUEUES=2 python -u tools/dm_fused_check.py 4" \
 "r6e_ab1:120:GPU_MAX_HW_QUEUES=1 $F 2 30 5 > gpurun_out/r6e_ab1.json" \
 "r6e_ab0:120:GPU_MAX_HW_QUEUES=1 BINE_DIRECT_SLICE_FLAGS=0 $F 2 30 5 > gpurun_out/r6e_ab0.json" \
 "r6e_ab1b:120:GPU_MAX_HW_QUEUES=1 $F 2 30 5 > gpurun_out/r6e_ab1b.json" \
 "r6e_ab0b:120:GPU_MAX_HW_QUEUES=1 BINE_DIRECT_SLICE_FLAGS=0 $F 2 30 5 > gpurun_out/r6e_ab0b.json" \
 "r6e_ab1p4:120:GPU_MAX_HW_QUEUES=1 $F 4 20 5 > gpurun_out/r6e_ab1p4.json" \
 "r6e_ab0p4:120:GPU_MAX_HW_QUEUES=1 BINE_DIRECT_SLICE_FLAGS=0 $F 4 20 5 > gpurun_out/r6e_ab0p4.json"
