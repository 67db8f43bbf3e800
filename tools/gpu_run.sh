# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "r6ab_ss1:200:BINE_SHARED_GPU_SINGLE_STREAM=1 GPU_MAX_HW_QUEUES=2 python -u tools/fullsize_multirank.py 8 > gpurun_out/r6ab_ss1.txt" \
 "r6ab_ss2:200:BINE_SHARED_GPU_SINGLE_STREAM=1 GPU_MAX_HW_QUEUES=2 python -u tools/fullsize_multirank.py 8 > gpurun_out/r6ab_ss2.txt" \
 "r6ab_ss3:200:BINE_SHARED_GPU_SINGLE_STREAM=1 GPU_MAX_HW_QUEUES=2 python -u tools/fullsize_multirank.py 8 > gpurun_out/r6ab_ss3.txt" \
 "r6ab_def:200:GPU_MAX_HW_QUEUES=2 python -u tools/fullsize_multirank.py 8 > gpurun_out/r6ab_def.txt"
