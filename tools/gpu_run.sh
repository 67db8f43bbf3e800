# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "r6g_res8q1:200:GPU_MAX_HW_QUEUES=1 python -u tools/residency8.py 8 > gpurun_out/r6g_res8q1.json" \
 "r6g_res8q2:200:GPU_MAX_HW_QUEUES=2 python -u tools/residency8.py 8 > gpurun_out/r6g_res8q2.json" \
 "r6g_res2q1:120:GPU_MAX_HW_QUEUES=1 python -u tools/residency8.py 2 > gpurun_out/r6g_res2q1.json"
