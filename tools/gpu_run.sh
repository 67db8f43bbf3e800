# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "r6u_p1_4m:150:python -u tools/e2e_staging.py 1 float 1048576 200 zc > gpurun_out/r6u_p1_4m.json" \
 "r6u_p1_16m:150:python -u tools/e2e_staging.py 1 float 4194304 100 zc > gpurun_out/r6u_p1_16m.json" \
 "r6u_p2_4m:150:GPU_MAX_HW_QUEUES=2 python -u tools/e2e_staging.py 2 float 1048576 200 zc > gpurun_out/r6u_p2_4m.json" \
 "r6u_p2_16m:150:GPU_MAX_HW_QUEUES=2 python -u tools/e2e_staging.py 2 float 4194304 100 zc > gpurun_out/r6u_p2_16m.json" \
 "r6u_p4_4m:150:GPU_MAX_HW_QUEUES=2 python -u tools/e2e_staging.py 4 float 1048576 200 zc > gpurun_out/r6u_p4_4m.json" \
 "r6u_p4_16m:150:GPU_MAX_HW_QUEUES=2 python -u tools/e2e_staging.py 4 float 4194304 100 zc > gpurun_out/r6u_p4_16m.json"
