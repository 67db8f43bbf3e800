# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
bash tools/gpu_steps.sh \
 "churn:200:$T tests/test_gpu.py -k 'freed_and_reallocated or match_mpich or pico_core_dropin or pico_core_c1'" \
 "staged:230:$T tests/test_gpu_rccl.py -k staged" \
 "e2e1:300:python -u tools/e2e_staging.py 1 float 67108864 20" \
 "rsg_q1:150:GPU_MAX_HW_QUEUES=1 BINE_SEGV_TRACE=1 BINE_SEGV_TRACE_DIR=\$PWD/gpurun_out python -u tools/rs_graph_probe.py 4 flatrs+flat+dm16 64 1"
