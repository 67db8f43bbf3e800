# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "r6af_suite_ss:800:BINE_SHARED_GPU_SINGLE_STREAM=1 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider"
