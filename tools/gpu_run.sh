# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "r6t_staged:300:python -u -m pytest tests/test_gpu.py -k 'staged' -v --timeout 200 --timeout-method thread -p no:cacheprovider"
