# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "smoke:120:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "ab2:200:python -u tools/dm_tree_ab.py 2 16,64 10" \
 "ab4:200:python -u tools/dm_tree_ab.py 4 16,64 10" \
 "ab8q1:300:GPU_MAX_HW_QUEUES=1 python -u tools/dm_tree_ab.py 8 16,64 10"
