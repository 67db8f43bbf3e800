# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "large4:300:python -u tools/rccl_large.py 4" \
 "rccl:400:python -u -m pytest tests/test_gpu_rccl.py -k 'matrix or orders or c1_four or fused_trees or staged' -x -v --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "ab4:200:python -u tools/dm_tree_ab.py 4 16,64 10" \
 "full8:300:python -u tools/fullsize_multirank.py 8"
