# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
 "ab2:150:python -u tools/dm_tree_ab.py 2 16,64 4" \
 "stamps2:600:python -u tools/dm_stamps.py 2 8 base: w64t128:BINE_DIRECT_WGS=64,BINE_DIRECT_TREE_WGS=128 w64t64:BINE_DIRECT_WGS=64,BINE_DIRECT_TREE_WGS=64 w96t128:BINE_DIRECT_WGS=96,BINE_DIRECT_TREE_WGS=128 w64t128p128:BINE_DIRECT_WGS=64,BINE_DIRECT_TREE_WGS=128,BINE_DIRECT_PULL_WGS=128 w64t128c64:BINE_DIRECT_WGS=64,BINE_DIRECT_TREE_WGS=128,BINE_CHUNK_BYTES=67108864 w128t256c64:BINE_DIRECT_WGS=128,BINE_DIRECT_TREE_WGS=256,BINE_CHUNK_BYTES=67108864" \
 "rccl:600:$T tests/test_gpu_rccl.py"
