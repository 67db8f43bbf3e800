# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
W="BINE_DIRECT_WGS=64,BINE_DIRECT_TREE_WGS=128"
bash tools/gpu_steps.sh \
 "ab2c:150:python -u tools/dm_tree_ab.py 2 16,64 6" \
 "stamps2c:700:python -u tools/dm_stamps.py 2 8 base: w64t128:$W w64t128g:$W,DM_STAMPS_GRAPHS=1 w64t128c64:$W,BINE_CHUNK_BYTES=67108864 w64t128c64s64:$W,BINE_CHUNK_BYTES=67108864,BINE_DIRECT_SLOT_BYTES=67108864 w64t128c64s64g:$W,BINE_CHUNK_BYTES=67108864,BINE_DIRECT_SLOT_BYTES=67108864,DM_STAMPS_GRAPHS=1 w128t256c64s64:BINE_DIRECT_WGS=128,BINE_DIRECT_TREE_WGS=256,BINE_CHUNK_BYTES=67108864,BINE_DIRECT_SLOT_BYTES=67108864" \
 "rcclc:600:$T tests/test_gpu_rccl.py" \
 "full8c:400:$T tests/test_gpu_fullsize.py -k eight_processes"
