set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "large4:400:PYTHONFAULTHANDLER=1 BINE_SEGV_TRACE=1 python -u tools/rccl_large.py 4" \
 "matrix4:500:python -u -m pytest tests/test_gpu_rccl.py -k 'matrix or orders or c1_four or fused_trees' -x -v --timeout 480 --timeout-method thread -p no:cacheprovider" \
 "ab4:300:python -u tools/dm_tree_ab.py 4 16,64 10" \
 "ab4nomc:300:BINE_DIRECT_MCAST=0 python -u tools/dm_tree_ab.py 4 16,64 10" \
 "full8:600:python -u tools/fullsize_multirank.py 8"
