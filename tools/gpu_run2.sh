set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "large4:400:PYTHONFAULTHANDLER=1 BINE_SEGV_TRACE=1 python -u tools/rccl_large.py 4" \
 "rs64:240:python -u tools/rs_graph_probe.py 4 flatrs+flat+dm 64 0" \
 "ab2w64:300:BINE_DIRECT_TREE_WGS=64 python -u tools/dm_tree_ab.py 2 16,64 10" \
 "ab2w256:300:python -u tools/dm_tree_ab.py 2 16,64 10" \
 "ab4w64:300:BINE_DIRECT_TREE_WGS=64 python -u tools/dm_tree_ab.py 4 16,64 10" \
 "ab4w256:300:python -u tools/dm_tree_ab.py 4 16,64 10" \
 "full8:600:python -u tools/fullsize_multirank.py 8"
