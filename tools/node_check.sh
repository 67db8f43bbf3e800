# On a multi-GPU node (one process per GPU, RCCL over xGMI): the multi-rank
# probes that run on the one-GPU box with every rank on GPU 0, here with rank
# r on GPU r (BINE_RANK_DEVICES=1, no fake RCCL host ids) -- the cross-GPU
# half of the direct transport's memory model and the RCCL paths over xGMI,
# every output checked against the oracle / the collective.  Not run by the
# one-GPU pool; usage on a node:  bash tools/node_check.sh [P]   (default 8)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${1:-8}
export BINE_RANK_DEVICES=1 TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_steps.sh \
 "node_large:400:python -u tools/rccl_large.py $P float" \
 "node_fullsize:400:python -u tools/fullsize_multirank.py $P" \
 "node_fused:300:python -u tools/dm_fused_check.py $P" \
 "node_rooted:300:python -u tools/rooted_check.py $P" \
 "node_matrix:600:python -u tools/rccl_matrix.py $P"
