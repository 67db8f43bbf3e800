set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "trace2:300:BINE_DIRECT_TREE_WGS=64 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace2 -o ab_%pid% -- python3 -u tools/dm_tree_ab.py 2 16 10"
