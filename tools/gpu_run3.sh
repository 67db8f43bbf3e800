set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "suite2:1100:python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_rccl.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
