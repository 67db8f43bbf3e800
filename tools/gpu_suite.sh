set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "suite:1120:python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
