# The whole -m gpu suite as one GPU call, with per-test durations (the round
# end's GPU step runs the same suite; its time budget is 900 s):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu_suite.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "suite:1120:python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider --durations=60"
