# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "r6ag_smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "r6ag_sub:400:python -u -m pytest tests/test_gpu.py tests/test_gpu_rccl.py -k 'pico_core or rebuilt or launch_caps or reduce_local' -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "r6ag_bench:240:python -u bench.py > gpurun_out/r6ag_bench.json"
