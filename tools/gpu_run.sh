# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "r6v_dropin:400:python -u -m pytest tests/test_gpu.py -k 'pico_core or libbine or op_check' -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "r6v_p2_8m:150:GPU_MAX_HW_QUEUES=2 python -u tools/e2e_staging.py 2 float 2097152 100 c1 > gpurun_out/r6v_p2_8m.json"
