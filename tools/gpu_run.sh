# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "r6k_suite:800:python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider --durations=15" \
 "r6k_smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "r6k_dmhi:150:PROBE_TRANSPORT=direct+dm PROBE_CHUNK_MIB=16 GPU_MAX_HW_QUEUES=1 python -u tools/fused8_probe.py 8 3 2 > gpurun_out/r6k_dmhi.json" \
 "r6k_dmlo:150:BINE_COMM_PRIORITY=0 PROBE_TRANSPORT=direct+dm PROBE_CHUNK_MIB=16 GPU_MAX_HW_QUEUES=1 python -u tools/fused8_probe.py 8 3 2 > gpurun_out/r6k_dmlo.json"
