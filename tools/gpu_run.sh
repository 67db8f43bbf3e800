# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "r6y_dm2s:150:PROBE_TRANSPORT=direct+dm PROBE_CHUNK_MIB=16 GPU_MAX_HW_QUEUES=1 python -u tools/fused8_probe.py 8 3 2 > gpurun_out/r6y_dm2s.json" \
 "r6y_dm1s:150:BINE_SINGLE_STREAM_BYTES=1073741824 PROBE_TRANSPORT=direct+dm PROBE_CHUNK_MIB=16 GPU_MAX_HW_QUEUES=1 python -u tools/fused8_probe.py 8 3 2 > gpurun_out/r6y_dm1s.json" \
 "r6y_fdm1s:150:BINE_SINGLE_STREAM_BYTES=1073741824 PROBE_TRANSPORT=flatrs+flat+dm PROBE_CHUNK_MIB=16 GPU_MAX_HW_QUEUES=1 python -u tools/fused8_probe.py 8 3 2 > gpurun_out/r6y_fdm1s.json" \
 "r6y_fdm2s:150:PROBE_TRANSPORT=flatrs+flat+dm PROBE_CHUNK_MIB=16 GPU_MAX_HW_QUEUES=1 python -u tools/fused8_probe.py 8 3 2 > gpurun_out/r6y_fdm2s.json"
