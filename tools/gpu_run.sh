# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
bash tools/gpu_steps.sh \
 "r6d_fusedck:200:GPU_MAX_HW_QUEUES=2 python -u tools/dm_fused_check.py 2 && GPU_MAX_HW_QUEUES=2 python -u tools/dm_fused_check.py 4" \
 "r6d_rccl:600:$T tests/test_gpu_rccl.py" \
 "r6d_full8:400:$T tests/test_gpu_fullsize.py -k eight_processes" \
 "r6d_b2:300:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 $R --nproc-per-node 2 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r6d_b2.json" \
 "r6d_f8q1:200:GPU_MAX_HW_QUEUES=1 python -u tools/fused8_probe.py 8 > gpurun_out/r6d_f8q1.json" \
 "r6d_f8q2:200:GPU_MAX_HW_QUEUES=2 python -u tools/fused8_probe.py 8 > gpurun_out/r6d_f8q2.json" \
 "r6d_f8q1t60:300:GPU_MAX_HW_QUEUES=1 BINE_DIRECT_TIMEOUT_S=60 python -u tools/fused8_probe.py 8 > gpurun_out/r6d_f8q1t60.json" \
 "r6d_f8q1w64:200:GPU_MAX_HW_QUEUES=1 BINE_DIRECT_FUSED_WGS=64 python -u tools/fused8_probe.py 8 > gpurun_out/r6d_f8q1w64.json"
