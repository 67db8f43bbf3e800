# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
bash tools/gpu_steps.sh \
 "r6b_rebuild:300:$T tests/test_gpu_rccl.py -k rebuilt_after" \
 "r6b_dmto:200:$T tests/test_gpu.py -k timed_out_call" \
 "r6b_b2:400:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 $R --nproc-per-node 2 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r6b_b2.json" \
 "r6b_b8:600:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 $R --nproc-per-node 8 --master-port 29515 bench.py --gpus 8 --steps 20 --warmup 5 > gpurun_out/r6b_b8.json"
