# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
bash tools/gpu_steps.sh \
 "r6ae_bench:240:python -u bench.py > gpurun_out/r6ae_bench.json" \
 "r6ae_b8:300:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 $R --nproc-per-node 8 --master-port 29515 bench.py --gpus 8 --steps 20 --warmup 5 > gpurun_out/r6ae_b8.json" \
 "r6ae_b2:300:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 $R --nproc-per-node 2 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r6ae_b2.json"
