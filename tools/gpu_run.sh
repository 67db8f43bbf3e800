set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "b8q1:700:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 8 --steps 20 --warmup 5 --no-graph-trial > gpurun_out/b8q1.json" \
 "b2q1:300:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --steps 20 --warmup 5 --no-graph-trial > gpurun_out/b2q1.json"
