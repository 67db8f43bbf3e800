set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "b8q1:700:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 8 --steps 20 --warmup 5 --no-graph-trial > gpurun_out/b8q1.json" \
 "b4:500:BINE_FAKE_HOSTS=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 20 --warmup 5 > gpurun_out/b4.json"
