# bench.py's N > 1 path rehearsed with several ranks on the box's ONE GPU
# (BINE_FAKE_HOSTS=1: distinct RCCL host ids, socket transport between the
# ranks; one HW queue per rank: the fewest queues on the shared GPU).  The
# numbers rank transports on one shared HBM; they say nothing about xGMI.
#   /usr/local/graft/bin/gpurun --timeout 1150 -- 'bash tools/gpu_rehearsal.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
bash tools/gpu_steps.sh \
 "b2:400:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 $R --nproc-per-node 2 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/b2.json" \
 "b4:450:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 $R --nproc-per-node 4 --master-port 29513 bench.py --gpus 4 --steps 20 --warmup 5 > gpurun_out/b4.json" \
 "b8:600:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 $R --nproc-per-node 8 --master-port 29515 bench.py --gpus 8 --steps 20 --warmup 5 > gpurun_out/b8.json"
