# the direct transport's workgroup autoscale: its GPU tests, the widening
# timings and bench.py's 2-rank rehearsal in one call
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
rm -f gpurun_out/steps.log
bash tools/gpu_steps.sh \
 "rccl:700:python -u -m pytest tests/test_gpu_rccl.py -x -q -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider" \
 "rb2:180:GPU_MAX_HW_QUEUES=2 python -u tools/rooted_bench.py 2 64" \
 "rb4:180:GPU_MAX_HW_QUEUES=2 python -u tools/rooted_bench.py 4 64" \
 "b2:400:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 $R --nproc-per-node 2 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/b2as.json"
