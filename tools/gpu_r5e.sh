set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
bash tools/gpu_steps.sh \
 "rooted:400:python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k 'rooted or gather or scatter or alltoall or GATHER or SCATTER or ALLTOALL or mpi_typed' > gpurun_out/rooted_r5.log 2>&1" \
 "b8:600:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 $R --nproc-per-node 8 --master-port 29515 bench.py --gpus 8 --steps 20 --warmup 5 > gpurun_out/b8r5e.json 2> gpurun_out/b8r5e.log"
