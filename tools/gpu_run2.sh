set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "prof:150:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py" \
 "pmcf:90:rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o bench -- python3 bench.py" \
 "pmcw:90:rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o bench -- python3 bench.py" \
 "ab8q1:400:GPU_MAX_HW_QUEUES=1 python -u tools/dm_tree_ab.py 8 16,64 10" \
 "ab4w32:300:BINE_DIRECT_TREE_WGS=32 python -u tools/dm_tree_ab.py 4 16,64 10" \
 "b8q1:700:GPU_MAX_HW_QUEUES=1 BINE_FAKE_HOSTS=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 8 --steps 20 --warmup 5 --no-graph-trial > gpurun_out/b8q1.json"
