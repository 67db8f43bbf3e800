set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "rooted:400:python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu.py tests/test_gpu_rccl.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k 'rooted or gather or scatter or alltoall or GATHER or SCATTER or ALLTOALL or mpi_typed or rebuilt' > gpurun_out/rooted_r5f.log 2>&1"
