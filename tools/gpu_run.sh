set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "staged:420:python -u tools/staged_check.py 4 1" \
 "fullsize8:600:python -u tools/fullsize_multirank.py 8" \
 "t_dropin:500:python -u -m pytest tests/test_gpu.py -k 'pico_core' tests/test_gpu_bench_multirank.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider" \
 "e2e4dm:240:BINE_DIRECT=1 python -u tools/e2e_staging.py 4 float 67108864 10 pipeline" \
 "prof:120:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py" \
 "pmcf:90:rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o bench -- python3 bench.py" \
 "pmcw:90:rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o bench -- python3 bench.py"
