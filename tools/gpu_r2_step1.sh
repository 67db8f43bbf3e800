set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bench_sizes.py tests/test_gpu_rccl.py > gpurun_out/r2_t1.txt 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r2_t1.txt; exit 1; }
tail -5 gpurun_out/r2_t1.txt
timeout -k 10 300 python -u bench.py > gpurun_out/r2_bench_n1.json 2> gpurun_out/r2_bench_n1.err || { echo BENCH_FAILED; tail -30 gpurun_out/r2_bench_n1.err; exit 1; }
cat gpurun_out/r2_bench_n1.json
