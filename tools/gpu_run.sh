# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
bash tools/gpu_steps.sh \
 "r6ad_suite:800:python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider --durations=15" \
 "r6ad_smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:240:python -u bench.py > gpurun_out/bench.json" \
 "prof:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline" \
 "pmcf:70:BENCH_NO_SMALL_WINDOWS=1 timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 5 --no-cpu-baseline" \
 "pmcw:70:BENCH_NO_SMALL_WINDOWS=1 timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 5 --no-cpu-baseline"
