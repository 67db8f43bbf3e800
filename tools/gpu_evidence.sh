# A round's GPU evidence in one call: the -m gpu suite, the N = 1 bench line,
# its rocprofv3 kernel trace and the two PMC passes (separate runs, as the
# MI355X guide prescribes), then on the host: python tools/pmc_summary.py rNN
# (writes profiles/rNN_pmc.json + latest_pmc.json, which bench.py's
# roofline.traffic reads when its kernels.hip hash matches).
#   /usr/local/graft/bin/gpurun --timeout 1150 -- 'bash tools/gpu_evidence.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
bash tools/gpu_steps.sh \
 "suite:700:python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider --durations=15" \
 "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:240:python -u bench.py > gpurun_out/bench.json" \
 "prof:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline" \
 "pmcf:70:BENCH_NO_SMALL_WINDOWS=1 timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 5 --no-cpu-baseline" \
 "pmcw:70:BENCH_NO_SMALL_WINDOWS=1 timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 5 --no-cpu-baseline"
