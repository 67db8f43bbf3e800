# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call;
# this is the last one of round 3.  Run as
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "smoke:300:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:300:python -u bench.py" \
 "prof:150:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py" \
 "pmcf:90:rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o bench -- python3 bench.py" \
 "pmcw:90:rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o bench -- python3 bench.py"
