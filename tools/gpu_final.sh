set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
bash tools/gpu_steps.sh \
 "suite:800:python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider --durations=10" \
 "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:240:python -u bench.py > gpurun_out/bench_final.json"
