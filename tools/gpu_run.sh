# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call;
# this one: kernel trace and HBM counters of the fused-tree A/B at P = 2.  Run as
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "abtrace:200:rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abtrace -o ab_%pid% -- python3 -u tools/dm_tree_ab.py 2 16 4" \
 "abfetch:200:rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/abfetch -o ab_%pid% -- python3 -u tools/dm_tree_ab.py 2 16 4" \
 "abwrite:200:rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/abwrite -o ab_%pid% -- python3 -u tools/dm_tree_ab.py 2 16 4"
