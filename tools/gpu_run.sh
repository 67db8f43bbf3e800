# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "r6w_sizes1:200:BINE_COPY_SMALL_U=1 python -u -m pytest tests/test_gpu_bench_sizes.py -q --timeout 150 --timeout-method thread -p no:cacheprovider" \
 "r6w_u8:100:python -u tools/e2e_staging.py 1 float 262144 500 zc > gpurun_out/r6w_u8.json" \
 "r6w_u4:100:BINE_COPY_SMALL_U=4 python -u tools/e2e_staging.py 1 float 262144 500 zc > gpurun_out/r6w_u4.json" \
 "r6w_u2:100:BINE_COPY_SMALL_U=2 python -u tools/e2e_staging.py 1 float 262144 500 zc > gpurun_out/r6w_u2.json" \
 "r6w_u1:100:BINE_COPY_SMALL_U=1 python -u tools/e2e_staging.py 1 float 262144 500 zc > gpurun_out/r6w_u1.json" \
 "r6w_u1_4m:100:BINE_COPY_SMALL_U=1 python -u tools/e2e_staging.py 1 float 1048576 200 zc > gpurun_out/r6w_u1_4m.json" \
 "r6w_u8_4m:100:python -u tools/e2e_staging.py 1 float 1048576 200 zc > gpurun_out/r6w_u8_4m.json"
