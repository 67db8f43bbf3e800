set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "c1trace:240:BINE_ROCTX=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c1prof -o c1_%pid% -- python3 tools/c1_probe.py 4 50" \
 "tree:120:tools/bin/tree_variants" \
 "calib_sdma0:120:HSA_ENABLE_SDMA=0 python -u tools/pcie_calib.py 256" \
 "e2e1:200:python -u tools/e2e_staging.py 1 float 67108864 20" \
 "e2e1_sdma0:200:HSA_ENABLE_SDMA=0 python -u tools/e2e_staging.py 1 float 67108864 20"
