set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "calib_sdma0:120:HSA_ENABLE_SDMA=0 python -u tools/pcie_calib.py 256" \
 "e2e1_sdma0:200:HSA_ENABLE_SDMA=0 python -u tools/e2e_staging.py 1 float 67108864 20" \
 "suite:1000:python -u -m pytest -v --timeout 400 --timeout-method thread tests -m gpu"
