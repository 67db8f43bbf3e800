#!/bin/bash
# copy-kernel survey incl. the XCD-aware tile orders (tools/copy_variants.hip)
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -I include -o /tmp/copy_variants tools/copy_variants.hip \
  -L pico_amd/lib -lbine_amd -Wl,-rpath,$PWD/pico_amd/lib > gpurun_out/cv_build.log 2>&1 || { tail gpurun_out/cv_build.log; exit 1; }
bash tools/gpu_steps.sh "cv:300:/tmp/copy_variants > gpurun_out/r2_copy_variants_xcd.txt"
