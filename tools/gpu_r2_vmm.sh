#!/bin/bash
cd "$(dirname "$0")/.."
T=$(python3 -c 'import os,torch;print(os.path.join(os.path.dirname(torch.__file__),"lib"))')
echo "== /opt/rocm runtime, by value"; timeout -k 5 60 ./tools/bin/vmm_ipc_probe; echo rc=$?
echo "== /opt/rocm runtime, by pointer"; timeout -k 5 60 ./tools/bin/vmm_ipc_probe ptr; echo rc=$?
echo "== torch runtime, by value"; LD_LIBRARY_PATH=$T timeout -k 5 60 ./tools/bin/vmm_ipc_probe; echo rc=$?
echo "== torch runtime, by pointer"; LD_LIBRARY_PATH=$T timeout -k 5 60 ./tools/bin/vmm_ipc_probe ptr; echo rc=$?
