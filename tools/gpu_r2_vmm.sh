#!/bin/bash
cd "$(dirname "$0")/.."
echo "== torch's HIP runtime (RPATH), by value"; timeout -k 5 60 ./tools/bin/vmm_ipc_probe_torch; echo rc=$?
echo "== torch's HIP runtime (RPATH), by pointer"; timeout -k 5 60 ./tools/bin/vmm_ipc_probe_torch ptr; echo rc=$?
