#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "suite:900:python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests -m gpu" \
  "smoke:200:python3 -c 'import __graft_entry__ as g; g.smoke()'"
