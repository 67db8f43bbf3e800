#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONFAULTHANDLER=1
bash tools/gpu_steps.sh \
  "glib_big:200:python3 -u tools/graph_probe.py 2 lib 67108864 direct,flatrs+flat" \
  "glib_big4:200:python3 -u tools/graph_probe.py 4 lib 67108864 direct,flatrs+flat,relay+flat" \
  "glib_c1:200:python3 -u tools/graph_probe.py 4 lib 262144 direct,flatrs+flat"
