#!/bin/bash
cd "$(dirname "$0")/.."
bash tools/gpu_steps.sh \
  "graph2:200:python3 -u tools/graph_probe.py 2 thread_local" \
  "graph4:200:python3 -u tools/graph_probe.py 4 relaxed"
