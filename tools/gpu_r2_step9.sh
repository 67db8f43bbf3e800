#!/bin/bash
cd "$(dirname "$0")/.."
bash tools/gpu_steps.sh "stripes4:300:python3 -u tools/stripe_probe.py 4 flatrs+flat" "stripes4d:300:python3 -u tools/stripe_probe.py 4 direct"
