#!/bin/bash
# round-2: full GPU suite (k_copy now runs every COPY primitive), bench N=1,
# C1 probe under the kernel + marker trace
cd "$(dirname "$0")/.." && rm -rf gpurun_out/c1trace
bash tools/gpu_steps.sh \
  "suite:900:python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu" \
  "bench_n1:300:python3 -u bench.py > gpurun_out/r2_bench_n1b.json" \
  "c1trace:300:BINE_ROCTX=1 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/c1trace -- python3 tools/c1_probe.py 4 200"
rm -rf gpurun_out/ovltrace
bash tools/gpu_steps.sh \
  "ovl_direct:300:rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ovltrace -- python3 tools/overlap_probe_rccl.py 4 direct" \
  "ovl_report:60:python3 tools/rccl_overlap_report.py gpurun_out/ovltrace"
rm -rf gpurun_out/a2atrace gpurun_out/p2ptrace
bash tools/gpu_steps.sh \
  "a2a_trace:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/a2atrace -- python3 tools/overlap_probe_rccl.py 4 flatrs+flat+a2a" \
  "p2p_trace:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p2ptrace -- python3 tools/overlap_probe_rccl.py 4 flatrs+flat"
