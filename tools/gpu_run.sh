# The GPU calls of a round, one step per line (tools/gpu_steps.sh: each step
# under its own time limit, output in gpurun_out/<name>.log).  Edited per call.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu_run.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "r6h_topo:30:for n in /sys/class/kfd/kfd/topology/nodes/*; do echo \"\$n gpu_id=\$(cat \$n/gpu_id) \$(grep -E '^(num_cp_queues|num_xcc|simd_count|max_waves_per_simd|num_sdma_engines|num_sdma_xgmi_engines)' \$n/properties | tr '\n' ' ')\"; done > gpurun_out/r6h_topo.txt; for p in hws_max_conc_proc sched_policy cwsr_enable mes; do echo \"\$p=\$(cat /sys/module/amdgpu/parameters/\$p 2>&1)\"; done >> gpurun_out/r6h_topo.txt" \
 "r6h_f8q1:240:GPU_MAX_HW_QUEUES=1 python -u tools/fused8_probe.py 8 12 5 > gpurun_out/r6h_f8q1.json" \
 "r6h_f8q2:240:GPU_MAX_HW_QUEUES=2 python -u tools/fused8_probe.py 8 12 5 > gpurun_out/r6h_f8q2.json" \
 "r6h_f8q3:300:GPU_MAX_HW_QUEUES=3 python -u tools/fused8_probe.py 8 12 5 > gpurun_out/r6h_f8q3.json" \
 "r6h_f8q4:300:GPU_MAX_HW_QUEUES=4 python -u tools/fused8_probe.py 8 12 5 > gpurun_out/r6h_f8q4.json"
