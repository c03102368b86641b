set -o pipefail
bash scripts/gpu_call_trace.sh || exit 1
timeout -k 10 300 python3 scripts/diag/pooled_probe2.py pooled:12 c4:2 pooled:4 > gpurun_out/pooled_probe.log 2>&1 || { tail -20 gpurun_out/pooled_probe.log; exit 1; }
cat gpurun_out/pooled_probe.log | grep -v amdgpu.ids
