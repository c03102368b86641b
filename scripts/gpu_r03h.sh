set -o pipefail
OUT=gpurun_out/r03h; mkdir -p $OUT; export TMPDIR=/tmp
CRISPR_NW_SEGV_TRACE=1 timeout -k 10 200 python -X faulthandler scripts/diag/pooled_probe2.py c4:1 > $OUT/c4_probe.log 2>&1; echo "c4 probe rc=$?"; grep -v amdgpu.ids $OUT/c4_probe.log | head -60
