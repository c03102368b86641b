set -o pipefail
OUT=gpurun_out/r03i; mkdir -p $OUT; export TMPDIR=/tmp
for t in 0 1; do
CRISPR_NW_QORDER=1 CRISPR_NW_HOST_TIMING=1 timeout -k 10 200 python scripts/diag/ab_call.py "CRISPR_NW_TAIL=$t" "CRISPR_NW_TAIL=$t,CRISPR_NW_DIRECT=0" 6 > $OUT/ht_tail$t.log 2>&1 || { tail -20 $OUT/ht_tail$t.log; exit 1; }
echo "== tail $t"; grep -v "^nw host\|^  chunk" $OUT/ht_tail$t.log | tail -2; grep -B9 "^nw host" $OUT/ht_tail$t.log | tail -20
done
HIP_LAUNCH_BLOCKING=1 CRISPR_NW_SEGV_TRACE=1 timeout -k 10 300 python -X faulthandler scripts/diag/pooled_probe2.py c4:1 > $OUT/c4_probe.log 2>&1; echo "c4 probe rc=$?"; grep -v amdgpu.ids $OUT/c4_probe.log | head -40
