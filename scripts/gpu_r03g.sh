set -o pipefail
OUT=gpurun_out/r03g; mkdir -p $OUT; export TMPDIR=/tmp
CRISPR_NW_TAIL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests_tail.log 2>&1 || { echo tail tests failed; tail -30 $OUT/tests_tail.log; exit 1; }
tail -1 $OUT/tests_tail.log
for q in 0 1; do
CRISPR_NW_QORDER=$q timeout -k 10 200 python scripts/diag/ab_call.py "" "CRISPR_NW_TAIL=1" 20 > $OUT/ab_q$q.log 2>&1 || { tail -20 $OUT/ab_q$q.log; exit 1; }
echo "qorder $q"; tail -2 $OUT/ab_q$q.log
done
for q in 0 1; do
CRISPR_NW_QORDER=$q timeout -k 10 200 python scripts/diag/ab_call.py "" "CRISPR_NW_TAIL=1" 5 pooled > $OUT/ab_pooled_q$q.log 2>&1 || { tail -20 $OUT/ab_pooled_q$q.log; exit 1; }
echo "pooled qorder $q"; tail -2 $OUT/ab_pooled_q$q.log
done
timeout -k 10 200 python -X faulthandler scripts/diag/pooled_probe2.py c4:2 > $OUT/c4_probe.log 2>&1; echo "c4 probe rc=$?"; grep -v amdgpu.ids $OUT/c4_probe.log | tail -30
