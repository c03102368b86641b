set -o pipefail
OUT=gpurun_out/r03k; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { echo tests failed; grep -E "^(FAILED|ERROR)" $OUT/tests.log | head -30; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
CRISPR_NW_QORDER=1 timeout -k 10 200 python scripts/diag/ab_call.py "CRISPR_NW_SPEC=1" "CRISPR_NW_SPEC=0" 20 > $OUT/ab_spec.log 2>&1 || { tail -20 $OUT/ab_spec.log; exit 1; }
tail -2 $OUT/ab_spec.log
CRISPR_NW_QORDER=0 timeout -k 10 200 python scripts/diag/ab_call.py "CRISPR_NW_SPEC=1" "CRISPR_NW_SPEC=0" 20 > $OUT/ab_spec_q0.log 2>&1 || { tail -20 $OUT/ab_spec_q0.log; exit 1; }
tail -2 $OUT/ab_spec_q0.log
CRISPR_NW_QORDER=1 CRISPR_NW_HOST_TIMING=1 timeout -k 10 200 python scripts/diag/ab_call.py "" "CRISPR_NW_TAIL=1" 4 > $OUT/ht.log 2>&1 || { tail -20 $OUT/ht.log; exit 1; }
grep -B8 "^nw host" $OUT/ht.log | tail -18
CRISPR_NW_QORDER=1 timeout -k 10 300 python scripts/diag/pooled_probe2.py pooled:6 c4:3 pooled:3 > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
grep -v amdgpu $OUT/probe.log
