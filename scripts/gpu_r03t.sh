set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03t; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { echo tests failed; grep -E "^(FAILED|ERROR)" $OUT/tests.log | head -30; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_SPEC=0" 20 > $OUT/ab_spec.log 2>&1 || { tail -20 $OUT/ab_spec.log; exit 1; }
tail -2 $OUT/ab_spec.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_SPEC=0" 5 pooled > $OUT/ab_spec_p.log 2>&1 || { tail -20 $OUT/ab_spec_p.log; exit 1; }
tail -2 $OUT/ab_spec_p.log
